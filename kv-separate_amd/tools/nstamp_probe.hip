// nstamp_probe.hip -- DIAGNOSTIC build of the narrow kernel with s_memrealtime stamps (100 MHz) per wave: entry,
// LDS fill + barrier done, after each 8-block group, exit.  Prints, relative to the earliest wave entry, the
// spread (p10 / p50 / p90 / max, us) of each stamp over all waves: where a small batch's time goes (launch ramp,
// fill, first data, last-group compute tail).  Never used for timing numbers.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o nstamp_probe nstamp_probe.hip
// Usage: nstamp_probe <block_len> <count> <kernel: 3 = narrow 16 waves, 4 = narrow 8 waves, 6 = claim>
#define KVSEP_STAMPS 1
#include "../csrc/crc32c_device.hip"
#include "../csrc/crc32c_host.cpp"
#include "../csrc/host_crc.cpp"
#include "../csrc/topology.cpp"

#include <algorithm>
#include <vector>

int main(int argc, char** argv) {
  const uint64_t blen = argc > 1 ? strtoull(argv[1], nullptr, 0) : 4096;
  const uint64_t count = argc > 2 ? strtoull(argv[2], nullptr, 0) : 65536;
  const int kernel = argc > 3 ? atoi(argv[3]) : 3;
  kvsep_crc32c_ctx* ctx = nullptr;
  if (kvsep_crc32c_ctx_create(0, &ctx)) { printf("ctx: %s\n", kvsep_last_error()); return 1; }
  kvsep_crc32c_ctx_set_kernel(ctx, kernel);
  uint8_t* data; uint64_t *doff, *dlen; uint32_t* out;
  hipMalloc(&data, blen * count + 64);
  kvsep_fill_splitmix64_device(nullptr, data, blen * count, 1, 0);
  std::vector<uint64_t> off(count), len(count, blen);
  for (uint64_t i = 0; i < count; ++i) off[i] = i * blen;
  hipMalloc(&doff, count * 8); hipMalloc(&dlen, count * 8); hipMalloc(&out, count * 4);
  hipMemcpy(doff, off.data(), count * 8, hipMemcpyHostToDevice);
  hipMemcpy(dlen, len.data(), count * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 4; ++rep) {
    std::vector<unsigned long long> z(8192 * 8, 0);
    hipMemcpyToSymbol(HIP_SYMBOL(kvsep::g_kvsep_stamps), z.data(), z.size() * 8);
    hipEvent_t ev0, ev1;
    hipEventCreate(&ev0); hipEventCreate(&ev1);
    hipEventRecord(ev0, nullptr);
    kvsep_crc32c_batch_device(ctx, nullptr, data, doff, dlen, nullptr, out, count, blen * count, blen);
    hipEventRecord(ev1, nullptr);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, ev0, ev1);
    hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(kvsep::g_kvsep_stamps), z.size() * 8);
    unsigned long long t0 = ~0ull;
    int nw = 0;
    for (int w = 0; w < 8192; ++w)
      if (z[w * 8]) { t0 = std::min(t0, z[w * 8]); ++nw; }
    printf("rep %d: event %.2f us, %d waves\n", rep, ms * 1e3, nw);
    const char* names[8] = {"entry", "fill done", "group 1", "group 2", "group 3", "group 4", "group 5", "exit"};
    for (int k = 0; k < 8; ++k) {
      std::vector<double> v;
      for (int w = 0; w < 8192; ++w)
        if (z[w * 8] && z[w * 8 + k]) v.push_back((z[w * 8 + k] - t0) / 100.0);
      if (v.empty()) continue;
      std::sort(v.begin(), v.end());
      auto q = [&](double f) { return v[std::min(v.size() - 1, size_t(f * v.size()))]; };
      printf("  %-9s n=%5zu  p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us\n", names[k], v.size(), q(0.1), q(0.5),
             q(0.9), v.back());
    }
    // exit time by XCD (workgroup id mod 8) and by wave slot within the workgroup: is the tail spatial?
    const int wpg = nw / 256 > 0 ? nw / 256 : 1;
    for (int by = 0; by < 2; ++by) {
      const int ng = by == 0 ? 8 : wpg;
      printf("  exit by %s:", by == 0 ? "XCD " : "wave");
      for (int gi = 0; gi < ng; ++gi) {
        std::vector<double> v;
        for (int w = 0; w < nw; ++w) {
          const int wg = w / wpg, ws = w % wpg;
          if ((by == 0 ? wg % 8 : ws) == gi && z[w * 8 + 7]) v.push_back((z[w * 8 + 7] - t0) / 100.0);
        }
        std::sort(v.begin(), v.end());
        if (!v.empty()) printf(" %d:%.1f/%.1f", gi, v[v.size() / 2], v.back());
      }
      printf("  (median/max us)\n");
    }
  }
  return 0;
}
