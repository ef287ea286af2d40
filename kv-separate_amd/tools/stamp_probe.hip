// stamp_probe.hip -- DIAGNOSTIC build of the CRC kernel with s_memtime stamps around the work-loop
// segments (cdna_hip_programming.md §7 "In-kernel stamps"); never used for timing numbers, only for the
// SHARES of a wave's time per item.  Build: hipcc --offload-arch=gfx950 -O3 -o stamp_probe stamp_probe.hip
// Usage: stamp_probe <block_len> <count>
#define KVSEP_STAMPS 1
#include "../csrc/crc32c_device.hip"
#include "../csrc/crc32c_host.cpp"

#include <algorithm>
#include <vector>

int main(int argc, char** argv) {
  const uint64_t blen = argc > 1 ? strtoull(argv[1], nullptr, 0) : 4096;
  const uint64_t count = argc > 2 ? strtoull(argv[2], nullptr, 0) : 65536;
  kvsep_crc32c_ctx* ctx = nullptr;
  if (kvsep_crc32c_ctx_create(0, &ctx)) { printf("ctx: %s\n", kvsep_last_error()); return 1; }
  uint8_t* data; uint64_t *doff, *dlen; uint32_t* out;
  hipMalloc(&data, blen * count + 64);
  kvsep_fill_splitmix64_device(nullptr, data, blen * count, 1, 0);
  std::vector<uint64_t> off(count), len(count, blen);
  for (uint64_t i = 0; i < count; ++i) off[i] = i * blen;
  hipMalloc(&doff, count * 8); hipMalloc(&dlen, count * 8); hipMalloc(&out, count * 4);
  hipMemcpy(doff, off.data(), count * 8, hipMemcpyHostToDevice);
  hipMemcpy(dlen, len.data(), count * 8, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; ++rep) {
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
    double s[3] = {0, 0, 0}, n = 0;
    double fill = 0, loop = 0, rt = 0, nw = 0;
    unsigned long long rmin = ~0ull, rmax = 0;
    for (int w = 0; w < 8192; ++w) {
      for (int k = 0; k < 3; ++k) s[k] += z[w * 8 + k];
      n += z[w * 8 + 3];
      if (z[w * 8 + 7]) {
        fill += z[w * 8 + 4]; loop += z[w * 8 + 5]; rt += z[w * 8 + 6]; nw += 1;
        rmin = std::min(rmin, z[w * 8 + 7]); rmax = std::max(rmax, z[w * 8 + 7] + z[w * 8 + 6]);
      }
    }
    printf("  event %.1f us | waves %.0f: mean fill %.0f cyc, loop %.0f cyc, wave span %.1f us (realtime), "
           "clock %.2f GHz | first entry -> last exit %.1f us\n", ms * 1e3, nw, fill / nw, loop / nw,
           rt / nw / 100.0, (fill + loop) / (rt / 100.0) / 1e3 / 1.0, (rmax - rmin) / 100.0);
    printf("len %lu count %lu: per item cycles  take-next %.0f  wait-data %.0f  compute %.0f  (items %.0f)\n",
           (unsigned long)blen, (unsigned long)count, s[0] / n, s[1] / n, s[2] / n, n);
  }
  return 0;
}
