// stamp_probe.hip -- DIAGNOSTIC build of the wide CRC kernel with s_memrealtime stamps (100 MHz) per wave: entry,
// LDS fill done, exit, the ticks spent in whole-block items and in pieces of split blocks, and the last item of the
// wave (crc32c_pieces_kernel's KVSEP_STAMPS block).  Never used for timing numbers, only for a per-wave time budget.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o stamp_probe stamp_probe.hip
// Usage: stamp_probe <layout.bin> <stamps_out.bin> [reps]
//   layout.bin: u64 count, then off[count], len[count] (tools/wstamp_analyze.py writes it); the span is filled with
//   the splitmix64 stream on the device.  stamps_out.bin: the 8192 x 8 u64 stamp words of the last rep.
#define KVSEP_STAMPS 1
#include "../csrc/crc32c_device.hip"
#include "../csrc/crc32c_host.cpp"
#include "../csrc/host_crc.cpp"
#include "../csrc/topology.cpp"

#include <algorithm>
#include <vector>

int main(int argc, char** argv) {
  if (argc < 3) {
    printf("usage: stamp_probe <layout.bin> <stamps_out.bin> [reps]\n");
    return 2;
  }
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  FILE* f = fopen(argv[1], "rb");
  if (!f) { printf("cannot open %s\n", argv[1]); return 1; }
  uint64_t count = 0;
  if (fread(&count, 8, 1, f) != 1) return 1;
  std::vector<uint64_t> off(count), len(count);
  if (fread(off.data(), 8, count, f) != count || fread(len.data(), 8, count, f) != count) return 1;
  fclose(f);
  uint64_t span = 0, total = 0, maxlen = 0;
  for (uint64_t i = 0; i < count; ++i) {
    span = std::max(span, off[i] + len[i]);
    total += len[i];
    maxlen = std::max(maxlen, len[i]);
  }
  kvsep_crc32c_ctx* ctx = nullptr;
  if (kvsep_crc32c_ctx_create(0, &ctx)) { printf("ctx: %s\n", kvsep_last_error()); return 1; }
  uint8_t* data; uint64_t *doff, *dlen; uint32_t* out;
  if (hipMalloc(&data, span + 64) != hipSuccess) { printf("hipMalloc %lu failed\n", (unsigned long)span); return 1; }
  kvsep_fill_splitmix64_device(nullptr, data, span, 1, 0);
  hipMalloc(&doff, count * 8); hipMalloc(&dlen, count * 8); hipMalloc(&out, count * 4);
  hipMemcpy(doff, off.data(), count * 8, hipMemcpyHostToDevice);
  hipMemcpy(dlen, len.data(), count * 8, hipMemcpyHostToDevice);
  std::vector<unsigned long long> z(8192 * 8, 0);
  for (int rep = 0; rep < reps; ++rep) {
    std::fill(z.begin(), z.end(), 0ull);
    hipMemcpyToSymbol(HIP_SYMBOL(kvsep::g_kvsep_stamps), z.data(), z.size() * 8);
    hipEvent_t ev0, ev1;
    hipEventCreate(&ev0); hipEventCreate(&ev1);
    hipEventRecord(ev0, nullptr);
    const int rc = kvsep_crc32c_batch_device(ctx, nullptr, data, doff, dlen, nullptr, out, count, total, maxlen);
    hipEventRecord(ev1, nullptr);
    hipDeviceSynchronize();
    if (rc) { printf("batch: %s\n", kvsep_last_error()); return 1; }
    float ms = 0;
    hipEventElapsedTime(&ms, ev0, ev1);
    printf("rep %d: %.3f ms (%.1f GB/s over %lu blocks, %lu B)\n", rep, ms, total / (ms * 1e6), (unsigned long)count,
           (unsigned long)total);
    fflush(stdout);
  }
  hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(kvsep::g_kvsep_stamps), z.size() * 8);
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 1;
  fwrite(z.data(), 8, z.size(), o);
  fclose(o);
  return 0;
}
