// stamp_probe.hip -- DIAGNOSTIC build of the CRC kernel with s_memtime stamps around the work-loop
// segments (cdna_hip_programming.md §7 "In-kernel stamps"); never used for timing numbers, only for the
// SHARES of a wave's time per item.  Build: hipcc --offload-arch=gfx950 -O3 -o stamp_probe stamp_probe.hip
// Usage: stamp_probe <block_len> <count>
#define KVSEP_STAMPS 1
#include "../csrc/crc32c_device.hip"
#include "../csrc/crc32c_host.cpp"

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
    std::vector<unsigned long long> z(8192 * 4, 0);
    hipMemcpyToSymbol(HIP_SYMBOL(kvsep::g_kvsep_stamps), z.data(), z.size() * 8);
    kvsep_crc32c_batch_device(ctx, nullptr, data, doff, dlen, nullptr, out, count, blen * count, blen);
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(kvsep::g_kvsep_stamps), z.size() * 8);
    double s[3] = {0, 0, 0}, n = 0;
    for (int w = 0; w < 8192; ++w) { for (int k = 0; k < 3; ++k) s[k] += z[w * 4 + k]; n += z[w * 4 + 3]; }
    printf("len %lu count %lu: per item cycles  take-next %.0f  wait-data %.0f  compute %.0f  (items %.0f)\n",
           (unsigned long)blen, (unsigned long)count, s[0] / n, s[1] / n, s[2] / n, n);
  }
  return 0;
}
