// nstamp_probe.hip -- DIAGNOSTIC build of the narrow kernel with s_memrealtime stamps (100 MHz) per wave: entry,
// LDS fill + barrier done, after each 8-block group, exit.  Prints, relative to the earliest wave entry, the
// spread (p10 / p50 / p90 / max, us) of each stamp over all waves: where a small batch's time goes (launch ramp,
// fill, first data, last-group compute tail).  Never used for timing numbers.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o nstamp_probe nstamp_probe.hip
// Usage: nstamp_probe <block_len> <count> <kernel: 3 = narrow 16 waves, 4 = narrow 8 waves, 6 = claim,
//                                              0 = the streaming-read ceiling over the same bytes>
#define KVSEP_STAMPS 1
#include "../csrc/crc32c_device.hip"
#include "../csrc/crc32c_host.cpp"
#include "../csrc/host_crc.cpp"
#include "../csrc/topology.cpp"

#include <algorithm>
#include <vector>

// kernel 0: stream_read_kernel (crc32c_device.hip) with the same per-wave stamps -- [0] entry, [1] the first round's
// data in registers (its loads issued at entry: nothing to fill), [2..6] after rounds 2, 4, 8, 12, 16 of its 1 MiB
// chunk, [7] exit -- so the CRC kernels' ramp and drain can be read against the streaming ceiling's own (round 5).
// kLds (kernel 5): the same kernel holding the CRC kernels' 157 KiB LDS image (unused), to see whether a workgroup that
// takes a whole CU's LDS is dispatched later than one that takes none.
template <bool kLds>
__global__ void __launch_bounds__(512) stamped_stream_kernel(uintptr_t src, uint64_t n16, uint32_t* sink) {
  using namespace kvsep;
  __shared__ uint8_t lds_pad[kLds ? kLdsBytes : 16];
  constexpr uint32_t kWavesPerWg = 8;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(w);
  KVSEP_NSTAMP_ENTRY();
  constexpr uint64_t kChunk16 = (1u << 20) / 16;
  constexpr uint64_t kStep = 8 * kStreamRows * kRowBytes;
  const uint64_t nchunks = n16 / kChunk16;
  uint32_t acc = 0;
  int round = 0;
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uintptr_t p = src + c * kChunk16 * 16 + uintptr_t(w) * kRowBytes + lane * 16u;
#pragma unroll 1
    for (uint64_t r = 0; r < kChunk16 * 16; r += kStep) {
      uint4 v[kStreamRows];
#pragma unroll
      for (int u = 0; u < kStreamRows; ++u) v[u] = ld16<true>(p + r + uint64_t(u) * 8 * kRowBytes);
#pragma unroll
      for (int u = 0; u < kStreamRows; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
      ++round;
      if (round == 1) {
        asm volatile("" : "+v"(acc));
        KVSEP_NSTAMP(1);
      } else if (round == 2 || round == 4 || round == 8 || round == 12 || round == 16) {
        asm volatile("" : "+v"(acc));
        KVSEP_NSTAMP(round == 2 ? 2 : round == 4 ? 3 : round == 8 ? 4 : round == 12 ? 5 : 6);
      }
    }
  }
  KVSEP_NSTAMP(7);
  if (acc == 0x9e3779b9u) {
    lds_pad[threadIdx.x] = uint8_t(acc);
    __syncthreads();
    atomicXor(sink, acc ^ lds_pad[threadIdx.x ^ 1u]);
  }
}

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
    std::vector<unsigned long long> z(8192 * 8, 0), f(8192, 0);
    hipMemcpyToSymbol(HIP_SYMBOL(kvsep::g_kvsep_stamps), z.data(), z.size() * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(kvsep::g_kvsep_first), f.data(), f.size() * 8);
    hipEvent_t ev0, ev1;
    hipEventCreate(&ev0); hipEventCreate(&ev1);
    hipEventRecord(ev0, nullptr);
    if (kernel == 0)
      stamped_stream_kernel<false><<<256, 512>>>(reinterpret_cast<uintptr_t>(data), blen * count / 16, out);
    else if (kernel == 5)
      stamped_stream_kernel<true><<<256, 512>>>(reinterpret_cast<uintptr_t>(data), blen * count / 16, out);
    else
      kvsep_crc32c_batch_device(ctx, nullptr, data, doff, dlen, nullptr, out, count, blen * count, blen);
    hipEventRecord(ev1, nullptr);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, ev0, ev1);
    hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(kvsep::g_kvsep_stamps), z.size() * 8);
    hipMemcpyFromSymbol(f.data(), HIP_SYMBOL(kvsep::g_kvsep_first), f.size() * 8);
    unsigned long long t0 = ~0ull;
    int nw = 0;
    for (int w = 0; w < 8192; ++w)
      if (z[w * 8]) { t0 = std::min(t0, z[w * 8]); ++nw; }
    printf("rep %d: event %.2f us, %d waves\n", rep, ms * 1e3, nw);
    const char* names[8] = {"entry", "fill done", "group 1", "group 2", "group 3", "group 4", "group 5", "exit"};
    const char* snames[8] = {"entry", "1st data", "round 2", "round 4", "round 8", "round 12", "round 16", "exit"};
    if (kernel == 0 || kernel == 5) std::copy(snames, snames + 8, names);
    for (int k = 0; k < 8; ++k) {
      std::vector<double> v;
      for (int w = 0; w < 8192; ++w)
        if (z[w * 8] && z[w * 8 + k]) v.push_back((z[w * 8 + k] - t0) / 100.0);
      if (v.empty()) continue;
      std::sort(v.begin(), v.end());
      auto q = [&](double f) { return v[std::min(v.size() - 1, size_t(f * v.size()))]; };
      printf("  %-9s n=%5zu  p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us\n", names[k], v.size(), q(0.1), q(0.5),
             q(0.9), v.back());
      if (k == 1 && kernel != 0 && kernel != 5) {  // the narrow kernels' first HBM data (KVSEP_NSTAMP_FIRST_DATA)
        std::vector<double> u;
        for (int w = 0; w < 8192; ++w)
          if (z[w * 8] && f[w]) u.push_back((f[w] - t0) / 100.0);
        std::sort(u.begin(), u.end());
        if (!u.empty())
          printf("  %-9s n=%5zu  p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us\n", "1st data", u.size(),
                 u[u.size() / 10], u[u.size() / 2], u[u.size() * 9 / 10], u.back());
      }
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
