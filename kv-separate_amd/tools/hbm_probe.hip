// hbm_probe.hip -- measurement tool (not part of the library): which read pattern gets closest to the
// MI355X HBM peak?  Times read-only kernels over a large buffer with hipEvents and prints GB/s.
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe hbm_probe.hip ; run: ./hbm_probe [GiB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gu32x4;

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));                         \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <int U, bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  gu32x4* g = reinterpret_cast<gu32x4*>(reinterpret_cast<uintptr_t>(p));
  if constexpr (NT) return __builtin_nontemporal_load(g);
  return *g;
}

// A: grid-stride, U independent loads in flight per thread
template <int U, bool NT>
__global__ void k_gridstride(const u32x4* src, size_t n16, unsigned* sink) {
  u32x4 acc = {0, 0, 0, 0};
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<U, NT>(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (; i < n16; i += stride) acc ^= ld<U, NT>(src + i);
  unsigned a = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (a == 0x12345678u) atomicXor(sink, a);
}

// B: each wave owns a contiguous chunk of `chunk16` x 16 B, read as 1 KiB rows, U rows in flight.
template <int U, bool NT>
__global__ void k_wavechunk(const u32x4* src, size_t n16, size_t chunk16, unsigned* sink) {
  const unsigned lane = threadIdx.x & 63;
  const size_t wave = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const size_t nwaves = (size_t(gridDim.x) * blockDim.x) >> 6;
  u32x4 acc = {0, 0, 0, 0};
  const size_t nchunks = n16 / chunk16;
  if (chunk16 % (64 * U)) return;  // whole U-row steps only (else reads overrun the buffer)
  for (size_t c = wave; c < nchunks; c += nwaves) {
    const u32x4* p = src + c * chunk16 + lane;
    for (size_t r = 0; r < chunk16; r += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld<U, NT>(p + r + 64 * u);
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
    }
  }
  unsigned a = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (a == 0x12345678u) atomicXor(sink, a);
}

// B': as B, but the loads are inline asm with an explicit gfx950 cache policy (POL: 0 = nt, 1 = sc1 nt,
// 2 = sc0 sc1 nt, 3 = sc0 nt), all U rows waited for at once.
template <int POL>
__device__ __forceinline__ u32x4 ld_pol(const u32x4* p) {
  u32x4 v;
  if constexpr (POL == 0) asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
  else if constexpr (POL == 1) asm volatile("global_load_dwordx4 %0, %1, off sc1 nt" : "=v"(v) : "v"(p) : "memory");
  else if constexpr (POL == 2) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt" : "=v"(v) : "v"(p) : "memory");
  else asm volatile("global_load_dwordx4 %0, %1, off sc0 nt" : "=v"(v) : "v"(p) : "memory");
  return v;
}
template <int U, int POL>
__global__ void k_wavechunk_pol(const u32x4* src, size_t n16, size_t chunk16, unsigned* sink) {
  const unsigned lane = threadIdx.x & 63;
  const size_t wave = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const size_t nwaves = (size_t(gridDim.x) * blockDim.x) >> 6;
  u32x4 acc = {0, 0, 0, 0};
  const size_t nchunks = n16 / chunk16;
  if (chunk16 % (64 * U)) return;
  for (size_t c = wave; c < nchunks; c += nwaves) {
    const u32x4* p = src + c * chunk16 + lane;
    for (size_t r = 0; r < chunk16; r += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld_pol<POL>(p + r + 64 * u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
    }
  }
  unsigned a = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (a == 0x12345678u) atomicXor(sink, a);
}

// C: each workgroup owns a contiguous chunk; its waves interleave rows (wave w reads rows w, w+W, ...).
template <int U, bool NT>
__global__ void k_wgchunk(const u32x4* src, size_t n16, size_t chunk16, unsigned* sink) {
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = blockDim.x >> 6;
  u32x4 acc = {0, 0, 0, 0};
  const size_t nchunks = n16 / chunk16;
  if (chunk16 % (size_t(64) * W * U)) return;  // a chunk must hold whole U-row steps (else reads overrun the buffer)
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const u32x4* p = src + c * chunk16 + lane + 64 * w;
    for (size_t r = 0; r < chunk16; r += size_t(64) * W * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ld<U, NT>(p + r + size_t(64) * W * u);
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
    }
  }
  unsigned a = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (a == 0x12345678u) atomicXor(sink, a);
}

__global__ void k_fill_random(u32x4* dst, size_t n16) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    dst[i] = u32x4{unsigned(z), unsigned(z >> 32), unsigned(z * 3), unsigned((z * 3) >> 32)};
  }
}

template <typename F>
double timeit(F f, int reps, double bytes) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int i = 0; i < reps; ++i) {
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return bytes / (ts[ts.size() / 2] * 1e-3) / 1e9;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 32.0;
  const size_t bytes = size_t(gib * (1ull << 30));
  const size_t n16 = bytes / 16;
  u32x4* buf;
  unsigned* sink;
  if (argc > 2 && argv[2][0] == 'c') {  // physically contiguous allocation (hipDeviceMallocContiguous)
    const hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&buf), bytes, hipDeviceMallocContiguous);
    printf("contiguous allocation of %.1f GiB: %s\n", gib, hipGetErrorString(e));
    if (e != hipSuccess) return 0;
  } else {
    CHECK(hipMalloc(&buf, bytes));
  }
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(buf, 0x5a, bytes));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int reps = 5;
  printf("buffer %.1f GiB, %d CUs\n", gib, cus);
#define GS(U, NT, BLK, WGPERCU)                                                                          \
  printf("gridstride U=%d nt=%d blk=%d wg/cu=%d : %.1f GB/s\n", U, NT, BLK, WGPERCU,                   \
         timeit([&] { k_gridstride<U, NT><<<cus * WGPERCU, BLK>>>(buf, n16, sink); }, reps, double(bytes)))
#define WC(U, NT, BLK, WGPERCU, CH)                                                                      \
  printf("wavechunk U=%d nt=%d blk=%d wg/cu=%d chunk=%zu KiB : %.1f GB/s\n", U, NT, BLK, WGPERCU,     \
         size_t(CH) / 1024,                                                                            \
         timeit([&] { k_wavechunk<U, NT><<<cus * WGPERCU, BLK>>>(buf, n16, size_t(CH) / 16, sink); }, reps, \
                double(bytes)))
#define WG(U, NT, BLK, WGPERCU, CH)                                                                       \
  printf("wgchunk U=%d nt=%d blk=%d wg/cu=%d chunk=%zu KiB : %.1f GB/s\n", U, NT, BLK, WGPERCU,        \
         size_t(CH) / 1024,                                                                              \
         timeit([&] { k_wgchunk<U, NT><<<cus * WGPERCU, BLK>>>(buf, n16, size_t(CH) / 16, sink); }, reps, \
                double(bytes)))
#define WP(U, POL, BLK, WGPERCU, CH)                                                                     \
  printf("wavechunk_pol U=%d pol=%d blk=%d wg/cu=%d chunk=%zu KiB : %.1f GB/s\n", U, POL, BLK, WGPERCU,  \
         size_t(CH) / 1024,                                                                             \
         timeit([&] { k_wavechunk_pol<U, POL><<<cus * WGPERCU, BLK>>>(buf, n16, size_t(CH) / 16, sink); }, \
                reps, double(bytes)))
  if (argc > 2 && (argv[2][0] == 'c' || argv[2][0] == 'p')) {  // allocation kind: contiguous ('c') vs plain ('p')
    k_fill_random<<<cus * 8, 256>>>(buf, n16);
    CHECK(hipDeviceSynchronize());
    for (int i = 0; i < 2; ++i) {
      WC(16, true, 512, 2, 1 << 20);
      WG(8, true, 512, 1, 1 << 20);
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'r') {  // constant vs random data, chunk size, at the best rows-in-flight
    WC(16, true, 512, 2, 1 << 20);
    WC(16, true, 512, 2, 128 << 10);
    WC(8, true, 512, 1, 128 << 10);
    k_fill_random<<<cus * 8, 256>>>(buf, n16);
    CHECK(hipDeviceSynchronize());
    printf("random data:\n");
    WC(16, true, 512, 2, 1 << 20);
    WC(16, true, 512, 2, 128 << 10);
    WC(8, true, 512, 1, 128 << 10);
    WC(4, true, 512, 1, 128 << 10);
    WC(8, true, 1024, 1, 1 << 20);
    WG(16, true, 512, 2, 1 << 20);
    WG(8, true, 512, 2, 1 << 20);
    WG(4, true, 512, 1, 1 << 20);
    WG(8, true, 512, 1, 1 << 20);
    WG(8, true, 512, 1, 128 << 10);
    WG(4, true, 512, 1, 128 << 10);
    WG(2, true, 512, 1, 1 << 20);
    WG(8, true, 1024, 1, 1 << 20);
    WG(4, true, 1024, 1, 1 << 20);
    return 0;
  }
  if (argc > 2) {  // rows-in-flight and cache-policy sweep on 1 MiB per-wave chunks
    WC(4, true, 1024, 1, 1 << 20);
    WC(8, true, 1024, 1, 1 << 20);
    WC(16, true, 1024, 1, 1 << 20);
    WC(8, true, 512, 2, 1 << 20);
    WC(16, true, 512, 2, 1 << 20);
    WC(8, true, 768, 1, 1 << 20);
    WP(8, 0, 1024, 1, 1 << 20);
    WP(8, 1, 1024, 1, 1 << 20);
    WP(8, 2, 1024, 1, 1 << 20);
    WP(8, 3, 1024, 1, 1 << 20);
    WP(16, 0, 1024, 1, 1 << 20);
    WP(16, 2, 1024, 1, 1 << 20);
    WC(8, true, 1024, 1, 256 << 10);
    WC(8, false, 1024, 1, 1 << 20);
    return 0;
  }
  WC(4, true, 1024, 1, 4 << 10);
  WC(4, true, 1024, 1, 16 << 10);
  WC(4, true, 1024, 1, 64 << 10);
  WC(4, true, 1024, 1, 1 << 20);
  WC(4, false, 1024, 1, 4 << 10);
  WC(4, true, 256, 8, 4 << 10);
  WC(4, true, 512, 4, 4 << 10);
  WG(4, true, 1024, 1, 64 << 10);
  WG(4, true, 1024, 1, 256 << 10);
  WG(1, true, 1024, 1, 16 << 10);
  GS(4, true, 256, 8);
  return 0;
}
