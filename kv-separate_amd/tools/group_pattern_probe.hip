// group_pattern_probe.hip -- measurement tool (not part of the library): is the narrow kernels' row pattern what keeps
// config 2 below the streaming ceiling's steady state (round 5)?  Read-only kernels over a small batch (default 256
// MiB of 4 KiB blocks, config 2), no CRC arithmetic, each timed as 20 back-to-back launches captured in one hipGraph
// (bench.py's config-2 form).  Every pattern reads every byte once, 256 workgroups x 8 waves, each workgroup owning
// the same contiguous run of 32 KiB groups (8 blocks) as crc32c_narrow_claim_kernel, wave w taking groups w, w + 8, ...:
//   0 slot rows   the claim kernel's: one load instruction reads one 128-B line of each of the group's 8 blocks
//                 (lanes 8s..8s+7 on block s), 32 such rows per group
//   1 1 KiB rows  the group read as 32 contiguous 1 KiB rows (the wide kernel's / the ceiling's row shape)
//   2 2-line slots each instruction reads two consecutive 128-B lines of 4 of the group's blocks (16 lanes per block)
//   3 stream      stream_read_kernel's pattern: the workgroup's 8 waves interleave 1 KiB rows of its 1 MiB run
//   4-7 (round 6) slot rows with each block's rows read in a rotated order -- by 4 rows per slot, per wave, per
//                 workgroup, or by 16 rows on every other wave -- so the lines in flight do not all sit at one offset
//                 in their 4 KiB blocks (is config 2's deficit address-channel camping?)
//   8 (round 6)   slot rows with the workgroup's 8 waves on the same 8 blocks: wave w reads rows 4w..4w+3 of each, so
//                 the workgroup's loads in flight sit in one 32 KiB window, as the streaming pattern's do
//   9 (round 6)   as 8 with wave w on rows w, w + 8, w + 16, w + 24
//   10, 11        slot rows with the waves in teams of 4 / 2, each team on its own group and each wave on a consecutive
//                 share of the group's rows: 2 / 4 groups in flight per workgroup (64 / 128 KiB windows)
// kRows loads in flight per wave (issued together, then consumed), as the kernels' row groups.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o group_pattern_probe group_pattern_probe.hip
// Usage: group_pattern_probe [MiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ldnt(uintptr_t a) { return __builtin_nontemporal_load(reinterpret_cast<gu32x4*>(a)); }

constexpr uint64_t kGroup = 32768, kBlock = 4096;

template <int kMode, int kRows>
__global__ void __launch_bounds__(512) pattern_kernel(uintptr_t src, uint64_t nbytes, unsigned* sink) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t groups = nbytes / kGroup;
  const uint64_t per = (groups + gridDim.x - 1) / gridDim.x;
  const uint64_t g0 = uint64_t(blockIdx.x) * per, g1 = g0 + per < groups ? g0 + per : groups;
  u32x4 acc = {0, 0, 0, 0};
  if (kMode == 10 || kMode == 11) {  // round 6: the workgroup's waves in teams of 4 (10) or 2 (11), each team on its own
    // group, wave t of a team reading its consecutive share of each block's 32 rows (8 or 16 rows, kRows at a time)
    constexpr uint32_t kTeam = kMode == 10 ? 4 : 2, kTeams = 8 / kTeam, kShare = 32 / kTeam;
    const uint32_t team = w / kTeam, t = w % kTeam;
    for (uint64_t g = g0 + team; g < g1; g += kTeams) {
      const uintptr_t gb = src + g * kGroup;
      for (uint32_t r = 0; r < kShare; r += kRows) {
        u32x4 v[kRows];
#pragma unroll
        for (int u = 0; u < kRows; ++u)
          v[u] = ldnt(gb + (lane >> 3) * kBlock + (t * kShare + r + u) * 128u + (lane & 7u) * 16u);
#pragma unroll
        for (int u = 0; u < kRows; ++u) acc ^= v[u];
      }
    }
  } else if (kMode == 8 || kMode == 9) {  // round 6: slot rows, the workgroup's 8 waves on the SAME 8 blocks per round (32
    // KiB window): wave w reads rows 4w .. 4w+3 (8) or rows w, w+8, w+16, w+24 (9) of each of the round's 8 blocks
    for (uint64_t g = g0; g < g1; ++g) {
      const uintptr_t gb = src + g * kGroup;
      u32x4 v[kRows];
#pragma unroll
      for (int u = 0; u < kRows; ++u) {
        const uint32_t row = kMode == 8 ? uint32_t(kRows) * w + u : w + 8u * u;
        v[u] = ldnt(gb + (lane >> 3) * kBlock + row * 128u + (lane & 7u) * 16u);
      }
#pragma unroll
      for (int u = 0; u < kRows; ++u) acc ^= v[u];
    }
  } else if (kMode == 3) {  // the workgroup's run as one contiguous span, 8 waves interleaving 1 KiB rows
    const uintptr_t base = src + g0 * kGroup, end = src + g1 * kGroup;
    for (uintptr_t r = base + uintptr_t(w) * 1024; r < end; r += uintptr_t(8) * 1024 * kRows) {
      u32x4 v[kRows];
#pragma unroll
      for (int u = 0; u < kRows; ++u) {
        const uintptr_t a = r + uintptr_t(u) * 8 * 1024;
        v[u] = ldnt((a < end ? a : base) + lane * 16u);
      }
#pragma unroll
      for (int u = 0; u < kRows; ++u) acc ^= v[u];
    }
  } else {
    for (uint64_t g = g0 + w; g < g1; g += 8) {
      const uintptr_t gb = src + g * kGroup;
      for (int r = 0; r < 32; r += kRows) {
        u32x4 v[kRows];
#pragma unroll
        for (int u = 0; u < kRows; ++u) {
          const uint32_t row = r + u;
          uintptr_t a;
          if (kMode == 0) a = gb + (lane >> 3) * kBlock + row * 128u + (lane & 7u) * 16u;
          else if (kMode >= 4) {  // round 6: slot rows with the row order rotated per slot / wave / workgroup
            const uint32_t rot = kMode == 4 ? 4u * (lane >> 3) : kMode == 5 ? 4u * w : kMode == 6 ? 4u * (blockIdx.x & 7u)
                                                                                            : 16u * (w & 1u);
            a = gb + (lane >> 3) * kBlock + ((row + rot) & 31u) * 128u + (lane & 7u) * 16u;
          }
          else if (kMode == 1) a = gb + row * 1024u + lane * 16u;
          else a = gb + ((row & 1u) * 4u + (lane >> 4)) * kBlock + (row >> 1) * 256u + (lane & 15u) * 16u;
          v[u] = ldnt(a);
        }
#pragma unroll
        for (int u = 0; u < kRows; ++u) acc ^= v[u];
      }
    }
  }
  const unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) atomicXor(sink, x);
}

template <int kMode, int kRows>
double time_us(uintptr_t src, uint64_t n, unsigned* sink, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  pattern_kernel<kMode, kRows><<<256, 512, 0, st>>>(src, n, sink);
  CK(hipStreamSynchronize(st));
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 20; ++i) pattern_kernel<kMode, kRows><<<256, 512, 0, st>>>(src, n, sink);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  double best = 1e30;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms * 1e3 / 20 < best ? ms * 1e3 / 20 : best;
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return best;
}

int main(int argc, char** argv) {
  const uint64_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 256;
  const uint64_t n = mib << 20;
  void* d = nullptr;
  unsigned* sink = nullptr;
  CK(hipMalloc(&d, n + 4096));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(d, 0x5a, n));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const uintptr_t s = reinterpret_cast<uintptr_t>(d);
  for (int round = 0; round < 3; ++round) {
    const double t[16] = {time_us<0, 4>(s, n, sink, st), time_us<0, 8>(s, n, sink, st), time_us<1, 4>(s, n, sink, st),
                          time_us<1, 8>(s, n, sink, st), time_us<2, 4>(s, n, sink, st), time_us<2, 8>(s, n, sink, st),
                          time_us<3, 4>(s, n, sink, st), time_us<3, 8>(s, n, sink, st), time_us<4, 4>(s, n, sink, st),
                          time_us<5, 4>(s, n, sink, st), time_us<6, 4>(s, n, sink, st), time_us<7, 4>(s, n, sink, st),
                          time_us<8, 4>(s, n, sink, st), time_us<9, 4>(s, n, sink, st), time_us<10, 4>(s, n, sink, st),
                          time_us<11, 4>(s, n, sink, st)};
    const char* nm[16] = {"slot rows x4", "slot rows x8", "1KiB rows x4", "1KiB rows x8", "2-line slots x4",
                          "2-line slots x8", "stream x4", "stream x8", "slot rows x4 rot/slot", "slot rows x4 rot/wave",
                          "slot rows x4 rot/wg", "slot rows x4 half/wave", "slot rows x4 wg-window",
                          "slot rows x4 wg-window il", "slot rows x4 teams of 4", "slot rows x4 teams of 2"};
    for (int i = 0; i < 16; ++i)
      std::printf("{\"round\": %d, \"mib\": %llu, \"pattern\": \"%s\", \"us\": %.2f, \"TBps\": %.3f}\n", round,
                  (unsigned long long)mib, nm[i], t[i], double(n) / (t[i] * 1e-6) / 1e12);
    std::fflush(stdout);
  }
  return 0;
}
