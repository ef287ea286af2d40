// host_crc.h -- the host legs of Extend (host_crc.cpp; no HIP).  Internal, not part of the public ABI.
#pragma once
#include <cstddef>
#include <cstdint>

namespace kvsep {

// Which leg host_crc runs on this CPU, chosen once at first use (KVSEP_HOST_CRC may force a slower one):
//   kFold      x86-64 with AVX-512F + VPCLMULQDQ (+ PCLMUL, SSE4.2): 512-bit carry-less folding, crc32 tail;
//   kSse42     x86-64 with SSE4.2: the crc32 instruction, three interleaved streams;
//   kPortable  any CPU: table-driven, 8 bytes per step (slicing-by-8; tables from gf2.h).
enum class HostLeg { kPortable = 0, kSse42 = 1, kFold = 2 };
HostLeg host_leg();
const char* host_leg_name(HostLeg leg);

// Extend(init, p[0, n)) on the host (util/crc32c.cc:276-377 semantics), on host_leg().
uint32_t host_crc(uint32_t init, const uint8_t* p, size_t n);
// The same on a named leg (tests and A/B); a leg this CPU cannot run falls back to the next slower one.
uint32_t host_crc_on(HostLeg leg, uint32_t init, const uint8_t* p, size_t n);

}  // namespace kvsep
