// The host legs of Extend built alone (tests/test_host_legs_cpu.py): with -DKVSEP_HOST_NO_X86 this is the form a
// non-x86 host compiles -- no x86 intrinsic, the portable leg only -- checked here against the oracle.
#include <cstddef>
#include <cstdint>

#include "host_crc.h"

extern "C" uint32_t hc_extend(uint32_t init, const char* p, size_t n) {
  return kvsep::host_crc(init, reinterpret_cast<const uint8_t*>(p), n);
}

extern "C" const char* hc_path() { return kvsep::host_leg_name(kvsep::host_leg()); }
