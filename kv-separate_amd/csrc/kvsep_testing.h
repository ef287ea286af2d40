// kvsep_testing.h -- test-only entry points of libkvsep_crc32c (not part of the public ABI, include/kvsep_crc32c.h).
// Exported so the test suite can reach them through ctypes, but inert unless the process runs with KVSEP_TEST_HOOKS=1
// (ADVICE r5): no production caller can make a batch call fail through them by accident.
#pragma once

#include "../../include/kvsep_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fault injection: the context's next batched call returns KVSEP_EHIP right after it enqueued its CRC kernel, before
 * the combine kernel of a planned batch -- the one point where an eager verify call's accumulators hold posts that no
 * kernel will publish.  The next verify call on the context resets them first, so its verdict is exact.  KVSEP_EINVAL
 * without KVSEP_TEST_HOOKS=1. */
int kvsep_crc32c_ctx_inject_failure(kvsep_crc32c_ctx* ctx);

#ifdef __cplusplus
}
#endif
