"""Seeded randomised parity sweep (kv-separate_amd/tools/soak.py, a fixed number of cases): random batch shapes --
up to 200 K blocks, uniform / Zipf / ~4 KiB / tiny / mixed lengths, packed or overlapping offsets, random or no
inits -- through every kernel choice, hint kind (none, exact, loose, understated), three piece sizes, the verify
form with planted mismatches, the host-span, pointer-per-block and device-group host forms, a hipGraph-captured
device call and the SST trailer / read-check forms; every result bit-exact against the oracle (util/crc32c.cc:276-377 restated) on the same bytes.
The time-bounded tool found the sorted-window verify bug of round 2; this keeps a slice of it in
the suite."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kv-separate_amd", "tools"))
import soak  # noqa: E402


@pytest.mark.parametrize("seed", [20261017, 7])
def test_seeded_soak(seed):
    cases, blocks, nbytes = soak.soak(seed, max_cases=300, log=lambda m: None, pool=64 << 20)
    assert cases == 300 and blocks > 0
