"""CPU checks of the N-rank reference goldens and of bench.py's result checker, no GPU:

  * full_cfg4_ranks.json's block ranges are exactly the ranges bench.py's config-4 ranks get today
    (kvsep_crc32c_partition over the N x 2^20 global batch), so the digests cannot go stale silently;
  * its digests agree with the per-block reference file full_cfg4.u32 wherever a range lies inside it;
  * check_results: a full N-rank result set drawn from the golden files passes with every block checked and none
    sampled; one flipped result is one mismatch (per block) or one mismatching range (by digest).
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import kvsep  # noqa: E402
from kvsep import shard  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def _json():
    with open(os.path.join(GOLDEN, "full_cfg4_ranks.json")) as f:
        return json.load(f)


def _u32(name):
    return np.fromfile(os.path.join(GOLDEN, name), dtype="<u4")


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_cfg4_rank_ranges_are_the_bench_partition(world):
    parts = _json()["ranks"][str(world)]
    assert len(parts) == world
    for r in range(world):
        plan = bench.Plan("4", world, r)
        (base, ib), = plan.passes
        assert (parts[r]["lo"], parts[r]["hi"]) == (ib, ib + plan.count)
        assert parts[r]["bytes"] == plan.useful
        assert plan.digest == parts[r]
    assert parts[0]["lo"] == 0 and parts[-1]["hi"] == world * (1 << 20)


def test_cfg4_digests_agree_with_per_block_reference():
    c4 = _u32("full_cfg4.u32")
    d = _json()["ranks"]
    inside = 0
    for world, parts in d.items():
        for p in parts:
            if p["hi"] <= c4.size:
                assert shard.crc_of_crcs(c4[p["lo"]:p["hi"]], kvsep.extend_host) == p["crc_of_crcs"], (world, p)
                assert int(np.bitwise_xor.reduce(c4[p["lo"]:p["hi"]])) == p["xor"]
                inside += 1
    assert inside >= 3  # N = 1, and rank 0 at N = 4 and N = 8


@pytest.mark.parametrize("cfg", ["2", "3a", "3b"])
def test_check_results_eight_ranks_every_block(cfg):
    gold = _u32({"2": "full_cfg2.u32", "3a": "full_cfg3a.u32", "3b": "full_cfg5.u32"}[cfg])
    plans = [bench.Plan(cfg, 8, r) for r in range(8)]
    results = [gold[r * 65536:(r + 1) * 65536].copy() for r in range(8)]
    par = bench.check_results(plans, results, oracle=None)
    assert par["every_block_checked"] and par["blocks_checked_vs_reference"] == 524288, par
    assert par["mismatches"] == 0 and par["blocks_sampled_vs_oracle"] == 0
    results[5][123] ^= 0x80000000
    assert bench.check_results(plans, results, oracle=None)["mismatches"] == 1


def test_check_results_cfg4_digest_path():
    c4 = _u32("full_cfg4.u32")
    plans = [bench.Plan("4", 2, r) for r in range(2)]
    # rank 0's range runs past the per-block file: per block up to 2^20, the rest of it only by the digest
    fake = [np.zeros(p.count, np.uint32) for p in plans]
    fake[0][:c4.size] = c4
    par = bench.check_results(plans, fake, oracle=None)
    assert par["blocks_checked_vs_reference"] == c4.size and par["mismatches"] == 0
    assert par["blocks_checked_vs_reference_digest"] == plans[0].count - c4.size + plans[1].count
    assert par["every_block_checked"] and par["mismatching_digest_ranges"] == 2  # zeros are not the reference
    for p, f in zip(plans, fake):  # with the digests of these vectors every range passes
        p.digest = dict(p.digest, crc_of_crcs=shard.crc_of_crcs(f, kvsep.extend_host))
    assert bench.check_results(plans, fake, oracle=None)["mismatching_digest_ranges"] == 0
