"""Every block of an N-rank bench line is checkable against the reference, run on the one-GPU
box: each rank's shard of bench.py's N-rank global batch -- bench.Plan(config, N, rank), the same layout, seed and
stream offsets the ranks of `bench.py --gpus N` use -- is generated in HBM and checksummed on cuda:0 one rank after
another, then bench.check_results checks the N per-rank result vectors exactly as rank 0 of a real N-GPU run does:

  config 3a at 8 ranks: 524,288 x 1 MiB (512 GiB), per block against tests/golden/full_cfg3a.u32
  config 2  at 8 ranks: 524,288 x 4 KiB, per block against full_cfg2.u32
  config 4  at 2, 4 and 8 ranks: N x 2^20 Zipf blocks cut by kvsep_crc32c_partition; per block where full_cfg4.u32
            covers (the first 2^20), every rank's whole range against the reference's digest (full_cfg4_ranks.json)
"""
import os
import sys

import numpy as np
import pytest

import kvsep

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def ctx():
    c = kvsep.Context(0)
    yield c
    c.close()


def _run_ranks(ctx, cfg, world):
    plans = [bench.Plan(cfg, world, r) for r in range(world)]
    span = max(p.span for p in plans)
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    results = []
    try:
        for p in plans:
            assert len(p.passes) == 1
            base, _ = p.passes[0]
            kvsep.fill_splitmix64(data.data_ptr(), p.span, p.seed, base)
            out = torch.zeros(max(p.count, 1), dtype=torch.int32, device=DEV)
            ctx.reserve(p.count, p.useful)
            ctx.batch_device(data.data_ptr(), bench.to_dev_u64(p.off, DEV), bench.to_dev_u64(p.ln, DEV), out,
                             count=p.count, total_bytes=p.useful, max_len=int(p.ln.max()))
            torch.cuda.synchronize()
            results.append(out[:p.count].cpu().numpy().view(np.uint32).copy())
    finally:
        del data
        torch.cuda.empty_cache()
    return plans, results


@pytest.mark.parametrize("cfg,world", [("3a", 8), ("2", 8), ("4", 2), ("4", 4), ("4", 8)])
def test_every_block_of_n_rank_batch_vs_reference(ctx, cfg, world):
    plans, results = _run_ranks(ctx, cfg, world)
    par = bench.check_results(plans, results, oracle=None)
    assert par["every_block_checked"] and par["blocks_sampled_vs_oracle"] == 0, par
    assert par["mismatches"] == 0 and par["mismatching_digest_ranges"] == 0, par
    assert par["blocks_total"] == sum(p.count for p in plans)
    if cfg != "4":
        assert par["blocks_checked_vs_reference"] == world * 65536
    # the checker is not vacuous: one wrong block in the last rank is caught
    results[-1][results[-1].size // 2] ^= 1
    bad = bench.check_results(plans, results, oracle=None)
    assert bad["mismatches"] + bad["mismatching_digest_ranges"] == 1, bad
