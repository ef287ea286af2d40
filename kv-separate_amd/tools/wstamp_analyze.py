#!/usr/bin/env python3
"""Per-wave time budget of the wide CRC kernel on one BASELINE layout (where config 4's last
0.86 ms to the read ceiling goes).  Writes the layout, runs tools/stamp_probe (the KVSEP_STAMPS build: realtime
stamps per wave, 100 MHz) as a child process, and splits every wave's time into the LDS fill, whole-block items,
pieces of split blocks and the rest (grabs, descriptor windows), then looks at the end of the kernel: when the waves
exit and what their last item was (a whole block, a block's first piece -- up to 2P bytes -- or a later piece).
Diagnostic only: the stamps perturb the kernel; the shares, not the times, are the result.
usage: wstamp_analyze.py [--config 4] [--out gpurun_out/wstamp_cfg4.json]"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from kvsep import workloads as W  # noqa: E402

P = 128 * 1024  # the default piece size (csrc/crc32c_device.hip, kvsep_crc32c_ctx::piece_bytes)
TICK_US = 0.01  # s_memrealtime: 100 MHz


def layout(cfg):
    if cfg == "4":
        return W.cfg4_layout()
    if cfg == "3a":
        return W.cfg3_layout()
    if cfg == "3b":
        return W.cfg3_layout(vlog=True)
    raise SystemExit("config must be 4, 3a or 3b")


def pct(a, q):
    return float(np.percentile(a, q)) if a.size else 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4")
    ap.add_argument("--probe", default=os.path.join(HERE, "stamp_probe"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    out_dir = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.join(HERE, "..", "..")), "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    off, ln = layout(args.config)
    n = off.size
    lay = os.path.join(out_dir, f"wstamp_layout_{args.config}.bin")
    with open(lay, "wb") as f:
        f.write(np.array([n], np.uint64).tobytes())
        f.write(off.astype(np.uint64).tobytes())
        f.write(ln.astype(np.uint64).tobytes())
    raw = os.path.join(out_dir, f"wstamp_raw_{args.config}.bin")
    r = subprocess.run([args.probe, lay, raw, str(args.reps)], capture_output=True, text=True, timeout=600)
    print(r.stdout, end="")
    if r.returncode:
        print(r.stderr)
        sys.exit(r.returncode)
    os.remove(lay)
    z = np.fromfile(raw, dtype=np.uint64).reshape(-1, 8)
    z = z[z[:, 4] != 0]  # waves that ran
    t0 = int(z[:, 4].min())
    entry = (z[:, 4].astype(np.int64) - t0) * TICK_US
    fill = (z[:, 5].astype(np.int64) - t0) * TICK_US
    exit_ = (z[:, 6].astype(np.int64) - t0) * TICK_US
    whole = z[:, 0].astype(np.float64) * TICK_US
    piece = z[:, 1].astype(np.float64) * TICK_US
    work = exit_ - fill
    other = work - whole - piece
    # the piece table as crc32c_plan_count_kernel builds it: a block of n >= 2P bytes gets n // P pieces
    ln64 = ln.astype(np.uint64)
    cnt = np.where(ln64 >= 2 * P, ln64 // P, 1).astype(np.int64)
    pstart = np.concatenate([[0], np.cumsum(cnt)])
    last = z[:, 7]
    last_whole = (last >> np.uint64(63)) & np.uint64(1)
    last_first = (last >> np.uint64(62)) & np.uint64(1)
    last_us = ((last >> np.uint64(40)) & np.uint64(0x3FFFFF)).astype(np.float64) * TICK_US
    last_item = (last & np.uint64(0xFFFFFFFFFF)).astype(np.int64)
    last_blk = np.searchsorted(pstart, last_item, side="right") - 1
    k = cnt[last_blk]
    j = last_item - pstart[last_blk]
    last_len = np.where(k == 1, ln64[last_blk].astype(np.int64),
                        np.where(j == 0, ln64[last_blk].astype(np.int64) - (k - 1) * P, P))
    span = float(exit_.max())
    med_exit = pct(exit_, 50)
    late = exit_ > med_exit
    res = {
        "config": args.config, "waves": int(z.shape[0]), "kernel_span_us": span,
        "items": {"whole_blocks": int(z[:, 2].sum()), "pieces": int(z[:, 3].sum()), "table_items": int(pstart[-1])},
        "entry_us": {"p50": pct(entry, 50), "max": float(entry.max())},
        "fill_done_us": {"p10": pct(fill, 10), "p50": pct(fill, 50), "p90": pct(fill, 90), "max": float(fill.max())},
        "exit_us": {"min": float(exit_.min()), "p10": pct(exit_, 10), "p50": med_exit, "p90": pct(exit_, 90),
                    "p99": pct(exit_, 99), "max": span},
        "per_wave_mean_us": {"fill": float(fill.mean() - entry.mean()), "whole_block_items": float(whole.mean()),
                             "pieces": float(piece.mean()), "other_in_loop": float(other.mean()),
                             "idle_after_exit_to_span": float((span - exit_).mean())},
        "share_of_wave_time": {"whole_block_items": float(whole.sum() / (exit_ - entry).sum()),
                               "pieces": float(piece.sum() / (exit_ - entry).sum()),
                               "fill": float((fill - entry).sum() / (exit_ - entry).sum()),
                               "other": float(other.sum() / (exit_ - entry).sum())},
        "mean_us_per_whole_block_item": float(whole.sum() / max(1, z[:, 2].sum())),
        "mean_us_per_piece": float(piece.sum() / max(1, z[:, 3].sum())),
        "tail": {
            "after_median_exit_us": span - med_exit,
            "late_waves": int(late.sum()),
            "late_last_item_kind": {"whole_block": int((late & (last_whole == 1)).sum()),
                                    "first_piece": int((late & (last_whole == 0) & (last_first == 1)).sum()),
                                    "later_piece": int((late & (last_whole == 0) & (last_first == 0)).sum())},
            "late_last_item_len_B": {"p50": pct(last_len[late], 50), "max": float(last_len[late].max()) if late.any()
                                     else 0.0},
            "late_last_item_us": {"p50": pct(last_us[late], 50), "p90": pct(last_us[late], 90),
                                  "max": float(last_us[late].max()) if late.any() else 0.0},
            "last_10_waves": [{"exit_us": float(exit_[i]), "kind": "whole" if last_whole[i] else
                               ("first_piece" if last_first[i] else "piece"), "len": int(last_len[i]),
                               "item_us": float(last_us[i])} for i in np.argsort(exit_)[-10:]],
        },
    }
    s = json.dumps(res, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
