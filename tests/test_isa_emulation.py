"""Functional emulation of the shipped CRC kernels' gfx950 assembly.  CPU only.

tools/wave_emu.py executes the compiled .s (the --save-temps output `make -C kv-separate_amd asm` keeps under build/)
instruction by instruction -- 64-lane VGPRs under EXEC, SGPRs, LDS, scalar / vector memory, ds_bpermute and DPP --
for one workgroup of the real 256-workgroup grid, and the CRCs it writes are compared with the oracle.  Round 3's
sorted-window fault was a code-generation error of exactly this kind (a rematerialised table base restored under the
narrowed EXEC of a nested divergent branch, so the slot-end lanes of every later group read the wrong table); the
emulator reproduced it from the diag build's assembly (tools/sorted_vin_emulate.py, retired in round 6: commit 8853f41) and
this test runs the same check
on every shipped narrow-family kernel, plain and verify forms, so a miscompile of that class fails on the CPU.  The
wide kernel runs too: unplanned (static runs, one workgroup of the grid) and planned (host-built piece table exactly
as the plan kernels build it, the guided schedule, then every workgroup of the combine kernel).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import load_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kv-separate_amd")
ASM = os.path.join(PKG, "build", "crc32c_device-hip-amdgcn-amd-amdhsa-gfx950.s")
sys.path.insert(0, os.path.join(PKG, "tools"))
sys.path.insert(0, PKG)

# the shipped narrow-family templates (launch_batch_in in csrc/crc32c_device.hip): name, threads per workgroup.  The
# claim kernel's waves take groups through an LDS counter; the emulator runs a workgroup's waves to each barrier in
# order, so its deal differs from the hardware's (a different interleaving, the same set of groups)
SORTED = "_ZN5kvsep27crc32c_narrow_sorted_kernelILi4ELb1ELi1024ELb%dENS_5ExactEEEvNS_10PiecesArgsE"
NARROW16 = "_ZN5kvsep20crc32c_narrow_kernelILi4ELb1ELi1024ELb0ELb1ENS_7LdsFullELb%dENS_5ExactEEEvNS_10PiecesArgsE"
NARROW8 = "_ZN5kvsep20crc32c_narrow_kernelILi4ELb1ELi512ELb1ELb1ENS_7LdsFullELb%dENS_5ExactEEEvNS_10PiecesArgsE"
CLAIM = "_ZN5kvsep26crc32c_narrow_claim_kernelILi4ELi512ELb%dELb1ELi8ELj3EEEvNS_10PiecesArgsE"  # kLean 3 (round 6)
CLAIM16 = "_ZN5kvsep26crc32c_narrow_claim_kernelILi4ELi512ELb%dELb1ELi16ELj0EEEvNS_10PiecesArgsE"
# the cooperative kernel (round 6, narrow form 12): the workgroup's 8 waves on one group, one barrier per group;
# init-less template (kInit false: no init word loaded)
COOP = "_ZN5kvsep25crc32c_narrow_coop_kernelILb%dELb0EEEvNS_10PiecesArgsE"
# (label, template, threads per workgroup, arrival levels of the verify publish: 8 = per-XCD shards, then the final word)
KERNELS = [("sorted", SORTED, 1024, 1), ("narrow16", NARROW16, 1024, 1), ("narrow8", NARROW8, 512, 1),
           ("claim", CLAIM, 512, 8), ("claim16", CLAIM16, 512, 8), ("coop", COOP, 512, 8)]


@pytest.fixture(scope="module")
def env():
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    subprocess.check_call(["make", "-s", "-C", PKG, "asm"], stdout=subprocess.DEVNULL)
    import wave_emu
    from kvsep import mask, splitmix64_bytes
    return wave_emu, wave_emu.dev_tables(), mask, splitmix64_bytes


def batch(kind, splitmix64_bytes):
    rng = np.random.default_rng(7)
    if kind == "short":  # the sorted-window probe's shape: 0..39 B, hint = max
        n, ln = 20000, rng.integers(0, 40, 20000)
        hint = 39
    else:  # up to 600 B with an understated hint of 256: the deferred-block path (narrow_deferred) runs too
        n, ln = 12000, rng.integers(0, 601, 12000)
        hint = 256
    ln = ln.astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    off += np.uint64(3)  # unaligned starts
    data = splitmix64_bytes(int(off[-1] + ln[-1]) + 4096, 11, 0)
    return data, off, ln, hint


@pytest.mark.parametrize("kind", ["short", "long"])
@pytest.mark.parametrize("label,tmpl,threads,shards", KERNELS)
def test_emulated_kernel_matches_oracle(env, label, tmpl, threads, shards, kind):
    E, tabs, mask, splitmix64_bytes = env
    data, off, ln, hint = batch(kind, splitmix64_bytes)
    exp = load_oracle().batch(data, off, ln, None, threads=8)
    wg = 5
    out, written, _, _, _ = E.run_batch_kernel(ASM, tmpl % 0, threads, data, off, ln, tabs, wg=wg, hint=hint)
    mine = np.nonzero(written)[0]
    assert mine.size > 0, "workgroup wrote nothing"
    assert np.array_equal(out[mine], exp[mine]), f"{label}: {np.count_nonzero(out[mine] != exp[mine])} wrong CRCs"
    if kind == "long":
        assert ln[mine].max() > hint, "the deferred path was not exercised"
    # verify form: the same workgroup with three wrong stored words among its blocks
    stored = np.array([mask(int(x)) for x in exp], np.uint32)
    plant = mine[[0, mine.size // 2, mine.size - 1]]
    stored[plant] ^= 0x100
    out_v, written_v, fb, nb, _ = E.run_batch_kernel(ASM, tmpl % 1, threads, data, off, ln, tabs, wg=wg, hint=hint,
                                                    expect=stored, shards=shards)
    assert np.array_equal(np.nonzero(written_v)[0], mine)
    assert np.array_equal(out_v[mine], exp[mine])
    assert (fb, nb) == (int(plant.min()), 3)  # published by this (last) workgroup, accumulators reset (batch_results)
    if kind == "short":  # every block of the workgroup bad: every wave's verdict, several mismatches per wave
        bad = np.array([mask(int(x)) for x in exp], np.uint32) ^ np.uint32(0x100)
        *_, fb, nb, _ = E.run_batch_kernel(ASM, tmpl % 1, threads, data, off, ln, tabs, wg=wg, hint=hint, expect=bad,
                                           shards=shards)
        assert (fb, nb) == (int(mine.min()), int(mine.size))
    _verify_tail(E, tmpl % 1, threads, data, off, ln, tabs, wg, hint, exp, mask, mine, plant, shards=shards)
    # the captured form (round 6): the workgroup's verdict in its own slot, nothing published, no accumulator touched
    st = {}
    out_s, written_s, fb, nb, _ = E.run_batch_kernel(ASM, tmpl % 1, threads, data, off, ln, tabs, wg=wg, hint=hint,
                                                     expect=stored, shards=shards, vslot=True, state=st)
    assert np.array_equal(np.nonzero(written_s)[0], mine) and np.array_equal(out_s[mine], exp[mine])
    assert (fb, nb) == (E.SENTINEL, E.SENTINEL)
    sl = st["slots"]
    assert sl[wg] == (int(plant.min()), 3), sl[wg]
    assert all(v == (E.SENTINEL, E.SENTINEL) for i, v in enumerate(sl) if i != wg)


def _verify_tail(E, name, threads, data, off, ln, tabs, wg, hint, exp, mask, mine, plant, lds_bytes=160768, shards=1):
    """The verify form's end (verify_publish): a clean batch publishes (-1, 0) from the last workgroup; a workgroup that
    is not the last leaves the caller's words alone and its posts -- lowest index, count, one arrival -- in the
    accumulators for the last one."""
    clean = np.array([mask(int(x)) for x in exp], np.uint32)
    *_, fb, nb, _ = E.run_batch_kernel(ASM, name, threads, data, off, ln, tabs, wg=wg, hint=hint, expect=clean,
                                       lds_bytes=lds_bytes, shards=shards)
    assert (fb, nb) == (-1, 0)
    stored = clean.copy()
    stored[plant] ^= 0x100
    st = {}
    *_, fb, nb, _ = E.run_batch_kernel(ASM, name, threads, data, off, ln, tabs, wg=wg, hint=hint, expect=stored,
                                       lds_bytes=lds_bytes, last=False, state=st, shards=shards)
    assert (fb, nb) == (E.SENTINEL, E.SENTINEL)  # not published
    # the workgroup's count travels with its arrival (round 5): on the final word (one level) or on the workgroup's
    # shard word (two levels); its lowest bad block on vacc[0]
    sh = [0] * E.VACC_SHARDS
    if shards > 1:
        sh[wg % shards] = (1 << 40) | len(plant)
    final = (len(plant) | (1 << 40)) if shards == 1 else 0
    assert st["vacc"] == (int(plant.min()), final, *sh), [hex(v) for v in st["vacc"]]


PIECES = "_ZN5kvsep20crc32c_pieces_kernelILb%dELb%dELi4ELb1ELb1ELi512ELb1ELb%dENS_5ExactEEEvNS_10PiecesArgsE"
COMBINE = "_ZN5kvsep21crc32c_combine_kernelILb%dEEEvNS_10PiecesArgsE"


def _planted(exp, mask, idx):
    stored = np.array([mask(int(x)) for x in exp], np.uint32)
    stored[idx] ^= 0x100
    return stored


@pytest.mark.parametrize("verify", [0, 1])
def test_emulated_wide_unplanned(env, verify):
    """The wide kernel on an unsplit batch (static contiguous runs): one workgroup of the grid."""
    E, tabs, mask, splitmix64_bytes = env
    rng = np.random.default_rng(3)
    n = 4096
    ln = rng.integers(0, 5000, n).astype(np.uint64)
    ln[rng.integers(0, n, 64)] = rng.integers(0, 16, 64)  # head/tail-only blocks
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + np.uint64(5), dtype=np.uint64)  # 5-B gaps: every start alignment
    data = splitmix64_bytes(int(off[-1] + ln[-1]) + 4096, 13, 0)
    exp = load_oracle().batch(data, off, ln, None, threads=8)
    out, written, _, _, _ = E.run_batch_kernel(ASM, PIECES % (0, 0, 0), 512, data, off, ln, tabs, wg=7,
                                               lds_bytes=160768)
    mine = np.nonzero(written)[0]
    assert mine.size > 0 and np.array_equal(out[mine], exp[mine])
    # per-block initial CRCs: the padded head rewinds each block's register to its 16-B boundary (x^-8k)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    exp_i = load_oracle().batch(data, off, ln, init, threads=8)
    out_i, wi, _, _, _ = E.run_batch_kernel(ASM, PIECES % (0, 0, 0), 512, data, off, ln, tabs, wg=7, init=init)
    assert np.array_equal(np.nonzero(wi)[0], mine) and np.array_equal(out_i[mine], exp_i[mine])
    if verify:
        plant = mine[[0, mine.size - 1]]
        out_v, wv, fb, nb, _ = E.run_batch_kernel(ASM, PIECES % (0, 0, 1), 512, data, off, ln, tabs, wg=7,
                                                  expect=_planted(exp, mask, plant))
        assert np.array_equal(np.nonzero(wv)[0], mine) and np.array_equal(out_v[mine], exp[mine])
        assert (fb, nb) == (int(plant.min()), 2)
        _verify_tail(E, PIECES % (0, 0, 1), 512, data, off, ln, tabs, 7, 0, exp, mask, mine, plant)


@pytest.mark.parametrize("verify", [0, 1])
def test_emulated_wide_planned_with_combine(env, verify):
    """A split batch as the large configs run it: piece table, the wide kernel's guided schedule (one workgroup takes
    every item here), the combine kernel's Horner step over the pieces; 16 KiB pieces, blocks up to 100 KiB."""
    E, tabs, mask, splitmix64_bytes = env
    rng = np.random.default_rng(4)
    n = 40
    ln = rng.integers(0, 100 * 1024, n).astype(np.uint64)
    ln[:4] = [0, 1, 32 * 1024, 32 * 1024 - 1]  # empty, one byte, exactly 2P (split), just under 2P (not split)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + np.uint64(3), dtype=np.uint64)
    data = splitmix64_bytes(int(off[-1] + ln[-1]) + 4096, 17, 0)
    exp = load_oracle().batch(data, off, ln, None, threads=8)
    expect = None
    plant = np.array([2, 5, n - 1])  # a split block and two others
    if verify:
        expect = _planted(exp, mask, plant)
    out, written, fb, nb, _ = E.run_planned_batch(ASM, PIECES % (1, 1, verify), COMBINE % verify, data, off, ln, tabs,
                                                  expect=expect)
    assert written.all()
    assert np.array_equal(out, exp), f"{np.count_nonzero(out != exp)} wrong CRCs"
    if verify:
        assert (fb, nb) == (2, 3)  # the combine kernel's last workgroup published; accumulators reset (batch_results)
        # captured: the pieces kernel's workgroup 5 (the whole blocks) and the combine kernel's one workgroup (the
        # split ones) each write their slot, clean or not; the reduce kernel's min / sum over the slots is the verdict
        st = {}
        out_s, _, fb, nb, _ = E.run_planned_batch(ASM, PIECES % (1, 1, 1), COMBINE % 1, data, off, ln, tabs,
                                                  expect=expect, state=st)
        assert np.array_equal(out_s, exp) and (fb, nb) == (E.SENTINEL, E.SENTINEL)
        sl = st["slots"]
        split = set(np.nonzero(ln >= 2 * 16 * 1024)[0].tolist())
        whole = [int(b) for b in plant if int(b) not in split]
        assert sl[5] == ((min(whole), len(whole)) if whole else ((1 << 64) - 1, 0)), sl[5]
        assert sl[256] == (min(int(b) for b in plant if int(b) in split), len(plant) - len(whole)), sl[256]
        written = [v for v in sl if v != (E.SENTINEL, E.SENTINEL)]
        assert len(written) == 2 and min(v[0] for v in written) == 2 and sum(v[1] for v in written) == 3
        _, _, fb, nb, _ = E.run_planned_batch(ASM, PIECES % (1, 1, 1), COMBINE % 1, data, off, ln, tabs,
                                              expect=_planted(exp, mask, np.array([], np.int64)))
        assert (fb, nb) == (-1, 0)
