"""Build-time guard on the shipped gfx950 kernels.  CPU only.

`make -C kv-separate_amd asm` compiles the shipped device code once more with --save-temps and
-Rpass-analysis=kernel-resource-usage (build/resource.txt, build/crc32c_device-hip-amdgcn-amd-amdhsa-gfx950.s;
nothing is rebuilt when the sources did not change).  Then, for every kvsep kernel:
  * no scratch and no VGPR spills, and VGPRs within the cap its launch bounds allow (512 / waves per SIMD);
  * tools/isa_audit.py: every memory-counter wait covers the registers read after it, under both the in-order
    vmcnt model and the loads-only model, and no ds_bpermute runs under a partial EXEC.
The two compiler traps DESIGN §3.2 records were spills at the 128-VGPR cap of the 16-wave narrow kernels; a spill that
reappears (a compiler update, an edit) fails here instead of showing up as a slow or wrong GPU run.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kv-separate_amd")
BUILD = os.path.join(PKG, "build")
ASM = os.path.join(BUILD, "crc32c_device-hip-amdgcn-amd-amdhsa-gfx950.s")
RES = os.path.join(BUILD, "resource.txt")
sys.path.insert(0, os.path.join(PKG, "tools"))

# kernel name fragment -> threads per workgroup of its launch (the caps follow: 4 SIMDs per CU, 512 VGPRs per lane
# slot per SIMD): the shipped templates, see launch_pieces_v / launch_batch_in in csrc/crc32c_device.hip
LAUNCH_THREADS = {
    "crc32c_pieces_kernel": 512,
    "crc32c_narrow_kernelILi4ELb1ELi512E": 512,
    "crc32c_narrow_kernelILi4ELb1ELi1024E": 1024,
    "crc32c_narrow_sorted_kernelILi4ELb1ELi1024E": 1024,
}


def _hipcc():
    return os.path.exists("/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def built():
    if not _hipcc():
        pytest.skip("hipcc not available")
    subprocess.check_call(["make", "-s", "-C", PKG, "asm"], stdout=subprocess.DEVNULL)
    assert os.path.exists(ASM) and os.path.exists(RES)
    return ASM, RES


def resources(path):
    rows, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark: \S+?:\d+:\d+:\s+(.+?): (\S+) \[", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = m.group(2)
    return {k: v for k, v in rows.items() if k.startswith("_ZN5kvsep")}


def test_every_shipped_kernel_is_reported(built):
    rows = resources(built[1])
    names = " ".join(rows)
    for frag in LAUNCH_THREADS:
        assert frag in names, f"{frag} missing from the resource report"
    assert "crc32c_combine_kernel" in names and "verify_finish_kernel" in names


def test_no_scratch_no_spills_vgprs_within_cap(built):
    rows = resources(built[1])
    bad = []
    for name, r in rows.items():
        if int(r["ScratchSize [bytes/lane]"]) != 0 or int(r["VGPRs Spill"]) != 0:
            bad.append((name, "scratch", r["ScratchSize [bytes/lane]"], "vgpr spill", r["VGPRs Spill"]))
        for frag, threads in LAUNCH_THREADS.items():
            if frag in name:
                cap = 512 // max(1, threads // 256)
                cap = min(cap, 256)
                if int(r["VGPRs"]) > cap:
                    bad.append((name, "VGPRs", r["VGPRs"], "cap", cap))
                # the launch must fit: occupancy (waves per SIMD) at least the waves one workgroup puts on a SIMD
                if int(r["Occupancy [waves/SIMD]"]) < threads // 256:
                    bad.append((name, "occupancy", r["Occupancy [waves/SIMD]"], "needs", threads // 256))
    assert not bad, bad


def test_isa_audit_waits_and_crosslane(built):
    import isa_audit as A

    nk = 0
    problems = []
    for name, body in A.functions(built[0]):
        if not name.startswith("_ZN5kvsep"):
            continue
        nk += 1
        blocks, succ = A.parse_function(body)
        for model in ("inorder", "loads"):
            for insn, reg, how, ents in A.audit(blocks, succ, model):
                problems.append((name, model, insn.line, reg, how, insn.text))
        # ds_bpermute (the sorted-window gather, the bitonic sort) reads 0 from an inactive source lane: none may run
        # under a partial EXEC.  (The EXEC model is a heuristic -- concrete lane masks, phis at joins -- so the DPP
        # moves of the slot trees, which it sometimes loses track of in the verify kernels, are not asserted on.)
        for lab, k, ex in A.crosslane_partial(blocks, succ):
            if k.op.startswith(("ds_bpermute", "ds_permute")):
                problems.append((name, "crosslane", k.line, lab, k.text))
    assert nk >= 10
    assert not problems, problems[:20]


def test_audit_catches_a_missing_wait(built, tmp_path):
    """The audit itself: drop one s_waitcnt from the shipped sorted-window kernel and it must complain."""
    import isa_audit as A

    lines = open(built[0]).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_ZN5kvsep27crc32c_narrow_sorted_kernel"))
    k = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_waitcnt lgkmcnt(0)"))
    del lines[k]
    p = tmp_path / "broken.s"
    p.write_text("\n".join(lines))
    hits = 0
    for name, body in A.functions(str(p)):
        if name.startswith("_ZN5kvsep27crc32c_narrow_sorted_kernel"):
            blocks, succ = A.parse_function(body)
            hits += len(A.audit(blocks, succ, "inorder"))
    assert hits > 0


def test_shipped_kernels_are_exact_only(built):
    """the kernel templates' replaceable steps come from an Ext type, and the shipped library has
    one, Exact -- the A/B forms and the ablations (wrong results by design) are types only the KVSEP_DIAG build
    defines (csrc/crc32c_diag.inc).  Every shipped CRC kernel is instantiated with Exact, and no diag type's name, nor
    the integer switches they replaced, is anywhere in the shipped assembly or the shipped kernel source."""
    asm, _ = built
    text = open(asm).read()
    names = set(re.findall(r"_ZN5kvsep\d+crc32c_(?:pieces|narrow|narrow_sorted)_kernel\w+", text))
    assert len(names) == 14, names  # 8 wide (planned x guided x verify), 4 narrow, 2 sorted
    assert all("NS_5ExactE" in n for n in names), [n for n in names if "NS_5ExactE" not in n]
    for diag_type in ("AblNoMerge", "AblXorRows", "AblNoHeadTail", "AblNoTree", "AblFreeShort", "SerialHead",
                      "SortedVIn", "SortedDrain"):
        assert diag_type not in text, diag_type
    src = "".join(open(os.path.join(PKG, "csrc", f)).read() for f in (
        "crc32c_device.hip", "crc32c_fold.inc", "crc32c_wide.inc", "crc32c_narrow.inc", "crc32c_support.inc"))
    for switch in ("kAbl", "kStrided", "kVIn", "c->variant", "c->narrow"):
        assert switch not in src, switch
    diag = open(os.path.join(PKG, "csrc", "crc32c_diag.inc")).read()
    head, shipped = diag.split("#else  // the shipped library", 1)
    assert "struct AblXorRows" in head and "struct" not in shipped  # the types live in the KVSEP_DIAG half only
