#!/usr/bin/env python3
"""Two builds' gfx950 assembly (build/crc32c_device-hip-amdgcn-amd-amdhsa-gfx950.s), compared instruction by
instruction: comments, directives and labels dropped, kvsep symbol names and basic-block labels normalised (a template
parameter list that changes a kernel's mangled name changes nothing else).  Prints both instruction counts, the
number of differing lines and the first hunks.  usage: asm_norm_diff.py <old.s> <new.s>"""
import re, sys
def norm(path):
    out = []
    for l in open(path):
        t = l.split(";")[0].rstrip()
        if not t.strip() or t.strip().startswith("."):
            continue
        t = re.sub(r"_ZN5kvsep\w+", "SYM", t)
        t = re.sub(r"\.LBB\d+_\d+", "LBB", t)
        t = re.sub(r"\.Lfunc_end\d+", "LFE", t)
        out.append(t)
    return out
a, b = norm(sys.argv[1]), norm(sys.argv[2])
print(len(a), len(b))
import difflib
d = list(difflib.unified_diff(a, b, lineterm="", n=0))
print("diff lines:", len([x for x in d if x.startswith(("+", "-")) and not x.startswith(("+++", "---"))]))
print("\n".join(d[:40]))
