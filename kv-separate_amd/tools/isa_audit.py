#!/usr/bin/env python3
"""Static audit of compiled gfx950 kernels: memory-counter waits and cross-lane operands.

Reads the device assembly hipcc writes with --save-temps (crc32c_device-hip-amdgcn-amd-amdhsa-gfx950.s) and, per
kernel, runs a forward data-flow pass over the control-flow graph that tracks every register a memory instruction
has yet to write back:

  * vmcnt: global/buffer loads (and atomics with return).  `s_waitcnt vmcnt(N)` retires a pending register when at
    least N vm-counted operations were issued after it.  Two models:  --vm-model inorder counts loads, stores and
    atomics in one in-order queue (what the compiler assumes on gfx9-family parts), --vm-model loads counts loads
    only (conservative: a store or atomic issued after a load is not taken to complete after it).
  * lgkmcnt: LDS operations (ds_read, ds_bpermute) return in order among themselves; scalar loads (s_load) may
    return in any order, so only lgkmcnt(0) retires them.

A read of a pending register, or a write to one (the late write-back would land on top of it), is a violation.  At a
join the pass keeps, per register, the smallest number of later operations over the incoming paths, so a wait is only
credited when it covers the register on every path.  The pass does not model wait states (s_nop hazards).

--crosslane also checks, with a concrete EXEC model (exec_audit below), that every cross-lane data instruction
(ds_bpermute, DPP) runs with the whole wave active: a ds_bpermute reads 0 from an inactive source lane.

Usage: isa_audit.py <file.s> [--kernel REGEX] [--vm-model inorder|loads] [--crosslane] [-v]
Exit status 1 if any violation is found (the CPU test tests/test_kernel_resources.py runs it on the shipped build).
"""
import argparse
import re
import sys
import zlib

REG_RE = re.compile(r'\b([vs])\[(\d+):(\d+)\]|\b([vs])(\d+)\b|\b(vcc|exec|m0|scc)\b')

NO_DST = ('v_cmp_', 's_cmp_', 's_bitcmp', 's_cbranch', 's_branch', 's_waitcnt', 's_nop', 's_barrier', 's_endpgm',
          's_setprio', 's_sleep', 's_sendmsg', 's_dcache', 'global_store', 'buffer_store', 'ds_write', 'scratch_store',
          'flat_store', 's_set', 's_trap', 'v_cmpx_', 'sched_')


def regs(text):
    out = []
    for m in REG_RE.finditer(text):
        if m.group(1):
            k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
            out += ['%s%d' % (k, i) for i in range(a, b + 1)]
        elif m.group(4):
            out.append('%s%s' % (m.group(4), m.group(5)))
        else:
            n = m.group(6)
            out += [n + '_lo', n + '_hi'] if n in ('vcc', 'exec') else [n]
    return out


def split_ops(rest):
    # operands are comma separated; modifiers (offset:, nt, sc0, dpp controls) follow the last one after spaces
    parts = [p.strip() for p in rest.split(',')]
    return parts


class Insn:
    __slots__ = ('line', 'text', 'op', 'dst', 'src', 'kind')

    def __init__(self, line, text):
        self.line = line
        self.text = text
        f = text.split(None, 1)
        self.op = f[0]
        rest = f[1] if len(f) > 1 else ''
        ops = split_ops(rest) if rest else []
        op = self.op
        self.kind = None
        dst, src = [], []
        if op.startswith(('global_load', 'buffer_load', 'scratch_load')):
            self.kind = ('vm', 'load')
            dst = regs(ops[0])
            for o in ops[1:]:
                src += regs(o)
        elif op.startswith(('global_store', 'buffer_store', 'scratch_store')):
            self.kind = ('vm', 'store')
            for o in ops:
                src += regs(o)
        elif op.startswith(('global_atomic', 'buffer_atomic')):
            # with a return value the form has four operands: vdst, vaddr, vdata, saddr|off (and sc0)
            if len(ops) >= 4:
                self.kind = ('vm', 'load')
                dst = regs(ops[0])
                for o in ops[1:]:
                    src += regs(o)
            else:
                self.kind = ('vm', 'store')
                for o in ops:
                    src += regs(o)
        elif op.startswith('flat_'):
            self.kind = ('flat', 'load' if 'load' in op or len(ops) >= 3 and 'atomic' in op else 'store')
            if self.kind[1] == 'load':
                dst = regs(ops[0])
                for o in ops[1:]:
                    src += regs(o)
            else:
                for o in ops:
                    src += regs(o)
        elif op.startswith('ds_'):
            if op.startswith(('ds_read', 'ds_bpermute', 'ds_permute', 'ds_swizzle')) or '_rtn' in op:
                self.kind = ('lgkm', 'ds')
                dst = regs(ops[0])
                for o in ops[1:]:
                    src += regs(o)
            else:
                self.kind = ('lgkm', 'dsw')
                for o in ops:
                    src += regs(o)
        elif op.startswith(('s_load', 's_buffer_load', 's_memtime', 's_memrealtime', 's_getreg')) and \
                not op.startswith('s_getreg'):
            self.kind = ('lgkm', 'smem')
            dst = regs(ops[0]) if ops else []
            for o in ops[1:]:
                src += regs(o)
        elif op.startswith(NO_DST):
            for o in ops:
                src += regs(o)
            if op.startswith('v_cmp_') and op.endswith('_e32'):
                dst = ['vcc_lo', 'vcc_hi']
            elif op.startswith('v_cmp_') and ops:
                dst = regs(ops[0])
                src = []
                for o in ops[1:]:
                    src += regs(o)
        else:
            if ops:
                dst = regs(ops[0])
                for o in ops[1:]:
                    src += regs(o)
            if op.endswith('_e32') and ('cndmask' in op or 'addc' in op or 'subb' in op):
                src += ['vcc_lo', 'vcc_hi']
            if op.startswith('s_') and ('saveexec' in op):
                src += ['exec_lo', 'exec_hi']
        self.dst = dst
        self.src = src


def parse_function(lines):
    """lines: the function body.  Returns (blocks, succ) with blocks = list of (label, [Insn])."""
    blocks = []
    cur_label, cur = '<entry>', []
    label_of_idx = {}

    def close():
        nonlocal cur
        blocks.append((cur_label, cur))
        cur = []

    for ln, raw in lines:
        s = raw.split(';', 1)[0].rstrip() if not raw.lstrip().startswith(';') else ''
        lab = re.match(r'^(\.LBB\w+):', raw)
        bb = re.match(r'^; %bb\.(\d+):', raw)
        if lab or bb:
            if cur or blocks or cur_label != '<entry>':
                close()
            cur_label = lab.group(1) if lab else '%%bb.%s' % bb.group(1)
            continue
        if not s.strip() or s.strip().startswith('.') or s.strip().endswith(':'):
            continue
        cur.append(Insn(ln, s.strip()))
    close()
    # successors
    idx = {lab: i for i, (lab, _) in enumerate(blocks)}
    succ = []
    for i, (lab, ins) in enumerate(blocks):
        ss = []
        fall = True
        for k in ins:
            if k.op == 's_branch':
                ss.append(idx[k.text.split()[1]])
                fall = False
            elif k.op.startswith('s_cbranch'):
                ss.append(idx[k.text.split()[1]])
            elif k.op in ('s_endpgm', 's_setpc_b64'):
                fall = False
        if fall and i + 1 < len(blocks):
            ss.append(i + 1)
        succ.append(ss)
    return blocks, succ


CAP = 64


def counts_for(kind, model):
    """Which issued operations age a pending entry of `kind`."""
    cnt, sub = kind
    if cnt == 'vm':
        return ('vm',) if model == 'inorder' else ('vm-load',)
    return ('ds',) if sub == 'ds' else ()


def issue_tags(insn, model):
    k = insn.kind
    if not k:
        return ()
    cnt, sub = k
    if cnt in ('vm', 'flat'):
        tags = ['vm']
        if sub == 'load':
            tags.append('vm-load')
        if cnt == 'flat':
            tags.append('ds')
        return tags
    if sub in ('ds', 'dsw'):
        return ('ds',)
    return ()


def waits(insn):
    out = {}
    for name, val in re.findall(r'(vmcnt|lgkmcnt|expcnt)\((\d+)\)', insn.text):
        out[name] = int(val)
    if insn.text.strip() in ('s_waitcnt 0', 's_waitcnt 0x0'):
        out = {'vmcnt': 0, 'lgkmcnt': 0}
    return out


def transfer(state, insn, model, report):
    """state: dict reg -> dict{(cnt, sub): d}.  Returns new state; appends violations to report."""
    if insn.op == 's_waitcnt':
        w = waits(insn)
        new = {}
        for r, ents in state.items():
            keep = {}
            for (cnt, sub), d in ents.items():
                if cnt in ('vm', 'flat') and 'vmcnt' in w and d >= w['vmcnt']:
                    if cnt == 'vm' or ('lgkmcnt' in w and w['lgkmcnt'] == 0):
                        continue
                if cnt == 'lgkm' and 'lgkmcnt' in w:
                    if sub == 'smem' and w['lgkmcnt'] == 0:
                        continue
                    if sub == 'ds' and d >= w['lgkmcnt']:
                        continue
                keep[(cnt, sub)] = d
            if keep:
                new[r] = keep
        return new
    for r in insn.src:
        if r in state:
            report.append((insn, r, 'read', dict(state[r])))
    for r in insn.dst:
        if r in state:
            # a later load of the same in-order queue into the same register writes back after the pending one:
            # not a hazard (the compiler does not wait there either)
            ents = state[r]
            same_queue = insn.kind is not None and insn.kind[1] in ('load', 'ds') and \
                all(k[0] == insn.kind[0] and k[1] == insn.kind[1] for k in ents)
            if not same_queue:
                report.append((insn, r, 'write', dict(ents)))
    tags = issue_tags(insn, model)
    if tags:
        new = {}
        for r, ents in state.items():
            ne = {}
            for key, d in ents.items():
                ages = counts_for(key, model)
                if key[0] == 'flat':
                    ages = ('vm',) if model == 'inorder' else ('vm-load',)
                ne[key] = min(CAP, d + 1) if any(a in tags for a in ages) else d
            new[r] = ne
        state = new
        if insn.kind[1] in ('load', 'ds', 'smem'):
            key = insn.kind if insn.kind[0] != 'flat' else ('flat', 'load')
            for r in insn.dst:
                state[r] = {key: 0}
    else:
        if insn.kind and insn.kind[1] == 'smem':
            state = dict(state)
            for r in insn.dst:
                state[r] = {insn.kind: 0}
    return state


def merge(a, b):
    out = {r: dict(e) for r, e in a.items()}
    for r, ents in b.items():
        t = out.setdefault(r, {})
        for k, d in ents.items():
            t[k] = min(t[k], d) if k in t else d
    return out


def audit(blocks, succ, model):
    n = len(blocks)
    ins = [None] * n
    ins[0] = {}
    work = [0]
    inq = {0}
    while work:
        i = work.pop()
        inq.discard(i)
        st = ins[i]
        scratch = []
        for k in blocks[i][1]:
            st = transfer(st, k, model, scratch)
        for s in succ[i]:
            m = st if ins[s] is None else merge(ins[s], st)
            if ins[s] is None or m != ins[s]:
                ins[s] = m
                if s not in inq:
                    work.append(s)
                    inq.add(s)
    report = []
    for i in range(n):
        if ins[i] is None:
            continue
        st = ins[i]
        for k in blocks[i][1]:
            st = transfer(st, k, model, report)
    return report



# ------------------------------------------------------------------------------------------------------------------
# EXEC model: concrete 64-bit masks.  Every per-lane compare (v_cmp) yields a pseudo-random lane mask fixed per
# instruction text; s_cselect of -1/0 and other scalar results are wave-uniform (all ones).  Mask arithmetic on SGPR pairs,
# VCC and EXEC (s_and/or/xor/andn2/orn2/mov and the *_saveexec forms) is evaluated exactly, so the structurizer's
# if / else / flow sequences restore EXEC to the entry mask exactly where the program really is uniform again.  At a
# join, a register whose incoming values differ becomes unknown (None).
ALL = (1 << 64) - 1


def _mask_of(state, ops_text):
    t = ops_text.strip()
    if t in ('exec',):
        return state.get('exec')
    if t == 'vcc':
        return state.get('vcc')
    if t in ('-1',):
        return ALL
    if t in ('0',):
        return 0
    m = re.match(r's\[(\d+):(\d+)\]$', t)
    if m:
        return state.get('s%s' % m.group(1))
    return None


def _set(state, dst_text, val):
    t = dst_text.strip()
    if t in ('exec', 'vcc'):
        state[t] = val
        return
    m = re.match(r's\[(\d+):(\d+)\]$', t)
    if m:
        state['s%s' % m.group(1)] = val
        return
    # any other SGPR write invalidates a pair starting there
    for r in regs(t):
        state.pop(r, None)


def _rand(line):
    x = (line * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & ALL
    x ^= x >> 29
    x = (x * 0xBF58476D1CE4E5B9) & ALL
    x ^= x >> 32
    return x | 1  # never empty


def exec_step(state, k):
    """Updates the mask state for one instruction; returns the EXEC in force while it executes."""
    ex = state.get('exec')
    op = k.op
    ops = [o.strip() for o in k.text.split(None, 1)[1].split(',')] if ' ' in k.text else []
    if op.startswith('v_cmp_') or op.startswith('v_cmpx_'):
        # keyed by the instruction text: the tail-duplicated copies of one compare (same registers) give one mask
        v = _rand(zlib.crc32(k.text.encode()))
        if ex is not None:
            v &= ex
        if op.endswith('_e32') or op.startswith('v_cmpx_'):
            state['vcc'] = v if not op.startswith('v_cmpx_') else state.get('vcc')
            if op.startswith('v_cmpx_'):
                state['exec'] = v
        elif ops:
            _set(state, ops[0], v)
        return ex
    if op in ('s_cselect_b64',):
        _set(state, ops[0], ALL)  # wave-uniform all-or-nothing: taken as "all lanes"
        return ex
    if op.endswith('_saveexec_b64'):
        src = _mask_of(state, ops[1])
        _set(state, ops[0], ex)
        if op.startswith('s_and_saveexec'):
            nv = None if src is None or ex is None else ex & src
        elif op.startswith('s_or_saveexec'):
            nv = None if src is None or ex is None else ex | src
        elif op.startswith('s_andn2_saveexec'):
            nv = None if src is None or ex is None else src & ~ex & ALL
        elif op.startswith('s_xor_saveexec'):
            nv = None if src is None or ex is None else ex ^ src
        else:
            nv = None
        state['exec'] = nv
        return ex
    m = re.match(r's_(and|or|xor|andn2|orn2|mov|not)_b64$', op)
    if m and ops:
        f = m.group(1)
        a = _mask_of(state, ops[1]) if len(ops) > 1 else None
        b = _mask_of(state, ops[2]) if len(ops) > 2 else None
        if f == 'mov':
            v = a
        elif f == 'or' and ops[0] == 'exec' and ops[1] == 'exec' and a is None and b is not None:
            v = b  # a join whose incoming EXECs differ (one path skipped a region): EXEC |= the mask saved at entry
        elif f == 'not':
            v = None if a is None else ~a & ALL
        elif a is None or b is None:
            v = None
        elif f == 'and':
            v = a & b
        elif f == 'or':
            v = a | b
        elif f == 'xor':
            v = a ^ b
        elif f == 'andn2':
            v = a & ~b & ALL
        else:
            v = a | (~b & ALL)
        _set(state, ops[0], v)
        return ex
    # any other writer of an SGPR pair / VCC loses its mask value
    for d in k.dst:
        if d.startswith('s'):
            state.pop(d, None)
            state.pop('s%d' % (int(d[1:]) - 1), None)
        elif d.startswith('vcc'):
            state.pop('vcc', None)
        elif d.startswith('exec'):
            state['exec'] = None
    return ex


def _merge_masks(a, b, where=0):
    """Join of two mask states.  EXEC that differs becomes unknown (the structurizer restores it from a saved mask
    right after the join, see exec_step); any other lane mask that differs (a divergent boolean carried across the
    join, e.g. `live`) becomes a phi: a fresh partial mask fixed per (join block, register), so later arithmetic on
    it stays consistent from one trip of a loop to the next."""
    out = {}
    for key in set(a) | set(b):
        va, vb = a.get(key, None), b.get(key, None)
        if va == vb:
            out[key] = va
        elif key == 'exec':
            out[key] = None
        else:
            out[key] = _rand(zlib.crc32(('%d:%s' % (where, key)).encode()))
    return out


def exec_audit(blocks, succ):
    """Returns [(insn, exec_mask)] for every instruction, the mask in force (None = unknown)."""
    n = len(blocks)
    ins = [None] * n
    ins[0] = {'exec': ALL}
    work = [0]
    rounds = 0
    while work and rounds < 200000:
        rounds += 1
        i = work.pop()
        st = dict(ins[i])
        for k in blocks[i][1]:
            exec_step(st, k)
        for s in succ[i]:
            m = dict(st) if ins[s] is None else _merge_masks(ins[s], st, s)
            if ins[s] is None or m != ins[s]:
                ins[s] = m
                work.append(s)
    out = []
    for i in range(n):
        if ins[i] is None:
            continue
        st = dict(ins[i])
        for k in blocks[i][1]:
            out.append((blocks[i][0], k, exec_step(st, k)))
    return out


# Cross-lane DATA movement whose result depends on other lanes being active: a ds_bpermute / ds_permute /
# ds_swizzle reads 0 from a disabled source lane, a DPP move takes the `old` operand (or 0) for one.  v_readlane reads
# its lane whatever EXEC says, and v_readfirstlane of a wave-uniform value is exact under any non-empty EXEC: those are
# not flagged.
CROSS = ('ds_bpermute', 'ds_permute', 'ds_swizzle', 'v_permlane')


def crosslane_partial(blocks, succ, unknown=False):
    """Cross-lane data ops executed under a partial EXEC (with unknown=True also those whose EXEC the model lost
    track of -- at joins of tail-duplicated regions that carry lane-mask phis it does)."""
    hits = []
    for lab, k, ex in exec_audit(blocks, succ):
        if ex == ALL or (ex is None and not unknown):
            continue
        if k.op.startswith(CROSS) or '_dpp' in k.op or 'row_shr' in k.text or 'quad_perm' in k.text or \
                'row_bcast' in k.text or 'row_ror' in k.text or 'wave_sh' in k.text or 'wave_ro' in k.text:
            hits.append((lab, k, ex))
    return hits


def functions(path):
    lines = open(path).read().split('\n')
    cur, name = None, None
    for i, raw in enumerate(lines, 1):
        m = re.match(r'^(_Z\w+):', raw)
        if m and not raw.startswith('.'):
            name, cur = m.group(1), []
            continue
        if cur is not None:
            if raw.strip().startswith('.Lfunc_end'):
                yield name, cur
                cur, name = None, None
            else:
                cur.append((i, raw))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('asm')
    ap.add_argument('--kernel', default='.')
    ap.add_argument('--vm-model', default='inorder', choices=('inorder', 'loads'))
    ap.add_argument('-v', action='store_true')
    ap.add_argument('--crosslane', action='store_true', help='also list cross-lane ops under a partial EXEC')
    ap.add_argument('--unknown', action='store_true', help='with --crosslane: also those under an EXEC the model lost')
    args = ap.parse_args()
    bad = 0
    nk = 0
    for name, body in functions(args.asm):
        if not re.search(args.kernel, name):
            continue
        nk += 1
        blocks, succ = parse_function(body)
        rep = audit(blocks, succ, args.vm_model)
        seen = set()
        for insn, r, how, ents in rep:
            key = (insn.line, r)
            if key in seen:
                continue
            seen.add(key)
            bad += 1
            print('%s:%d: %s of pending %s %s: %s' % (name, insn.line, how, r, ents, insn.text))
        if args.crosslane:
            for lab, k, ex in crosslane_partial(blocks, succ, args.unknown):
                bad += 1
                print('%s:%d: cross-lane data op under %s EXEC (%s): %s' % (name, k.line, 'unknown' if ex is None else
                                                                             'partial', lab, k.text))
        if args.v:
            print('%s: %d blocks, %d violations' % (name, len(blocks), len(rep)))
    print('audited %d kernel(s), %d violation(s)' % (nk, bad))
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main())
