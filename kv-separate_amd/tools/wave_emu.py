#!/usr/bin/env python3
"""A functional emulator of one gfx950 workgroup, for the instruction subset the kvsep kernels compile to.

Tools-only (never loaded by the package, the tests or bench.py).  It executes the compiled assembly of a kernel --
the .s hipcc writes with --save-temps -- instruction by instruction: 64-lane VGPRs under EXEC, SGPRs / VCC / SCC,
scalar and vector memory, LDS and the cross-lane ops (ds_bpermute, DPP row shifts, readlane).  Every memory operation
completes before the next instruction, so s_waitcnt is a no-op, and there is no notion of time: it answers "does this
instruction sequence, executed as the ISA defines it, compute the right result?" -- separating a logic error in the
generated code from a timing or hardware effect.

Semantics follow the CDNA3/4 ISA for the opcodes listed in VALU / SALU / MEM below; anything else raises.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile

import numpy as np

M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1
LANES = np.arange(64, dtype=np.uint32)


class EmuError(RuntimeError):
    pass


# ------------------------------------------------------------------------------------------------------------------
class Memory:
    """Sparse flat address space of byte regions."""

    def __init__(self):
        self.regions = []  # (base, np.uint8 array)
        self.next = 0x10000000

    def alloc(self, nbytes: int, align: int = 256, data=None) -> int:
        base = (self.next + align - 1) // align * align
        arr = np.zeros(max(1, nbytes), dtype=np.uint8)
        if data is not None:
            b = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else \
                data.view(np.uint8).reshape(-1)
            arr[:b.size] = b
        self.regions.append((base, arr))
        self.next = base + arr.size + 4096
        return base

    def find(self, addr: int, n: int):
        for base, arr in self.regions:
            if base <= addr and addr + n <= base + arr.size:
                return arr, addr - base
        raise EmuError("bad address 0x%x (+%d)" % (addr, n))

    def read(self, addr: int, n: int) -> bytes:
        arr, o = self.find(addr, n)
        return arr[o:o + n].tobytes()

    def write(self, addr: int, data: bytes):
        arr, o = self.find(addr, len(data))
        arr[o:o + len(data)] = np.frombuffer(data, dtype=np.uint8)

    def r32(self, addr):
        return struct.unpack('<I', self.read(addr, 4))[0]

    def r64(self, addr):
        return struct.unpack('<Q', self.read(addr, 8))[0]

    def view(self, addr: int, n: int) -> np.ndarray:
        arr, o = self.find(addr, n)
        return arr[o:o + n]


# ------------------------------------------------------------------------------------------------------------------
REG = re.compile(r'^([vs])(\d+)$|^([vs])\[(\d+):(\d+)\]$')
FLOAT_INLINE = {'0.5': 0x3F000000, '-0.5': 0xBF000000, '1.0': 0x3F800000, '-1.0': 0xBF800000, '2.0': 0x40000000,
                '-2.0': 0xC0000000, '4.0': 0x40800000, '-4.0': 0xC0800000}


def f32(u):
    return np.array(u, dtype=np.uint32).view(np.float32)


def u32f(f):
    return np.asarray(f, dtype=np.float32).view(np.uint32)


class Insn:
    __slots__ = ('op', 'ops', 'mods', 'line', 'text')

    def __init__(self, line, text):
        self.line = line
        self.text = text
        f = text.split(None, 1)
        self.op = f[0]
        rest = f[1] if len(f) > 1 else ''
        parts = [p.strip() for p in rest.split(',')] if rest else []
        self.mods = {}
        if parts:
            last = parts[-1].split()
            parts[-1] = last[0] if last else ''
            for m in last[1:]:
                if ':' in m:
                    k, v = m.split(':', 1)
                    self.mods[k] = v
                else:
                    self.mods[m] = True
            if parts[-1] == '':
                parts.pop()
        self.ops = parts


def load_function(path: str, name: str):
    lines = open(path).read().split('\n')
    insns, labels = [], {}
    on = False
    for i, raw in enumerate(lines, 1):
        if raw.startswith(name + ':'):
            on = True
            continue
        if not on:
            continue
        if raw.strip().startswith('.Lfunc_end'):
            break
        m = re.match(r'^(\.LBB\w+):', raw)
        if m:
            labels[m.group(1)] = len(insns)
            continue
        s = raw.split(';', 1)[0].strip()
        if not s or s.startswith('.') or s.endswith(':'):
            continue
        insns.append(Insn(i, s))
    if not insns:
        raise EmuError('function %s not found' % name)
    return insns, labels


# ------------------------------------------------------------------------------------------------------------------
class Wave:
    def __init__(self, wg, wave_id: int):
        self.wg = wg
        self.id = wave_id
        self.v = np.zeros((512, 64), dtype=np.uint32)  # v509-v511: SDWA temporaries
        self.s = [0] * 128
        self.vcc = 0
        self.exec = M64
        self.scc = 0
        self.m0 = 0
        self.pc = 0
        self.done = False
        self.at_barrier = False
        self.count = 0

    # ---- scalar operand access
    def sget(self, t: str, width=32) -> int:
        t = t.strip()
        if t in ('vcc', 'vcc_lo', 'vcc_hi', 'exec', 'exec_lo', 'exec_hi'):
            full = self.vcc if t.startswith('vcc') else self.exec
            if t.endswith('_lo'):
                return full & M32
            if t.endswith('_hi'):
                return full >> 32
            return full if width == 64 else full & M32
        if t == 'scc':
            return self.scc
        if t == 'm0':
            return self.m0
        if t == 'off':
            return 0
        m = REG.match(t)
        if m:
            if m.group(1) == 's':
                return self.s[int(m.group(2))]
            if m.group(3) == 's':
                a, b = int(m.group(4)), int(m.group(5))
                v = 0
                for k in range(b, a - 1, -1):
                    v = (v << 32) | self.s[k]
                return v
            raise EmuError('vector operand where scalar expected: ' + t)
        if t in FLOAT_INLINE:
            return FLOAT_INLINE[t]
        v = int(t, 0)
        if width == 64:
            return v & M64  # inline constants sign-extend to 64 bits
        return v & M32

    def sset(self, t: str, val: int):
        t = t.strip()
        if t in ('vcc', 'exec'):
            if t == 'vcc':
                self.vcc = val & M64
            else:
                self.exec = val & M64
            return
        if t in ('vcc_lo', 'vcc_hi', 'exec_lo', 'exec_hi'):
            full = self.vcc if t.startswith('vcc') else self.exec
            if t.endswith('_lo'):
                full = (full & ~M32 & M64) | (val & M32)
            else:
                full = (full & M32) | ((val & M32) << 32)
            if t.startswith('vcc'):
                self.vcc = full
            else:
                self.exec = full
            return
        if t == 'm0':
            self.m0 = val & M32
            return
        m = REG.match(t)
        if m and m.group(1) == 's':
            self.s[int(m.group(2))] = val & M32
            return
        if m and m.group(3) == 's':
            a, b = int(m.group(4)), int(m.group(5))
            for k in range(a, b + 1):
                self.s[k] = val & M32
                val >>= 32
            return
        raise EmuError('bad scalar destination ' + t)

    # ---- vector operand access (returns np.uint64 per-lane values for 64-bit, uint32 otherwise)
    def vget(self, t: str, width=32):
        t = t.strip()
        m = REG.match(t)
        if m and m.group(1) == 'v':
            return self.v[int(m.group(2))].copy()
        if m and m.group(3) == 'v':
            a, b = int(m.group(4)), int(m.group(5))
            if width == 64 or b == a + 1:
                return self.v[a].astype(np.uint64) | (self.v[a + 1].astype(np.uint64) << np.uint64(32))
            raise EmuError('wide vector operand ' + t)
        x = self.sget(t, width)
        if width == 64:
            return np.full(64, x, dtype=np.uint64)
        return np.full(64, x & M32, dtype=np.uint32)

    def vset(self, t: str, val, mask=None):
        t = t.strip()
        act = self.active() if mask is None else mask
        m = REG.match(t)
        if m and m.group(1) == 'v':
            r = int(m.group(2))
            self.v[r][act] = np.asarray(val).astype(np.uint64)[act].astype(np.uint32) if \
                np.asarray(val).dtype == np.uint64 else np.asarray(val, dtype=np.uint32)[act]
            return
        if m and m.group(3) == 'v':
            a, b = int(m.group(4)), int(m.group(5))
            val = np.asarray(val)
            if b == a + 1:
                v64 = val.astype(np.uint64)
                self.v[a][act] = (v64 & np.uint64(M32)).astype(np.uint32)[act]
                self.v[a + 1][act] = (v64 >> np.uint64(32)).astype(np.uint32)[act]
                return
            raise EmuError('wide vset ' + t)
        raise EmuError('bad vector destination ' + t)

    def active(self):
        return ((np.uint64(self.exec) >> LANES.astype(np.uint64)) & np.uint64(1)).astype(bool)

    @staticmethod
    def bits(mask: int):
        return ((np.uint64(mask) >> LANES.astype(np.uint64)) & np.uint64(1)).astype(bool)

    @staticmethod
    def pack(boolarr) -> int:
        return int(np.sum(np.asarray(boolarr, dtype=np.uint64) << LANES.astype(np.uint64)))


# ------------------------------------------------------------------------------------------------------------------
def sdwa_sel(val, sel):
    val = val.astype(np.uint32)
    if sel in (None, 'DWORD'):
        return val
    if sel == 'WORD_0':
        return val & np.uint32(0xFFFF)
    if sel == 'WORD_1':
        return val >> np.uint32(16)
    if sel.startswith('BYTE_'):
        k = int(sel[5:])
        return (val >> np.uint32(8 * k)) & np.uint32(0xFF)
    raise EmuError('sdwa sel ' + sel)


def perm_byte(s0, s1, sel):
    """v_perm_b32 byte select: 0-7 bytes of {s0, s1} (s1 = bytes 0-3), 8-11 sign bits, 12 zero, >= 13 0xFF."""
    cat = (s0.astype(np.uint64) << np.uint64(32)) | s1.astype(np.uint64)
    out = np.zeros(64, dtype=np.uint32)
    for k in range(4):
        sb = (sel >> np.uint32(8 * k)) & np.uint32(0xFF)
        by = ((cat >> (np.uint64(8) * (sb.astype(np.uint64) & np.uint64(7)))) & np.uint64(0xFF)).astype(np.uint32)
        r = np.where(sb < 8, by, 0).astype(np.uint32)
        r = np.where(sb == 8, np.where((s1 >> np.uint32(15)) & np.uint32(1), 0xFF, 0), r)
        r = np.where(sb == 9, np.where((s1 >> np.uint32(31)) & np.uint32(1), 0xFF, 0), r)
        r = np.where(sb == 10, np.where((s0 >> np.uint32(15)) & np.uint32(1), 0xFF, 0), r)
        r = np.where(sb == 11, np.where((s0 >> np.uint32(31)) & np.uint32(1), 0xFF, 0), r)
        r = np.where(sb == 12, 0, r)
        r = np.where(sb >= 13, 0xFF, r)
        out |= (r.astype(np.uint32) & np.uint32(0xFF)) << np.uint32(8 * k)
    return out


CMP = {'eq': np.equal, 'ne': np.not_equal, 'lt': np.less, 'le': np.less_equal, 'gt': np.greater,
       'ge': np.greater_equal, 'lg': np.not_equal}


class Workgroup:
    def __init__(self, mem: Memory, insns, labels, nthreads: int, lds_bytes: int, kernarg: int, wg_id: int,
                 trace=None):
        self.mem = mem
        self.insns = insns
        self.labels = labels
        self.lds = np.zeros(lds_bytes, dtype=np.uint8)
        self.waves = []
        for w in range((nthreads + 63) // 64):
            wv = Wave(self, w)
            wv.s[0], wv.s[1] = kernarg & M32, kernarg >> 32
            wv.s[2] = wg_id
            wv.v[0] = LANES + np.uint32(64 * w)
            self.waves.append(wv)
        self.trace = trace

    # -- memory helpers
    def lds_read32(self, addrs, act):
        out = np.zeros(64, dtype=np.uint32)
        for l in np.nonzero(act)[0]:
            a = int(addrs[l])
            out[l] = struct.unpack('<I', self.lds[a:a + 4].tobytes())[0]
        return out

    def run(self, max_steps=10_000_000, waves=None):
        steps = 0
        pending = list(range(len(self.waves))) if waves is None else list(waves)
        # phase: run every wave to its barrier / end, release the barrier, repeat
        while True:
            progressed = False
            for wi in pending:
                w = self.waves[wi]
                while not w.done and not w.at_barrier:
                    self.step(w)
                    steps += 1
                    progressed = True
                    if steps > max_steps:
                        raise EmuError('step limit')
            live = [self.waves[i] for i in pending if not self.waves[i].done]
            if not live:
                return steps
            if all(w.at_barrier for w in live):
                for w in live:
                    w.at_barrier = False
                continue
            if not progressed:
                raise EmuError('deadlock')

    # -- one instruction
    def step(self, w: Wave):
        k = self.insns[w.pc]
        w.pc += 1
        w.count += 1
        op, o = k.op, k.ops
        try:
            self.exec_insn(w, k, op, o)
        except EmuError:
            raise
        except Exception as e:  # pragma: no cover
            raise EmuError('line %d: %s: %s' % (k.line, k.text, e))
        if self.trace:
            self.trace(w, k)

    def branch(self, w, label):
        w.pc = self.labels[label]

    def exec_insn(self, w, k, op, o):
        act = w.active()
        # ---------------- scalar control
        if op in ('s_waitcnt', 's_nop', 's_setprio', 's_sleep', 'buffer_wbl2', 'buffer_inv') or op.startswith('sched_'):
            return  # every memory op completes before the next instruction: waits and cache maintenance are no-ops
        if op == 's_endpgm':
            w.done = True
            return
        if op == 's_barrier':
            w.at_barrier = True
            return
        if op == 's_branch':
            return self.branch(w, o[0])
        if op.startswith('s_cbranch_'):
            c = op[10:]
            take = {'scc0': w.scc == 0, 'scc1': w.scc == 1, 'vccz': w.vcc == 0, 'vccnz': w.vcc != 0,
                    'execz': w.exec == 0, 'execnz': w.exec != 0}[c]
            if take:
                self.branch(w, o[0])
            return
        # ---------------- scalar memory
        if op.startswith('s_load_dword'):
            n = {'s_load_dword': 1, 's_load_dwordx2': 2, 's_load_dwordx4': 4, 's_load_dwordx8': 8,
                 's_load_dwordx16': 16}[op]
            base = w.sget(o[1], 64) & ~3
            off = w.sget(o[2]) if len(o) > 2 else 0
            data = self.mem.read(base + off, 4 * n)
            vals = struct.unpack('<%dI' % n, data)
            m = REG.match(o[0])
            first = int(m.group(2)) if m.group(1) else int(m.group(4))
            for i, v in enumerate(vals):
                w.s[first + i] = v
            return
        # ---------------- SALU
        if op.startswith('s_'):
            return self.salu(w, k, op, o)
        # ---------------- vector memory
        if op.startswith('global_'):
            return self.gmem(w, k, op, o, act)
        if op.startswith('ds_'):
            return self.lds_op(w, k, op, o, act)
        if op.startswith('v_'):
            return self.valu(w, k, op, o, act)
        raise EmuError('unknown opcode ' + k.text)

    # ------------------------------------------------------------------------------------------------------------
    def salu(self, w, k, op, o):
        g = w.sget

        def b64(t):
            return g(t, 64)

        if op in ('s_mov_b32', 's_movk_i32'):
            v = g(o[1])
            if op == 's_movk_i32':
                v = v & 0xFFFF
                v = v - 0x10000 if v & 0x8000 else v
            w.sset(o[0], v & M32)
            return
        if op == 's_mov_b64':
            w.sset(o[0], b64(o[1]))
            return
        if op in ('s_and_saveexec_b64', 's_or_saveexec_b64', 's_andn2_saveexec_b64', 's_xor_saveexec_b64'):
            src = b64(o[1])
            old = w.exec
            w.sset(o[0], old)
            if op == 's_and_saveexec_b64':
                w.exec = src & old
            elif op == 's_or_saveexec_b64':
                w.exec = src | old
            elif op == 's_andn2_saveexec_b64':
                w.exec = src & ~old & M64
            else:
                w.exec = src ^ old
            w.scc = int(w.exec != 0)
            return
        m = re.match(r's_(and|or|xor|andn2|orn2|nand|nor|xnor)_b(32|64)$', op)
        if m:
            f, wd = m.group(1), int(m.group(2))
            msk = M64 if wd == 64 else M32
            a, b = g(o[1], wd) & msk, g(o[2], wd) & msk
            r = {'and': a & b, 'or': a | b, 'xor': a ^ b, 'andn2': a & ~b, 'orn2': a | ~b, 'nand': ~(a & b),
                 'nor': ~(a | b), 'xnor': ~(a ^ b)}[f] & msk
            w.sset(o[0], r)
            w.scc = int(r != 0)
            return
        if op in ('s_not_b32', 's_not_b64'):
            wd = 64 if op.endswith('64') else 32
            msk = M64 if wd == 64 else M32
            r = ~g(o[1], wd) & msk
            w.sset(o[0], r)
            w.scc = int(r != 0)
            return
        if op == 's_add_u32':
            a, b = g(o[1]), g(o[2])
            r = a + b
            w.sset(o[0], r & M32)
            w.scc = int(r > M32)
            return
        if op == 's_addc_u32':
            a, b = g(o[1]), g(o[2])
            r = a + b + w.scc
            w.sset(o[0], r & M32)
            w.scc = int(r > M32)
            return
        if op == 's_sub_u32':
            a, b = g(o[1]), g(o[2])
            w.sset(o[0], (a - b) & M32)
            w.scc = int(b > a)
            return
        if op == 's_subb_u32':
            a, b = g(o[1]), g(o[2])
            r = a - b - w.scc
            w.sset(o[0], r & M32)
            w.scc = int(r < 0)
            return
        if op in ('s_add_i32', 's_sub_i32'):
            a, b = g(o[1]), g(o[2])
            sa = a - (1 << 32) if a >> 31 else a
            sb = b - (1 << 32) if b >> 31 else b
            r = sa + sb if op == 's_add_i32' else sa - sb
            w.sset(o[0], r & M32)
            w.scc = int(r < -(1 << 31) or r >= (1 << 31))
            return
        if op in ('s_addk_i32', 's_mulk_i32'):  # sdst op= sign-extended 16-bit immediate
            a, k16 = g(o[0]), g(o[1]) & 0xFFFF
            sa = a - (1 << 32) if a >> 31 else a
            sk = k16 - 0x10000 if k16 & 0x8000 else k16
            r = sa + sk if op == 's_addk_i32' else sa * sk
            w.sset(o[0], r & M32)
            if op == 's_addk_i32':
                w.scc = int(r < -(1 << 31) or r >= (1 << 31))
            return
        if op == 's_mul_i32':
            w.sset(o[0], (g(o[1]) * g(o[2])) & M32)
            return
        if op == 's_mul_hi_u32':
            w.sset(o[0], ((g(o[1]) * g(o[2])) >> 32) & M32)
            return
        if op in ('s_lshl_b32', 's_lshr_b32', 's_lshl_b64', 's_lshr_b64', 's_ashr_i32'):
            wd = 64 if op.endswith('64') else 32
            msk = M64 if wd == 64 else M32
            a, sh = g(o[1], wd) & msk, g(o[2]) & (wd - 1)
            if op.startswith('s_lshl'):
                r = (a << sh) & msk
            elif op.startswith('s_lshr'):
                r = a >> sh
            else:
                sa = a - (1 << 32) if a >> 31 else a
                r = (sa >> sh) & M32
            w.sset(o[0], r)
            w.scc = int(r != 0)
            return
        if op in ('s_min_u32', 's_max_u32', 's_min_i32', 's_max_i32'):
            a, b = g(o[1]), g(o[2])
            if op.endswith('i32'):
                a2 = a - (1 << 32) if a >> 31 else a
                b2 = b - (1 << 32) if b >> 31 else b
            else:
                a2, b2 = a, b
            if 'min' in op:
                r, w.scc = (a, 1) if a2 < b2 else (b, 0)
            else:
                r, w.scc = (a, 1) if a2 > b2 else (b, 0)
            w.sset(o[0], r)
            return
        if op in ('s_cselect_b32', 's_cselect_b64'):
            wd = 64 if op.endswith('64') else 32
            w.sset(o[0], g(o[1], wd) if w.scc else g(o[2], wd))
            return
        m = re.match(r's_cmp_(eq|lg|lt|le|gt|ge)_(u32|i32|u64)$', op)
        if m:
            c, t = m.group(1), m.group(2)
            wd = 64 if t == 'u64' else 32
            a, b = g(o[0], wd), g(o[1], wd)
            if t == 'i32':
                a = a - (1 << 32) if a >> 31 else a
                b = b - (1 << 32) if b >> 31 else b
            w.scc = int({'eq': a == b, 'lg': a != b, 'lt': a < b, 'le': a <= b, 'gt': a > b, 'ge': a >= b}[c])
            return
        if op == 's_bfe_u32':
            x, c = g(o[1]), g(o[2])
            r = (x >> (c & 31)) & ((1 << ((c >> 16) & 0x7F)) - 1) & M32
            w.sset(o[0], r)
            w.scc = int(r != 0)
            return
        if op == 's_bfe_i32':
            x, c = g(o[1]), g(o[2])
            wd = (c >> 16) & 0x7F
            r = (x >> (c & 31)) & ((1 << wd) - 1) if wd else 0
            if wd and r >> (wd - 1) & 1:
                r -= 1 << wd
            r &= M32
            w.sset(o[0], r)
            w.scc = int(r != 0)
            return
        if op == 's_bitset1_b32':
            w.sset(o[0], g(o[0]) | (1 << (g(o[1]) & 31)))
            return
        if op == 's_bitcmp1_b32':
            w.scc = (g(o[0]) >> (g(o[1]) & 31)) & 1
            return
        if op == 's_bitcmp0_b32':
            w.scc = 1 - ((g(o[0]) >> (g(o[1]) & 31)) & 1)
            return
        if op == 's_bcnt1_i32_b64':
            r = bin(g(o[1], 64)).count('1')
            w.sset(o[0], r)
            w.scc = int(r != 0)
            return
        if op == 's_bcnt1_i32_b32':
            r = bin(g(o[1])).count('1')
            w.sset(o[0], r)
            w.scc = int(r != 0)
            return
        if op == 's_ff1_i32_b64':
            v = g(o[1], 64)
            w.sset(o[0], (v & -v).bit_length() - 1 if v else M32)
            return
        if op == 's_ff1_i32_b32':
            v = g(o[1])
            w.sset(o[0], (v & -v).bit_length() - 1 if v else M32)
            return
        raise EmuError('unknown SALU ' + k.text)

    # ------------------------------------------------------------------------------------------------------------
    def gmem(self, w, k, op, o, act):
        mem = self.mem
        off_imm = int(k.mods.get('offset', 0), 0) if 'offset' in k.mods else 0

        def addrs(vaddr_t, saddr_t):
            if saddr_t == 'off' or saddr_t is None:
                a = w.vget(vaddr_t, 64)
            else:
                base = w.sget(saddr_t, 64)
                a = w.vget(vaddr_t).astype(np.uint64) + np.uint64(base)
            return a + np.uint64(off_imm & M64 if off_imm >= 0 else (off_imm + (1 << 64)))

        if op.startswith('global_load_'):
            n = {'global_load_dword': 1, 'global_load_dwordx2': 2, 'global_load_dwordx3': 3,
                 'global_load_dwordx4': 4}[op]
            a = addrs(o[1], o[2] if len(o) > 2 else 'off')
            m = REG.match(o[0])
            first = int(m.group(2)) if m.group(1) else int(m.group(4))
            for l in np.nonzero(act)[0]:
                vals = struct.unpack('<%dI' % n, mem.read(int(a[l]), 4 * n))
                for i in range(n):
                    w.v[first + i][l] = vals[i]
            return
        if op.startswith('global_store_'):
            n = {'global_store_dword': 1, 'global_store_dwordx2': 2, 'global_store_dwordx4': 4}[op]
            a = addrs(o[0], o[2] if len(o) > 2 else 'off')
            m = REG.match(o[1])
            first = int(m.group(2)) if m.group(1) else int(m.group(4))
            for l in np.nonzero(act)[0]:
                mem.write(int(a[l]), struct.pack('<%dI' % n, *[int(w.v[first + i][l]) for i in range(n)]))
            return
        m = re.match(r'global_atomic_(add|umin|umax|smin|smax|or|and|xor|swap)(_x2)?$', op)
        if m:
            f, x2 = m.group(1), bool(m.group(2))
            ret = len(o) >= 4
            if ret:
                dst, vaddr, vdata, saddr = o[0], o[1], o[2], o[3]
            else:
                vaddr, vdata, saddr = o[0], o[1], o[2] if len(o) > 2 else 'off'
            a = addrs(vaddr, saddr)
            d = w.vget(vdata, 64) if x2 else w.vget(vdata)
            old_vals = np.zeros(64, dtype=np.uint64)
            for l in np.nonzero(act)[0]:
                ad = int(a[l])
                old = mem.r64(ad) if x2 else mem.r32(ad)
                x = int(d[l])
                new = {'add': old + x, 'umin': min(old, x), 'umax': max(old, x), 'or': old | x, 'and': old & x,
                       'xor': old ^ x, 'swap': x}[f] if f not in ('smin', 'smax') else None
                if new is None:
                    raise EmuError('atomic ' + op)
                new &= M64 if x2 else M32
                mem.write(ad, struct.pack('<Q' if x2 else '<I', new))
                old_vals[l] = old
            if ret:
                w.vset(dst, old_vals if x2 else old_vals.astype(np.uint32))
            return
        raise EmuError('unknown global op ' + k.text)

    def lds_op(self, w, k, op, o, act):
        off = int(k.mods.get('offset', 0), 0) if 'offset' in k.mods else 0
        if op == 'ds_read_b32':
            a = w.vget(o[1]).astype(np.int64) + off
            w.vset(o[0], self.lds_read32(a, act))
            return
        if op in ('ds_read_b64', 'ds_read_b96', 'ds_read_b128'):  # wider reads (the verify form's slot reads, round 5)
            n = {'ds_read_b64': 2, 'ds_read_b96': 3, 'ds_read_b128': 4}[op]
            a = w.vget(o[1]).astype(np.int64) + off
            m = REG.match(o[0])
            first = int(m.group(2)) if m.group(1) else int(m.group(4))
            for l in np.nonzero(act)[0]:
                ad = int(a[l])
                vals = struct.unpack('<%dI' % n, self.lds[ad:ad + 4 * n].tobytes())
                for i in range(n):
                    w.v[first + i][l] = vals[i]
            return
        if op in ('ds_write_b32', 'ds_write_b64', 'ds_write_b128'):
            n = {'ds_write_b32': 1, 'ds_write_b64': 2, 'ds_write_b128': 4}[op]
            a = w.vget(o[0]).astype(np.int64) + off
            m = REG.match(o[1])
            first = int(m.group(2)) if m.group(1) else int(m.group(4))
            for l in np.nonzero(act)[0]:
                ad = int(a[l])
                self.lds[ad:ad + 4 * n] = np.frombuffer(
                    struct.pack('<%dI' % n, *[int(w.v[first + i][l]) for i in range(n)]), dtype=np.uint8)
            return
        if op in ('ds_add_rtn_u32', 'ds_add_u32'):  # LDS atomic add; active lanes in lane order
            ret = op == 'ds_add_rtn_u32'
            a = w.vget(o[1] if ret else o[0]).astype(np.int64) + off
            data = w.vget(o[2] if ret else o[1])
            old_vals = np.zeros(64, dtype=np.uint32)
            for l in np.nonzero(act)[0]:
                ad = int(a[l])
                cur = struct.unpack('<I', self.lds[ad:ad + 4].tobytes())[0]
                old_vals[l] = cur
                self.lds[ad:ad + 4] = np.frombuffer(struct.pack('<I', (cur + int(data[l])) & M32), dtype=np.uint8)
            if ret:
                w.vset(o[0], old_vals)
            return
        if op in ('ds_min_u32', 'ds_min_u64'):  # non-returning LDS atomic min (the verify form's slot, round 5)
            x2 = op == 'ds_min_u64'
            a = w.vget(o[0]).astype(np.int64) + off
            data = w.vget(o[1], 64) if x2 else w.vget(o[1])
            fmt, nb = ('<Q', 8) if x2 else ('<I', 4)
            for l in np.nonzero(act)[0]:
                ad = int(a[l])
                cur = struct.unpack(fmt, self.lds[ad:ad + nb].tobytes())[0]
                self.lds[ad:ad + nb] = np.frombuffer(struct.pack(fmt, min(cur, int(data[l]))), dtype=np.uint8)
            return
        if op == 'ds_bpermute_b32':
            addr = w.vget(o[1]).astype(np.int64) + off
            data = w.vget(o[2])
            src = (addr >> 2) & 63
            out = np.where(act[src], data[src], 0).astype(np.uint32)  # a disabled source lane reads 0
            w.vset(o[0], out)
            return
        raise EmuError('unknown ds op ' + k.text)

    # ------------------------------------------------------------------------------------------------------------
    SDWA_TMP = (509, 510, 511)  # scratch VGPRs of the emulator (the kernels use at most 256)

    def sdwa(self, w, k, op, o, act):
        """VOP1/VOP2 SDWA: select bytes/words of the sources, run the plain op on temporaries, place the result per
        dst_sel / dst_unused."""
        if any(x.startswith('sext(') for x in o) or 'clamp' in k.mods:
            raise EmuError('sdwa modifier ' + k.text)
        t0, t1, td = self.SDWA_TMP
        if op.startswith('v_cmp_'):  # VOPC SDWA: the destination is an SGPR pair / VCC
            m = re.match(r'v_cmp_(\w+)_([ui])(16|32)_sdwa$', op)
            if not m:
                raise EmuError('sdwa compare ' + k.text)
            wide = m.group(3) == '32'  # a 32-bit compare of the (zero-extended, no sext) selected fields
            for i, (t, sel) in enumerate(zip(o[1:3], (k.mods.get('src0_sel'), k.mods.get('src1_sel')))):
                w.v[(t0, t1)[i]] = sdwa_sel(w.vget(t), sel) & np.uint32(0xFFFFFFFF if wide else 0xFFFF)
            plain = Insn(k.line, 'v_cmp_%s_%s32_e64 %s, v%d, v%d' % (m.group(1), m.group(2), o[0], t0, t1))
            if m.group(2) == 'i' and not wide:
                for t in (t0, t1):
                    w.v[t] = (w.v[t].astype(np.uint16).view(np.int16).astype(np.int32)).view(np.uint32)
            return self.valu(w, plain, plain.op, plain.ops, act)
        srcs = o[1:]
        ops = ['v%d' % td]
        for i, (t, sel) in enumerate(zip(srcs, (k.mods.get('src0_sel'), k.mods.get('src1_sel')))):
            if t == 'vcc':
                ops.append(t)
                continue
            w.v[(t0, t1)[i]] = sdwa_sel(w.vget(t), sel)
            ops.append('v%d' % (t0, t1)[i])
        plain = Insn(k.line, op[:-5] + ('_e64' if op[:-5].startswith('v_cmp') else '') + ' ' + ', '.join(ops))
        self.valu(w, plain, plain.op, plain.ops, act)
        r = w.v[td].copy()
        dsel, unused = k.mods.get('dst_sel', 'DWORD'), k.mods.get('dst_unused', 'UNUSED_PAD')
        if dsel != 'DWORD':
            old = w.vget(o[0])
            if dsel.startswith('BYTE_'):
                sh, m = 8 * int(dsel[5:]), np.uint32(0xFF)
            else:
                sh, m = 16 * int(dsel[5:]), np.uint32(0xFFFF)
            field = (r & m) << np.uint32(sh)
            fmask = m << np.uint32(sh)
            if unused == 'UNUSED_PRESERVE':
                r = (old & ~fmask) | field
            elif unused == 'UNUSED_PAD':
                r = field
            else:
                raise EmuError('sdwa dst_unused ' + k.text)
        w.vset(o[0], r)

    def valu(self, w, k, op, o, act):
        if op.endswith('_sdwa'):
            return self.sdwa(w, k, op, o, act)
        V = w.vget
        base = re.sub(r'_(e32|e64|sdwa|dpp)$', '', op)
        # compares
        m = re.match(r'v_cmp_(eq|ne|lt|le|gt|ge|lg)_(u32|i32|u64|i64)$', base)
        if m:
            c, t = m.group(1), m.group(2)
            wd = 64 if t.endswith('64') else 32
            if op.endswith('_e32'):
                dst, a_t, b_t = 'vcc', o[0] if o[0] != 'vcc' else o[1], o[-1]
                if o[0] == 'vcc':
                    a_t, b_t = o[1], o[2]
            else:
                dst, a_t, b_t = o[0], o[1], o[2]
            a, b = V(a_t, wd), V(b_t, wd)
            if t.startswith('i'):
                a = a.astype(np.int64 if wd == 64 else np.int32) if wd == 32 else a.astype(np.uint64).view(np.int64)
                b = b.astype(np.int64 if wd == 64 else np.int32) if wd == 32 else b.astype(np.uint64).view(np.int64)
                if wd == 32:
                    a = a.astype(np.uint32).view(np.int32)
                    b = b.astype(np.uint32).view(np.int32)
            r = CMP[c](a, b) & act  # inactive lanes write 0
            w.sset(dst, Wave.pack(r))
            return
        if base == 'v_mov_b32' and op.endswith('_dpp'):
            src = V(o[1])
            old = V(o[0])
            rs = int(k.mods.get('row_shr', '0'), 0) if 'row_shr' in k.mods else None
            if rs is None:
                raise EmuError('dpp control ' + k.text)
            bc = 'bound_ctrl' in k.mods
            lane_in_row = LANES % 16
            valid = lane_in_row >= rs
            srcl = (LANES - rs) % 64
            valid = valid & act[srcl]
            val = np.where(valid, src[srcl], np.uint32(0) if bc else old).astype(np.uint32)
            w.vset(o[0], val)
            return
        if op == 'v_readlane_b32':
            lane = w.sget(o[2]) & 63
            w.sset(o[0], int(V(o[1])[lane]))
            return
        if op == 'v_readfirstlane_b32':
            idx = np.nonzero(act)[0]
            lane = int(idx[0]) if idx.size else 0
            w.sset(o[0], int(V(o[1])[lane]))
            return
        if op == 'v_writelane_b32':
            lane = w.sget(o[2]) & 63
            w.v[int(REG.match(o[0]).group(2))][lane] = w.sget(o[1])
            return
        u = np.uint32
        if base == 'v_mov_b32':
            w.vset(o[0], V(o[1]))
            return
        if base == 'v_mov_b64':
            w.vset(o[0], V(o[1], 64))
            return
        if base == 'v_not_b32':
            w.vset(o[0], ~V(o[1]))
            return
        if base == 'v_bfrev_b32':
            x = V(o[1])
            r = np.zeros(64, dtype=np.uint32)
            for i in range(32):
                r |= ((x >> u(i)) & u(1)) << u(31 - i)
            w.vset(o[0], r)
            return
        if base in ('v_and_b32', 'v_or_b32', 'v_xor_b32'):
            a, b = V(o[1]), V(o[2])
            r = {'v_and_b32': a & b, 'v_or_b32': a | b, 'v_xor_b32': a ^ b}[base]
            w.vset(o[0], r)
            return
        if base == 'v_bitop3_b32':
            a, b, c = V(o[1]), V(o[2]), V(o[3])
            imm = int(k.mods['bitop3'], 0)
            r = np.zeros(64, dtype=np.uint32)
            for idx in range(8):
                if (imm >> idx) & 1:
                    ta = a if idx & 4 else ~a
                    tb = b if idx & 2 else ~b
                    tc = c if idx & 1 else ~c
                    r |= ta & tb & tc
            w.vset(o[0], r)
            return
        if base == 'v_and_or_b32':
            w.vset(o[0], (V(o[1]) & V(o[2])) | V(o[3]))
            return
        if base == 'v_perm_b32':
            w.vset(o[0], perm_byte(V(o[1]), V(o[2]), V(o[3])))
            return
        if base in ('v_add_u32', 'v_sub_u32', 'v_subrev_u32'):
            a, b = V(o[1]).astype(np.int64), V(o[2]).astype(np.int64)
            r = a + b if base == 'v_add_u32' else (a - b if base == 'v_sub_u32' else b - a)
            if 'clamp' in k.mods:
                r = np.clip(r, 0, M32)
            w.vset(o[0], (r & M32).astype(np.uint32))
            return
        if base == 'v_add3_u32':
            r = V(o[1]).astype(np.uint64) + V(o[2]).astype(np.uint64) + V(o[3]).astype(np.uint64)
            w.vset(o[0], (r & np.uint64(M32)).astype(np.uint32))
            return
        if base in ('v_add_co_u32', 'v_sub_co_u32', 'v_subrev_co_u32', 'v_addc_co_u32', 'v_subb_co_u32'):
            dst, cd, a_t, b_t = o[0], o[1], o[2], o[3]
            a, b = V(a_t).astype(np.int64), V(b_t).astype(np.int64)
            cin = Wave.bits(w.sget(o[4], 64)).astype(np.int64) if len(o) > 4 else 0
            if base == 'v_add_co_u32':
                r = a + b
                co = r > M32
            elif base == 'v_addc_co_u32':
                r = a + b + cin
                co = r > M32
            elif base == 'v_sub_co_u32':
                r = a - b
                co = r < 0
            elif base == 'v_subrev_co_u32':
                r = b - a
                co = r < 0
            else:
                r = a - b - cin
                co = r < 0
            w.vset(dst, (r & M32).astype(np.uint32))
            w.sset(cd, Wave.pack(co & act))
            return
        if base in ('v_lshlrev_b32', 'v_lshrrev_b32', 'v_ashrrev_i32'):
            sh, x = V(o[1]) & u(31), V(o[2])
            if base == 'v_lshlrev_b32':
                r = x << sh
            elif base == 'v_lshrrev_b32':
                r = x >> sh
            else:
                r = (x.view(np.int32) >> sh.astype(np.int32)).view(np.uint32)
            w.vset(o[0], r)
            return
        if base in ('v_lshlrev_b64', 'v_lshrrev_b64'):
            sh, x = (V(o[1]) & u(63)).astype(np.uint64), V(o[2], 64)
            r = (x << sh) if base == 'v_lshlrev_b64' else (x >> sh)
            w.vset(o[0], r)
            return
        if base == 'v_lshl_add_u64':
            a, sh, b = V(o[1], 64), (V(o[2]) & u(7)).astype(np.uint64), V(o[3], 64)
            w.vset(o[0], (a << sh) + b)
            return
        if base == 'v_lshl_or_b32':
            a, sh, b = V(o[1]), V(o[2]) & u(31), V(o[3])
            w.vset(o[0], (a << sh) | b)
            return
        if base == 'v_mad_u32_u24':
            a, b, c = V(o[1]) & u(0xFFFFFF), V(o[2]) & u(0xFFFFFF), V(o[3])
            w.vset(o[0], ((a.astype(np.uint64) * b.astype(np.uint64) + c) & np.uint64(M32)).astype(np.uint32))
            return
        if base == 'v_lshl_add_u32':
            a, sh, b = V(o[1]), V(o[2]) & u(31), V(o[3])
            w.vset(o[0], ((a << sh) + b) & u(M32))
            return
        if base == 'v_alignbit_b32':
            a, b, sh = V(o[1]).astype(np.uint64), V(o[2]).astype(np.uint64), (V(o[3]) & u(31)).astype(np.uint64)
            w.vset(o[0], (((a << np.uint64(32)) | b) >> sh) & np.uint64(M32))
            return
        if base in ('v_bfe_u32', 'v_bfe_i32'):
            x, off, wd = V(o[1]), V(o[2]) & u(31), V(o[3]) & u(31)
            mask = np.where(wd == 0, 0, (np.uint64(1) << wd.astype(np.uint64)) - np.uint64(1)).astype(np.uint64)
            r = ((x.astype(np.uint64) >> off.astype(np.uint64)) & mask).astype(np.uint64)
            if base == 'v_bfe_i32':
                sign = np.where(wd > 0, (r >> (wd.astype(np.uint64) - np.uint64(1)).clip(0)) & np.uint64(1), 0)
                r = np.where(sign.astype(bool), r | (~mask & np.uint64(M32)), r)
            w.vset(o[0], (r & np.uint64(M32)).astype(np.uint32))
            return
        if base in ('v_min_u32', 'v_max_u32', 'v_min_i32', 'v_max_i32'):
            a, b = V(o[1]), V(o[2])
            if base.endswith('i32'):
                a, b = a.view(np.int32), b.view(np.int32)
            r = np.minimum(a, b) if 'min' in base else np.maximum(a, b)
            w.vset(o[0], r.view(np.uint32) if r.dtype == np.int32 else r)
            return
        if base in ('v_min3_u32', 'v_max3_u32'):
            a, b, c = V(o[1]), V(o[2]), V(o[3])
            r = np.minimum(np.minimum(a, b), c) if 'min' in base else np.maximum(np.maximum(a, b), c)
            w.vset(o[0], r)
            return
        if base == 'v_cndmask_b32':
            a, b = V(o[1]), V(o[2])
            msk = Wave.bits(w.sget(o[3], 64) if len(o) > 3 else w.vcc)
            w.vset(o[0], np.where(msk, b, a))
            return
        if base in ('v_mbcnt_lo_u32_b32', 'v_mbcnt_hi_u32_b32'):
            msk, src = w.sget(o[1]), V(o[2])
            r = np.zeros(64, dtype=np.uint32)
            for l in range(64):
                if base.endswith('lo_u32_b32'):
                    tm = ((1 << l) - 1) & M32 if l < 32 else M32
                else:
                    tm = 0 if l < 32 else ((1 << (l - 32)) - 1) & M32
                r[l] = bin(msk & tm).count('1')
            w.vset(o[0], r + src)
            return
        if base == 'v_mul_lo_u32':
            w.vset(o[0], ((V(o[1]).astype(np.uint64) * V(o[2]).astype(np.uint64)) & np.uint64(M32)).astype(np.uint32))
            return
        if base == 'v_mul_hi_u32':
            w.vset(o[0], ((V(o[1]).astype(np.uint64) * V(o[2]).astype(np.uint64)) >> np.uint64(32)).astype(np.uint32))
            return
        if base == 'v_mad_u64_u32':
            a, b, c = V(o[2]).astype(object), V(o[3]).astype(object), V(o[4], 64).astype(object)
            r = [(int(a[l]) * int(b[l]) + int(c[l])) for l in range(64)]
            w.vset(o[0], np.array([x & M64 for x in r], dtype=np.uint64))
            w.sset(o[1], Wave.pack(np.array([x > M64 for x in r]) & act))
            return
        # floats (used by the integer division sequences)
        if base == 'v_cvt_f32_u32':
            w.vset(o[0], u32f(V(o[1]).astype(np.float32)))
            return
        if base == 'v_cvt_f32_ubyte0':
            w.vset(o[0], u32f((V(o[1]) & u(0xFF)).astype(np.float32)))
            return
        if base == 'v_cvt_u32_f32':
            f = f32(V(o[1])).astype(np.float64)
            f = np.nan_to_num(f, nan=0.0)
            w.vset(o[0], np.clip(np.trunc(f), 0, M32).astype(np.uint64).astype(np.uint32))
            return
        if base == 'v_trunc_f32':
            w.vset(o[0], u32f(np.trunc(f32(V(o[1])))))
            return
        if base in ('v_rcp_f32', 'v_rcp_iflag_f32'):
            with np.errstate(divide='ignore'):
                w.vset(o[0], u32f(np.float32(1.0) / f32(V(o[1]))))
            return
        if base == 'v_mul_f32':
            w.vset(o[0], u32f(f32(V(o[1])) * f32(V(o[2]))))
            return
        if base == 'v_fmac_f32':
            a, b, c = f32(V(o[1])).astype(np.float64), f32(V(o[2])).astype(np.float64), f32(V(o[0])).astype(
                np.float64)
            w.vset(o[0], u32f((a * b + c).astype(np.float32)))
            return
        if base == 'v_fmamk_f32':
            a, kk, c = f32(V(o[1])).astype(np.float64), f32(V(o[2])).astype(np.float64), f32(V(o[3])).astype(
                np.float64)
            w.vset(o[0], u32f((a * kk + c).astype(np.float32)))
            return
        raise EmuError('unknown VALU ' + k.text)


# ------------------------------------------------------------------------------------------------------------------
# PiecesArgs (csrc/crc32c_fold.inc) field offsets; the hidden arguments follow the 184-byte struct
PIECES_ARGS = {"base": 0, "off": 8, "len": 16, "init": 24, "out": 32, "count": 40, "pstart": 48, "pblk": 56,
               "partial": 64, "work_counter": 72, "piece_bytes": 80, "zpiece": 88, "max_pieces": 96,
               "static_contig": (104, "<I"), "guided_div": (108, "<I"), "guided_cap": (112, "<I"), "hint": 120,
               "expect": 128, "first_bad": 136, "nbad": 144, "tabs": 152, "vacc": 160, "vslot": 168,
               "vslot_base": (176, "<I")}
ARGS_BYTES = 184
# the verify accumulators (crc32c_device.hip, PiecesArgs::vacc): u64 words; [0] lowest block, [1] final arrival word
# (arrived << 40) | mismatches, shard s's arrival word at [16 (s + 1)] (the combine kernel's two-level arrival)
VACC_STRIDE, VACC_SHARDS = 16, 8


def pieces_kernarg(fields: dict, grid: int, threads: int) -> bytes:
    ka = bytearray(ARGS_BYTES + 256)
    for k, v in fields.items():
        spec = PIECES_ARGS[k]
        o, fmt = spec if isinstance(spec, tuple) else (spec, "<Q")
        struct.pack_into(fmt, ka, o, v)
    struct.pack_into("<III", ka, ARGS_BYTES, grid, 1, 1)         # hidden_block_count_x/y/z
    struct.pack_into("<HHH", ka, ARGS_BYTES + 12, threads, 1, 1)  # hidden_group_size_x/y/z
    struct.pack_into("<H", ka, ARGS_BYTES + 64, 1)                # hidden_grid_dims
    return bytes(ka)


_FN_CACHE = {}


def kernel_code(asm: str, name: str):
    key = (asm, name, os.path.getmtime(asm))
    if key not in _FN_CACHE:
        _FN_CACHE[key] = load_function(asm, name)
    return _FN_CACHE[key]


def group_segment_bytes(asm: str, name: str) -> int:
    """The kernel's LDS size from its .amdhsa_kernel descriptor in the assembly (0 if not found)."""
    key = ("lds", asm, name, os.path.getmtime(asm))
    if key not in _FN_CACHE:
        text = open(asm).read()
        m = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"\s.*?\.amdhsa_group_segment_fixed_size (\d+)", text,
                      re.S)
        _FN_CACHE[key] = int(m.group(1)) if m else 0
    return _FN_CACHE[key]


def launch(mem: Memory, asm: str, name: str, threads: int, lds_bytes: int, fields: dict, grid: int, wgs=None) -> int:
    """Run workgroups `wgs` (default: the whole grid, one after another) of a PiecesArgs kernel; returns the number of
    wave-instructions executed.  Workgroups run to completion in order, so a dynamic (atomic-counter) schedule hands
    every item to the first workgroup -- functionally the same result, a different interleaving.  The LDS is at least
    the kernel's own group segment size."""
    insns, labels = kernel_code(asm, name)
    lds_bytes = max(lds_bytes, group_segment_bytes(asm, name))
    d_ka = mem.alloc(ARGS_BYTES + 256, data=pieces_kernarg(fields, grid, threads))
    steps = 0
    for g in (range(grid) if wgs is None else wgs):
        steps += Workgroup(mem, insns, labels, threads, lds_bytes, d_ka, g).run()
    return steps


SENTINEL = 0xDEADBEEF


def batch_memory(data, off, ln, tabs: bytes, expect=None, last_of=None, shards: int = 1):
    """Device image of one batch call: payload, descriptors, results (sentinel-filled), tables, verify words.  The
    caller's result words start as a sentinel (the kernels must write them); the accumulators in their reset state,
    except with last_of = (wg, grid): every other workgroup of the grid counts as arrived already, so emulating that
    one workgroup is the last, publishing one (shards > 1: a two-level arrival, verify_publish<kShards>: the rest of
    its shard on the shard word, the other shards' last workgroups on the final word)."""
    n = int(np.asarray(off).size)
    mem = Memory()
    f = {"base": mem.alloc(data.size + 65536, data=data), "off": mem.alloc(8 * n, data=np.asarray(off, np.uint64)),
         "len": mem.alloc(8 * n, data=np.asarray(ln, np.uint64)),
         "out": mem.alloc(4 * n, data=np.full(n, SENTINEL, np.uint32)), "count": n, "piece_bytes": 128 * 1024,
         "max_pieces": n, "static_contig": 1, "tabs": mem.alloc(len(tabs), data=tabs)}
    if expect is not None:
        f["expect"] = mem.alloc(4 * n, data=np.asarray(expect, np.uint32))
        f["first_bad"] = mem.alloc(8, data=np.array([SENTINEL], np.uint64))
        f["nbad"] = mem.alloc(8, data=np.array([SENTINEL], np.uint64))
        v = np.zeros(VACC_STRIDE * (1 + VACC_SHARDS), np.uint64)
        v[0] = ~np.uint64(0)
        if last_of is not None:
            wg, grid = last_of
            if shards == 1:  # one level: every workgroup on the final word
                v[1] = np.uint64(grid - 1) << np.uint64(40)
            else:
                sh = wg % shards
                v[VACC_STRIDE * (1 + sh)] = np.uint64((grid - sh + shards - 1) // shards - 1) << np.uint64(40)
                v[1] = np.uint64(min(grid, shards) - 1) << np.uint64(40)
        f["vacc"] = mem.alloc(8 * v.size, data=v)
    return mem, f


def accumulators(mem: Memory, f: dict):
    """The verify accumulators: (lowest posted block, final arrival word, the 8 shard arrival words)."""
    return (mem.r64(f["vacc"]), mem.r64(f["vacc"] + 8)) + tuple(
        mem.r64(f["vacc"] + 8 * VACC_STRIDE * (1 + s)) for s in range(VACC_SHARDS))


def batch_results(mem: Memory, f: dict, published: bool = True):
    """(out words, mask of blocks written, first_bad or -1, nbad); a verify call must also leave its accumulators in
    their reset state (~0, 0) for the next call"""
    out = mem.view(f["out"], 4 * f["count"]).view(np.uint32).copy()
    fb = mem.r64(f["first_bad"]) if "first_bad" in f else (1 << 64) - 1
    nb = mem.r64(f["nbad"]) if "nbad" in f else 0
    if published and "vacc" in f and accumulators(mem, f) != ((1 << 64) - 1,) + (0,) * (1 + VACC_SHARDS):
        raise EmuError("verify accumulators not reset: %s" % [hex(x) for x in accumulators(mem, f)])
    # a written word equals the sentinel only by chance (1 in 2^32): callers compare against the oracle
    return out, out != SENTINEL, (-1 if fb == (1 << 64) - 1 else fb), nb


def alloc_slots(mem: Memory, f: dict, n: int):
    """Verdict slots of a captured verify call (PiecesArgs::vslot, round 6): n (lowest block, count) pairs, sentinel-
    filled so an unwritten slot shows."""
    f["vslot"] = mem.alloc(16 * n, data=np.full(2 * n, SENTINEL, np.uint64))


def slots(mem: Memory, f: dict, n: int):
    v = mem.view(f["vslot"], 16 * n).view(np.uint64).reshape(n, 2)
    return [(int(a), int(b)) for a, b in v]


def run_batch_kernel(asm: str, name: str, threads: int, data: np.ndarray, off, ln, tabs: bytes, wg: int = 0,
                     grid: int = 256, hint: int = 0, expect=None, lds_bytes: int = 160768, last: bool = True,
                     state: dict | None = None, init=None, shards: int = 1, vslot: bool = False):
    """Run workgroup `wg` of a batch kernel (a PiecesArgs kernel in static, unplanned mode) over the given batch.
    Verify form: with `last` the other grid - 1 workgroups count as arrived, so this one publishes the verdict; without
    it, it is an early one and `state` (a dict) receives the accumulators it leaves.  vslot: a captured call's form --
    the workgroup writes its verdict slot (state["slots"]: every slot of the grid) and touches neither the
    accumulators nor the caller's words.
    Returns (out words, mask of blocks written, first_bad or -1, nbad, instructions executed)."""
    mem, f = batch_memory(data, off, ln, tabs, expect, last_of=(wg, grid) if last and not vslot else None,
                          shards=shards)
    f["hint"] = hint
    if vslot:
        alloc_slots(mem, f, grid)
    if init is not None:  # per-block initial CRCs (Extend(init[i], block i))
        f["init"] = mem.alloc(4 * len(init), data=np.asarray(init, np.uint32))
    steps = launch(mem, asm, name, threads, lds_bytes, f, grid, [wg])
    if state is not None and "vacc" in f:
        state["vacc"] = accumulators(mem, f)
    if state is not None and vslot:
        state["slots"] = slots(mem, f, grid)
    return batch_results(mem, f, published=last or vslot) + (steps,)


# DevTables field offsets (bytes), csrc/crc32c_device.hip
TAB_ZSMALL = 4096 * 9 + 1024 + 4096   # z1024, z4, ztree[6], byte1, zpiece, znarrow -> zsmall[0]


def run_planned_batch(asm: str, pieces: str, combine: str, data: np.ndarray, off, ln, tabs: bytes, piece_k: int = 0,
                      grid: int = 256, expect=None, state: dict | None = None):
    """One planned (split-block) call as launch_batch_in issues it: the piece table built on the host exactly as
    crc32c_plan_count_kernel / InclusiveSum / crc32c_plan_expand_kernel build it, the pieces kernel (dynamic
    schedule; one workgroup takes every item), then every workgroup of the combine kernel.  Pieces are
    zsmall[piece_k]'s 16 KiB << piece_k.  state (a dict, verify form): the call as captured -- verdict slots, the
    combine kernel's after the pieces kernel's (vslot_base = grid); state["slots"] receives them all.
    Returns (out, written, first_bad, nbad, instructions)."""
    ln = np.asarray(ln, np.uint64)
    n = ln.size
    P = (16 * 1024) << piece_k
    counts = np.where(ln < 2 * P, 1, ln // P).astype(np.uint64)
    pstart = np.zeros(n + 1, np.uint64)
    pstart[1:] = np.cumsum(counts, dtype=np.uint64)
    npieces = int(pstart[-1])
    pblk = np.repeat(np.arange(n, dtype=np.uint32), counts.astype(np.int64))
    mem, f = batch_memory(data, off, ln, tabs, expect)  # a split batch: the combine kernel's last workgroup publishes
    f.update(pstart=mem.alloc(8 * (n + 1), data=pstart), pblk=mem.alloc(4 * npieces, data=pblk),
             partial=mem.alloc(4 * npieces), work_counter=mem.alloc(16), piece_bytes=P, max_pieces=npieces,
             zpiece=f["tabs"] + TAB_ZSMALL + 4096 * piece_k, guided_div=0, guided_cap=0)
    # one workgroup takes every item; not workgroup 0, so its shard (5) is one the combine grid below may not have:
    # the planned kernel's counts must reach the publishing grid anyway
    cgrid = min((n + 255) // 256, 2048)  # kCombineMaxGrid
    if state is not None:
        alloc_slots(mem, f, grid + cgrid)
    steps = launch(mem, asm, pieces, 512, 160768, f, grid, [5])
    if state is not None:
        f["vslot_base"] = grid
    steps += launch(mem, asm, combine, 256, 4096, f, cgrid)
    if state is not None:
        state["slots"] = slots(mem, f, grid + cgrid)
    return batch_results(mem, f) + (steps,)


TABLES_DUMP = r'''
#include <cstdio>
#include "gf2.h"
using namespace kvsep;
struct DevTables { uint32_t z1024[4][256], z4[4][256], ztree[6][4][256], byte1[256], zpiece[4][256], znarrow[4][256],
                   zsmall[3][4][256], x2n[64], xinv[16]; };
int main() {
  static DevTables h;
  gf2::byte_tables(gf2::zero_bytes_map(1024), &h.z1024[0][0]);
  gf2::byte_tables(gf2::zero_bytes_map(4), &h.z4[0][0]);
  for (int j = 0; j < 6; ++j) gf2::byte_tables(gf2::zero_bytes_map(16ull << j), &h.ztree[j][0][0]);
  for (uint32_t b = 0; b < 256; ++b) h.byte1[b] = gf2::byte_table_entry(b);
  gf2::byte_tables(gf2::zero_bytes_map(128 * 1024), &h.zpiece[0][0]);
  for (int k = 0; k < 3; ++k) gf2::byte_tables(gf2::zero_bytes_map((16 * 1024ull) << k), &h.zsmall[k][0][0]);
  gf2::byte_tables(gf2::zero_bytes_map(128), &h.znarrow[0][0]);
  gf2::x2n_table(h.x2n);
  gf2::xinv_table(h.xinv);
  fwrite(&h, sizeof h, 1, stdout);
}
'''


def dev_tables(csrc=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc")) -> bytes:
    """The DevTables image upload_tables (csrc/crc32c_device.hip) copies to the device, built from the same gf2.h."""
    with tempfile.TemporaryDirectory() as t:
        src, exe = os.path.join(t, "d.cpp"), os.path.join(t, "d")
        open(src, "w").write(TABLES_DUMP)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", csrc, src, "-o", exe])
        img = subprocess.check_output([exe])
    assert len(img) == 4096 * 13 + 1024 + 256 + 64
    return img
