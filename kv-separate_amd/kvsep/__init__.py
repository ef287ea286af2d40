"""kvsep -- Python binding (ctypes) of libkvsep_crc32c.so for tests and bench.

The product is the C ABI in include/kvsep_crc32c.h (C++ host code + gfx950 HIP kernels); this module
only marshals arguments.  It mirrors the reference's util/crc32c.h interface (extend / value / mask /
unmask, util/crc32c.h:17-38) and adds the batched device/host entry points.

There is no CPU fallback here: if the shared library is missing, importing the GPU entry points
raises; if no gfx950 device is present, Context() raises.  The oracle under oracle/ is never used.
"""
from __future__ import annotations

import ctypes
import os
import re
import sys

try:  # torch first: its libamdhip64.so.7 then serves our library too (same soname, one HIP runtime)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host-only entry points
    torch = None

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkvsep_crc32c.so")
HEADER_PATH = os.path.join(_HERE, "..", "..", "include", "kvsep_crc32c.h")

KVSEP_OK = 0
MASK_DELTA = 0xA282EAD8  # util/crc32c.h:22

_lib = None


class KvsepError(RuntimeError):
    pass


def _u32p():
    return ctypes.POINTER(ctypes.c_uint32)


def _u64p():
    return ctypes.POINTER(ctypes.c_uint64)


_SIGS = {
    "kvsep_crc32c_extend": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    "kvsep_crc32c_value": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_size_t]),
    "kvsep_crc32c_mask": (ctypes.c_uint32, [ctypes.c_uint32]),
    "kvsep_crc32c_unmask": (ctypes.c_uint32, [ctypes.c_uint32]),
    "kvsep_accelerated_crc32c": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    "kvsep_set_offload_threshold": (None, [ctypes.c_uint64]),
    "kvsep_set_offload_wait": (None, [ctypes.c_int]),
    "kvsep_offload_stats": (None, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kvsep_crc32c_kernel_name": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
    "kvsep_crc32c_extend_host": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    "kvsep_crc32c_host_path": (ctypes.c_char_p, []),
    "kvsep_crc32c_ctx_set_host_node": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "kvsep_crc32c_ctx_host_placement": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                       ctypes.c_void_p, ctypes.c_int]),
    "kvsep_crc32c_ctx_inject_failure": (ctypes.c_int, [ctypes.c_void_p]),
    "kvsep_device_pci_bus_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "kvsep_pci_numa_node": (ctypes.c_int, [ctypes.c_char_p]),
    "kvsep_device_numa_node": (ctypes.c_int, [ctypes.c_int]),
    "kvsep_numa_node_cpus": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "kvsep_bind_process_numa": (ctypes.c_int, [ctypes.c_int]),
    "kvsep_host_page_node": (ctypes.c_int, [ctypes.c_void_p]),
    "kvsep_crc32c_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "kvsep_crc32c_ctx_destroy": (None, [ctypes.c_void_p]),
    "kvsep_crc32c_ctx_set_piece_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]),
    "kvsep_crc32c_ctx_set_schedule": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "kvsep_crc32c_ctx_set_kernel": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "kvsep_crc32c_reserve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]),
    "kvsep_crc32c_reserve_captures": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "kvsep_crc32c_release_captures": (ctypes.c_int, [ctypes.c_void_p]),
    "kvsep_crc32c_capture_sets": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "kvsep_crc32c_ctx_set_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "kvsep_crc32c_ctx_get_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                                   ctypes.POINTER(ctypes.c_uint64)]),
    "kvsep_crc32c_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_uint64]),
    "kvsep_crc32c_verify_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_uint64]),
    "kvsep_crc32c_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_uint64]),
    "kvsep_crc32c_batch_host_span": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_uint64]),
    "kvsep_fill_splitmix64_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                    ctypes.c_uint64]),
    "kvsep_stream_read_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                ctypes.c_void_p]),
    "kvsep_vlog_walk": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "kvsep_vlog_verify_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kvsep_vlog_frame_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "kvsep_log_walk": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]),
    "kvsep_log_verify_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.c_void_p]),
    "kvsep_log_frame_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "kvsep_log_accept": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_void_p]),
    "kvsep_sst_trailers_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_uint64]),
    "kvsep_sst_verify_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
    "kvsep_sst_trailers_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_uint64]),
    "kvsep_sst_verify_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint64]),
    "kvsep_crc32c_partition": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]),
    "kvsep_crc32c_group_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "kvsep_crc32c_group_destroy": (None, [ctypes.c_void_p]),
    "kvsep_crc32c_group_size": (ctypes.c_int, [ctypes.c_void_p]),
    "kvsep_crc32c_group_ctx": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int]),
    "kvsep_crc32c_group_batch_host_span": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_uint64]),
    "kvsep_crc32c_group_verify_host_span": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                           ctypes.c_void_p, ctypes.c_uint64]),
    "kvsep_vlog_verify_host_group": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "kvsep_crc32c_group_batch_device": (ctypes.c_int, [ctypes.c_void_p] * 9),
    "kvsep_crc32c_group_verify_device": (ctypes.c_int, [ctypes.c_void_p] * 13),
    "kvsep_host_alloc_pinned": (ctypes.c_void_p, [ctypes.c_uint64]),
    "kvsep_host_free_pinned": (None, [ctypes.c_void_p]),
    "kvsep_last_error": (ctypes.c_char_p, []),
    "kvsep_build_info": (ctypes.c_char_p, []),
    "kvsep_abi_version": (ctypes.c_int, []),
    "kvsep_device_count": (ctypes.c_int, []),
}


def lib():
    """Load libkvsep_crc32c.so (raises loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise KvsepError(f"{LIB_PATH} missing: run `make -C kv-separate_amd` (or __graft_entry__.build())")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def header_functions(path: str = HEADER_PATH):
    """Names of every function declared in include/kvsep_crc32c.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kvsep_[a-z0-9_]+)\s*\(", src)))


def _check(rc: int, what: str):
    if rc != KVSEP_OK:
        raise KvsepError(f"{what} failed ({rc}): {lib().kvsep_last_error().decode(errors='replace')}")


def _buf(data):
    """(ctypes pointer, keepalive) for bytes / bytearray / numpy arrays."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data)
        return a.ctypes.data_as(ctypes.c_void_p), a
    if isinstance(data, (bytes, bytearray, memoryview)):
        a = np.frombuffer(data, dtype=np.uint8)
        return a.ctypes.data_as(ctypes.c_void_p), a
    raise TypeError(type(data))


def _checked_len(keep, n):
    """n defaults to the whole buffer; a larger n would read past it."""
    if n is None:
        return keep.nbytes
    if n < 0 or n > keep.nbytes:
        raise ValueError(f"n = {n} outside the {keep.nbytes}-byte buffer")
    return n


# ------------------------------------------------------------------ scalar mirror of util/crc32c.h
def extend(init_crc: int, data, n: int | None = None) -> int:
    """leveldb::crc32c::Extend (util/crc32c.h:17)."""
    p, keep = _buf(data)
    n = _checked_len(keep, n)
    return lib().kvsep_crc32c_extend(init_crc & 0xFFFFFFFF, p, n)


def value(data, n: int | None = None) -> int:
    """leveldb::crc32c::Value (util/crc32c.h:20)."""
    return extend(0, data, n)


def mask(crc: int) -> int:
    """leveldb::crc32c::Mask (util/crc32c.h:29)."""
    return lib().kvsep_crc32c_mask(crc & 0xFFFFFFFF)


def unmask(masked: int) -> int:
    """leveldb::crc32c::Unmask (util/crc32c.h:35)."""
    return lib().kvsep_crc32c_unmask(masked & 0xFFFFFFFF)


def extend_host(init_crc: int, data, n: int | None = None) -> int:
    p, keep = _buf(data)
    n = _checked_len(keep, n)
    return lib().kvsep_crc32c_extend_host(init_crc & 0xFFFFFFFF, p, n)


def host_path() -> str:
    """The host leg this process runs ("fold", "sse42" or "portable"; kvsep_crc32c_host_path)."""
    return lib().kvsep_crc32c_host_path().decode()


# ------------------------------------------------------------------ device context
def _stream_handle(stream):
    if stream is None:
        if torch is not None and torch.cuda.is_available():
            return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        return ctypes.c_void_p(0)
    if hasattr(stream, "cuda_stream"):
        return ctypes.c_void_p(stream.cuda_stream)
    return ctypes.c_void_p(int(stream))


def _dptr(t):
    if t is None:
        return ctypes.c_void_p(0)
    if isinstance(t, int):
        return ctypes.c_void_p(t)
    return ctypes.c_void_p(t.data_ptr())


DEFAULT_PIECE_BYTES = 128 * 1024  # the library default (kvsep_crc32c_ctx, crc32c_device.hip)


class Context:
    """One per device: uploads the Z_d tables once, owns scratch and staging."""

    def __init__(self, device: int = 0, piece_bytes: int | None = None, dynamic: bool | None = None):
        h = ctypes.c_void_p()
        _check(lib().kvsep_crc32c_ctx_create(device, ctypes.byref(h)), "kvsep_crc32c_ctx_create")
        self._h = h
        self.device = device
        if piece_bytes is not None:
            self.set_piece_bytes(piece_bytes)
        if dynamic is not None:
            self.set_schedule(dynamic)

    def close(self):
        if getattr(self, "_h", None):
            lib().kvsep_crc32c_ctx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_piece_bytes(self, n: int):
        _check(lib().kvsep_crc32c_ctx_set_piece_bytes(self._h, n), "set_piece_bytes")

    def set_schedule(self, dynamic):
        """True = guided dynamic, False = static contiguous runs, "rr" = static round-robin items, None = auto
        (guided only when long blocks are split)."""
        v = -1 if dynamic is None else 2 if dynamic == "rr" else (1 if dynamic else 0)
        _check(lib().kvsep_crc32c_ctx_set_schedule(self._h, v), "set_schedule")

    KERNELS = {"auto": 0, "wide": 1, "narrow": 2, "narrow16": 3, "narrow8": 4, "sorted": 5, "claim": 6, "claim16": 7,
               "coop": 8}

    def set_kernel(self, kernel: str):
        """Kernel choice for unsplit batches (kvsep_crc32c_ctx_set_kernel): "auto" (default), "wide", or the narrow
        kernel whenever the max_len hint is <= 64 KiB ("narrow"; "narrow16" / "narrow8" pin its workgroup size,
        "sorted" its sorted-window form for ragged batches, "claim" / "claim16" its workgroup-run form with LDS claims,
        8 / 16 lanes per block, "coop" the form whose 8 waves share each 8-block group).  Never changes a result."""
        _check(lib().kvsep_crc32c_ctx_set_kernel(self._h, self.KERNELS[kernel]), "set_kernel")

    def set_host_node(self, node: int):
        """NUMA node for this context's pinned staging and copier threads (-1: no placement; default: the device's)."""
        _check(lib().kvsep_crc32c_ctx_set_host_node(self._h, node), "set_host_node")

    def host_placement(self):
        """-> {"device_node", "staging_node", "copier_cpus"} (kvsep_crc32c_ctx_host_placement)."""
        dn, sn = ctypes.c_int(), ctypes.c_int()
        cpus = (ctypes.c_int * 4096)()
        n = lib().kvsep_crc32c_ctx_host_placement(self._h, ctypes.byref(dn), ctypes.byref(sn), cpus, 4096)
        if n < 0:
            _check(n, "host_placement")
        return {"device_node": dn.value, "staging_node": sn.value, "copier_cpus": list(cpus[:min(n, 4096)])}

    def inject_failure(self):
        """Fault injection (tests; csrc/kvsep_testing.h): the next batched call fails right after enqueuing its CRC
        kernel.  The library honours it only under KVSEP_TEST_HOOKS=1 (tests/conftest.py sets it)."""
        _check(lib().kvsep_crc32c_ctx_inject_failure(self._h), "inject_failure")

    def reserve(self, count: int, total_bytes: int):
        _check(lib().kvsep_crc32c_reserve(self._h, count, total_bytes), "reserve")

    def reserve_captures(self, nsets: int):
        """At least `nsets` capture sets (one per graph capture that may be held at once)."""
        _check(lib().kvsep_crc32c_reserve_captures(self._h, nsets), "reserve_captures")

    def release_captures(self):
        """Every capture set free again: only once the graphs captured so far are destroyed."""
        _check(lib().kvsep_crc32c_release_captures(self._h), "release_captures")

    def capture_sets(self):
        """(number of capture sets, how many a graph holds)."""
        held = ctypes.c_int(0)
        n = lib().kvsep_crc32c_capture_sets(self._h, ctypes.byref(held))
        _check(n if n < 0 else 0, "capture_sets")
        return n, held.value

    def kernel_name(self, count: int, max_len: int, total_bytes: int = 0) -> str:
        """The main kernel a batch of `count` blocks with these max_len / total_bytes hints runs on."""
        return lib().kvsep_crc32c_kernel_name(self._h, count, total_bytes, max_len).decode()

    def set_timing(self, on: bool):
        _check(lib().kvsep_crc32c_ctx_set_timing(self._h, 1 if on else 0), "set_timing")

    def get_timing(self):
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        _check(lib().kvsep_crc32c_ctx_get_timing(self._h, ctypes.byref(ms), ctypes.byref(n)), "get_timing")
        return ms.value, n.value

    # -- device form (torch tensors or raw device addresses)
    def batch_device(self, base, off, length, out, init=None, count=None, total_bytes=None, max_len=0, stream=None):
        count = int(off.numel()) if count is None else count
        if total_bytes is None:
            total_bytes = int(length.sum().item()) if count else 0
        _check(lib().kvsep_crc32c_batch_device(self._h, _stream_handle(stream), _dptr(base), _dptr(off),
                                               _dptr(length), _dptr(init), _dptr(out), count, total_bytes,
                                               max_len), "kvsep_crc32c_batch_device")
        return out

    def verify_device(self, base, off, length, expected_masked, out, first_bad, nbad, init=None, count=None,
                      total_bytes=None, max_len=0, stream=None):
        count = int(off.numel()) if count is None else count
        if total_bytes is None:
            total_bytes = int(length.sum().item()) if count else 0
        _check(lib().kvsep_crc32c_verify_device(self._h, _stream_handle(stream), _dptr(base), _dptr(off),
                                                _dptr(length), _dptr(init), _dptr(expected_masked), _dptr(out),
                                                _dptr(first_bad), _dptr(nbad), count, total_bytes, max_len),
               "kvsep_crc32c_verify_device")
        return out

    def stream_read(self, src, nbytes: int, sink, stream=None):
        _check(lib().kvsep_stream_read_device(self._h, _stream_handle(stream), _dptr(src), nbytes, _dptr(sink)),
               "kvsep_stream_read_device")

    # -- host forms (numpy / bytes)
    def batch_host_span(self, buf, off, length, init=None):
        p, keep = _buf(buf)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        out = np.zeros(off.size, dtype=np.uint32)
        ip = None
        if init is not None:
            init = np.ascontiguousarray(init, dtype=np.uint32)
            ip = init.ctypes.data_as(ctypes.c_void_p)
        _check(lib().kvsep_crc32c_batch_host_span(self._h, p, keep.nbytes, off.ctypes.data_as(ctypes.c_void_p),
                                                  length.ctypes.data_as(ctypes.c_void_p), ip,
                                                  out.ctypes.data_as(ctypes.c_void_p), off.size),
               "kvsep_crc32c_batch_host_span")
        return out

    def batch_host(self, blocks, init=None):
        """blocks: list of bytes-like objects (gathered through pinned staging)."""
        keep = [_buf(b) for b in blocks]
        n = len(blocks)
        ptrs = (ctypes.c_void_p * n)(*[k[0].value for k in keep])
        lens = np.array([k[1].nbytes for k in keep], dtype=np.uint64)
        out = np.zeros(n, dtype=np.uint32)
        ip = None
        if init is not None:
            init = np.ascontiguousarray(init, dtype=np.uint32)
            ip = init.ctypes.data_as(ctypes.c_void_p)
        _check(lib().kvsep_crc32c_batch_host(self._h, ip, ptrs, lens.ctypes.data_as(ctypes.c_void_p),
                                             out.ctypes.data_as(ctypes.c_void_p), n), "kvsep_crc32c_batch_host")
        return out


    # -- framings (vlog / log / SST call sites)
    def vlog_verify(self, image, with_drop=False):
        """db/value_log_reader.cc:86-138 over a whole vlog image -> (records, good, good_bytes), plus the byte count
        reported with "checksum mismatch" (0 if none) when with_drop."""
        p, keep = _buf(image)
        n, g, gb, dr = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().kvsep_vlog_verify_host(self._h, p, keep.nbytes, ctypes.byref(n), ctypes.byref(g),
                                            ctypes.byref(gb), ctypes.byref(dr)), "kvsep_vlog_verify_host")
        return (n.value, g.value, gb.value, dr.value) if with_drop else (n.value, g.value, gb.value)

    def vlog_frame(self, payloads, out=None):
        """db/value_log_writer.cc:46-76 for a batch of payloads -> bytes of the framed records; with `out` (a
        writable uint8 numpy array of >= sum(8 + len) bytes) the records are framed into it and the byte count
        is returned instead."""
        keep = [_buf(b) for b in payloads]
        k = len(payloads)
        ptrs = (ctypes.c_void_p * max(k, 1))(*[x[0].value for x in keep])
        lens = np.array([x[1].nbytes for x in keep], dtype=np.uint64)
        need = int(lens.sum()) + 8 * k
        dst = np.zeros(max(need, 1), dtype=np.uint8) if out is None else out
        w = ctypes.c_uint64()
        _check(lib().kvsep_vlog_frame_host(self._h, ptrs, lens.ctypes.data_as(ctypes.c_void_p), k,
                                           dst.ctypes.data_as(ctypes.c_void_p), dst.nbytes, ctypes.byref(w)),
               "kvsep_vlog_frame_host")
        return dst[:w.value].tobytes() if out is None else w.value

    def log_frame(self, records, dest_length: int = 0, out=None):
        """db/log_writer.cc:35-115: AddRecord of each record onto a log of length dest_length -> appended bytes;
        with `out` (a writable uint8 numpy array, large enough) they are written into it and the count returned."""
        keep = [_buf(b) for b in records]
        k = len(records)
        ptrs = (ctypes.c_void_p * max(k, 1))(*[x[0].value for x in keep])
        lens = np.array([x[1].nbytes for x in keep], dtype=np.uint64)
        w = ctypes.c_uint64()
        if out is None:
            lib().kvsep_log_frame_host(self._h, ptrs, lens.ctypes.data_as(ctypes.c_void_p), k, dest_length, None, 0,
                                       ctypes.byref(w))  # sizing call: *written even when dst is short
        dst = np.zeros(max(w.value, 1), dtype=np.uint8) if out is None else out
        _check(lib().kvsep_log_frame_host(self._h, ptrs, lens.ctypes.data_as(ctypes.c_void_p), k, dest_length,
                                          dst.ctypes.data_as(ctypes.c_void_p), dst.nbytes, ctypes.byref(w)),
               "kvsep_log_frame_host")
        return dst[:w.value].tobytes() if out is None else w.value

    def frame_raw(self, kind: str, addrs, lens, out, dest_length: int = 0) -> int:
        """The framing writers on prebuilt arrays: addrs = uint64 host addresses of the payloads, lens = their
        uint64 lengths, out = a writable uint8 numpy array (kind "vlog" or "log").  No per-record Python work,
        so a caller framing thousands of records pays only the C-ABI call.  Returns the bytes written."""
        addrs = np.ascontiguousarray(addrs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        w = ctypes.c_uint64()
        vp = ctypes.c_void_p
        if kind == "vlog":
            rc = lib().kvsep_vlog_frame_host(self._h, addrs.ctypes.data_as(vp), lens.ctypes.data_as(vp), lens.size,
                                             out.ctypes.data_as(vp), out.nbytes, ctypes.byref(w))
        else:
            rc = lib().kvsep_log_frame_host(self._h, addrs.ctypes.data_as(vp), lens.ctypes.data_as(vp), lens.size,
                                            dest_length, out.ctypes.data_as(vp), out.nbytes, ctypes.byref(w))
        _check(rc, f"kvsep_{kind}_frame_host")
        return w.value

    def log_verify(self, image):
        """db/log_reader.cc:246-259 per physical record of a log/MANIFEST image -> array of 0/1."""
        p, keep = _buf(image)
        cnt = log_walk(image)[0].size
        ok = np.zeros(max(cnt, 1), dtype=np.uint8)
        n = ctypes.c_uint64()
        _check(lib().kvsep_log_verify_host(self._h, p, keep.nbytes, ok.ctypes.data_as(ctypes.c_void_p), ok.size,
                                           ctypes.byref(n)), "kvsep_log_verify_host")
        return ok[:n.value]

    def sst_trailers_device(self, base, off, length, types, masked_out, count=None, total_bytes=None, max_len=0,
                            stream=None):
        count = int(off.numel()) if count is None else count
        if total_bytes is None:
            total_bytes = int(length.sum().item()) if count else 0
        _check(lib().kvsep_sst_trailers_device(self._h, _stream_handle(stream), _dptr(base), _dptr(off),
                                               _dptr(length), _dptr(types), _dptr(masked_out), count, total_bytes,
                                               max_len), "kvsep_sst_trailers_device")

    def sst_verify_device(self, file_base, off, length, out, first_bad, nbad, count=None, total_bytes=None,
                          max_len=0, stream=None):
        count = int(off.numel()) if count is None else count
        if total_bytes is None:
            total_bytes = int(length.sum().item()) if count else 0
        _check(lib().kvsep_sst_verify_device(self._h, _stream_handle(stream), _dptr(file_base), _dptr(off),
                                             _dptr(length), _dptr(out), _dptr(first_bad), _dptr(nbad), count,
                                             total_bytes, max_len), "kvsep_sst_verify_device")

    def sst_trailers(self, blocks, types):
        """table/table_builder.cc:209-232 for host-resident blocks -> uint32 trailer words
        Mask(Extend(Value(block), &type, 1)) (kvsep_sst_trailers_host)."""
        keep = [_buf(b) for b in blocks]
        k = len(blocks)
        ptrs = (ctypes.c_void_p * max(k, 1))(*[x[0].value for x in keep])
        lens = np.array([x[1].nbytes for x in keep], dtype=np.uint64)
        t = np.ascontiguousarray(types, dtype=np.uint8)
        if t.size != k:
            raise ValueError("blocks and types must have the same length")
        out = np.zeros(max(k, 1), dtype=np.uint32)
        _check(lib().kvsep_sst_trailers_host(self._h, ptrs, lens.ctypes.data_as(ctypes.c_void_p),
                                             t.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), k),
               "kvsep_sst_trailers_host")
        return out[:k]

    def sst_trailers_raw(self, addrs, lens, types, out):
        """kvsep_sst_trailers_host on prebuilt arrays: addrs = uint64 host addresses of the blocks, lens their uint64
        lengths, types uint8, out a uint32 array filled with the trailer words.  No per-block Python work."""
        addrs = np.ascontiguousarray(addrs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        t = np.ascontiguousarray(types, dtype=np.uint8)
        if addrs.size != lens.size or t.size != lens.size:
            raise ValueError("addrs, lens and types must have the same length")
        if not (isinstance(out, np.ndarray) and out.dtype == np.uint32 and out.flags.c_contiguous
                and out.size >= lens.size):
            raise ValueError("out must be a contiguous uint32 array with room for every block")
        vp = ctypes.c_void_p
        _check(lib().kvsep_sst_trailers_host(self._h, addrs.ctypes.data_as(vp), lens.ctypes.data_as(vp),
                                             t.ctypes.data_as(vp), out.ctypes.data_as(vp), lens.size),
               "kvsep_sst_trailers_host")
        return out

    def sst_verify(self, image, off, length):
        """table/format.cc:73-108 for every block handle (off, length) of a host SST file image -> (out, first_bad,
        nbad): out[i] = Value(block, len + 1); first_bad = -1 when every block matches its stored trailer word."""
        p, keep = _buf(image)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        if off.size != length.size:
            raise ValueError("off and length must have the same length")
        k = off.size
        out = np.zeros(max(k, 1), dtype=np.uint32)
        fb, nb = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().kvsep_sst_verify_host(self._h, p, keep.nbytes, off.ctypes.data_as(ctypes.c_void_p),
                                           length.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.byref(fb), ctypes.byref(nb), k), "kvsep_sst_verify_host")
        first = -1 if fb.value == 0xFFFFFFFFFFFFFFFF else fb.value
        return out[:k], first, nb.value


def vlog_walk(image):
    """Header walk of a vlog image (db/value_log_reader.cc:86-108) -> (off, len, stored, consumed)."""
    p, keep = _buf(image)
    cnt = lib().kvsep_vlog_walk(p, keep.nbytes, None, None, None, 0, None)
    off = np.zeros(cnt, np.uint64)
    ln = np.zeros(cnt, np.uint64)
    st = np.zeros(cnt, np.uint32)
    used = ctypes.c_uint64()
    lib().kvsep_vlog_walk(p, keep.nbytes, off.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p),
                          st.ctypes.data_as(ctypes.c_void_p), cnt, ctypes.byref(used))
    return off, ln, st, used.value


def log_walk(image):
    """Physical-record walk of a log/MANIFEST image (db/log_reader.cc:189-272) -> (off, len, stored, type)."""
    p, keep = _buf(image)
    cnt = lib().kvsep_log_walk(p, keep.nbytes, None, None, None, None, 0)
    off = np.zeros(cnt, np.uint64)
    ln = np.zeros(cnt, np.uint64)
    st = np.zeros(cnt, np.uint32)
    ty = np.zeros(cnt, np.uint8)
    lib().kvsep_log_walk(p, keep.nbytes, off.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p),
                         st.ctypes.data_as(ctypes.c_void_p), ty.ctypes.data_as(ctypes.c_void_p), cnt)
    return off, ln, st, ty


def log_accept(off, ok, n: int):
    """log::Reader acceptance (db/log_reader.cc:250-258) from the walk and per-record checksum verdicts ->
    (accept 0/1 array, bytes reported dropped with "checksum mismatch")."""
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ok = np.ascontiguousarray(ok, dtype=np.uint8)
    acc = np.zeros(max(off.size, 1), np.uint8)
    dropped = lib().kvsep_log_accept(off.ctypes.data_as(ctypes.c_void_p), ok.ctypes.data_as(ctypes.c_void_p),
                                     off.size, n, acc.ctypes.data_as(ctypes.c_void_p))
    return acc[:off.size], int(dropped)


def partition(length, parts: int) -> np.ndarray:
    """kvsep_crc32c_partition: block-range bounds (parts + 1 entries) balanced by bytes."""
    length = np.ascontiguousarray(length, dtype=np.uint64)
    b = np.zeros(parts + 1, dtype=np.uint64)
    _check(lib().kvsep_crc32c_partition(length.ctypes.data_as(ctypes.c_void_p), length.size, parts,
                                        b.ctypes.data_as(ctypes.c_void_p)), "kvsep_crc32c_partition")
    return b


class Group:
    """Several devices in one process (kvsep_crc32c_group_*): one context and stream per listed device."""

    def __init__(self, devices):
        arr = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        _check(lib().kvsep_crc32c_group_create(arr, len(devices), ctypes.byref(h)), "kvsep_crc32c_group_create")
        self._h = h
        self.devices = list(devices)

    def close(self):
        if getattr(self, "_h", None):
            lib().kvsep_crc32c_group_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return lib().kvsep_crc32c_group_size(self._h)

    def batch_host_span(self, buf, off, length, init=None, expected_masked=None):
        """-> out, or (out, first_bad, nbad) with expected_masked."""
        p, keep = _buf(buf)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        out = np.zeros(off.size, dtype=np.uint32)
        vp = ctypes.c_void_p
        ip = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
        ipp = None if ip is None else ip.ctypes.data_as(vp)
        if expected_masked is None:
            _check(lib().kvsep_crc32c_group_batch_host_span(self._h, p, keep.nbytes, off.ctypes.data_as(vp),
                                                            length.ctypes.data_as(vp), ipp, out.ctypes.data_as(vp),
                                                            off.size), "kvsep_crc32c_group_batch_host_span")
            return out
        ex = np.ascontiguousarray(expected_masked, dtype=np.uint32)
        fb, nb = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().kvsep_crc32c_group_verify_host_span(self._h, p, keep.nbytes, off.ctypes.data_as(vp),
                                                         length.ctypes.data_as(vp), ipp, ex.ctypes.data_as(vp),
                                                         out.ctypes.data_as(vp), ctypes.byref(fb), ctypes.byref(nb),
                                                         off.size), "kvsep_crc32c_group_verify_host_span")
        return out, fb.value, nb.value

    def vlog_verify(self, image):
        """kvsep_vlog_verify_host_group -> (records, good, good_bytes, drop_bytes)."""
        p, keep = _buf(image)
        v = [ctypes.c_uint64() for _ in range(4)]
        _check(lib().kvsep_vlog_verify_host_group(self._h, p, keep.nbytes, *[ctypes.byref(x) for x in v]),
               "kvsep_vlog_verify_host_group")
        return tuple(x.value for x in v)

    def batch_device(self, shards, expected_masked=None, index_base=None):
        """shards: per member a dict(base=, off=, len=, out=, [init=], total_bytes=, max_len=) of device tensors /
        addresses on that member's device.  -> None, or (first_bad, nbad) over all shards with expected_masked
        (per-member device arrays) and index_base (global index of each shard's first block)."""
        n = len(shards)
        P = ctypes.c_void_p * n
        U = ctypes.c_uint64 * n
        base = P(*[_dptr(s["base"]).value for s in shards])
        off = P(*[_dptr(s["off"]).value for s in shards])
        ln = P(*[_dptr(s["len"]).value for s in shards])
        out = P(*[_dptr(s["out"]).value for s in shards])
        init = P(*[_dptr(s.get("init")).value for s in shards])
        cnt = U(*[int(s["off"].numel()) for s in shards])
        tot = U(*[int(s["total_bytes"]) for s in shards])
        ml = U(*[int(s.get("max_len", 0)) for s in shards])
        if expected_masked is None:
            _check(lib().kvsep_crc32c_group_batch_device(self._h, base, off, ln, init, out, cnt, tot, ml),
                   "kvsep_crc32c_group_batch_device")
            return None
        ex = P(*[_dptr(e).value for e in expected_masked])
        ib = U(*[int(x) for x in index_base])
        fb, nb = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().kvsep_crc32c_group_verify_device(self._h, base, off, ln, init, ex, out, ib, cnt, tot, ml,
                                                      ctypes.byref(fb), ctypes.byref(nb)),
               "kvsep_crc32c_group_verify_device")
        return fb.value, nb.value


def fill_splitmix64(dst, nbytes: int, seed: int, stream_offset: int = 0, stream=None):
    """Device synthetic data (same stream as oracle_fill_splitmix64 / splitmix64_bytes below)."""
    _check(lib().kvsep_fill_splitmix64_device(_stream_handle(stream), _dptr(dst), nbytes, seed & (2**64 - 1),
                                              stream_offset), "kvsep_fill_splitmix64_device")


def splitmix64_bytes(nbytes: int, seed: int, stream_offset: int = 0) -> np.ndarray:
    """Host (numpy) version of the synthetic byte stream, for small test cases."""
    w0 = stream_offset >> 3
    w1 = (stream_offset + nbytes + 7) >> 3
    j = np.arange(w0, w1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (j + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    s = stream_offset - (w0 << 3)
    return b[s:s + nbytes].copy()


def device_count() -> int:
    return lib().kvsep_device_count()


# ------------------------------------------------------------------ topology and host placement
def pci_bus_id(device: int) -> str:
    """PCI bus ID of a device, as sysfs spells it ("0000:75:00.0"; kvsep_device_pci_bus_id)."""
    buf = ctypes.create_string_buffer(64)
    _check(lib().kvsep_device_pci_bus_id(device, buf, 64), "kvsep_device_pci_bus_id")
    return buf.value.decode()


def pci_numa_node(bus_id: str) -> int:
    """NUMA node of a PCI function from sysfs (-1 unknown); no device needed."""
    return lib().kvsep_pci_numa_node(bus_id.encode())


def device_numa_node(device: int) -> int:
    return lib().kvsep_device_numa_node(device)


def numa_node_cpus(node: int) -> list:
    n = lib().kvsep_numa_node_cpus(node, None, 0)
    cpus = (ctypes.c_int * max(n, 1))()
    lib().kvsep_numa_node_cpus(node, cpus, n)
    return list(cpus[:n])


def bind_process_numa(node: int) -> int:
    """Every thread of this process onto the CPUs of `node` it may use, `node` the calling thread's preferred memory
    node (kvsep_bind_process_numa) -> number of CPUs bound to (0: nothing changed)."""
    return lib().kvsep_bind_process_numa(node)


def host_page_node(addr: int) -> int:
    """NUMA node of the page at host address `addr` (-1 unknown)."""
    return lib().kvsep_host_page_node(ctypes.c_void_p(addr))


def format_cpulist(cpus) -> str:
    """[0, 1, 2, 3, 8] -> "0-3,8" (the sysfs cpulist spelling)."""
    cpus = sorted(set(int(c) for c in cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if j == i else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def build_info() -> str:
    return lib().kvsep_build_info().decode()
