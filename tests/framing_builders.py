"""Reference-format image builders for the framing tests -- TEST INFRASTRUCTURE, checksums from the
oracle.  Each follows the reference writer it names, so the engine's walkers/verifiers are checked
against independently framed bytes."""
import struct

import numpy as np


def vlog_image(payloads, oracle):
    """db/value_log_writer.cc:46-76: [Mask(Value(p)) LE32][len LE32][p] back to back."""
    out = bytearray()
    for p in payloads:
        c = oracle.lib.oracle_crc32c_mask(oracle.extend(0, p))
        out += struct.pack("<II", c, len(p)) + p
    return bytes(out)


BLOCK, HEADER = 32768, 7  # db/log_format.h:30,33
FULL, FIRST, MIDDLE, LAST = 1, 2, 3, 4


def log_image(records, oracle):
    """log::Writer::AddRecord (db/log_writer.cc:35-82) + EmitPhysicalRecord (:84-115).
    Returns (image, physical) with physical = [(header_offset, type, payload_len)]."""
    out = bytearray()
    phys = []
    block_off = 0
    for rec in records:
        left, pos, begin = len(rec), 0, True
        while True:
            leftover = BLOCK - block_off
            if leftover < HEADER:
                out += b"\x00" * leftover
                block_off = 0
            avail = BLOCK - block_off - HEADER
            frag = min(left, avail)
            end = left == frag
            t = FULL if (begin and end) else FIRST if begin else LAST if end else MIDDLE
            data = rec[pos:pos + frag]
            crc = oracle.lib.oracle_crc32c_mask(oracle.extend(oracle.extend(0, bytes([t])), data))
            phys.append((len(out), t, frag))
            out += struct.pack("<IHB", crc, frag, t) + data
            block_off += HEADER + frag
            pos += frag
            left -= frag
            begin = False
            if left == 0:
                break
    return bytes(out), phys


def sst_image(blocks, types, oracle):
    """TableBuilder::WriteRawBlock (table/table_builder.cc:209-232): block, then [type][Mask(crc)]
    with crc = Extend(Value(block), &type, 1).  Returns (image, offsets, trailer words)."""
    out = bytearray()
    offs, words = [], []
    for b, t in zip(blocks, types):
        crc = oracle.extend(oracle.extend(0, b), bytes([t]))
        w = oracle.lib.oracle_crc32c_mask(crc)
        offs.append(len(out))
        words.append(w)
        out += b + bytes([t]) + struct.pack("<I", w)
    return bytes(out), np.array(offs, np.uint64), np.array(words, np.uint32)
