"""Chunk blob v1 — the wire / on-disk format of stored records (include/pixiu_amd.h,
px_save / px_load).  This module reads and writes it in pure Python for hosts that
only move blobs (the multi-GPU gather, tests); the GPU library writes and loads it
natively.  Layout (little-endian):

    header  64 B : magic "PXCB", version 1, n_chunks, n_records, data_off, data_bytes, flags
    chunks  16 B : shard, chunk (sequence in that shard), first record, records
    records 16 B : offset into data, comp_len, doc_len | 1 << 31 (dead)
    data         : compressed bytes, each record 8-byte aligned

Record i of a chunk is its chunk-local slot: the `idx` that reference tokens carry
(PiXiuStr.cpp:56-82), so every chunk decodes on its own.
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

MAGIC = 0x42435850  # "PXCB"
VERSION = 1
DEAD = 1 << 31
_HDR = struct.Struct("<IIIIQQI28x")
CHUNK_DTYPE = np.dtype([("shard", "<u4"), ("chunk", "<u4"), ("first", "<u4"), ("n", "<u4")])
REC_DTYPE = np.dtype([("off", "<u8"), ("comp_len", "<u4"), ("doc_len", "<u4")])
assert _HDR.size == 64 and CHUNK_DTYPE.itemsize == 16 and REC_DTYPE.itemsize == 16


@dataclasses.dataclass
class Chunk:
    shard: int
    chunk: int
    records: list      # compressed bytes per slot
    doc_len: list      # escaped doc length per slot
    dead: list         # bool per slot


def write(chunks: list) -> bytes:
    """Chunks (in order) -> blob bytes."""
    recs, data, tabs = [], [], []
    off = 0
    first = 0
    for c in chunks:
        tabs.append((c.shard, c.chunk, first, len(c.records)))
        for comp, dl, dead in zip(c.records, c.doc_len, c.dead):
            recs.append((off, len(comp), dl | (DEAD if dead else 0)))
            pad = (-len(comp)) % 8
            data.append(comp + b"\0" * pad)
            off += len(comp) + pad
        first += len(c.records)
    ct = np.array(tabs, CHUNK_DTYPE) if tabs else np.zeros(0, CHUNK_DTYPE)
    rt = np.array(recs, REC_DTYPE) if recs else np.zeros(0, REC_DTYPE)
    tables = _HDR.size + ct.nbytes + rt.nbytes
    data_off = (tables + 63) // 64 * 64
    head = _HDR.pack(MAGIC, VERSION, len(ct), len(rt), data_off, off, 0)
    return head + ct.tobytes() + rt.tobytes() + b"\0" * (data_off - tables) + b"".join(data)


def read(blob) -> list:
    """Blob bytes -> chunks; raises ValueError on a malformed blob."""
    blob = bytes(blob)
    if len(blob) < _HDR.size:
        raise ValueError("blob shorter than its header")
    magic, ver, nc, nr, data_off, data_bytes, _ = _HDR.unpack_from(blob, 0)
    if magic != MAGIC or ver != VERSION:
        raise ValueError(f"not a v{VERSION} chunk blob")
    tables = _HDR.size + 16 * nc + 16 * nr
    if data_off < tables or data_off + data_bytes > len(blob):
        raise ValueError("blob tables / data out of range")
    ct = np.frombuffer(blob, CHUNK_DTYPE, nc, _HDR.size)
    rt = np.frombuffer(blob, REC_DTYPE, nr, _HDR.size + 16 * nc)
    out, nxt, seen = [], 0, {}
    for shard, chunk, first, n in ct.tolist():
        if first != nxt or n == 0 or chunk != seen.get(shard, 0):
            raise ValueError("chunk table does not tile the records")
        seen[shard] = chunk + 1
        nxt += n
        recs, dls, dead = [], [], []
        for o, cl, dl in rt[first:first + n].tolist():
            if o + cl > data_bytes:
                raise ValueError("record out of range")
            recs.append(blob[data_off + o:data_off + o + cl])
            dls.append(dl & ~DEAD)
            dead.append(bool(dl & DEAD))
        out.append(Chunk(shard, chunk, recs, dls, dead))
    if nxt != nr:
        raise ValueError("chunk table does not cover every record")
    return out
