"""Chunk blob v1 (pixiu_amd/blob.py, include/pixiu_amd.h px_save/px_load) on the CPU:
write/read round trip, rejection of malformed blobs, and that a blob of oracle-encoded
chunks decodes every record back to its escaped doc (each chunk on its own)."""
import pytest

from _oracle import EXACT, assemble
from pixiu_amd import blob, synth


def _chunks_from_oracle(oracle, cp, rows, shard=0):
    docs = [assemble(cp.key(i), cp.val(i)) for i in rows]
    comp, ch, idx = oracle.encode_docs(docs)
    out = []
    for c in sorted(set(ch)):
        sel = [k for k in range(len(rows)) if ch[k] == c]
        assert [idx[k] for k in sel] == list(range(len(sel)))
        out.append(blob.Chunk(shard, c, [comp[k] for k in sel], [len(docs[k]) for k in sel], [False] * len(sel)))
    return out, docs


def test_round_trip_and_decode(oracle):
    cp = synth.make(2, 1500)
    chunks, docs = _chunks_from_oracle(oracle, cp, range(1500))
    chunks[0].dead[3] = True
    b = blob.write(chunks)
    back = blob.read(b)
    assert [(c.shard, c.chunk, c.records, c.doc_len, c.dead) for c in back] == \
           [(c.shard, c.chunk, c.records, c.doc_len, c.dead) for c in chunks]
    k = 0
    for c in back:
        for i in range(len(c.records)):
            assert oracle.decode_chunk(c.records, i, mode=EXACT) == docs[k]
            k += 1


def test_rejects_malformed():
    good = blob.write([blob.Chunk(0, 0, [b"ab\xfb\x00"], [4], [False])])
    blob.read(good)
    with pytest.raises(ValueError):
        blob.read(b"XXXX" + good[4:])
    with pytest.raises(ValueError):
        blob.read(good[:40])
    bad = bytearray(good)
    bad[64 + 4:64 + 8] = (1).to_bytes(4, "little")  # chunk sequence 1 without a chunk 0
    with pytest.raises(ValueError):
        blob.read(bytes(bad))
