"""Reinsert compaction on the GPU runtime (px_runtime.cpp set_ctrl / reinsert_chunk):
the reinsert scenarios of tests/_reinsert.py run as batches through the C-ABI must
reach the reference's end state (tests/golden/reinsert.json) and the oracle's chunk
placement, whatever the batch split."""
import json
import os

import numpy as np
import pytest

import _reinsert as R

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reinsert.json")))


def _split(ops, batch):
    if not batch:
        return ops
    out = []
    for op in ops:
        if op[0] == "reinsert":
            out.append(op)
            continue
        for a in range(0, len(op[1]), batch):
            out.append((op[0],) + tuple(x[a:a + batch] for x in op[1:]))
    return out


def _key_of(doc: bytes) -> bytes:
    """Unescape a doc's key part (up to the 251,0 key terminator)."""
    out, i = bytearray(), 0
    while i < len(doc):
        if doc[i] == 251:
            if doc[i + 1] == 0:
                return bytes(out)
            out.append(doc[i + 1])
            i += 2
        else:
            out.append(doc[i])
            i += 1
    raise AssertionError("no key terminator")


@pytest.mark.parametrize("batch", [0, 7777])
@pytest.mark.parametrize("name", sorted(GOLD))
def test_gpu_reinsert_matches_reference(name, batch, store_factory, oracle):
    ops = R.scenarios()[name]
    g = GOLD[name]
    st = store_factory(records_per_shard=0)
    rets = []
    for op in _split(ops, batch):
        if op[0] == "set":
            r = st.set_batch(list(op[1]), list(op[2]))
            assert int(r["status"].max()) == 0
            rets += r["replaced"].tolist()
        elif op[0] == "reinsert":
            st.reinsert(0, op[1])
            rets.append(0)
        else:
            rets += st.delete(list(op[1])).tolist()
    keys = R.touched(ops)
    got = st.get_batch(keys)
    recs = st.iter(b"r")
    docs = st.parse_batch(recs)
    comps = st.export(recs)
    where = {_key_of(d): (int(rc["chunk"]), int(rc["idx"]), c) for rc, d, c in zip(recs, docs, comps)}
    state = []
    for k, gv in zip(keys, got):
        w = where.get(k)
        assert (gv is None) == (w is None)
        state.append((k, gv is not None, gv, w[1] if w else None, w[2] if w else None))
    d = R.digest(rets, state)
    assert d == {k: g[k] for k in d}
    # chunk placement equals the oracle's
    sh = oracle.new()
    R.run_scalar(sh, ops)
    for k in keys[:: 97]:
        loc = sh.locate(k)
        assert (loc is None and k not in where) or (loc is not None and where[k][:2] == loc)
