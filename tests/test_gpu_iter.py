"""px_iter (PiXiuCtrl::iter, CritBitTree.h:55-157) on the GPU store against the oracle:
same records in the same yield order, expanded through px_parse_batch (compat)."""
import random

import numpy as np
import pytest

from _oracle import COMPAT, Oracle

pytestmark = pytest.mark.gpu

ALPHA = [b"A", b"B", b"C", b"D", b"E"]
PREFIXES = [b"", b"A", b"C", b"CA", b"EEE", b"F", b"A.", bytes([251]), b"B" * 9 + b"."]


def ops_for(seed, n=300, dels=True):
    rng = random.Random(seed)
    live, ops = {}, []
    for _ in range(n):
        k = b"".join(rng.choice(ALPHA) for _ in range(rng.randint(0, 9))) + b"."
        if not dels and k in live:
            continue
        v = bytes(rng.randint(33, 126) for _ in range(rng.randint(0, 40)))
        if seed % 3 == 0 and rng.random() < 0.1:
            v += bytes([251]) * rng.randint(1, 3)
        ops.append(("set", k, v))
        live[k] = v
        if dels and rng.random() < 0.4:
            kd = rng.choice(sorted(live))
            ops.append(("del", kd, b""))
            del live[kd]
    return ops


def run_store(st, ops):
    """Apply ops: runs of sets as one batch, deletes one by one (same order)."""
    batch = []
    for op, k, v in ops + [("end", b"", b"")]:
        if op == "set":
            batch.append((k, v))
            continue
        if batch:
            st.set_batch([b[0] for b in batch], [b[1] for b in batch])
            batch = []
        if op == "del":
            st.delete([k])


def gpu_docs(st, prefix):
    recs = st.iter(prefix)
    if recs is None:
        return None
    return st.parse_batch(recs, COMPAT) if len(recs) else []


def oracle_docs(sh, prefix):
    recs = sh.iter(prefix)
    return None if recs is None else [sh.parse(c, i, 0, 65535, COMPAT) for c, i in recs]


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_iter_single_instance(store_factory, seed):
    ops = ops_for(seed)
    st = store_factory(records_per_shard=0)
    run_store(st, ops)
    sh = Oracle().new()
    for op, k, v in ops:
        if op == "set":
            sh.set(k, v)
        else:
            sh.delete(k)
    for p in PREFIXES:
        assert gpu_docs(st, p) == oracle_docs(sh, p), p


def test_iter_empty(store_factory):
    st = store_factory(records_per_shard=0)
    assert st.iter(b"A") is None


def test_iter_sharded(store_factory):
    ops = ops_for(7, n=200, dels=False)
    keys = [k for _, k, _ in ops]
    vals = [v for _, _, v in ops]
    rps = 9
    st = store_factory(records_per_shard=rps)
    st.set_batch(keys, vals)
    orc = Oracle()
    shards = []
    for s0 in range(0, len(keys), rps):
        sh = orc.new()
        for k, v in zip(keys[s0:s0 + rps], vals[s0:s0 + rps]):
            sh.set(k, v)
        shards.append(sh)
    for p in PREFIXES:
        want = []
        for sh in shards:
            d = oracle_docs(sh, p)
            if d:
                want += d
        assert gpu_docs(st, p) == want, p


def test_iter_long_prefix_checks_value_bytes(store_factory):
    """A prefix running past the key into the value: startswith needs a GPU decode."""
    st = store_factory(records_per_shard=0)
    keys = [b"k%03d" % i for i in range(50)]
    vals = [b"value-%d-" % (i % 3) + bytes([97 + i % 26]) * 50 for i in range(50)]
    st.set_batch(keys, vals)
    sh = Oracle().new()
    for k, v in zip(keys, vals):
        sh.set(k, v)
    for p in [b"k0", b"k001\xfb\x00value-1", b"k001\xfb\x00value-2", b"k01"]:
        assert gpu_docs(st, p) == oracle_docs(sh, p), p
