"""getitem resolves stored keys through the key map's record hint (verified: the hinted
record must be live and its stored compat key prefix must equal the query) before the
CritBit walk.  Deletes, replaces in the same shard, moves to a newer shard (a later
batch re-sets a key) and missing keys must all answer like the reference's single
map semantics (the last set wins; deleted keys are gone)."""
import random

import pytest

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def test_hints_follow_deletes_replaces_and_moves(store_factory):
    rng = random.Random(5)
    st = store_factory(records_per_shard=3)
    model = {}
    keys = [b"k%03d" % i for i in range(300)]
    for rnd in range(6):
        ks = rng.sample(keys, 120)
        vs = [bytes(rng.choice(b"abcxyz") for _ in range(rng.randint(1, 30))) for _ in ks]
        r = st.set_batch(ks, vs)
        assert int(r["status"].max()) == 0
        for k, v in zip(ks, vs):
            model[k] = v
        dels = rng.sample(keys, 40)
        res = st.delete(dels)
        for k, rr in zip(dels, res):
            assert int(rr) == (0 if k in model else 1)
            model.pop(k, None)
        got = st.get_batch(keys + [b"missing", b"k"])
        for k, g in zip(keys + [b"missing", b"k"], got):
            if k in model:
                assert g is not None and g[:len(k)] == k and g.endswith(model[k] + b"\xfb\x02"), k
            else:
                assert g is None, k
