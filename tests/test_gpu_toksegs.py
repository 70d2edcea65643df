"""The segment index built from the encoder's own record tokens (k_gst_emit -> k_tok_segs)
must equal the one k_tokenize parses out of the compressed bytes (the grammar of PXSGen,
PiXiuStr.h:139-192), entry for entry: segment entries, lane entries, position index, counts.
PX_DEBUG_TOKSEGS=1 makes every set batch build both and fail on any difference."""
import os

import numpy as np
import pytest

from _oracle import assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


@pytest.fixture
def toksegs_check():
    old = os.environ.get("PX_DEBUG_TOKSEGS")
    os.environ["PX_DEBUG_TOKSEGS"] = "1"
    yield
    if old is None:
        os.environ.pop("PX_DEBUG_TOKSEGS", None)
    else:
        os.environ["PX_DEBUG_TOKSEGS"] = old


@pytest.mark.parametrize("cfg,n,rps", [(2, 4000, 500), (3, 278, 139), (4, 40000, 8000), (5, 252, 126), (3, 400, 0)])
def test_tokens_equal_parse(cfg, n, rps, store_factory, toksegs_check):
    from pixiu_amd import synth
    cp = synth.make(cfg, n)
    st = store_factory(records_per_shard=rps)
    r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    assert int(r["status"].max()) == 0
    rows = range(0, n, max(1, n // 200))
    got = st.get_batch([cp.key(i) for i in rows], mode=px.EXACT)
    if cfg != 5:  # (config 5's length-251 runs alias the escape: some exact expansions are not their docs)
        assert got == [assemble(cp.key(i), cp.val(i)) for i in rows]


def test_tokens_equal_parse_small_alphabets(store_factory, toksegs_check):
    """251-heavy docs: runs of length 251 (the alias) and wrapping `from`s go to the parse."""
    rng = np.random.default_rng(11)
    for alpha in (b"ab", b"\xfb\xfba", b"a\xfb<"):
        a = np.frombuffer(alpha, np.uint8)
        keys, vals = [], []
        for i in range(60):
            v = a[rng.integers(0, len(a), int(rng.integers(100, 9000)))].tobytes()
            keys.append(b"t%04d" % i)
            vals.append(v + v[: int(rng.integers(0, len(v)))])
        st = store_factory(records_per_shard=0)
        r = st.set_batch(keys, vals)
        assert int(r["status"].max()) == 0
        got = st.get_batch(keys, mode=px.EXACT)
        assert sum(g == assemble(k, v) for g, k, v in zip(got, keys, vals)) > 0
