"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: compressed bytes, chunk/slot placement and compat-decoded bytes are
bit-exact with oracle/pxo (itself pinned to the reference, tests/test_oracle_*);
exact-mode decode equals the original escaped doc wherever the compressed
bytes are lossless (everything but the len-251 alias).
"""
import random

import numpy as np
import pytest

from _oracle import COMPAT, EXACT, assemble

pytestmark = pytest.mark.gpu

px = pytest.importorskip("pixiu_amd")


def _store(**kw):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return px.Store(**kw)


def _gen(rng, n, alpha, kmax, vmax):
    keys, vals, seen = [], [], set()
    while len(keys) < n:
        k = bytes(rng.choice(alpha) for _ in range(rng.randint(1, kmax)))
        if k in seen:
            continue
        seen.add(k)
        keys.append(k)
        vals.append(bytes(rng.choice(alpha) for _ in range(rng.randint(0, vmax))))
    return keys, vals


ALPHAS = [b"ab", b"abc", b"ABCDE", bytes([97, 98, 251]), bytes([251, 0, 2, 1, 97]), bytes(range(256)),
          b"abcdefghij"]


def _check_shard(st, res, keys, vals, oracle, rows):
    """Records `rows` of one store shard vs a fresh oracle instance fed the same records."""
    ks = [keys[i] for i in rows]
    vs = [vals[i] for i in rows]
    try:
        ref = oracle.run(ks, vs, do_get=True, mode=COMPAT)
    except RuntimeError:
        # the oracle (and the reference) fail on this input: the product must flag it
        assert any(int(res["status"][i]) != 0 for i in rows)
        return "both_fail"
    assert all(int(res["status"][i]) == 0 for i in rows), [int(res["status"][i]) for i in rows]
    recs = px.records_of(res[rows])
    comp = st.export(recs)
    assert comp == ref["comp"]
    assert [int(x) for x in res["chunk"][rows]] == ref["chunk"]
    assert [int(x) for x in res["idx"][rows]] == ref["idx"]
    got = st.get_batch(ks, COMPAT)
    want = [g if g else None for g in ref["get"]]
    assert got == want
    ex = st.parse_batch(recs, EXACT)
    for i, r in enumerate(rows):
        doc = assemble(keys[r], vals[r])
        # exact == original unless the record (transitively) holds the len-251 alias
        if ex[i] != doc:
            assert any(b"\xfb\xfb" in c for c in comp), (r, ex[i][:40], doc[:40])
    return "eq"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_single_shard(seed, oracle):
    rng = random.Random(seed)
    stats = {"eq": 0, "both_fail": 0}
    for trial in range(25):
        alpha = rng.choice(ALPHAS)
        n = rng.randint(1, 30)
        keys, vals = _gen(rng, n, alpha, 6, rng.choice([5, 30, 200, 1000]))
        with _store(records_per_shard=0) as st:
            res = st.set_batch(keys, vals, check=False)
            stats[_check_shard(st, res, keys, vals, oracle, list(range(n)))] += 1
    assert stats["eq"] > 0


def test_incremental_batches(oracle):
    rng = random.Random(7)
    keys, vals = _gen(rng, 60, b"abcdefgh", 8, 400)
    with _store(records_per_shard=0) as st:
        parts = [0, 1, 5, 17, 18, 40, 60]
        res = np.concatenate([st.set_batch(keys[a:b], vals[a:b]) for a, b in zip(parts, parts[1:])])
        assert _check_shard(st, res, keys, vals, oracle, list(range(60))) == "eq"


@pytest.mark.parametrize("rps", [1, 3, 8])
def test_sharded(rps, oracle):
    rng = random.Random(100 + rps)
    keys, vals = _gen(rng, 40, b"abcdefghij<>/", 10, 600)
    with _store(records_per_shard=rps) as st:
        res = st.set_batch(keys, vals)
        for s in range(0, 40, rps):
            rows = list(range(s, min(40, s + rps)))
            assert set(int(x) for x in res["shard"][rows]) == {s // rps}
            assert _check_shard(st, res, keys, vals, oracle, rows) == "eq"


def test_decoder_bug_repro(oracle):
    """the reference's getitem('k1') yields 'abaabbbba'."""
    keys, vals = [b"k0", b"k1"], [b"abaabaabaabba", b"abaababba"]
    with _store() as st:
        res = st.set_batch(keys, vals)
        comp = st.export(px.records_of(res))
        assert comp[0] == bytes([107, 48, 251, 0, 97, 98, 97, 97, 251, 7, 0, 0, 12, 0, 98, 97, 251, 2])
        assert comp[1] == bytes([107, 49, 251, 8, 0, 0, 10, 0, 98, 98, 97, 251, 2])
        got = st.get_batch([b"k1"], COMPAT)[0]
        assert got == b"k1\xfb\x00abaabbbba\xfb\x02"
        ex = st.get_batch([b"k1"], EXACT)[0]
        assert ex == b"k1\xfb\x00abaababba\xfb\x02"


def test_len251_alias(oracle):
    rng = random.Random(5)
    a = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(400))
    keys, vals = [b"K1", b"K2"], [a, b"Q" + a[:251] + b"#"]
    ref = oracle.run(keys, vals)
    with _store() as st:
        res = st.set_batch(keys, vals)
        comp = st.export(px.records_of(res))
        assert comp == ref["comp"]
        assert comp[1].endswith(bytes([81, 251, 251, 0, 0, 255, 0, 35, 251, 2]))
        assert st.get_batch(keys, COMPAT) == ref["get"]


def test_partial_parse(oracle):
    rng = random.Random(11)
    keys, vals = _gen(rng, 20, b"ab\xfbc", 5, 300)
    sh = oracle.new()
    for k, v in zip(keys, vals):
        assert sh.set(k, v)[0] >= 0
    with _store() as st:
        res = st.set_batch(keys, vals)
        recs = []
        for i in range(20):
            for _ in range(10):
                dl = int(res["doc_len"][i])
                a = rng.randint(0, dl)
                b = rng.randint(a, dl + 3)
                recs.append((0, int(res["chunk"][i]), int(res["idx"][i]), a, b))
        ra = np.array(recs, px.REC_DTYPE)
        for mode in (COMPAT, EXACT):
            got = st.parse_batch(ra, mode)
            for (s, c, i, a, b), g in zip(recs, got):
                assert g == sh.parse(c, i, a, b, mode), (c, i, a, b, mode)


def test_missing_and_contains_delete(oracle):
    with _store() as st:
        st.set_batch([b"alpha", b"beta", b"gamma"], [b"1", b"2", b""])
        assert st.get_batch([b"zzz", b"beta"]) == [None, b"beta\xfb\x002\xfb\x02"]
        assert list(st.contains([b"alpha", b"nope", b"gamma"])) == [True, False, True]
        assert list(st.delete([b"alpha", b"alpha"])) == [0, 1]
        assert st.get_batch([b"alpha"]) == [None]
        r = st.set_batch([b"beta"], [b"22"])
        assert int(r["replaced"][0]) == 1
        assert st.get_batch([b"beta"]) == [b"beta\xfb\x0022\xfb\x02"]


@pytest.mark.parametrize("cfg,n,rps", [(1, 300, 0), (2, 200, 50), (3, 12, 4), (4, 3000, 1000), (5, 6, 3)])
def test_config_corpora(cfg, n, rps, oracle):
    from pixiu_amd import synth
    cp = synth.make(cfg, n)
    keys = [cp.key(i) for i in range(n)]
    vals = [cp.val(i) for i in range(n)]
    with _store(records_per_shard=rps) as st:
        res = st.set_batch(keys, vals)
        step = rps or n
        for s in range(0, n, step):
            rows = list(range(s, min(n, s + step)))
            assert _check_shard(st, res, keys, vals, oracle, rows) == "eq"


def test_device_resident_inputs(oracle):
    import torch
    from pixiu_amd import synth
    cp = synth.make(3, 6)
    with _store(records_per_shard=3) as st:
        kb = torch.from_numpy(cp.keys).cuda()
        ko = torch.from_numpy(cp.koff.astype(np.uint64).view(np.int64)).cuda()
        vb = torch.from_numpy(cp.vals).cuda()
        vo = torch.from_numpy(cp.voff.astype(np.uint64).view(np.int64)).cuda()
        torch.cuda.synchronize()
        res = st.set_batch_device(cp.n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr())
        keys = [cp.key(i) for i in range(cp.n)]
        vals = [cp.val(i) for i in range(cp.n)]
        for s in (0, 3):
            assert _check_shard(st, res, keys, vals, oracle, [s, s + 1, s + 2]) == "eq"


def _edge_docs(rng):
    """Records whose encoder runs end on, just before and just after the 64-message
    steps of k_gst_emit (the open-run carry), runs of exactly 6/7/255/256 bytes (the
    literal / small / big token limits) and 251 pairs split across a step boundary."""
    base = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(3000))
    keys, vals = [b"base"], [base]
    # copies of base slices: the key plus the 2-byte separator shifts them by len(key)+2
    for n, (lo, ln) in enumerate([(0, 6), (0, 7), (10, 255), (10, 256), (5, 57), (5, 58), (5, 59),
                                  (100, 121), (100, 122), (100, 123), (7, 1000), (200, 2047)]):
        keys.append(b"c%02d" % n)
        vals.append(base[lo:lo + ln] + b"#" + base[lo + 1:lo + ln] + b"!")
    # 251 pairs (escaped 251 = 251,251) straddling positions 63/64 and 127/128
    for n, at in enumerate([57, 58, 59, 60, 121, 122, 123]):
        v = bytearray(base[:400])
        v[at] = 251
        v[at + 1] = 251
        keys.append(b"e%02d" % n)
        vals.append(bytes(v))
        keys.append(b"f%02d" % n)
        vals.append(bytes(v[:at + 1]) + b"\xfb" + base[500:700])
    return keys, vals


def test_encoder_step_boundaries(oracle):
    keys, vals = _edge_docs(random.Random(64))
    with _store(records_per_shard=0) as st:
        res = st.set_batch(keys, vals)
        assert _check_shard(st, res, keys, vals, oracle, list(range(len(keys)))) == "eq"
