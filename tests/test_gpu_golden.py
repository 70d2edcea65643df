"""The HIP path against golden vectors generated from the reference itself
(tests/golden/, see tools/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from _oracle import assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _store(**kw):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return px.Store(**kw)


@pytest.fixture(scope="module")
def kats():
    return json.load(open(os.path.join(GOLD, "kats.json")))


def h(x):
    return bytes.fromhex(x) if x is not None else None


def test_readme_transcript(kats):
    with _store() as st:
        for step in kats["readme"]["steps"]:
            r = st.set_batch([h(step["key"])], [h(step["val"])])
            comp = st.export(px.records_of(r))[0]
            assert comp == h(step["comp"])
            assert len(step["cmd"]) - len(comp) == step["saved"]
        assert kats["readme"]["steps"][-1]["saved"] == 27
        keys = list(kats["readme"]["gets"])
        assert st.get_batch([k.encode() for k in keys]) == [h(kats["readme"]["gets"][k]) for k in keys]


def test_hand_built_chunk_decode(kats):
    cd = kats["chunk_decode"]
    with _store() as st:
        sid = st.import_chunk([h(c) for c in cd["chunk"]])
        recs = np.array([(sid, 0, q["idx"], q["from"], q["to"]) for q in cd["queries"]], px.REC_DTYPE)
        assert st.parse_batch(recs, px.COMPAT) == [h(q["out"]) for q in cd["queries"]]


def test_decoder_bug_and_len251(kats):
    for key in ("decoder_bug", "len251"):
        case = kats[key]
        with _store() as st:
            r = st.set_batch([h(k) for k in case["keys"]], [h(v) for v in case["vals"]])
            assert st.export(px.records_of(r)) == [h(c) for c in case["comp"]]
            if key == "decoder_bug":
                assert st.get_batch([b"k1"])[0] == h(case["get_k1"])
            else:
                assert st.get_batch([h(k) for k in case["keys"]]) == [h(g) for g in case["gets"]]


def test_max_size_records(kats):
    with _store() as st:
        big = bytes([233]) + bytes([1]) * 65532
        r = st.set_batch([big], [b""])
        comp = st.export(px.records_of(r))[0]
        assert hashlib.sha256(comp).hexdigest() == kats["max_elem"]["comp_sha256"]
        g = st.get_batch([big])[0]
        assert len(g) == 65535 and hashlib.sha256(g).hexdigest() == kats["max_elem"]["get_sha256"]
    with _store() as st:  # the golden max-kv record was stored in a fresh instance
        mk, mv = bytes([6]) * 100, bytes([2]) * kats["max_kv"]["vlen"]
        r = st.set_batch([mk], [mv])
        assert hashlib.sha256(st.export(px.records_of(r))[0]).hexdigest() == kats["max_kv"]["comp_sha256"]
        assert hashlib.sha256(st.get_batch([mk])[0]).hexdigest() == kats["max_kv"]["get_sha256"]
        r = st.set_batch([bytes([1]) * 65534, b"ok"], [b"", b"v"], check=False)
        assert list(r["status"]) == [px.PX_EINVAL, 0]  # oversize doc rejected, neighbour stored


def test_crud_script(kats):
    with _store() as st:
        for op in kats["crud"]:
            if op[0] == "set":
                r = st.set_batch([h(op[1])], [h(op[2])])
                assert int(r["replaced"][0]) == op[3]
                assert st.export(px.records_of(r))[0] == h(op[4])
            elif op[0] == "get":
                assert st.get_batch([h(op[1])])[0] == h(op[2])
            elif op[0] == "contains":
                assert int(st.contains([h(op[1])])[0]) == op[2]
            elif op[0] == "del":
                assert int(st.delete([h(op[1])])[0]) == op[2]


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_config_corpora(cfg):
    from pixiu_amd import synth
    z = np.load(os.path.join(GOLD, f"corpus_c{cfg}.npz"), allow_pickle=False)
    n = int(z["n"])
    cp = synth.make(cfg, n)
    assert hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest() == z["input_sha256"].tobytes().decode()
    with _store() as st:
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        comp, coff = z["comp"], z["comp_off"]
        assert st.export(px.records_of(r)) == [comp[coff[i]:coff[i + 1]].tobytes() for i in range(n)]
        assert r["chunk"].tolist() == z["chunk"].tolist() and r["idx"].tolist() == z["idx"].tolist()
        g, go = z["get"], z["get_off"]
        assert st.get_batch((cp.keys, cp.koff.astype(np.uint64))) == [g[go[i]:go[i + 1]].tobytes() for i in range(n)]


@pytest.mark.parametrize("name", ["slots_tiny", "pools_c2", "pools_c4"])
def test_rotation(name):
    from pixiu_amd import synth
    rot = json.load(open(os.path.join(GOLD, "rotation.json")))[name]
    cp = synth.make(rot["config"], rot["n"]) if rot["config"] else synth.tiny_keys(rot["n"])
    with _store() as st:
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        comp = st.export(px.records_of(r))
        for ch in rot["chunks"]:
            rows = range(ch["first"], ch["first"] + ch["records"])
            assert all(int(r["chunk"][i]) == ch["chunk"] for i in rows)
            assert [int(r["idx"][i]) for i in rows] == list(range(ch["records"]))
            assert hashlib.sha256(b"".join(comp[i] for i in rows)).hexdigest() == ch["sha256"]
        # every record still round-trips after the rotation (exact mode)
        sample = list(range(0, cp.n, max(1, cp.n // 200)))
        ex = st.parse_batch(px.records_of(r[sample]), px.EXACT)
        assert ex == [assemble(cp.key(i), cp.val(i)) for i in sample]
