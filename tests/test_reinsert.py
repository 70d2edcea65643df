"""Reinsert compaction (PiXiuCtrl.cpp:12-29, 63-69, 88-114) in the oracle, against the
reference's own end state (tests/golden/reinsert.json, tools/make_golden.py reinsert)."""
import json
import os

import pytest

import _reinsert as R

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reinsert.json")))


@pytest.mark.parametrize("name", sorted(GOLD))
def test_oracle_reinsert_matches_reference(name, oracle):
    ops = R.scenarios()[name]
    g = GOLD[name]
    assert R.ops_sha256(ops) == g["ops_sha256"]
    sh = oracle.new()
    rets = R.run_scalar(sh, ops)
    keys = R.touched(ops)
    state, where = R.oracle_state(sh, keys)
    d = R.digest(rets, state)
    assert d == {k: g[k] for k in d}
    # the compaction happened: nothing live is left in chunk 0
    assert all(w is None or w[0] > 0 for w in where)
