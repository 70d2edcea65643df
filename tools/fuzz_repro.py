"""Debug aid: re-run one failing fuzz case of tests/test_gpu_parity.py (seed, trial)
several times and print where the GPU's compressed bytes differ from the oracle."""
import os, random, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import pixiu_amd as px
from _oracle import COMPAT, Oracle
from test_gpu_parity import ALPHAS, _gen

seed = int(sys.argv[1])
orc = Oracle()
rng = random.Random(seed)
for trial in range(25):
    alpha = rng.choice(ALPHAS)
    n = rng.randint(1, 30)
    keys, vals = _gen(rng, n, alpha, 6, rng.choice([5, 30, 200, 1000]))
    try:
        ref = orc.run(keys, vals, do_get=True, mode=COMPAT)
    except RuntimeError:
        continue
    for rep in range(3):
        with px.Store(records_per_shard=0) as st:
            res = st.set_batch(keys, vals, check=False)
            if any(int(s) for s in res["status"]):
                print("trial", trial, "rep", rep, "status", list(res["status"]))
                continue
            comp = st.export(px.records_of(res))
            for i, (a, b) in enumerate(zip(comp, ref["comp"])):
                if a != b:
                    j = next((t for t in range(min(len(a), len(b))) if a[t] != b[t]), min(len(a), len(b)))
                    print(f"trial {trial} rep {rep} rec {i}/{n} len gpu {len(a)} ref {len(b)} first diff {j}: "
                          f"gpu {list(a[max(0,j-8):j+12])} ref {list(b[max(0,j-8):j+12])} doc {len(keys[i])+len(vals[i])}")
                    break
print("done")
