"""Debug aid: run the single-shard fuzz on the GPU and dump the first mismatching
case (inputs + both outputs) to gpurun_out/fuzz_case.json."""
import json, random, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import pixiu_amd as px
from _oracle import Oracle
from test_gpu_parity import _gen, ALPHAS

orc = Oracle()
seeds = [int(x) for x in sys.argv[1:]] or [1]
found = 0
for seed in seeds:
    rng = random.Random(seed)
    for trial in range(25):
        alpha = rng.choice(ALPHAS)
        n = rng.randint(1, 30)
        keys, vals = _gen(rng, n, alpha, 6, rng.choice([5, 30, 200, 1000]))
        try:
            ref = orc.run(keys, vals)
        except RuntimeError:
            continue
        with px.Store() as st:
            res = st.set_batch(keys, vals, check=False)
            if any(int(s) for s in res["status"]):
                print("status fail", seed, trial, res["status"].tolist()); continue
            comp = st.export(px.records_of(res))
        for i in range(n):
            if comp[i] != ref["comp"][i]:
                print("MISMATCH seed", seed, "trial", trial, "rec", i)
                if not found:
                    json.dump({"keys": [k.hex() for k in keys[:i+1]], "vals": [v.hex() for v in vals[:i+1]],
                               "got": comp[i].hex(), "want": ref["comp"][i].hex()}, open("gpurun_out/fuzz_case.json", "w"))
                found += 1
                break
print("mismatching trials:", found)
