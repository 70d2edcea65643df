"""Debug aid: many small single-shard batches (the fuzz shapes of
tests/test_gpu_parity.py), each in a fresh Store, compressed bytes checked against
the oracle; counts mismatches to expose rare nondeterminism.
  python tools/fuzz_stress.py SEED0 NSEEDS"""
import os, random, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import pixiu_amd as px
from _oracle import COMPAT, Oracle
from test_gpu_parity import ALPHAS, _gen

s0, ns = int(sys.argv[1]), int(sys.argv[2])
orc = Oracle()
bad = tot = 0
t0 = time.time()
for seed in range(s0, s0 + ns):
    rng = random.Random(seed)
    for trial in range(25):
        alpha = rng.choice(ALPHAS)
        n = rng.randint(1, 30)
        keys, vals = _gen(rng, n, alpha, 6, rng.choice([5, 30, 200, 1000]))
        try:
            ref = orc.run(keys, vals, do_get=False, mode=COMPAT)
        except RuntimeError:
            continue
        with px.Store(records_per_shard=0) as st:
            res = st.set_batch(keys, vals, check=False)
            tot += 1
            if any(int(s) for s in res["status"]):
                bad += 1
                print(f"seed {seed} trial {trial}: status {list(res['status'])}", flush=True)
                continue
            comp = st.export(px.records_of(res))
            if comp != ref["comp"]:
                bad += 1
                i = next(i for i, (a, b) in enumerate(zip(comp, ref["comp"])) if a != b)
                print(f"seed {seed} trial {trial}: rec {i}/{n} gpu {len(comp[i])} B ref {len(ref['comp'][i])} B "
                      f"comp_len {list(res['comp_len'])}", flush=True)
    if seed % 20 == 0:
        print(f"seed {seed}: {tot} batches, {bad} bad, {time.time() - t0:.0f} s", flush=True)
print(f"done: {tot} batches, {bad} bad")
