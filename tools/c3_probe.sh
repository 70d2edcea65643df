#!/bin/bash
# config 3 at 64-record shards: per-step group classes of the segmented doubling sort
mkdir -p gpurun_out
PX_PSA_SEGSORT=1 PX_PSA_VERBOSE=1 timeout -k 10 120 python -u - > gpurun_out/c3_steps.log 2>&1 <<'PY'
import sys, time
sys.path.insert(0, '.')
import numpy as np
import pixiu_amd as px
from pixiu_amd import synth
cp = synth.make(3, 10000)
st = px.Store(records_per_shard=64)
for _ in range(2):
    st.reset()
    t = time.time()
    r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    print("set", time.time() - t, int(r["status"].max()), st.stats()["last_psa_ms"], flush=True)
PY
