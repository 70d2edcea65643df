import sys, time, os
sys.path.insert(0, '.')
import numpy as np
import pixiu_amd as px
from pixiu_amd import synth
cp = synth.make(5, int(sys.argv[1]))
st = px.Store(records_per_shard=126)
t = time.time()
r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
print("set", time.time() - t, int(r["status"].max()), st.stats()["last_psa_ms"], flush=True)
