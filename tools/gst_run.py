"""Debug aid: one k_gst_encode batch (config, records, rps) with the product library,
for rocprofv3 counter passes."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import pixiu_amd as px
from pixiu_amd import synth
cfg, n, rps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cp = synth.make(cfg, n)
with px.Store(records_per_shard=rps) as st:
    st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    stt = st.stats()
    print(f"config {cfg} n {n} rps {rps}: kernel {stt['last_set_stage_ms']:.1f} ms raw {int(cp.koff[-1] + cp.voff[-1])} B "
          f"ratio {stt['comp_bytes'] / max(stt['raw_bytes'], 1):.4f}")
