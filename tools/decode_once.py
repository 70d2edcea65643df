"""Debug aid: one get_batch (compat) over a config batch, product library (for rocprofv3)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import pixiu_amd as px
from pixiu_amd import synth
cfg, n, rps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cp = synth.make(cfg, n)
keys_host = (np.ascontiguousarray(cp.keys), cp.koff.astype(np.uint64))
out_cap = int(2 * cp.raw_bytes + 256 * n + (1 << 20))
out = torch.empty(out_cap, dtype=torch.uint8, device="cuda")
with px.Store(records_per_shard=rps) as st:
    st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    rc, off, ln, sts, need = st.get_batch_device(keys_host, out.data_ptr(), out_cap, px.COMPAT)
    print(f"decode kernel {st.stats()['last_decode_kernel_ms']:.2f} ms rc {rc}")
