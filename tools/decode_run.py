"""Debug aid: k_decode timing for one config-3 batch under several decode_waves settings."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import pixiu_amd as px
from pixiu_amd import synth
cfg, n, rps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
waves = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0]
cp = synth.make(cfg, n)
keys_host = (np.ascontiguousarray(cp.keys), cp.koff.astype(np.uint64))
out_cap = int(2 * cp.raw_bytes + 256 * n + (1 << 20))
out = torch.empty(out_cap, dtype=torch.uint8, device="cuda")
for w in waves:
    with px.Store(records_per_shard=rps, decode_waves=w) as st:
        st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        for rep in range(2):
            rc, off, ln, sts, need = st.get_batch_device(keys_host, out.data_ptr(), out_cap, px.COMPAT)
        ms = st.stats()["last_decode_kernel_ms"]
        print(f"waves {w}: decode kernel {ms:.2f} ms, expanded {int(np.asarray(ln).sum())} B -> {np.asarray(ln).sum() / ms / 1e3:.0f} MB/s rc {rc}")
