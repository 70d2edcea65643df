"""Debug aid: host-side getitem phases (key lookups, whole C call) on one config-3
batch under several host_threads settings; contains() is the single-threaded lookup."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import pixiu_amd as px
from pixiu_amd import synth
n, rps = int(sys.argv[1]), int(sys.argv[2])
threads = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
cp = synth.make(3, n)
keys_host = (np.ascontiguousarray(cp.keys), cp.koff.astype(np.uint64))
out_cap = int(2 * cp.raw_bytes + 256 * n + (1 << 20))
out = torch.empty(out_cap, dtype=torch.uint8, device="cuda")
for t in threads:
    with px.Store(records_per_shard=rps, host_threads=t) as st:
        st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        look, call, wall = [], [], []
        for rep in range(8):
            t0 = time.perf_counter()
            rc, off, ln, sts, need = st.get_batch_device(keys_host, out.data_ptr(), out_cap, px.COMPAT)
            wall.append((time.perf_counter() - t0) * 1e3)
            s = st.stats()
            look.append(s["last_get_lookup_ms"])
            call.append(s["last_get_call_ms"])
        t0 = time.perf_counter()
        c = st.contains(keys_host)
        cms = (time.perf_counter() - t0) * 1e3
        print(f"threads {t}: lookup {np.median(look):.3f} ms (min {min(look):.3f}), call {np.median(call):.3f}, "
              f"wall {np.median(wall):.3f}, decode {s['last_decode_kernel_ms']:.3f}; contains (1 thread) {cms:.3f} ms "
              f"found {int(np.sum(c))} rc {rc}", flush=True)
