import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pixiu_amd as px
from pixiu_amd import synth
cp = synth.make(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
dev = torch.device("cuda", 0)
kb = torch.from_numpy(cp.keys).to(dev); ko = torch.from_numpy(cp.koff.astype(np.int64)).to(dev)
vb = torch.from_numpy(cp.vals).to(dev); vo = torch.from_numpy(cp.voff.astype(np.int64)).to(dev)
keys = (np.ascontiguousarray(cp.keys), cp.koff.astype(np.uint64))
cap = int(2 * cp.raw_bytes + 256 * cp.n + (1 << 20))
out = torch.empty(cap, dtype=torch.uint8, device=dev)
st = px.Store(records_per_shard=int(sys.argv[1]), device=0)
for i in range(3):
    st.reset()
    t0 = time.perf_counter()
    st.set_batch_device(cp.n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=False)
    t1 = time.perf_counter()
    for j in range(3):
        t2 = time.perf_counter()
        rc, off, ln, sts, _ = st.get_batch_device(keys, out.data_ptr(), cap, px.COMPAT)
        t3 = time.perf_counter()
        s = st.stats()
        print(f"round {i} get {j}: {(t3-t2)*1e3:.3f} ms  stage {s['last_decode_kernel_ms']:.3f}  device keys {int(s['last_get_device_keys'])}  gq {int(s['last_gather_queries'])}  set {(t1-t0)*1e3:.1f} ms", flush=True)
