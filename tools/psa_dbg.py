import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import torch; assert torch.cuda.is_available()
import pixiu_amd as px
from pixiu_amd import synth
from _oracle import Oracle, assemble
cp = synth.make(3, int(sys.argv[1]))
with px.Store(records_per_shard=int(sys.argv[2])) as st:
    r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)), check=False)
    print("status max", int(r["status"].max()), st.stats()["last_psa_iters"])
