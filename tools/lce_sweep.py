"""LCE span sweep (one GPU): config 3 stored at the bench's shard size with PX_LCE_SPAN set
to each value (a fresh process per value: the span is read per launch), reporting the
links + lcp stage and the whole encode stage."""
import os
import subprocess
import sys

CHILD = r'''
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.getcwd())
import pixiu_amd as px
from pixiu_amd import synth
cp = synth.make(3)
dev = torch.device("cuda", 0)
kb = torch.from_numpy(cp.keys).to(dev); ko = torch.from_numpy(cp.koff.astype(np.int64)).to(dev)
vb = torch.from_numpy(cp.vals).to(dev); vo = torch.from_numpy(cp.voff.astype(np.int64)).to(dev)
st = px.Store(records_per_shard=139, device=0)
lcp, enc, comp = [], [], 0
for i in range(4):
    st.reset()
    res = st.set_batch_device(cp.n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=False)
    s = st.stats()
    if i:
        lcp.append(s["last_psa_lcp_ms"]); enc.append(s["last_encode_stage_ms"])
    comp = int(res["comp_len"].sum())
print(f"PX_LCE_SPAN={os.environ.get('PX_LCE_SPAN', 'default')}: links+lcp {np.median(lcp):.2f} ms  encode {np.median(enc):.2f} ms  comp {comp}", flush=True)
'''


def main():
    for v in (sys.argv[1] if len(sys.argv) > 1 else "256,128,64,32").split(","):
        env = dict(os.environ)
        env["PX_LCE_SPAN"] = v
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
