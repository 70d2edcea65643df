"""Set-batch phase timing (one GPU): one config stored three times at its bench shard size
with PX_SET_VERBOSE=1 (px_runtime.cpp PhaseClock prints each phase to stderr)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PX_SET_VERBOSE"] = "1"
import pixiu_amd as px  # noqa: E402
from pixiu_amd import synth  # noqa: E402

RPS = {2: 2000, 3: 139, 4: 8000, 5: 126}


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cp = synth.make(cfg)
    dev = torch.device("cuda", 0)
    kb = torch.from_numpy(cp.keys).to(dev)
    ko = torch.from_numpy(cp.koff.astype(np.int64)).to(dev)
    vb = torch.from_numpy(cp.vals).to(dev)
    vo = torch.from_numpy(cp.voff.astype(np.int64)).to(dev)
    st = px.Store(records_per_shard=RPS[cfg], device=0)
    for i in range(3):
        st.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.set_batch_device(cp.n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=False)
        print(f"--- set {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
