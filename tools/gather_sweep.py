"""Getitem tuning sweep (one GPU): config 3 stored once (argv[2]: records per shard, 139), then
20 full-record getitem batches per setting of PX_GATHER_WG (k_gather workgroups per CU);
prints the median stage (HIP events) and call wall per setting."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pixiu_amd as px  # noqa: E402
from pixiu_amd import synth  # noqa: E402


def main():
    settings = [s for s in (sys.argv[1] if len(sys.argv) > 1 else "16,5,8,32").split(",")]
    rps = int(sys.argv[2]) if len(sys.argv) > 2 else 139
    cp = synth.make(3)
    dev = torch.device("cuda", 0)
    kb = torch.from_numpy(cp.keys).to(dev)
    ko = torch.from_numpy(cp.koff.astype(np.int64)).to(dev)
    vb = torch.from_numpy(cp.vals).to(dev)
    vo = torch.from_numpy(cp.voff.astype(np.int64)).to(dev)
    st = px.Store(records_per_shard=rps, device=0)
    st.set_batch_device(cp.n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=False)
    keys = (np.ascontiguousarray(cp.keys), cp.koff.astype(np.uint64))
    cap = int(2 * cp.raw_bytes + 256 * cp.n + (1 << 20))
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    ref = None
    for s in settings:
        os.environ["PX_GATHER_WG"] = s
        ks, ws = [], []
        for _ in range(20):
            t0 = time.perf_counter()
            rc, off, ln, sts, _ = st.get_batch_device(keys, out.data_ptr(), cap, px.COMPAT)
            ws.append((time.perf_counter() - t0) * 1e3)
            ks.append(st.stats()["last_decode_kernel_ms"])
            assert rc == px.PX_OK
        h = hash(out[: int(off[-1]) + int(ln[-1])].cpu().numpy().tobytes())
        ref = h if ref is None else ref
        print(f"PX_GATHER_WG={s}: stage {np.median(ks):.3f} ms  wall {np.median(ws):.3f} ms (first {ws[0]:.3f}) "
              f"device keys {int(st.stats()['last_get_device_keys'])}  gather queries "
              f"{int(st.stats()['last_gather_queries'])}  same={h == ref}", flush=True)


if __name__ == "__main__":
    main()
