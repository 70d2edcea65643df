"""GPU probe: store config-3 records at a shard size, get every key back, report misses
(index, chunk, slot, exact round trip, contains).  python tools/get_probe.py N RPS"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

assert torch.cuda.is_available()
import pixiu_amd as px  # noqa: E402
from pixiu_amd import synth  # noqa: E402
from _oracle import assemble  # noqa: E402

n, rps = int(sys.argv[1]), int(sys.argv[2])
cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cp = synth.make(cfg, n)
dev = len(sys.argv) > 4 and sys.argv[4] == "dev"
with px.Store(records_per_shard=rps) as st:
    if dev:  # inputs resident in HBM, as bench.py stores them
        kb = torch.from_numpy(cp.keys).cuda()
        ko = torch.from_numpy(cp.koff.astype(np.int64)).cuda()
        vb = torch.from_numpy(cp.vals).cuda()
        vo = torch.from_numpy(cp.voff.astype(np.int64)).cuda()
        st.reset()
        r = st.set_batch_device(n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=False)
    else:
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    print("set: status max", int(r["status"].max()), "chunks", int(r["chunk"].max()) + 1, flush=True)
    got = st.get_batch([cp.key(i) for i in range(n)])
    miss = [i for i, g in enumerate(got) if g is None]
    print("missing", len(miss), miss[:20], flush=True)
    if miss:
        m = miss[:20]
        ex = st.parse_batch(px.records_of(r[m]), px.EXACT)
        co = st.parse_batch(px.records_of(r[m]), px.COMPAT)
        for j, i in enumerate(m):
            d = assemble(cp.key(i), cp.val(i))
            print(i, "chunk", int(r["chunk"][i]), "idx", int(r["idx"][i]), "shard", int(r["shard"][i]),
                  "exact==doc", ex[j] == d, "compat==doc", co[j] == d, "keylen", len(cp.key(i)),
                  "compat key prefix ok", co[j][:len(cp.key(i))] == cp.key(i), flush=True)
        # chunk boundaries
        ch = r["chunk"].tolist()
        b = [0] + [i for i in range(1, n) if ch[i] != ch[i - 1]]
        print("chunk starts", b[:80])
