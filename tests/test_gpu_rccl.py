"""The multi-GPU exchange over RCCL itself (backend "nccl" = RCCL on ROCm), on the one GPU
of a test box: a world-size-1 NCCL process group, as bench.py:main opens it.

* ``gather_blobs`` (pixiu_amd/dist.py): the size all_gather runs over RCCL;
* the blob then goes through RCCL point to point, with the same ``batch_isend_irecv``
  P2POp batch gather_blobs issues on N > 1 (here a send to self and the matching receive);
* the received copy is ``px_load``-ed into a fresh store and every key read back (EXACT ==
  the escaped doc, COMPAT == the live store's).

The 1 -> 8 GPU curve is the driver's (SCALE_rNN.json); this pins that the RCCL calls the
N > 1 path makes execute on MI355X."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.environ["PX_ROOT"])
import numpy as np
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
import pixiu_amd as px
from pixiu_amd import synth
from pixiu_amd.dist import gather_blobs

assert dist.get_backend() == "nccl"
cp = synth.make(2, 3000)
keys = [cp.key(i) for i in range(cp.n)]
vals = [cp.val(i) for i in range(cp.n)]
dev = torch.device("cuda", 0)
out = {}
with px.Store(records_per_shard=1000) as st:
    st.set_batch(keys, vals)
    nb = st.save_device(0, 0)
    buf = torch.empty(nb, dtype=torch.uint8, device=dev)
    st.save_device(buf.data_ptr(), nb)
    got = gather_blobs(buf, dst=0)                      # size all_gather over RCCL
    out["gathered"] = len(got)
    recv = torch.empty_like(buf)                        # RCCL point to point: send to self + receive
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, got[0], 0), dist.P2POp(dist.irecv, recv, 0)])
    for q in reqs:
        q.wait()
    torch.cuda.synchronize()
    out["p2p_equal"] = bool(torch.equal(recv, buf))
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev)]
    dist.all_gather(sizes, torch.tensor([nb], dtype=torch.int64, device=dev))
    out["allgather_size"] = int(sizes[0].item()) == nb
    live = st.get_batch(keys, px.COMPAT)
    with px.Store(records_per_shard=1000) as st2:
        st2.load(recv.data_ptr(), on_device=True, length=nb)
        ex = st2.get_batch(keys, px.EXACT)
        co = st2.get_batch(keys, px.COMPAT)
    docs = [k + b"\xfb\x00" + v + b"\xfb\x02" for k, v in zip(keys, vals)]
    out["exact_equal"] = sum(a == b for a, b in zip(ex, docs))
    out["compat_equal_live"] = sum(a == b for a, b in zip(co, live))
    out["records"] = len(keys)
    out["blob_bytes"] = nb
dist.destroy_process_group()
print(json.dumps(out))
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_gather_p2p_load():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", PX_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(out)
    assert out["gathered"] == 1 and out["p2p_equal"] and out["allgather_size"]
    assert out["exact_equal"] == out["records"] == 3000
    assert out["compat_equal_live"] == out["records"]
