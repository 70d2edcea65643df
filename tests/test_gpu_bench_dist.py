"""bench.py's own N > 1 branch on one GPU: two ranks (torch.distributed.run, gloo) run the
timed step -- setitem, save_device, the chunk-blob gather to rank 0, getitem -- and the
MAX / SUM reductions; rank 0 then loads both gathered blobs into a fresh store and reads
back a sample of each rank's keys (EXACT == the regenerated doc; its own records' compat
expansion == its live store's, served by span-table gathers of the loaded chunks)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("rps", [None, 0], ids=["bench_rps", "rps0"])
def test_bench_two_ranks_gloo(rps):
    """rps 0: every rank is one single-instance shard; rank 0 loads each gathered blob into
    a store of its own (a single shard takes one blob)"""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--records", "300", "--configs", "", "--steps", "1",
           "--warmup", "0", "--no-cpu", "--no-single", "--no-pcie", "--no-cliff"]
    if rps is not None:
        cmd += ["--rps", str(rps)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["backend"] == "gloo"
    assert out["config"]["records_per_gpu"] == 300
    g = out["gather_check"]
    assert g["ranks"] == 2 and len(g["blob_bytes"]) == 2 and min(g["blob_bytes"]) > 0
    assert g["records_checked"] == 2 * g["records_per_rank_sampled"] > 0
    assert g["exact_equal"] == g["records_checked"]
    assert g["rank0_compat_equal_live"] == g["records_per_rank_sampled"]
    assert g["rank0_gather_served"] > 0
    assert out["parity_counts"]["exact_ne_original"] == 0
    assert g["stores"] == (2 if rps == 0 else 1)
