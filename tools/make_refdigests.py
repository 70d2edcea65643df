#!/usr/bin/env python3
"""Per-record digests of the REFERENCE's compressed bytes and compat getitem at the
bench's full sizes (tests/_refdig.py has the format).  Build container only: the
reference is oracle/_ref/libpxref.so, compiled from /root/reference/src by
`make -C oracle ref`; the outputs are data.

    python tools/make_refdigests.py                 # every (config, rps) below
    python tools/make_refdigests.py 3:139 4:8000    # some of them
    python tools/make_refdigests.py 4:0:50000       # the first 50,000 records only

Each shard is one fresh reference PiXiuCtrl (PiXiuCtrl.cpp:77-81) fed its records in
order (PiXiuCtrl.cpp:12-47); after the last setitem every key of the shard is read back
through PiXiuCtrl::getitem and the PXSGen drained (PiXiuCtrl.cpp:59-61). The reference
keeps process-global state (PiXiuStr.cpp:4, 17-26; SuffixTree.cpp:5-6), so shards run
in separate worker processes.
"""
from __future__ import annotations

import hashlib
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pixiu_amd import synth  # noqa: E402
import _refdig  # noqa: E402

# the bench's shard sizes (bench.DEFAULT_RPS) and the reference's own single instance
JOBS = [(3, 0, None), (3, 139, None), (5, 126, None), (2, 2000, None), (4, 8000, None),
        (4, 0, 50000)]  # (bench.py one_record_per_call: config 4's first 50,000 records, one instance)

_CORPUS = {}
_REF = None


def _shard(job):
    """(config, rps, first, count) -> per-record arrays of one shard"""
    global _REF
    cfg, rps, a, cnt = job
    if _REF is None:
        from _oracle import Reference
        _REF = Reference()
    cp = _CORPUS[cfg]
    keys = [cp.key(i) for i in range(a, a + cnt)]
    vals = [cp.val(i) for i in range(a, a + cnt)]
    t = time.time()
    r = _REF.run(keys, vals, do_get=True)
    d = _refdig.digest64
    return (cfg, rps, a, np.array([len(g) for g in r["get"]], np.uint32), np.array([d(g) for g in r["get"]], np.uint64),
            np.array([len(c) for c in r["comp"]], np.uint32), np.array([d(c) for c in r["comp"]], np.uint64),
            np.array(r["chunk"], np.uint32), np.array(r["idx"], np.uint32), time.time() - t)


def main():
    want = JOBS
    if len(sys.argv) > 1:
        want = [tuple(int(x) for x in s.split(":")) for s in sys.argv[1:]]
        want = [w if len(w) == 3 else w + (None,) for w in want]
    for cfg in sorted({w[0] for w in want}):
        _CORPUS[cfg] = synth.make(cfg)
    tasks = []
    limit = {}
    for cfg, rps, lim in want:
        n = lim or _CORPUS[cfg].n
        limit[(cfg, rps)] = lim
        step = rps or n
        tasks += [(cfg, rps, a, min(step, n - a)) for a in range(0, n, step)]
    want = [(c, r) for c, r, _ in want]
    # the longest shards first (the single instance alone is ~45 minutes)
    tasks.sort(key=lambda t: -int(_CORPUS[t[0]].koff[t[2] + t[3]] - _CORPUS[t[0]].koff[t[2]]
                                   + _CORPUS[t[0]].voff[t[2] + t[3]] - _CORPUS[t[0]].voff[t[2]]))
    res = {(c, r): {} for c, r in want}
    secs = {(c, r): 0.0 for c, r in want}
    workers = int(os.environ.get("REFDIG_WORKERS", "7"))
    t0 = time.time()
    with mp.get_context("fork").Pool(workers, maxtasksperchild=8) as pool:
        for out in pool.imap_unordered(_shard, tasks):
            cfg, rps, a = out[:3]
            res[(cfg, rps)][a] = out[3:9]
            secs[(cfg, rps)] += out[9]
            lim = limit[(cfg, rps)]
            n = lim or _CORPUS[cfg].n
            step = rps or n
            if len(res[(cfg, rps)]) == (n + step - 1) // step:
                parts = [res[(cfg, rps)][k] for k in sorted(res[(cfg, rps)])]
                cols = [np.concatenate([p[j] for p in parts]) for j in range(6)]
                cp = _CORPUS[cfg]
                h = hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest()  # (the full corpus)
                np.savez_compressed(_refdig.path(cfg, rps, lim), config=np.int64(cfg), rps=np.int64(rps),
                                    n=np.int64(n), get_len=cols[0], get_d64=cols[1], comp_len=cols[2],
                                    comp_d64=cols[3], chunk=cols[4], idx=cols[5],
                                    input_sha256=np.frombuffer(h.encode(), np.uint8),
                                    generator=np.frombuffer(b"Reference (oracle/_ref/libpxref.so)", np.uint8),
                                    reference_seconds=np.float64(secs[(cfg, rps)]))
                print(f"config {cfg} rps {rps}: {n} records, get {int(cols[0].sum())} B, comp "
                      f"{int(cols[2].sum())} B, {secs[(cfg, rps)]:.0f} s of reference time, "
                      f"{time.time() - t0:.0f} s wall", flush=True)
                del res[(cfg, rps)]


if __name__ == "__main__":
    main()
