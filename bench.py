#!/usr/bin/env python3
"""bench.py — PiXiu batch setitem + getitem on MI355X (BASELINE.json metric).

One step = batch setitem of the whole per-rank corpus into a fresh store (escape,
GST walk + encoder, packed store, segment index, CritBit inserts) followed by a
batch getitem (CritBit lookup + compat PXSGen expansion) of every key, with
inputs resident in HBM when the timed region starts.  With N > 1 GPUs every
rank runs its own corpus part (weak scaling, no cross-GPU references) and the
compressed output is gathered to rank 0 over RCCL, the one exchange step.

value = setitem MB/s (raw key+value bytes ingested) + getitem MB/s (expanded
bytes), both whole-job aggregates; the two parts are reported separately.

  python bench.py                       # N=1, config 3 (10k x 60 KB HTML-shape)
  torchrun --nproc-per-node 8 bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
# records per shard (independent GST instances) benchmarked for each BASELINE config;
# DESIGN.md §6 has the compression-vs-shard-size curve.  Config 3: 139 pages (8.35 MB) is
# the largest shard whose live chunk cannot rotate (kPsaMaxText), and
# compresses within 0.5 % of the reference's single instance (0.7734 vs 0.7698)
DEFAULT_RPS = {1: 0, 2: 2000, 3: 139, 4: 8000, 5: 126}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, help="the headline config (BASELINE.json metric: 3)")
    ap.add_argument("--records", type=int, default=None, help="records per rank (default: full config)")
    ap.add_argument("--rps", type=int, default=None, help="records per shard (default: DEFAULT_RPS[config])")
    ap.add_argument("--configs", default="2,4,5",
                    help="further BASELINE configs reported under per_config ('' for none)")
    ap.add_argument("--extra-steps", type=int, default=2, help="timed steps of each further config")
    ap.add_argument("--no-checks", action="store_true", help="skip the compat/exact/original parity counts")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the single-instance leg (config 3 as one shard, GPU and CPU)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) leg")
    ap.add_argument("--no-cliff", action="store_true", help="skip the walk-fallback leg (one forced-flag shard)")
    ap.add_argument("--no-exact", action="store_true",
                    help="skip the exact-mode getitem (profiling runs: one compat batch per step only)")
    ap.add_argument("--retain-mb", type=int, default=0,
                    help="px_opts.retain_mb of the benchmarked stores (0: the batch's own peak stays cached)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N > 1 (nccl = RCCL over xGMI; gloo: CPU transport, for tests)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_r06.json"),
                    help="per-kernel PMC summary (tools/pmc_summary.py); used only if its workload matches")
    return ap.parse_args()


def cpu_baseline(corpus, rps, budget_s):
    """Time the oracle (clean-room CPU restatement, 1 thread) on whole shards of the
    same corpus and shard size, until the budget is spent; also spot-check parity."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import Oracle
    orc = Oracle()
    rps = rps or corpus.n
    t_set = t_get = 0.0
    raw = exp = 0
    nrec = 0
    shards = []
    s = 0
    while s < corpus.n and (t_set + t_get) < budget_s:
        rows = range(s, min(corpus.n, s + rps))
        sh = orc.new()
        ks = [corpus.key(i) for i in rows]
        vs = [corpus.val(i) for i in rows]
        t0 = time.perf_counter()
        for k, v in zip(ks, vs):
            rc, _, _ = sh.set(k, v)
            if rc < 0:
                raise RuntimeError(f"oracle setitem failed: {rc}")
        t1 = time.perf_counter()
        outs = [sh.get(k) for k in ks]
        t2 = time.perf_counter()
        t_set += t1 - t0
        t_get += t2 - t1
        raw += sum(len(k) + len(v) for k, v in zip(ks, vs))
        exp += sum(len(o) for o in outs if o)
        nrec += len(ks)
        shards.append((s, sh, ks, outs))
        s += rps
    return {"set_MBps": raw / t_set / 1e6, "get_MBps": exp / t_get / 1e6, "records": nrec, "raw": raw,
            "shards": shards, "seconds": t_set + t_get}


def walk_cliff(local, corpus, records=8):
    """The walk fallback's cost: the first `records` records as one shard, once through
    the suffix-array path and once with the stale-pair check forced to fire
    (PX_DEBUG_PSA_FLAG_ROUND=1: the shard is re-walked by k_gst_encode).
    Both must give the same bytes (the configs hold no stale state)."""
    import pixiu_amd as px
    kv = ((np.ascontiguousarray(corpus.keys[:corpus.koff[records]]), corpus.koff[:records + 1].astype(np.uint64)),
          (np.ascontiguousarray(corpus.vals[:corpus.voff[records]]), corpus.voff[:records + 1].astype(np.uint64)))
    raw = int(corpus.koff[records] + corpus.voff[records])
    out = {}
    for name, flag in (("psa", None), ("psa", None), ("walk", "1")):
        if flag:
            os.environ["PX_DEBUG_PSA_FLAG_ROUND"] = flag
        try:
            with px.Store(records_per_shard=records, device=local) as st:
                t0 = time.perf_counter()
                r = st.set_batch(*kv)
                dt = time.perf_counter() - t0
                s = st.stats()
                out[name] = {"s": dt, "walk_shards": int(s["last_walk_shards"]),
                             "comp": st.export(px.records_of(r))}
        finally:
            os.environ.pop("PX_DEBUG_PSA_FLAG_ROUND", None)
    return {"records": records, "raw_bytes": raw, "psa_MBps": round(raw / out["psa"]["s"] / 1e6, 3),
            "walk_MBps": round(raw / out["walk"]["s"] / 1e6, 3),
            "walk_over_psa_time": round(out["walk"]["s"] / out["psa"]["s"], 1),
            "walked_shards": out["walk"]["walk_shards"], "bytes_equal": out["walk"]["comp"] == out["psa"]["comp"],
            "note": "one shard forced to the walk fallback (PX_DEBUG_PSA_FLAG_ROUND=1), host buffers, one call"}


def small_batches(local, calls=50000, defer_mb=8):
    """Facade-shaped setitem: one record per call (PiXiuCtrl::setitem, PiXiuCtrl.cpp:12-47,
    through px_set_batch with n = 1) into one store at records_per_shard = 0: config 4's
    first `calls` records (256 B; 50,000 cross a chunk rotation), through the write-behind
    queue the facade uses (px_opts.defer_bytes = defer_mb MB, include/pixiu_amd.h px_flush).
    Timed: every call plus the final flush.  Then (untimed) every record's compressed bytes,
    slot and compat getitem against the reference's own digests for the same records
    (tests/golden/refdig_c4_r0_n50000.npz)."""
    import pixiu_amd as px
    from pixiu_amd import synth
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _refdig
    cp = synth.make(4)
    keys = [cp.key(i) for i in range(calls)]
    vals = [cp.val(i) for i in range(calls)]
    raw = sum(len(k) + len(v) for k, v in zip(keys, vals))
    ts = np.zeros(calls)
    one = np.zeros(1, np.uint64)
    with px.Store(records_per_shard=0, device=local, defer_bytes=defer_mb << 20) as st:
        lib, h = st._lib, st._h
        res = np.zeros(1, px.SET_RESULT_DTYPE)
        rp = res.ctypes.data
        ko = np.zeros(2, np.uint64)
        vo = np.zeros(2, np.uint64)
        kop, vop = ko.ctypes.data, vo.ctypes.data
        replaced = 0
        t_all = time.perf_counter()
        for i in range(calls):
            k, v = keys[i], vals[i]
            ko[1], vo[1] = len(k), len(v)
            t0 = time.perf_counter()
            rc = lib.px_set_batch(h, 1, k, kop, v, vop, 0, rp)
            ts[i] = time.perf_counter() - t0
            if rc != px.PX_OK:
                raise SystemExit(f"one_record_per_call: setitem {i} rc={rc}")
            replaced += int(res["replaced"][0])
        t0 = time.perf_counter()
        st.flush()
        t_flush = time.perf_counter() - t0
        total = time.perf_counter() - t_all
        s = st.stats()
        out = {"calls": calls, "record_bytes": raw // calls, "chunks": int(s["chunks"]),
               "defer_bytes": defer_mb << 20, "flushes": int(s["deferred_flushes"]),
               "ms_per_call_first1000": round(float(ts[:1000].mean()) * 1e3, 4),
               "ms_per_call_last1000": round(float(ts[-1000:].mean()) * 1e3, 4),
               "ms_per_call_max": round(float(ts.max()) * 1e3, 3), "final_flush_ms": round(t_flush * 1e3, 3),
               "MBps": round(raw / total / 1e6, 3), "replaced": replaced,
               "deferred_mismatch": int(s["deferred_mismatch"])}
        ref = _refdig.load(4, 0, calls)
        if ref is not None:  # every record vs the reference fed the same records one call at a time
            recs, sts = st.locate(keys)
            r2 = np.zeros(calls, px.SET_RESULT_DTYPE)
            r2["shard"], r2["chunk"], r2["idx"] = recs["shard"], recs["chunk"], recs["idx"]
            import torch
            buf, off, ln = _refdig.compat_all(st, keys, torch.device("cuda", local))
            chk = _refdig.check_store(ref, st, r2, buf, off, ln)
            out["reference_check"] = dict(chk, fixture=os.path.relpath(_refdig.path(4, 0, calls), ROOT))
    return out


def cpu_calibration():
    """The oracle-vs-reference speed factors measured in the build container (the GPU box
    has no reference): profiles/cpu_calibration_r03.json, or None."""
    path = os.path.join(ROOT, "profiles", "cpu_calibration_r03.json")
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def cpu_single_instance(corpus, budget_s):
    """The reference-shaped CPU baseline: ONE oracle instance (records_per_shard = 0, the
    reference's single PiXiuCtrl with its chunk rotation), records set in order until half
    the budget is spent, then every stored key read back."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import Oracle
    sh = Oracle().new()
    ks, raw = [], 0
    t0 = time.perf_counter()
    while len(ks) < corpus.n and time.perf_counter() - t0 < budget_s / 2:
        k, v = corpus.key(len(ks)), corpus.val(len(ks))
        if sh.set(k, v)[0] < 0:
            raise RuntimeError("oracle setitem failed")
        ks.append(k)
        raw += len(k) + len(v)
    t1 = time.perf_counter()
    exp = sum(len(sh.get(k) or b"") for k in ks)
    t2 = time.perf_counter()
    return {"set_MBps": raw / (t1 - t0) / 1e6, "get_MBps": exp / (t2 - t1) / 1e6, "records": len(ks), "raw": raw,
            "seconds": t2 - t0}


def cpu_baseline_mt(corpus, rps, set_MBps_1t, budget_s):
    """The same oracle with N threads = min(#shards, host cores), one independent
    instance per shard (SURVEY.md §8d second row).  ctypes drops the GIL inside the
    oracle calls; shards are sized so the set phase takes about budget_s."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import Oracle
    orc = Oracle()
    rps = rps or corpus.n
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))  # a GPU box gives one process a 16-core share
    shard_bytes = corpus.raw_bytes / corpus.n * rps
    per_thread = max(1, int(set_MBps_1t * 1e6 * budget_s / shard_bytes))
    nshards = min(corpus.n // rps, cores * per_thread)
    threads = max(1, min(cores, nshards))
    starts = [i * rps for i in range(nshards)]

    def do_set(s0):
        sh = orc.new()
        ks = [corpus.key(i) for i in range(s0, s0 + rps)]
        vs = [corpus.val(i) for i in range(s0, s0 + rps)]
        for k, v in zip(ks, vs):
            if sh.set(k, v)[0] < 0:
                raise RuntimeError("oracle setitem failed")
        return sh, ks, sum(len(k) + len(v) for k, v in zip(ks, vs))

    def do_get(item):
        sh, ks, _ = item
        return sum(len(sh.get(k) or b"") for k in ks)

    with cf.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        done = list(ex.map(do_set, starts))
        t1 = time.perf_counter()
        exp = sum(ex.map(do_get, done))
        t2 = time.perf_counter()
    raw = sum(d[2] for d in done)
    return {"set_MBps": raw / (t1 - t0) / 1e6, "get_MBps": exp / (t2 - t1) / 1e6, "threads": threads,
            "records": nshards * rps, "raw": raw, "seconds": t2 - t0}


def pcie_leg(st, px, corpus, keys_host, out_cap):
    """The same batch through host buffers, as the PiXiuCtrl facade hands them over:
    setitem uploads the raw records, getitem downloads the expanded bytes into host
    memory. Reported beside `value` (never as it); the second of two passes is kept
    (the first touches the host pages)."""
    vals_host = (np.ascontiguousarray(corpus.vals), corpus.voff.astype(np.uint64))
    out_h = np.empty(out_cap, np.uint8)
    for _ in range(2):
        st.reset()
        t0 = time.perf_counter()
        res = st.set_batch(keys_host, vals_host)
        t1 = time.perf_counter()
        rc, off, ln, sts, need = st.get_batch_host(keys_host, out_h, px.COMPAT)
        t2 = time.perf_counter()
        if rc != px.PX_OK or int(res["status"].max()) != 0 or int(sts.max()) != 0:
            raise SystemExit(f"host-buffer leg: rc={rc}")
    return {"set_MBps": round(corpus.raw_bytes / (t1 - t0) / 1e6, 3),
            "get_MBps": round(int(ln.sum()) / (t2 - t1) / 1e6, 3),
            "set_ms": round((t1 - t0) * 1e3, 3), "get_ms": round((t2 - t1) * 1e3, 3),
            "note": "host (pageable) inputs and output buffer, PCIe transfers inside the timed calls"}


def _docs_np(corpus):
    """Every record's escaped doc (PiXiuCtrl.cpp:31-44) as one host buffer + offsets."""
    if not (corpus.keys == 251).any() and not (corpus.vals == 251).any():
        n = corpus.n
        kl, vl = np.diff(corpus.koff), np.diff(corpus.voff)
        dl = kl + 2 + np.where(vl > 0, vl + 2, 0)
        off = np.zeros(n + 1, np.int64)
        np.cumsum(dl, out=off[1:])
        buf = np.empty(int(off[-1]), np.uint8)
        for i in range(n):  # vectorising this buys little next to the decode
            o = int(off[i])
            k = corpus.keys[corpus.koff[i]:corpus.koff[i + 1]]
            buf[o:o + len(k)] = k
            buf[o + len(k):o + len(k) + 2] = (251, 0)
            if vl[i]:
                v = corpus.vals[corpus.voff[i]:corpus.voff[i + 1]]
                p = o + len(k) + 2
                buf[p:p + len(v)] = v
                buf[p + len(v):p + len(v) + 2] = (251, 2)
        return buf, off
    parts = []
    for i in range(corpus.n):
        k, v = corpus.key(i), corpus.val(i)
        d = k.replace(b"\xfb", b"\xfb\xfb") + b"\xfb\x00"
        if v:
            d += v.replace(b"\xfb", b"\xfb\xfb") + b"\xfb\x02"
        parts.append(d)
    off = np.zeros(corpus.n + 1, np.int64)
    np.cumsum([len(x) for x in parts], out=off[1:])
    return np.frombuffer(b"".join(parts), np.uint8), off


def _count_ne(a, a_off, a_len, b, b_off, b_len, dev, piece=1 << 26):
    """Records whose byte ranges differ: a[a_off[i]:+a_len[i]] vs b[b_off[i]:+b_len[i]]
    (device buffers; compared on the GPU in pieces of about `piece` bytes)."""
    import torch
    a_off = np.asarray(a_off, np.int64)
    b_off = np.asarray(b_off, np.int64)
    a_len = np.asarray(a_len, np.int64)
    b_len = np.asarray(b_len, np.int64)
    n = len(a_len)
    bad = int((a_len != b_len).sum())
    same = np.nonzero(a_len == b_len)[0]
    lens = a_len[same]
    i = 0
    while i < len(same):
        j = i
        tot = 0
        while j < len(same) and (tot == 0 or tot + lens[j] <= piece):
            tot += int(lens[j])
            j += 1
        sel = same[i:j]
        ln = torch.from_numpy(lens[i:j]).to(dev)
        seg = torch.repeat_interleave(torch.arange(j - i, device=dev), ln)
        start = torch.cumsum(ln, 0) - ln
        within = torch.arange(int(ln.sum()), device=dev) - torch.repeat_interleave(start, ln)
        ia = torch.from_numpy(a_off[sel]).to(dev)[seg] + within
        ib = torch.from_numpy(b_off[sel]).to(dev)[seg] + within
        neq = (a[ia] != b[ib]).to(torch.int32)
        per = torch.zeros(j - i, dtype=torch.int32, device=dev).index_add_(0, seg, neq)
        bad += int((per > 0).sum())
        i = j
    assert n >= bad
    return bad


def run_config(cfg, a, rank, world, local, steps, warmup, rps, records=None, checks=True):
    """One BASELINE config on this rank: warmup + `steps` timed steps of batch setitem
    (+ the blob gather when world > 1) and compat getitem, then (untimed) an exact-mode
    getitem and the compat / exact / original parity counts over every record."""
    import torch
    import torch.distributed as dist
    import pixiu_amd as px
    from pixiu_amd import synth
    from pixiu_amd.dist import gather_blobs

    corpus = synth.make(cfg, records, part=rank)  # weak scaling: an independent part per rank
    n = corpus.n
    dev = torch.device("cuda", local)
    kb = torch.from_numpy(corpus.keys).to(dev)
    ko = torch.from_numpy(corpus.koff.astype(np.int64)).to(dev)
    vb = torch.from_numpy(corpus.vals).to(dev)
    vo = torch.from_numpy(corpus.voff.astype(np.int64)).to(dev)
    keys_host = (np.ascontiguousarray(corpus.keys), corpus.koff.astype(np.uint64))
    raw_bytes = corpus.raw_bytes
    # every doc is <= 2*raw + 4 escaped bytes; the decoder gets doc_len + 64 per record
    out_cap = int(2 * raw_bytes + 256 * n + (1 << 20))
    out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    gather_buf = [None]
    gathered = [None]
    st = px.Store(records_per_shard=rps, device=local, retain_mb=a.retain_mb)
    # getitem takes the keys where setitem took them (HBM: kb / ko) and leaves its offsets,
    # lengths and statuses in HBM (px_get_batch_dev); the pcie_inclusive leg times host keys
    # and host results
    r_off = torch.empty(n, dtype=torch.int64, device=dev)
    r_len = torch.empty(n, dtype=torch.int32, device=dev)
    r_sts = torch.empty(n, dtype=torch.int32, device=dev)

    # (the caller's device pointers, taken once: a torch data_ptr() per argument per call was
    # part of the timed getitem)
    ptrs = (kb.data_ptr(), ko.data_ptr(), r_off.data_ptr(), r_len.data_ptr(), r_sts.data_ptr())

    def get_dev(buf, mode):
        rc, need = st.get_batch_dev(n, ptrs[0], ptrs[1], buf.data_ptr(), out_cap, ptrs[2], ptrs[3], ptrs[4], mode)
        return rc, need

    def step():
        tr = time.perf_counter()
        st.reset()
        t0 = time.perf_counter()
        res = st.set_batch_device(n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=False)
        t_set = time.perf_counter() - t0
        sst = st.stats()
        set_kms, walk_kms, emit_kms = sst["last_set_stage_ms"], sst["last_encode_stage_ms"], sst["last_emit_kernel_ms"]
        psa = (sst["last_psa_ms"], int(sst["last_psa_shards"]), int(sst["last_walk_shards"]),
               sst["last_psa_sort_ms"], sst["last_psa_lcp_ms"], sst["last_psa_msg_ms"], int(sst["last_psa_iters"]),
               int(sst["last_psa_rounds"]), int(sst["last_psa_rotations"]), sst["last_psa_pool_ms"], int(sst["chunks"]))
        t1 = time.perf_counter()  # (the set stats above are instrumentation, outside both timings)
        rc, need = get_dev(out, px.COMPAT)
        t2 = time.perf_counter()
        gst = st.stats()
        dec_kms, look_ms, call_ms = gst["last_decode_kernel_ms"], gst["last_get_lookup_ms"], gst["last_get_call_ms"]
        spans = (int(gst["last_gather_queries"]), int(sst["span_entries"]), sst["last_span_build_ms"],
                 int(sst["device_bytes"]), int(sst["last_set_peak_bytes"]), int(sst["device_live_bytes"]))
        g_ms = 0.0
        if world > 1:  # every rank's chunk blob (pixiu_amd/blob.py) to rank 0, RCCL over xGMI
            tg = time.perf_counter()
            nb = st.save_device(0, 0)
            if gather_buf[0] is None or gather_buf[0].numel() < nb:
                gather_buf[0] = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            st.save_device(gather_buf[0].data_ptr(), nb)
            blob = gather_buf[0][:nb]
            if a.backend == "gloo":  # (gloo moves CPU tensors)
                blob = blob.cpu()
            gathered[0] = gather_blobs(blob, dst=0)
            torch.cuda.synchronize()
            g_ms = (time.perf_counter() - tg) * 1e3
        if rc != px.PX_OK or int(res["status"].max()) != 0:
            bad = int((res["status"] != 0).sum())
            raise SystemExit(f"rank {rank} config {cfg}: setitem failures={bad} getitem rc={rc}")
        # setitem's one exchange (the compressed-blob gather to rank 0) counts as setitem time
        return {"set_s": t_set + g_ms * 1e-3, "get_s": t2 - t1, "reset_s": t0 - tr, "set_kms": set_kms, "walk_kms": walk_kms,
                "emit_kms": emit_kms, "dec_kms": dec_kms, "gather_ms": g_ms, "look_ms": look_ms,
                "call_ms": call_ms, "comp": int(res["comp_len"].sum()), "exp": int(r_len.sum(dtype=torch.int64)),
                "res": res, "psa": psa, "spans": spans,
                "mem": {k[4:-6]: int(sst[k]) for k in sst if k.startswith("mem_") and k.endswith("_bytes")}}

    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    T0 = time.perf_counter()
    runs = [step() for _ in range(steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    T1 = time.perf_counter()
    r = {"corpus": corpus, "st": st, "runs": runs, "elapsed": T1 - T0, "n": n, "raw": raw_bytes,
         "out": out, "out_cap": out_cap, "keys_host": keys_host, "gathered": gathered[0]}
    last = runs[-1]
    last["off"] = r_off.cpu().numpy().astype(np.uint64)  # (the last step's results, for the checks)
    last["len"] = r_len.cpu().numpy().astype(np.uint32)
    # every record against the reference's own output (per-record digests made from the
    # compiled reference over the same corpus part and shards, tests/_refdig.py); only the
    # canonical part 0 at full size has them (not in --no-checks runs: the profiling legs)
    if rank == 0 and checks:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _refdig
        ref = _refdig.load(cfg, rps)
        if ref is not None and int(ref["n"]) == n:
            r["reference_check"] = dict(_refdig.check_store(ref, st, last["res"], out, last["off"], last["len"]),
                                        fixture=os.path.relpath(_refdig.path(cfg, rps), ROOT))
    # exact-mode getitem (one timed call, outside the step loop) and parity counts
    if a.no_exact:
        r["exact_s"], r["exact_dec_kms"], r["exact_exp"], r["exact_gather"] = 0.0, 0.0, 0, 0
        return r
    out2 = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    te = time.perf_counter()
    rc, _ = get_dev(out2, px.EXACT)
    r["exact_s"] = time.perf_counter() - te
    eoff, eln = r_off.cpu().numpy().astype(np.uint64), r_len.cpu().numpy().astype(np.uint32)
    r["exact_dec_kms"] = st.stats()["last_decode_kernel_ms"]
    r["exact_gather"] = int(st.stats()["last_gather_queries"])
    r["exact_exp"] = int(eln.sum())
    if rc != px.PX_OK:
        raise SystemExit(f"config {cfg}: exact getitem rc={rc}")
    if checks:
        docs, doff = _docs_np(corpus)
        dbuf = torch.from_numpy(docs).to(dev)
        ne_ce = _count_ne(out, last["off"], last["len"], out2, eoff, eln, dev)
        ne_eo = _count_ne(out2, eoff, eln, dbuf, doff[:-1], np.diff(doff), dev)
        r["parity_counts"] = {"records": n, "compat_ne_exact": ne_ce, "exact_ne_original": ne_eo}
        if "reference_check" in r:
            rc_ = r["reference_check"]
            r["parity_counts"].update(compat_ne_reference=rc_["compat_ne_reference"],
                                      comp_ne_reference=rc_["comp_ne_reference"],
                                      placement_ne_reference=rc_["placement_ne_reference"],
                                      reference_fixture=rc_["fixture"])
        del dbuf
    del out2
    return r


def check_gathered(cfg, r, rps, world, records, sample=300):
    """Rank 0, outside the timed region: load every rank's gathered chunk blob (the last
    step's) into a fresh store and read back a sample of each rank's keys.  EXACT getitem
    must equal the record's escaped doc (regenerated from that rank's corpus part), and
    the compat getitem of rank 0's own records must equal its live store's."""
    import numpy as np
    import pixiu_amd as px
    from pixiu_amd import synth
    blobs = r["gathered"]
    # every blob into one store; with records_per_shard = 0 (one shard: the reference's single
    # instance) a store takes one blob only (px_load refuses a second into a non-empty single
    # shard), so each rank's blob gets a store of its own
    stores = [px.Store(records_per_shard=rps) for _ in (blobs if rps == 0 else [0])]
    try:
        for i, b in enumerate(blobs):
            st = stores[i if rps == 0 else 0]
            if b.is_cuda:
                st.load(b.data_ptr(), on_device=True, length=b.numel())
            else:
                st.load(np.ascontiguousarray(b.numpy()).tobytes())
        checked = exact_eq = 0
        gathered_q = 0
        for rk in range(world):
            st = stores[rk if rps == 0 else 0]
            cp = r["corpus"] if rk == 0 else synth.make(cfg, records, part=rk)
            rows = np.linspace(0, cp.n - 1, min(sample, cp.n)).astype(int).tolist()
            keys = [cp.key(i) for i in rows]
            got = st.get_batch(keys, px.EXACT)
            for i, g in zip(rows, got):
                v = cp.val(i)
                d = cp.key(i).replace(b"\xfb", b"\xfb\xfb") + b"\xfb\x00"
                if v:
                    d += v.replace(b"\xfb", b"\xfb\xfb") + b"\xfb\x02"
                exact_eq += g == d
                checked += 1
            if rk == 0:
                comp_loaded = st.get_batch(keys, px.COMPAT)
                gathered_q = int(st.stats()["last_gather_queries"])
                comp_live = r["st"].get_batch(keys, px.COMPAT)
                own_compat_eq = sum(x == y for x, y in zip(comp_loaded, comp_live))
        return {"ranks": world, "blob_bytes": [int(b.numel()) for b in blobs], "records_checked": checked,
                "exact_equal": exact_eq, "rank0_compat_equal_live": own_compat_eq,
                "rank0_gather_served": gathered_q, "records_per_rank_sampled": min(sample, r["n"]),
                "stores": len(stores)}
    finally:
        for st in stores:
            st.close()


def check_single(r0):
    """The single-instance leg against the reference (outside the timed region): every
    chunk's first record, record count and sha256 of its compressed bytes must equal
    tests/golden/c3_single.json, which the reference produced over the same corpus
    (tools/make_golden.py c3_single)."""
    import hashlib
    import pixiu_amd as px
    path = os.path.join(ROOT, "tests", "golden", "c3_single.json")
    if not os.path.exists(path):
        return None
    g = json.load(open(path))
    cp = r0["corpus"]
    if cp.n != g["n"]:
        return {"skipped": f"{cp.n} records, the golden holds {g['n']}"}
    res = r0["runs"][-1]["res"]
    comp = r0["st"].export(px.records_of(res))
    rows = {}
    for i, c in enumerate(res["chunk"].tolist()):
        rows.setdefault(c, []).append(i)
    got = [(v[0], len(v), hashlib.sha256(b"".join(comp[i] for i in v)).hexdigest()) for _, v in sorted(rows.items())]
    want = [(c["first"], c["records"], c["sha256"]) for c in g["chunks"]]
    return {"golden": "tests/golden/c3_single.json", "chunks": len(got), "golden_chunks": len(want),
            "chunks_equal": sum(x == y for x, y in zip(got, want)),
            "comp_bytes_equal": sum(map(len, comp)) == g["comp_bytes"]}


def _mmm(v, nd=3):
    """[min, median, max] of a list (rounded to nd places; nd = 0: ints)."""
    v = sorted(v)
    q = [v[0], v[len(v) // 2] if len(v) % 2 else (v[len(v) // 2 - 1] + v[len(v) // 2]) / 2, v[-1]]
    return [int(x) for x in q] if nd == 0 else [round(float(x), nd) for x in q]


def summarize(cfg, r, rps, world, a, pmc_path):
    """Aggregate one config's runs (whole-job volumes over ranks) into its report."""
    import torch
    import torch.distributed as dist
    runs = r["runs"]
    steps = len(runs)
    dev = r["out"].device if a.backend == "nccl" else torch.device("cpu")
    set_s = sum(x["set_s"] for x in runs)
    get_s = sum(x["get_s"] for x in runs)
    tot = torch.tensor([r["elapsed"], set_s, get_s, r["exact_s"]], dtype=torch.float64, device=dev)
    vol = torch.tensor([r["raw"], runs[-1]["comp"], runs[-1]["exp"], r["exact_exp"]], dtype=torch.float64, device=dev)
    if world > 1:  # slowest rank's clock, every rank's bytes
        dist.all_reduce(tot, op=dist.ReduceOp.MAX)
        dist.all_reduce(vol, op=dist.ReduceOp.SUM)
    elapsed, set_s, get_s, exact_s = (float(x) for x in tot.tolist())
    job_raw, job_comp, job_exp, job_exact = (float(x) for x in vol.tolist())
    set_MBps = job_raw * steps / set_s / 1e6
    get_MBps = job_exp * steps / get_s / 1e6
    comp, exp, raw = runs[-1]["comp"], runs[-1]["exp"], r["raw"]
    walk_kms = float(np.mean([x["walk_kms"] for x in runs]))
    emit_kms = float(np.mean([x["emit_kms"] for x in runs]))
    dec_kms = float(np.mean([x["dec_kms"] for x in runs]))
    # roofline: algorithmic bytes per launch / avg launch time, HIP events
    # on the context's stream (px_stats).  The setitem encode stage is the suffix-array
    # pipeline (px_psa.hip + px_sort.hip: hand-written segmented radix sorts and k_psa_* / k_dbl_* /
    # k_pool_*) for PSA shards and k_gst_encode for
    # walked ones; its span is timed as one stage.
    psa_shards = int(np.mean([x["psa"][1] for x in runs]))
    walk_shards = int(np.mean([x["psa"][2] for x in runs]))
    enc_name = ("k_psa (suffix-array pipeline)" if walk_shards == 0 else "k_psa + k_gst_encode") if psa_shards \
        else "k_gst_encode"
    set_gbps = (raw + comp) / (walk_kms * 1e-3) / 1e9   # encode stage: raw in + compressed out
    emit_gbps = (raw * 5 + comp) / (emit_kms * 1e-3) / 1e9
    dec_gbps = (comp + exp) / (dec_kms * 1e-3) / 1e9     # getitem stage: compressed in + expanded out
    dec_name = "k_gather + k_decode"
    dominant = enc_name if walk_kms >= dec_kms else dec_name
    ach = set_gbps if dominant == enc_name else dec_gbps
    traffic, tsrc = None, None
    if pmc_path and os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            w = pmc.get("workload", {})
            # only a profile of this exact workload counts (config, shard size, records)
            if w.get("config") == cfg and w.get("rps") == rps and w.get("records") == r["n"]:
                if dominant == dec_name:  # the stage's launches (one compat batch in the profile run)
                    tot_b = sum(v["hbm_bytes_per_launch"] * v["dispatches"] for k, v in pmc.items()
                                if isinstance(v, dict) and k in ("k_decode", "k_gather", "k_gather_tasks", "k_dk_lookup"))
                    traffic = tot_b or None
                else:  # every kernel of the encode stage, summed over its launches
                    tot_b = 0.0
                    for k, v in pmc.items():
                        # (tools/pmc_summary.py names rocPRIM's sort / scan kernels by their
                        # k_id_wrapper / k_scan_determinism template pieces)
                        if isinstance(v, dict) and (k.startswith(("k_psa", "k_seg", "k_cmp", "k_pool", "k_dbl", "k_big", "k_stat")) or "rocprim" in k
                                                    or k in ("k_gst_encode", "k_id_wrapper", "k_scan_determinism")):
                            tot_b += v["hbm_bytes_per_launch"] * v["dispatches"]
                    traffic = tot_b or None
                tsrc = f"{os.path.relpath(pmc_path, ROOT)} ({pmc.get('source', '')})"
        except Exception:
            traffic = None
    out = {
        "records_per_gpu": r["n"], "raw_bytes_per_gpu": raw, "records_per_shard": rps,
        "shards_per_gpu": int(r["st"].stats()["shards"]), "steps": steps,
        "value": round(set_MBps + get_MBps, 3), "unit": "MB/s",
        "ms_per_step": round(elapsed / steps * 1e3, 3),
        "setitem_MBps": round(set_MBps, 3), "getitem_MBps": round(get_MBps, 3),
        "getitem_exact_MBps": round(job_exact / exact_s / 1e6, 3) if exact_s else None,
        "compression_ratio": round(job_comp / job_raw, 4),
        "kernel_ms": {"encode_stage": round(walk_kms, 3), "k_gst_emit": round(emit_kms, 3),
                      "getitem_stage": round(dec_kms, 3), "getitem_stage_exact": round(r["exact_dec_kms"], 3)},
        "getitem_path": {"kernels": dec_name, "gather_queries": runs[-1]["spans"][0],
                         "exact_gather_queries": r.get("exact_gather", 0), "queries": r["n"],
                         "span_entries": runs[-1]["spans"][1],
                         "span_table_vs_comp": round(runs[-1]["spans"][1] * 8 / max(comp, 1), 4),
                         "span_build_ms": round(float(np.mean([x["spans"][2] for x in runs])), 3),
                         "device_bytes": runs[-1]["spans"][3]},
        "encode_stage": {"kernels": enc_name, "psa_shards": psa_shards, "walked_shards": walk_shards,
                         "psa_host_ms": round(float(np.mean([x["psa"][0] for x in runs])), 3),
                         "psa_split_ms": {"sort": round(float(np.mean([x["psa"][3] for x in runs])), 3),
                                          "links_lcp": round(float(np.mean([x["psa"][4] for x in runs])), 3),
                                          "messages": round(float(np.mean([x["psa"][5] for x in runs])), 3),
                                          "pool_emulation": round(float(np.mean([x["psa"][9] for x in runs])), 3)},
                         "doubling_steps": runs[-1]["psa"][6],
                         # last set batch: suffix-array rounds (chunk windows) and the rotations
                         # the MemPool emulation found; chunks = the store's chunk count
                         "psa_rounds": runs[-1]["psa"][7], "psa_rotations": runs[-1]["psa"][8],
                         "chunks": runs[-1]["psa"][10]},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(ach, 3), "peak": PEAK_HBM_GBPS,
                     "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBPS, 6), "traffic": traffic,
                     "traffic_source": tsrc,
                     # what the stage's kernels actually move (PMC bytes / stage time): how busy
                     # HBM is, next to the algorithmic rate above
                     "traffic_GBps": round(traffic / ((walk_kms if dominant == enc_name else dec_kms) * 1e-3) / 1e9, 1)
                     if traffic else None,
                     "traffic_per_algorithmic_byte": round(traffic / ((raw + comp) if dominant == enc_name
                                                                      else (comp + exp)), 1) if traffic else None},
        "roofline_kernels_GBps": {"encode_stage": round(set_gbps, 3), "k_gst_emit": round(emit_gbps, 3),
                                  "getitem_stage": round(dec_gbps, 3)},
        "gather_ms": round(float(np.mean([x["gather_ms"] for x in runs])), 3),
        # every timed step on this rank (min / median / max): set and get are the two timed
        # calls, reset the untimed px_reset before each set; device bytes after the set batch
        # (heap held + store arena), at its peak, and live
        "per_step": {k: _mmm([x[f] * 1e3 for x in runs]) for k, f in
                     (("set_ms", "set_s"), ("get_ms", "get_s"), ("reset_ms", "reset_s"))},
    }
    out["per_step"]["set_max_over_min"] = round(out["per_step"]["set_ms"][2] / max(out["per_step"]["set_ms"][0], 1e-9), 3)
    out["per_step"]["device_bytes_after_set"] = _mmm([x["spans"][3] for x in runs], 0)
    out["per_step"]["device_peak_bytes_in_set"] = _mmm([x["spans"][4] for x in runs], 0)
    out["per_step"]["device_live_bytes"] = runs[-1]["spans"][5]
    # the stored data's device bytes by structure (px_stats mem_*), and per raw byte
    mem = runs[-1].get("mem", {})
    if mem:
        raw = max(1, int(r["raw"]))
        out["per_step"]["device_mem_bytes"] = mem
        out["per_step"]["device_mem_per_raw_byte"] = {k: round(v / raw, 3) for k, v in mem.items()}
    if "parity_counts" in r:
        out["parity_counts"] = r["parity_counts"]
    return out


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # (ranks beyond the visible GPUs share them: tests on one GPU)
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    import pixiu_amd as px

    rps = a.rps if a.rps is not None else DEFAULT_RPS[a.config]
    r = run_config(a.config, a, rank, world, local, a.steps, a.warmup, rps, a.records, checks=not a.no_checks)
    main_sum = summarize(a.config, r, rps, world, a, a.pmc)
    per_config = {}
    extra = [int(c) for c in a.configs.split(",") if c.strip()] if a.configs else []
    for cfg in extra:
        if cfg == a.config:
            continue
        rc_ = run_config(cfg, a, rank, world, local, a.extra_steps, 1, DEFAULT_RPS[cfg], None,
                         checks=not a.no_checks)
        per_config[str(cfg)] = summarize(cfg, rc_, DEFAULT_RPS[cfg], world, a, a.pmc)
        rc_["st"].close()
        del rc_
        torch.cuda.empty_cache()

    if rank != 0:
        r["st"].close()
        if world > 1:
            dist.destroy_process_group()
        return
    gather_check = check_gathered(a.config, r, rps, world, a.records) if world > 1 else None

    st, corpus, runs = r["st"], r["corpus"], r["runs"]
    n, raw_bytes = r["n"], r["raw"]
    get_split = {"lookup_ms": float(np.mean([x["look_ms"] for x in runs])),
                 "call_ms": float(np.mean([x["call_ms"] for x in runs])),
                 "wall_ms": float(np.mean([x["get_s"] for x in runs])) * 1e3}
    line = {
        "metric": "MB/s ingested (setitem) + MB/s expanded (getitem), 10k×60KB corpus, 1/2/4/8 GPU",
        "value": main_sum["value"],
        "unit": "MB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": main_sum["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (pixiu_amd/synth.py, splitmix64 seed 0x5049585500+config, one part per rank)",
        "config": {"workload": (f"config{a.config}: {n} records x {raw_bytes // max(n, 1)} B per GPU "
                                f"(HTML-shape pages)") if a.config == 3 else f"config{a.config}: {n} records per GPU",
                   "records_per_gpu": n, "raw_bytes_per_gpu": raw_bytes, "records_per_shard": rps,
                   "shards_per_gpu": main_sum["shards_per_gpu"], "decode_mode": "compat",
                   "parallelism": f"dp{world} (record-range shards, no cross-GPU refs)"},
    }
    for k in ("setitem_MBps", "getitem_MBps", "getitem_exact_MBps", "compression_ratio", "kernel_ms",
              "encode_stage", "getitem_path", "roofline", "roofline_kernels_GBps", "gather_ms", "per_step",
              "parity_counts"):
        if k in main_sum:
            line[k] = main_sum[k]
    line["getitem_split_ms"] = {k: round(v, 3) for k, v in get_split.items()}
    if gather_check:
        line["gather_check"] = gather_check
        line["config"]["backend"] = a.backend
    line["ub_reads"] = int(st.stats()["ub_reads"])
    if per_config:
        line["per_config"] = per_config
    if not a.no_cpu and world == 1:
        cb = cpu_baseline(corpus, rps, a.cpu_seconds)
        # parity spot-check: the sampled shards' compressed bytes and compat getitems
        res = runs[-1]["res"]
        eq_c = eq_g = tot_c = 0
        for s0, sh, ks, outs in cb["shards"]:
            recs = px.records_of(res[s0:s0 + len(ks)])
            comp_gpu = st.export(recs)
            for j, (cg, o) in enumerate(zip(comp_gpu, outs)):
                tot_c += 1
                eq_c += cg == sh.comp(int(res["chunk"][s0 + j]), int(res["idx"][s0 + j]))
            got = st.get_batch(ks, px.COMPAT)
            eq_g += sum(g == o for g, o in zip(got, outs))
        line["cpu_baseline"] = {"value": round(cb["set_MBps"] + cb["get_MBps"], 4), "unit": "MB/s",
                                "set_MBps": round(cb["set_MBps"], 4), "get_MBps": round(cb["get_MBps"], 4),
                                "cores": 1, "kind": "port",
                                "sample": f"first {cb['records']} records ({cb['raw'] / 1e6:.1f} MB) of the same "
                                          f"corpus, same {rps}-record shards, oracle/pxo.cpp single-threaded, "
                                          f"{cb['seconds']:.1f} s"}
        cal = cpu_calibration()
        if cal:  # the reference's own speed relative to the port, timed on one shared host
            line["cpu_baseline"]["calibration"] = {
                "ref_over_port_set": round(cal["ref_over_port_set"], 4),
                "ref_over_port_get": round(cal["ref_over_port_get"], 4),
                "reference_equivalent_value": round(cb["set_MBps"] * cal["ref_over_port_set"]
                                                    + cb["get_MBps"] * cal["ref_over_port_get"], 4),
                "source": "profiles/cpu_calibration_r03.json (tools/calibrate_cpu.py: " + cal["workload"] + ")"}
        line["parity_sample"] = {"records": tot_c, "compressed_equal": eq_c, "getitem_equal": eq_g}
        mt = cpu_baseline_mt(corpus, rps, cb["set_MBps"], a.cpu_seconds / 2)
        line["cpu_baseline_mt"] = {"value": round(mt["set_MBps"] + mt["get_MBps"], 4), "unit": "MB/s",
                                   "set_MBps": round(mt["set_MBps"], 4), "get_MBps": round(mt["get_MBps"], 4),
                                   "cores": mt["threads"], "kind": "port",
                                   "sample": f"{mt['records']} records ({mt['raw'] / 1e6:.1f} MB), one oracle "
                                             f"instance per {rps}-record shard, {mt['threads']} threads, "
                                             f"{mt['seconds']:.1f} s"}
    if not a.no_pcie and world == 1:
        line["pcie_inclusive"] = pcie_leg(st, px, corpus, r["keys_host"], r["out_cap"])
    if not a.no_cliff and world == 1:
        line["walk_fallback"] = walk_cliff(local, corpus)
        line["one_record_per_call"] = small_batches(local)
    st.close()
    if not a.no_single and world == 1 and a.config == 3 and rps != 0:
        # the same corpus as ONE shard (records_per_shard = 0): the reference's single
        # instance, chunks rotated by its MemPool rule (suffix-array path with the pool
        # emulation), next to the oracle's single instance on the CPU
        torch.cuda.empty_cache()
        # (checks: every record's compat getitem, compressed bytes and slot against the
        # reference's own single instance, tests/golden/refdig_c3_r0.npz, outside the timing)
        r0 = run_config(a.config, a, rank, world, local, 1, 1, 0, None, checks=not a.no_checks)
        s0 = summarize(a.config, r0, 0, world, a, None)
        line["single_instance"] = {
            "records_per_shard": 0, "setitem_MBps": s0["setitem_MBps"], "getitem_MBps": s0["getitem_MBps"],
            "getitem_exact_MBps": s0.get("getitem_exact_MBps"), "compression_ratio": s0["compression_ratio"],
            "ms_per_step": s0.get("ms_per_step"), "chunks": s0["encode_stage"].get("chunks"),
            "psa_rounds": s0["encode_stage"].get("psa_rounds"),
            "encode_stage_ms": s0["kernel_ms"]["encode_stage"],
            "psa_split_ms": s0["encode_stage"].get("psa_split_ms"), "reference_check": check_single(r0)}
        if "reference_check" in r0:  # every record's compat getitem / bytes / slot vs the reference's digests
            line["single_instance"]["reference_digests"] = r0["reference_check"]
        if "parity_counts" in r0:
            line["single_instance"]["parity_counts"] = r0["parity_counts"]
        if not a.no_cpu:
            c0 = cpu_single_instance(corpus, a.cpu_seconds)
            line["single_instance"]["cpu_baseline"] = {
                "value": round(c0["set_MBps"] + c0["get_MBps"], 4), "unit": "MB/s",
                "set_MBps": round(c0["set_MBps"], 4), "get_MBps": round(c0["get_MBps"], 4), "cores": 1,
                "kind": "port", "sample": f"first {c0['records']} records ({c0['raw'] / 1e6:.2f} MB) into one "
                                          f"oracle instance, {c0['seconds']:.1f} s"}
            cal = cpu_calibration()
            if cal:
                line["single_instance"]["cpu_baseline"]["reference_equivalent_value"] = round(
                    c0["set_MBps"] * cal["ref_over_port_set"] + c0["get_MBps"] * cal["ref_over_port_get"], 4)
        r0["st"].close()
    # the headline's parts again at the end of the line (a reader of the line's tail sees them)
    line["headline_parts"] = {
        "setitem_MBps": line.get("setitem_MBps"), "getitem_MBps": line.get("getitem_MBps"),
        "setitem_MBps_pcie_inclusive": line.get("pcie_inclusive", {}).get("set_MBps"),
        "ms_per_step": line["ms_per_step"], "per_step": line.get("per_step")}
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
