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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--records", type=int, default=None, help="records per rank (default: full config)")
    ap.add_argument("--rps", type=int, default=2, help="records per shard (independent GST); DESIGN.md §6 has the ratio curve")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_r01h.json"))
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


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import pixiu_amd as px
    from pixiu_amd import synth
    from pixiu_amd.dist import gather_blobs

    corpus = synth.make(a.config, a.records, part=rank) if a.config == 3 else synth.make(a.config, a.records)
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
    gather_buf = None

    st = px.Store(records_per_shard=a.rps, device=local)

    def step():
        st.reset()
        t0 = time.perf_counter()
        res = st.set_batch_device(n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=False)
        t1 = time.perf_counter()
        sst = st.stats()
        set_kms, walk_kms, emit_kms = sst["last_set_kernel_ms"], sst["last_walk_kernel_ms"], sst["last_emit_kernel_ms"]
        rc, off, ln, sts, need = st.get_batch_device(keys_host, out.data_ptr(), out_cap, px.COMPAT)
        t2 = time.perf_counter()
        gst = st.stats()
        dec_kms, look_ms, call_ms = gst["last_decode_kernel_ms"], gst["last_get_lookup_ms"], gst["last_get_call_ms"]
        g_ms = 0.0
        if world > 1:  # gather every rank's compressed blob to rank 0 (RCCL over xGMI)
            nonlocal gather_buf
            tg = time.perf_counter()
            nb = st.last_store_bytes()
            if gather_buf is None or gather_buf.numel() < nb:
                gather_buf = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            st.copy_last_store(gather_buf.data_ptr(), gather_buf.numel(), True)
            gather_blobs(gather_buf[:nb], dst=0)
            torch.cuda.synchronize()
            g_ms = (time.perf_counter() - tg) * 1e3
        if rc != px.PX_OK or int(res["status"].max()) != 0:
            bad = int((res["status"] != 0).sum())
            raise SystemExit(f"rank {rank}: setitem failures={bad} getitem rc={rc}")
        # setitem's one exchange (the compressed-blob gather to rank 0) counts as setitem time
        return {"set_s": t1 - t0 + g_ms * 1e-3, "get_s": t2 - t1, "set_kms": set_kms, "walk_kms": walk_kms,
                "emit_kms": emit_kms,
                "dec_kms": dec_kms, "gather_ms": g_ms, "look_ms": look_ms, "call_ms": call_ms,
                "comp": int(res["comp_len"].sum()), "exp": int(ln.sum()), "res": res}

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    T0 = time.perf_counter()
    runs = [step() for _ in range(a.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    T1 = time.perf_counter()

    elapsed = T1 - T0
    set_s = sum(r["set_s"] for r in runs)
    get_s = sum(r["get_s"] for r in runs)
    tot = torch.tensor([elapsed, set_s, get_s], dtype=torch.float64, device=dev)
    vol = torch.tensor([raw_bytes, runs[-1]["comp"], runs[-1]["exp"]], dtype=torch.float64, device=dev)
    if world > 1:  # slowest rank's clock, every rank's bytes
        dist.all_reduce(tot, op=dist.ReduceOp.MAX)
        dist.all_reduce(vol, op=dist.ReduceOp.SUM)
    elapsed, set_s, get_s = (float(x) for x in tot.tolist())
    job_raw, job_comp, job_exp = (float(x) for x in vol.tolist())
    comp = runs[-1]["comp"]
    exp = runs[-1]["exp"]
    set_kms = float(np.mean([r["set_kms"] for r in runs]))
    walk_kms = float(np.mean([r["walk_kms"] for r in runs]))
    emit_kms = float(np.mean([r["emit_kms"] for r in runs]))
    dec_kms = float(np.mean([r["dec_kms"] for r in runs]))
    # getitem wall time split: host key lookups, the rest of the C call (query upload,
    # k_decode, length/status download), and the Python binding around it
    get_split = {"lookup_ms": float(np.mean([r["look_ms"] for r in runs])),
                 "call_ms": float(np.mean([r["call_ms"] for r in runs])),
                 "wall_ms": float(np.mean([r["get_s"] for r in runs])) * 1e3}
    stats = st.stats()

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    K = a.steps
    set_MBps = job_raw * K / set_s / 1e6
    get_MBps = job_exp * K / get_s / 1e6
    # roofline: algorithmic bytes per launch / avg launch time
    set_alg = raw_bytes + comp                  # raw in + compressed out
    dec_alg = comp + exp                        # compressed in + expanded out
    # the setitem path is two launches: k_gst_encode (suffix-tree walk -> encoder
    # messages) and k_gst_emit (lane-parallel stream encoder); the walk bounds it
    set_gbps = set_alg / (walk_kms * 1e-3) / 1e9
    emit_alg = raw_bytes * 5 + comp             # doc bytes + 4-byte messages in, compressed out
    emit_gbps = emit_alg / (emit_kms * 1e-3) / 1e9
    dec_gbps = dec_alg / (dec_kms * 1e-3) / 1e9
    pmc = {}
    if os.path.exists(a.pmc):
        try:
            pmc = json.load(open(a.pmc))
        except Exception:
            pmc = {}
    dominant = "k_gst_encode" if walk_kms >= dec_kms else "k_decode"
    if dominant == "k_gst_encode":
        ach, tr = set_gbps, pmc.get("k_gst_encode", {}).get("hbm_bytes_per_launch")
    else:
        ach, tr = dec_gbps, pmc.get("k_decode", {}).get("hbm_bytes_per_launch")
    line = {
        "metric": "MB/s ingested (setitem) + MB/s expanded (getitem), 10k×60KB corpus, 1/2/4/8 GPU",
        "value": round(set_MBps + get_MBps, 3),
        "unit": "MB/s",
        "n_gpus": world,
        "steps": K,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (pixiu_amd/synth.py, splitmix64 seed 0x5049585500+config)",
        "config": {"workload": f"config{a.config}: {n} records x {raw_bytes // max(n, 1)} B per GPU "
                               f"(HTML-shape pages)" if a.config == 3 else f"config{a.config}: {n} records per GPU",
                   "records_per_gpu": n, "raw_bytes_per_gpu": raw_bytes, "records_per_shard": a.rps,
                   "shards_per_gpu": int(stats["shards"]), "decode_mode": "compat",
                   "parallelism": f"dp{world} (record-range shards, no cross-GPU refs)"},
        "setitem_MBps": round(set_MBps, 3),
        "getitem_MBps": round(get_MBps, 3),
        "compression_ratio": round(job_comp / job_raw, 4),
        "kernel_ms": {"k_gst_encode": round(walk_kms, 3), "k_gst_emit": round(emit_kms, 3), "k_decode": round(dec_kms, 3)},
        "getitem_split_ms": {k: round(v, 3) for k, v in get_split.items()},
        "gather_ms": round(float(np.mean([r["gather_ms"] for r in runs])), 3),
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(ach, 3), "peak": PEAK_HBM_GBPS,
                     "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBPS, 6), "traffic": tr},
        "roofline_other": {"kernel": "k_decode" if dominant == "k_gst_encode" else "k_gst_encode",
                           "achieved": round(dec_gbps if dominant == "k_gst_encode" else set_gbps, 3),
                           "unit": "GB/s"},
        "roofline_emit": {"kernel": "k_gst_emit", "achieved": round(emit_gbps, 3), "unit": "GB/s",
                          "frac": round(emit_gbps / PEAK_HBM_GBPS, 6)},
        "ub_reads": int(stats["ub_reads"]),
    }
    if not a.no_cpu and world == 1:
        cb = cpu_baseline(corpus, a.rps, a.cpu_seconds)
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
                                          f"corpus, same {a.rps}-record shards, oracle/pxo.cpp single-threaded, "
                                          f"{cb['seconds']:.1f} s"}
        line["parity_sample"] = {"records": tot_c, "compressed_equal": eq_c, "getitem_equal": eq_g}
        mt = cpu_baseline_mt(corpus, a.rps, cb["set_MBps"], a.cpu_seconds / 2)
        line["cpu_baseline_mt"] = {"value": round(mt["set_MBps"] + mt["get_MBps"], 4), "unit": "MB/s",
                                   "set_MBps": round(mt["set_MBps"], 4), "get_MBps": round(mt["get_MBps"], 4),
                                   "cores": mt["threads"], "kind": "port",
                                   "sample": f"{mt['records']} records ({mt['raw'] / 1e6:.1f} MB), one oracle "
                                             f"instance per {a.rps}-record shard, {mt['threads']} threads, "
                                             f"{mt['seconds']:.1f} s"}
    if not a.no_pcie and world == 1:
        line["pcie_inclusive"] = pcie_leg(st, px, corpus, keys_host, out_cap)
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
