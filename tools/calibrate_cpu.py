#!/usr/bin/env python3
"""Calibrate bench.py's cpu_baseline (the clean-room oracle, oracle/pxo.cpp) against the
reference compiled from its own sources (oracle/_ref/libpxref.so), in the build container:
the same config-3 shard (the first 139 pages, bench.py's records_per_shard), the same
single thread, setitem of every record in order into one fresh instance, then getitem of
a fixed sample of them.  Writes profiles/cpu_calibration_r03.json; bench.py carries the
factors beside its cpu_baseline (the GPU box has no reference to time).

    python tools/calibrate_cpu.py [records] [repeats]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from _oracle import Oracle, Reference, have_reference  # noqa: E402
from pixiu_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 139
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if not have_reference():
        raise SystemExit("no reference build (oracle/_ref): run in the build container")
    cp = synth.make(3, n)
    keys = [cp.key(i) for i in range(n)]
    vals = [cp.val(i) for i in range(n)]
    raw = sum(len(k) + len(v) for k, v in zip(keys, vals))
    sample = list(range(0, n, 7))
    orc = Oracle()
    ref = Reference()

    def run_oracle():
        sh = orc.new()
        t0 = time.perf_counter()
        for k, v in zip(keys, vals):
            if sh.set(k, v)[0] < 0:
                raise RuntimeError("oracle setitem failed")
        t1 = time.perf_counter()
        outs = [sh.get(keys[i]) for i in sample]
        return t1 - t0, time.perf_counter() - t1, outs

    def run_ref():
        ref.init()
        t0 = time.perf_counter()
        for k, v in zip(keys, vals):
            if ref.set(k, v) < 0:
                raise RuntimeError("reference setitem failed")
        t1 = time.perf_counter()
        outs = [ref.get(keys[i]) for i in sample]
        return t1 - t0, time.perf_counter() - t1, outs

    res = {}
    for name, fn in (("oracle", run_oracle), ("reference", run_ref)):
        best_s = best_g = float("inf")
        outs = None
        for _ in range(reps):
            s, g, outs = fn()
            best_s, best_g = min(best_s, s), min(best_g, g)
        exp = sum(len(o) for o in outs if o)
        res[name] = {"set_MBps": raw / best_s / 1e6, "get_MBps": exp / best_g / 1e6, "set_s": best_s, "get_s": best_g,
                     "outs": outs}
    same = res["oracle"].pop("outs") == res["reference"].pop("outs")
    out = {
        "workload": f"config3 first {n} pages ({raw / 1e6:.2f} MB), one instance, setitem in order, then getitem of "
                    f"every 7th record ({len(sample)}), best of {reps}, 1 thread",
        "host": os.uname().nodename, "cpu_threads": os.cpu_count(),
        "oracle": res["oracle"], "reference": res["reference"], "getitem_outputs_equal": same,
        # multiply the oracle's MB/s by these for the reference's speed on the same host
        "ref_over_port_set": res["reference"]["set_MBps"] / res["oracle"]["set_MBps"],
        "ref_over_port_get": res["reference"]["get_MBps"] / res["oracle"]["get_MBps"],
        "generator": "tools/calibrate_cpu.py",
    }
    path = os.path.join(ROOT, "profiles", "cpu_calibration_r03.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
