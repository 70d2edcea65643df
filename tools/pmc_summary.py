"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs (separate passes) into the
per-kernel JSON bench.py reads for roofline.traffic.  Usage:
  python tools/pmc_summary.py FETCH.csv WRITE.csv OUT.json "source description" [CONFIG RPS RECORDS]
bench.py uses the file only when CONFIG / RPS / RECORDS match the run it reports.
"""
import collections, csv, json, re, sys

fetch_csv, write_csv, out, source = sys.argv[1:5]
workload = None
if len(sys.argv) >= 8:
    workload = {"config": int(sys.argv[5]), "rps": int(sys.argv[6]), "records": int(sys.argv[7])}


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        m = re.search(r"(k_[a-z_]+)", name)
        key = m.group(1) if m else name.split("(")[0]
        agg[key].append(float(r["Counter_Value"]) * 1024.0)  # KB counters
    return agg


f = per_kernel(fetch_csv, "FETCH_SIZE")
w = per_kernel(write_csv, "WRITE_SIZE")
res = {"source": source, "workload": workload,
       "formula": "hbm_bytes = (FETCH_SIZE + WRITE_SIZE) * 1024 (KB counters, separate passes); no gfx950 "
                  "wide-stream correction applied: these kernels issue scattered narrow accesses"}
for k in sorted(set(f) | set(w)):
    fv, wv = f.get(k, [0.0]), w.get(k, [0.0])
    n = max(len(fv), len(wv))
    fa, wa = sum(fv) / len(fv), sum(wv) / len(wv)
    res[k] = {"dispatches": n, "fetch_bytes_per_launch_avg": fa, "write_bytes_per_launch_avg": wa,
              "fetch_bytes_max_dispatch": max(fv), "write_bytes_max_dispatch": max(wv),
              "hbm_bytes_per_launch": fa + wa}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in res.items() if isinstance(v, dict)}, indent=1))
