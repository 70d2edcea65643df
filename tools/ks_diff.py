"""Per-kernel totals of rocprofv3 kernel_stats.csv files side by side:
python tools/ks_diff.py A.csv B.csv [C.csv ...]"""
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    while "<" in name:
        new = re.sub(r"<[^<>]*>", "", name)
        if new == name:
            break
        name = new
    return name.replace("void ", "").strip()[-50:]


cols = []
for f in sys.argv[1:]:
    d = {}
    for r in csv.DictReader(open(f)):
        k = short(r["Name"])
        d[k] = d.get(k, 0.0) + float(r["TotalDurationNs"]) / 1e6
    cols.append(d)
keys = sorted(set().union(*cols), key=lambda k: -max(c.get(k, 0.0) for c in cols))
print(f"{'total':50s} " + " ".join(f"{sum(c.values()):9.2f}" for c in cols))
for k in keys[:40]:
    print(f"{k:50s} " + " ".join(f"{c.get(k, 0.0):9.2f}" for c in cols))
