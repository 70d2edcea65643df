"""Top kernels of a rocprofv3 kernel_stats.csv: python tools/ks_top.py FILE [N]"""
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)  # parameter list
    while "<" in name:  # template arguments
        new = re.sub(r"<[^<>]*>", "", name)
        if new == name:
            break
        name = new
    return name.replace("void ", "").strip()[-60:]


rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f'{short(r["Name"]):60s} {r["Calls"]:>6s} {float(r["TotalDurationNs"]) / 1e6:9.3f} ms {float(r["AverageNs"]) / 1e3:9.1f} us')
