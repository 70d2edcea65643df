"""The dispatch sequence of a rocprofv3 kernel_trace.csv, compacted: one line per dispatch
of the kernels matching a pattern (default: the suffix-array pipeline's), in launch order,
with its duration -- e.g. the doubling's per-step costs.

    python tools/trace_seq.py TRACE.csv [REGEX] > out.txt
"""
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


pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_(psa|dbl|big|seg|scan|stat|pool)")
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows:
    nm = short(r["Kernel_Name"])
    if not pat.search(nm):
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e6:10.3f} ms  {(e - s) / 1e3:9.1f} us  {nm}")
