"""Round timeline of a single-instance kernel trace (rocprofv3 --kernel-trace CSV, .gz ok):
per suffix-array round (a round starts at k_psa_gather) its wall time, the time kernels
were busy, the idle gaps, and the busiest kernels.   python tools/round_timeline.py TRACE"""
import collections
import csv
import gzip
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
    return name.replace("void ", "").split("::")[-1].strip()


path = sys.argv[1]
f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
rows = list(csv.DictReader(f))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
rounds, cur = [], None
for s, e, n in ev:
    if n == "k_psa_gather":
        cur = []
        rounds.append(cur)
    if cur is not None:
        cur.append((s, e, n))
print(f"{len(ev)} dispatches, {len(rounds)} rounds")
agg = collections.Counter()
tot_wall = tot_busy = 0
for i, r in enumerate(rounds):
    # a round ends where the next begins; trailing non-PSA work (emit, spans) is cut at the
    # last k_pool_scan / k_psa_place
    last = max(j for j, x in enumerate(r) if x[2].startswith(("k_pool", "k_psa")))
    r = r[:last + 1]
    wall = r[-1][1] - r[0][0]
    busy, end = 0, r[0][0]
    for s, e, n in r:
        busy += max(0, e - max(s, end))
        end = max(end, e)
        agg[n] += e - s
    tot_wall += wall
    tot_busy += busy
    if i < 3 or i == len(rounds) - 1:
        per = collections.Counter()
        for s, e, n in r:
            per[n] += e - s
        top = ", ".join(f"{n} {t / 1e6:.2f}" for n, t in per.most_common(8))
        print(f"round {i}: wall {wall / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, {len(r)} kernels; {top}")
print(f"all rounds: wall {tot_wall / 1e6:.1f} ms, busy {tot_busy / 1e6:.1f} ms, idle {(tot_wall - tot_busy) / 1e6:.1f} ms")
for n, t in agg.most_common(20):
    print(f"  {n:28s} {t / 1e6:8.2f} ms")
