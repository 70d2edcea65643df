"""Print one kernel's counters from rocprofv3 --pmc CSVs (summed over its dispatches).
  python tools/pmc_kernel.py KERNEL_SUBSTRING a.csv [b.csv ...]"""
import collections, csv, sys

want = sys.argv[1]
tot = collections.OrderedDict()
dur = {}
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        if want not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        dur[(path, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in tot.items():
    print(f"{k:28s} {v:20.1f}")
if dur:
    print(f"{'avg dispatch ms':28s} {sum(dur.values()) / len(dur) / 1e6:20.3f}")
