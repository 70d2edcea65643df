#!/usr/bin/env python3
"""Kernel time summary from a rocprofv3 rocpd database (prof_results.db):
    python tools/prof_db.py gpurun_out/<dir>/prof_results.db [top] [--csv out.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 40
    con = sqlite3.connect(db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    q = (f"select s.kernel_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start) "
         f"from {kd} d join {ks} s on d.kernel_id = s.id group by s.kernel_name order by 3 desc")
    rows = con.execute(q).fetchall()
    tot = sum(r[2] for r in rows)
    for name, n, t, mn, mx in rows[:top]:
        short = name.split("(")[0].replace("px::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
        if "rocprim" in short:
            short = "rocprim:" + ("radix_sort" if "radix" in name else "scan" if "scan" in name else short[-60:])
        print(f"{t / 1e6:9.3f} ms {n:6d}  avg {t / n / 1e3:9.1f} us  {short[:90]}")
    print(f"{tot / 1e6:9.3f} ms total")
    if "--csv" in sys.argv:
        out = sys.argv[sys.argv.index("--csv") + 1]
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for name, n, t, mn, mx in rows:
                w.writerow([name, n, t, t / n, 100.0 * t / tot, mn, mx])


if __name__ == "__main__":
    main()
