"""Per-kernel SQ counter summary of a rocprofv3 counter_collection.csv (tools/gpu_run.sh sq):
waves, cycles per wave, the shares of cycles waiting / stalled on issue / issuing, and
instructions per wave.   python tools/sq_summary.py FILE"""
import collections
import csv
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_[a-z_0-9]+)", r["Kernel_Name"])
    k = m.group(1) if m else r["Kernel_Name"][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg, key=lambda k: -agg[k].get("SQ_WAVE_CYCLES", 0))[:20]:
    a = agg[k]
    w = max(a.get("SQ_WAVES", 1), 1)
    cyc = max(a.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{k:22s} waves {w:9.0f} cyc/wave {a.get('SQ_WAVE_CYCLES', 0) / w:10.0f} wait {a.get('SQ_WAIT_ANY', 0) / cyc:5.2f} "
          f"issue-stall {a.get('SQ_WAIT_INST_ANY', 0) / cyc:5.2f} active {a.get('SQ_ACTIVE_INST_ANY', 0) / cyc:5.2f} "
          f"valu/wave {a.get('SQ_INSTS_VALU', 0) / w:9.0f} salu/wave {a.get('SQ_INSTS_SALU', 0) / w:9.0f} "
          f"vmem_wr/wave {a.get('SQ_INSTS_VMEM_WR', 0) / w:8.0f}")
