"""Print the headline fields of a bench.py log's JSON line: python tools/line_summary.py LOG"""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
keys = ["value", "setitem_MBps", "getitem_MBps", "getitem_exact_MBps", "compression_ratio", "kernel_ms",
        "getitem_split_ms", "parity_counts"]
print({k: d.get(k) for k in keys})
print("encode:", {k: d["encode_stage"].get(k) for k in ("psa_split_ms", "psa_rounds", "doubling_steps")})
