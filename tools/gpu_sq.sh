#!/bin/bash
# SQ counters (one pass, 8 SQ counters) of one config-3 bench step: where the serial
# per-record kernels (k_tokenize, k_decode_addr, k_gst_emit) spend their wave cycles
#   gpurun -- 'bash tools/gpu_sq.sh r05m'
set -o pipefail
TAG=${1:?tag}
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR \
  -d $O/${TAG}_sq -o sq --output-format csv -- python3 $R/bench.py --no-cpu --no-single --no-pcie --no-cliff --no-exact --no-checks \
  --configs= --steps 1 --warmup 0 > $O/${TAG}_sq.log 2>&1 || { echo SQ FAILED; tail -5 $O/${TAG}_sq.log; exit 1; }
F=$(find $O/${TAG}_sq -name '*counter_collection.csv' | head -1)
python3 - "$F" > $O/${TAG}_sq_summary.txt <<'PY'
import csv, collections, re, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_[a-z_0-9]+)", r["Kernel_Name"])
    k = m.group(1) if m else r["Kernel_Name"][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg, key=lambda k: -agg[k].get("SQ_WAVE_CYCLES", 0))[:20]:
    a = agg[k]
    w = max(a.get("SQ_WAVES", 1), 1)
    print(f"{k:22s} waves {w:9.0f} cyc/wave {a.get('SQ_WAVE_CYCLES',0)/w:10.0f} wait {a.get('SQ_WAIT_ANY',0)/max(a.get('SQ_WAVE_CYCLES',1),1):5.2f} "
          f"issue-stall {a.get('SQ_WAIT_INST_ANY',0)/max(a.get('SQ_WAVE_CYCLES',1),1):5.2f} active {a.get('SQ_ACTIVE_INST_ANY',0)/max(a.get('SQ_WAVE_CYCLES',1),1):5.2f} "
          f"valu/wave {a.get('SQ_INSTS_VALU',0)/w:9.0f} salu/wave {a.get('SQ_INSTS_SALU',0)/w:9.0f} vmem_wr/wave {a.get('SQ_INSTS_VMEM_WR',0)/w:8.0f}")
PY
gzip -f $F
cat $O/${TAG}_sq_summary.txt
