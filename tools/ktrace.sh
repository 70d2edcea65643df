#!/bin/bash
# kernel-trace summary of one bench step: gpurun -- 'bash tools/ktrace.sh TAG [bench args]'
TAG=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_ks -o ks --output-format csv \
  -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-pcie --no-checks --no-exact --configs= "$@" > gpurun_out/${TAG}_ks.log 2>&1 || { echo KTRACE FAILED; tail -20 gpurun_out/${TAG}_ks.log; exit 1; }
F=$(find gpurun_out/${TAG}_ks -name '*kernel_stats.csv' | head -1)
python3 - "$F" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {int(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}%")
PY
