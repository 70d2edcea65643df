#!/bin/bash
# GPU box: kernel-trace stats of one config-3 bench step at records_per_shard $1.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${1:-64}
TAG=${2:-psaprof}
PX_PSA_VERBOSE=1 timeout -k 10 300 python3 bench.py --rps $R --configs= --no-cpu --no-pcie --no-checks --steps 1 --warmup 0 2>&1 | grep -E "^psa:" || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_ks -o ks --output-format csv \
  -- python3 bench.py --rps $R --configs= --no-cpu --no-pcie --no-checks --steps 1 --warmup 1 > gpurun_out/${TAG}.log 2>&1 || { echo FAILED; tail -20 gpurun_out/${TAG}.log; exit 1; }
grep '^{' gpurun_out/${TAG}.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['setitem_MBps'], d['kernel_ms'], d['encode_stage'])"
python3 - <<PY
import csv
rows = list(csv.DictReader(open("gpurun_out/${TAG}_ks/ks_kernel_stats.csv")))
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:10.3f} ms  {int(r['Calls']):5d}  {r['Name'][:110]}")
PY
