#!/bin/bash
# A/B of one environment switch on one config: VAR=0 vs VAR=1, bench lines into
# gpurun_out/ab_<VAR><0|1>_c<CFG>.log.   gpurun -- 'bash tools/ab_env.sh PX_PSA_SEGSORT 3'
set -o pipefail
VAR=${1:?var}
CFG=${2:-3}
mkdir -p gpurun_out
export TMPDIR=/tmp
for X in 0 1; do
  L=gpurun_out/ab_${VAR}${X}_c$CFG.log
  env $VAR=$X timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-pcie --no-checks --configs= --config $CFG \
    > $L 2>&1 || { echo "BENCH FAILED"; tail -20 $L; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$L') if l.startswith('{')][-1])
print('$VAR=$X', 'set', d['setitem_MBps'], 'get', d['getitem_MBps'], 'ratio', d['compression_ratio'], d['kernel_ms'], d['encode_stage']['psa_split_ms'])"
done
