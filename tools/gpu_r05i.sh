#!/bin/bash
# single instance with / without retirement; getitem phase clocks on configs 3 and 4
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-exact --no-checks"
for R in 0 1; do
  PX_PSA_RETIRE=$R PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py $B --rps 0 > $O/r05i_single_ret$R.log 2>&1 || { echo SINGLE $R FAILED; tail -5 $O/r05i_single_ret$R.log; exit 1; }
  tail -1 $O/r05i_single_ret$R.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('ret', $R, l['setitem_MBps'], l['kernel_ms'], l['encode_stage']['psa_split_ms'])"
done
PX_GET_VERBOSE=1 timeout -k 10 300 python -u bench.py $B > $O/r05i_get3.log 2>&1 || { echo GET3 FAILED; exit 1; }
tail -1 $O/r05i_get3.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('cfg3', l['getitem_MBps'], l['getitem_split_ms'], l['per_step'])"
PX_GET_VERBOSE=1 timeout -k 10 300 python -u bench.py $B --config 4 > $O/r05i_get4.log 2>&1 || { echo GET4 FAILED; exit 1; }
tail -1 $O/r05i_get4.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('cfg4', l['getitem_MBps'], l['getitem_split_ms'], l['per_step'])"
