#!/bin/bash
# links to text order: gathered (default) against scattered from suffix-array order
set -o pipefail
O=gpurun_out
mkdir -p $O
PX_LINKS_SCATTER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_psa.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/r05y_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05y_tests.log; exit 1; }
tail -1 $O/r05y_tests.log
B="--steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for V in 0 1 0 1; do
  PX_LINKS_SCATTER=$V timeout -k 10 200 python -u bench.py $B > $O/r05y_$V.log 2>&1 || { echo BENCH $V FAILED; tail -3 $O/r05y_$V.log; exit 1; }
  tail -1 $O/r05y_$V.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('scatter=$V', l['setitem_MBps'], l['kernel_ms']['encode_stage'], l['encode_stage']['psa_split_ms'], l['ms_per_step'])"
done
