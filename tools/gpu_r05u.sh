#!/bin/bash
# working set of the suffix-array pass: positions per round (PX_PSA_ROUND_MAX) against the
# encode stage (a round's random reads and writes stay inside its own arrays)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_spans.py tests/test_gpu_toksegs.py tests/test_gpu_golden.py tests/test_gpu_refdig.py tests/test_gpu_psa.py -x -q --timeout 300 --timeout-method thread > $O/r05u_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05u_tests.log; exit 1; }
tail -1 $O/r05u_tests.log
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for M in 0 300000000 150000000 75000000 40000000 20000000; do
  if [ $M = 0 ]; then E=""; else E="PX_PSA_ROUND_MAX=$M"; fi
  env $E timeout -k 10 200 python -u bench.py $B > $O/r05u_$M.log 2>&1 || { echo BENCH $M FAILED; tail -3 $O/r05u_$M.log; exit 1; }
  tail -1 $O/r05u_$M.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); e=l['encode_stage']; print('$M', l['setitem_MBps'], l['kernel_ms']['encode_stage'], e['psa_rounds'], e['psa_split_ms'], l['ms_per_step'])"
done
