#!/bin/bash
# compat span tables in pieces: spans tests, then configs 3 and 5 with every record checked,
# then getitem phase clocks on configs 4 and 2
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_spans.py -x -v --timeout 300 --timeout-method thread > $O/r05n_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05n_tests.log; exit 1; }
tail -1 $O/r05n_tests.log
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff"
for C in 3 5; do
  PX_SET_VERBOSE=1 timeout -k 10 300 python -u bench.py $B --config $C > $O/r05n_c$C.log 2>&1 || { echo BENCH $C FAILED; tail -3 $O/r05n_c$C.log; exit 1; }
  tail -1 $O/r05n_c$C.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print($C, l['setitem_MBps'], l['getitem_MBps'], l['getitem_exact_MBps'], l['getitem_path']['span_build_ms'], l['parity_counts'])"
done
PX_GET_VERBOSE=1 timeout -k 10 300 python -u tools/get_after_reset.py 8000 4 > $O/r05n_get4.log 2>&1 || { echo GET4 FAILED; tail -5 $O/r05n_get4.log; exit 1; }
PX_GET_VERBOSE=1 timeout -k 10 300 python -u tools/get_after_reset.py 2000 2 > $O/r05n_get2.log 2>&1 || { echo GET2 FAILED; tail -5 $O/r05n_get2.log; exit 1; }
grep "round 2" $O/r05n_get4.log $O/r05n_get2.log
