#!/bin/bash
# exact-table split with whole-record redo: config 5 (length-251 aliases) and 3, every record checked
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff"
for C in 5 3; do
  PX_SET_VERBOSE=1 timeout -k 10 300 python -u bench.py $B --config $C > $O/r05m_c$C.log 2>&1 || { echo BENCH $C FAILED; tail -3 $O/r05m_c$C.log; exit 1; }
  tail -1 $O/r05m_c$C.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print($C, l['setitem_MBps'], l['getitem_MBps'], l['getitem_exact_MBps'], l['getitem_path']['span_build_ms'], l['parity_counts'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_spans.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/r05m_tests.log 2>&1 || { echo TESTS FAILED; tail -5 $O/r05m_tests.log; exit 1; }
tail -1 $O/r05m_tests.log
