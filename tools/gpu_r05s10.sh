#!/bin/bash
# exact span tables' piece size (PX_SPAN_XPIECE; compat pieces stay 4 KB), with the phase clock
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for V in 1024 2048 4096 1024 2048 4096; do
  PX_SET_VERBOSE=1 PX_SPAN_XPIECE=$V timeout -k 10 200 python -u bench.py $B > $O/r05s10_$V.log 2>&1 || { echo BENCH $V FAILED; tail -3 $O/r05s10_$V.log; exit 1; }
  X=$(grep -A8 "build_spans (exact)" $O/r05s10_$V.log | grep "total" | tail -1)
  tail -1 $O/r05s10_$V.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('xpiece $V', l['setitem_MBps'], l['getitem_path']['span_build_ms'], '$X', l['ms_per_step'])"
done
timeout -k 10 300 env PX_SPAN_XPIECE=1024 python -u -m pytest tests/test_gpu_spans.py -x -q --timeout 200 --timeout-method thread > $O/r05s10_tests.log 2>&1 || { echo TESTS FAILED; tail -20 $O/r05s10_tests.log; exit 1; }
tail -1 $O/r05s10_tests.log
