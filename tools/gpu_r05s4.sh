#!/bin/bash
# deep reference chains: the new span test, and the decoder counters of its set batch
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_spans.py -x -v --timeout 200 --timeout-method thread > $O/r05s4_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05s4_tests.log; exit 1; }
tail -3 $O/r05s4_tests.log
for A in "96 48" "160 160"; do
  timeout -k 10 120 python -u tools/chain_profile.py $A > $O/r05s4_chain.log 2>&1 || { echo CHAIN FAILED; tail -5 $O/r05s4_chain.log; exit 1; }
  cat $O/r05s4_chain.log
done
timeout -k 10 120 python -u tools/decode_profile.py 3 2000 139 > $O/r05s4_decprof.log 2>&1 || { echo DECPROF FAILED; tail -5 $O/r05s4_decprof.log; exit 1; }
grep -E "d_spill|df_depth|d_serial" $O/r05s4_decprof.log
