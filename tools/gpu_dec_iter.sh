#!/bin/bash
# Decode iteration: GPU tests, prof-build decode counters, bench line without the CPU leg.
#   gpurun -- 'bash tools/gpu_dec_iter.sh TAG'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=gpurun_out/${TAG}; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u tools/decode_profile.py 3 10000 2 > $O/decprof.log 2>&1 || { echo PROF FAILED; tail -20 $O/decprof.log; exit 1; }
cat $O/decprof.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
