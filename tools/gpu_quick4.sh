#!/bin/bash
# tests first, then the headline bench, then kernel traces with and without $AB
set -o pipefail
TAG=${1:?tag}
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_psa.py tests/test_gpu_pools.py tests/test_gpu_rounds.py tests/test_gpu_golden.py $EXTRA_TESTS \
  -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/${TAG}_tests.log | head; tail -5 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
B="--steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff"
show() { grep -E "psa: N=|retired" $1 | tail -2; tail -1 $1 | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['setitem_MBps'], l['kernel_ms'], l['encode_stage']['psa_split_ms'], l['parity_counts'])"; }
PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py $B > $O/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -5 $O/${TAG}_bench.log; exit 1; }
show $O/${TAG}_bench.log
bash tools/gpu_trace.sh $TAG
if [ -n "$AB" ]; then env $AB bash tools/gpu_trace.sh ${TAG}_ab; fi
