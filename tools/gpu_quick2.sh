#!/bin/bash
# headline config only: a short bench with every record checked against the reference
# digests (PSA verbose), then the psa/pool/rounds tests, then a kernel trace of one step
#   gpurun -- 'bash tools/gpu_quick2.sh TAG'
set -o pipefail
TAG=${1:?tag}
O=gpurun_out
mkdir -p $O
if [ -n "$AB" ]; then  # an A/B leg first: the same bench under the environment in $AB
env $AB PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff \
  > $O/${TAG}_bench_ab.log 2>&1 || { echo AB BENCH FAILED; tail -5 $O/${TAG}_bench_ab.log; exit 1; }
grep "psa: N=" $O/${TAG}_bench_ab.log | tail -1
tail -1 $O/${TAG}_bench_ab.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('AB', l['value'], l['setitem_MBps'], l['kernel_ms'], l['encode_stage']['psa_split_ms'], l['parity_counts'])"
fi
PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff \
  > $O/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -5 $O/${TAG}_bench.log; exit 1; }
grep -E "psa: N=|retired" $O/${TAG}_bench.log | tail -2
tail -1 $O/${TAG}_bench.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['setitem_MBps'], l['kernel_ms'], l['encode_stage']['psa_split_ms'], l['parity_counts'])"
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_psa.py tests/test_gpu_pools.py tests/test_gpu_rounds.py tests/test_gpu_golden.py $EXTRA_TESTS \
  -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/${TAG}_tests.log | head; tail -5 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
fi
bash tools/gpu_trace.sh $TAG
