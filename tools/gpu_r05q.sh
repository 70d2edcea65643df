#!/bin/bash
# full GPU suite, then the bench with its default legs (every record checked)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05q_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05q_gpu_tests.log; exit 1; }
tail -1 $O/r05q_gpu_tests.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > $O/r05q_bench.log 2>&1 || { echo BENCH FAILED; tail -5 $O/r05q_bench.log; exit 1; }
tail -1 $O/r05q_bench.log | python3 -c "
import json,sys; l=json.loads(sys.stdin.read())
print('value', l['value'], 'set', l['setitem_MBps'], 'get', l['getitem_MBps'], 'ms/step', l['ms_per_step'], 'span', l['getitem_path']['span_build_ms'])
for k,v in l.get('per_config',{}).items(): print(k, v['setitem_MBps'], v['getitem_MBps'], v.get('getitem_exact_MBps'), v['getitem_path']['span_build_ms'], v.get('parity_counts'))
print('single', l['single_instance']['setitem_MBps'], l['single_instance']['reference_digests'])
print(l['parity_counts'])"
