#!/bin/bash
# full GPU suite, the bench's default legs (every record checked), the decoder's counters of a
# config-3 set batch, SQ counters of one bench step
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 560 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05r_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05r_gpu_tests.log; exit 1; }
tail -1 $O/r05r_gpu_tests.log
timeout -k 10 330 python -u bench.py --steps 3 --warmup 1 > $O/r05r_bench.log 2>&1 || { echo BENCH FAILED; tail -5 $O/r05r_bench.log; exit 1; }
tail -1 $O/r05r_bench.log | python3 -c "
import json,sys; l=json.loads(sys.stdin.read())
print('value', l['value'], 'set', l['setitem_MBps'], 'get', l['getitem_MBps'], 'ms/step', l['ms_per_step'], 'span', l['getitem_path']['span_build_ms'], 'enc', l['kernel_ms']['encode_stage'])
for k,v in l.get('per_config',{}).items(): print(k, v['setitem_MBps'], v['getitem_MBps'], v.get('getitem_exact_MBps'), v['getitem_path']['span_build_ms'], v.get('parity_counts'))
print('single', l['single_instance']['setitem_MBps'], l['single_instance']['reference_digests'])
print(l['parity_counts'])"
timeout -k 10 120 python -u tools/decode_profile.py 3 10000 139 > $O/r05r_decprof.log 2>&1 || { echo DECPROF FAILED; tail -5 $O/r05r_decprof.log; exit 1; }
head -30 $O/r05r_decprof.log
bash tools/gpu_sq.sh r05r
