#!/bin/bash
# round-5 final, part 1 (log prefix $P, default r05z): the whole GPU suite, smoke(), and the bench with the driver's flags
set -o pipefail
O=gpurun_out
P=${P:-r05z}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${P}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/${P}_gpu_tests.log; exit 1; }
tail -1 $O/${P}_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${P}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -10 $O/${P}_smoke.log; exit 1; }
tail -1 $O/${P}_smoke.log
timeout -k 10 420 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/${P}_bench.log 2>&1 || { echo BENCH FAILED; tail -5 $O/${P}_bench.log; exit 1; }
tail -1 $O/${P}_bench.log | python3 -c "
import json,sys; l=json.loads(sys.stdin.read())
print('value', l['value'], 'set', l['setitem_MBps'], 'get', l['getitem_MBps'], 'ms/step', l['ms_per_step'], 'max/min', l['per_step']['set_max_over_min'])
print('roofline', l['roofline'])
for k,v in l.get('per_config',{}).items(): print(k, v['setitem_MBps'], v['getitem_MBps'], v.get('parity_counts'))
print('single', l['single_instance']['setitem_MBps'], l['single_instance']['reference_digests'])
print('one_record_per_call', l['one_record_per_call']['MBps'], 'walk', l['walk_fallback']['walk_over_psa_time'], 'pcie', l['pcie_inclusive'])
print(l['parity_counts'])"
