#!/bin/bash
# big groups placed in one look-back pass (k_big_place): parity tests, kernel times, bench
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_psa.py tests/test_gpu_golden.py tests/test_gpu_refdig.py tests/test_gpu_pools.py -x -q --timeout 300 --timeout-method thread > $O/r05w_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05w_tests.log; exit 1; }
tail -1 $O/r05w_tests.log
B="--steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
timeout -k 10 200 python -u bench.py $B > $O/r05w_c3.log 2>&1 || { echo BENCH FAILED; tail -3 $O/r05w_c3.log; exit 1; }
tail -1 $O/r05w_c3.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['setitem_MBps'], l['getitem_MBps'], l['kernel_ms']['encode_stage'], l['getitem_path']['span_build_ms'], l['ms_per_step'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OLDPWD/$O/r05w_ks -o ks --output-format csv -- python3 $OLDPWD/bench.py --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --configs= --steps 1 --warmup 0 > $OLDPWD/$O/r05w_ks.log 2>&1 || { echo KS FAILED; tail -5 $OLDPWD/$O/r05w_ks.log; exit 1; }
cd $OLDPWD
F=$(find $O/r05w_ks -name '*kernel_stats.csv' | head -1)
cp $F $O/r05w_cfg3_kernel_stats.csv
find $O/r05w_ks -name '*kernel_trace.csv' -delete
python3 - $F <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:24]:
    n = re.sub(r'\(.*', '', r['Name'].replace('(anonymous namespace)::', '').replace('void ', ''))
    print(f"{n[:44]:44s} {r['Calls']:>5s} {float(r['TotalDurationNs'])/1e6:9.2f} ms")
print('total', round(sum(float(r['TotalDurationNs']) for r in rows)/1e6, 1))
PY
