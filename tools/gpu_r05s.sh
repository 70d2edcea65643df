#!/bin/bash
# decoder look-ahead: spans / refdig / parity tests, kernel times of a config-3 step, span
# piece sweep, config 4 set phases, decoder counters
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_spans.py tests/test_gpu_parity.py tests/test_gpu_refdig.py tests/test_gpu_toksegs.py -x -q --timeout 300 --timeout-method thread > $O/r05s_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05s_tests.log; exit 1; }
tail -1 $O/r05s_tests.log
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff"
for P in 1024 4096 16384; do
  PX_SPAN_PIECE=$P timeout -k 10 200 python -u bench.py $B --no-checks --no-exact --config 3 > $O/r05s_piece$P.log 2>&1 || { echo BENCH $P FAILED; tail -3 $O/r05s_piece$P.log; exit 1; }
  tail -1 $O/r05s_piece$P.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('piece', $P, l['setitem_MBps'], l['getitem_path']['span_build_ms'], l['ms_per_step'])"
done
PX_SET_VERBOSE=1 timeout -k 10 300 python -u bench.py $B --config 4 > $O/r05s_c4.log 2>&1 || { echo BENCH 4 FAILED; tail -3 $O/r05s_c4.log; exit 1; }
tail -1 $O/r05s_c4.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(4, l['setitem_MBps'], l['getitem_MBps'], l['getitem_path']['span_build_ms'], l['parity_counts'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OLDPWD/$O/r05s_ks -o ks --output-format csv -- python3 $OLDPWD/bench.py --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --configs= --steps 1 --warmup 0 > $OLDPWD/$O/r05s_ks.log 2>&1 || { echo KS FAILED; tail -5 $OLDPWD/$O/r05s_ks.log; exit 1; }
cd $OLDPWD
F=$(find $O/r05s_ks -name '*kernel_stats.csv' | head -1)
cp $F $O/r05s_cfg3_kernel_stats.csv
python3 - $F <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:28]:
    n = re.sub(r'\(.*', '', r['Name'].replace('(anonymous namespace)::', '').replace('void ', ''))
    print(f"{n[:44]:44s} {r['Calls']:>5s} {float(r['TotalDurationNs'])/1e6:9.2f} ms")
PY
timeout -k 10 150 python -u tools/decode_profile.py 3 10000 139 > $O/r05s_decprof.log 2>&1 || { echo DECPROF FAILED; tail -5 $O/r05s_decprof.log; exit 1; }
head -32 $O/r05s_decprof.log | tail -30
