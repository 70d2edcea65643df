#!/bin/bash
# decoder lane frames spilled to scratch past the LDS stack: parity, depth flags, A/B s0/s24/s48
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_spans.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_refdig.py -x -q --timeout 300 --timeout-method thread > $O/r05s2_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/r05s2_tests.log; exit 1; }
tail -1 $O/r05s2_tests.log
timeout -k 10 120 python -u tools/decode_profile.py 3 10000 139 > $O/r05s2_decprof.log 2>&1 || { echo DECPROF FAILED; tail -5 $O/r05s2_decprof.log; exit 1; }
head -30 $O/r05s2_decprof.log
B="--steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for V in s0 s24 s48 s0 s24; do
  L=$PWD/pixiu_amd/libpixiu_amd.so; [ $V != s24 ] && L=$PWD/pixiu_amd/libpixiu_amd_$V.so
  PIXIU_AMD_LIB=$L timeout -k 10 200 python -u bench.py $B > $O/r05s2_$V.log 2>&1 || { echo BENCH $V FAILED; tail -3 $O/r05s2_$V.log; exit 1; }
  tail -1 $O/r05s2_$V.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('$V', l['setitem_MBps'], l['getitem_path']['span_build_ms'], l['kernel_ms']['encode_stage'], l['ms_per_step'])"
done
