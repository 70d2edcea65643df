set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/dec_tests.log; exit 1; }
tail -1 $O/dec_tests.log
for w in 0 5120 6144 10000; do timeout -k 10 120 python -u tools/decode_profile.py 3 10000 2 $w > $O/decprof_$w.log 2>&1 || { echo PROF FAILED; cat $O/decprof_$w.log; exit 1; }; head -3 $O/decprof_$w.log | tail -2; done
timeout -k 10 300 python -u bench.py --no-cpu > $O/dec_bench.log 2>&1 || exit 1
tail -1 $O/dec_bench.log
