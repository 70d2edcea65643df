#!/bin/bash
# One GPU call: (optional) GPU test suite, the default bench line, a rocprofv3
# kernel-trace summary of the headline config, and the two PMC passes (FETCH_SIZE,
# WRITE_SIZE) folded into gpurun_out/<tag>_pmc.json for the same workload.
#   gpurun --timeout 1200 -- 'bash tools/gpu_profile.sh r02a'
# Outputs land in gpurun_out/<tag>_*; copy the ones to keep into profiles/.
set -o pipefail
TAG=${1:?tag}
SKIP_TESTS=${SKIP_TESTS:-0}
CFG=${CFG:-3}
RPS=${RPS:-}
BENCH_ARGS=${BENCH_ARGS:-}
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
  tail -2 $O/${TAG}_gpu_tests.log
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > $O/${TAG}_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/${TAG}_bench.log; exit 1; }
  tail -1 $O/${TAG}_bench.log
fi
# a counter-collection pass prints nothing for minutes: a ticker keeps the run visibly alive
( while sleep 50; do echo "tick $(date +%T)" >> $O/${TAG}_ticks.log; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
PROF="bench.py --steps 1 --warmup 0 --no-cpu --no-pcie --no-cliff --no-checks --no-exact --no-single --configs= --config $CFG ${RPS:+--rps $RPS}"
if [ "${SKIP_KS:-0}" != 1 ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_ks -o ks --output-format csv \
  -- python3 $PROF > $O/${TAG}_ks.log 2>&1 || { echo "KTRACE FAILED"; tail -20 $O/${TAG}_ks.log; exit 1; }
fi
if [ "${SKIP_PMC:-0}" = 1 ]; then find $O/${TAG}_ks -name '*kernel_trace.csv' -delete 2>/dev/null; echo DONE; exit 0; fi
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/${TAG}_pmc_f -o f --output-format csv \
  -- python3 $PROF > $O/${TAG}_pmc_f.log 2>&1 || { echo "PMC FETCH FAILED"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/${TAG}_pmc_w -o w --output-format csv \
  -- python3 $PROF > $O/${TAG}_pmc_w.log 2>&1 || { echo "PMC WRITE FAILED"; exit 1; }
F=$(find $O/${TAG}_pmc_f -name '*counter_collection.csv' | head -1)
W=$(find $O/${TAG}_pmc_w -name '*counter_collection.csv' | head -1)
REC=$(python3 -c "from pixiu_amd import synth; print(synth.FULL_SIZES[$CFG])")
RPSV=${RPS:-$(python3 -c "import bench; print(bench.DEFAULT_RPS[$CFG])")}
python3 tools/pmc_summary.py "$F" "$W" $O/${TAG}_pmc.json "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), python3 $PROF ($TAG)" $CFG $RPSV $REC > /dev/null
find $O/${TAG}_ks -name '*kernel_stats.csv' 2>/dev/null | sort
# the per-dispatch traces are large (gpurun copies back at most 64 MiB): keep the summaries
find $O/${TAG}_ks $O/${TAG}_pmc_f $O/${TAG}_pmc_w -name '*kernel_trace.csv' -delete 2>/dev/null
gzip -f $O/${TAG}_pmc_f/*counter_collection.csv $O/${TAG}_pmc_w/*counter_collection.csv 2>/dev/null
echo DONE
