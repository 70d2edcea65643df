#!/bin/bash
# The one GPU runner: a tag and a list of steps, run in order, each under its own time limit;
# the first failing step ends the call (nothing more touches the GPU after a fault).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_run.sh r06a tests bench ktrace pmc'
#
# steps (ARGS after ':' replace the step's defaults; spaces inside ARGS as '+'):
#   tests[:PYTEST ARGS]  the -m gpu suite (or the named tests)      -> TAG_tests.log
#   smoke                __graft_entry__ smoke                          -> TAG_smoke.log
#   bench[:BENCH ARGS]   one bench line (default: the driver's flags)  -> TAG_bench.log
#   quick[:BENCH ARGS]   the headline only, 2 steps, no CPU / single / PCIe / cliff legs
#   single[:BENCH ARGS]  the single instance (rps 0) headline, 1 step
#   ktrace[:BENCH ARGS]  rocprofv3 --kernel-trace --stats of one headline step -> TAG_ks/
#   pmc[:BENCH ARGS]     FETCH_SIZE and WRITE_SIZE in separate passes, folded -> TAG_pmc.json
#   sq[:BENCH ARGS]      8 SQ counters per kernel (one pass)            -> TAG_sq_summary.txt
#   phases[:BENCH ARGS]  PX_SET_VERBOSE phase clock of one set batch    -> TAG_phases.log
# Environment: CFG (default 3) and RPS select the profiled config of ktrace / pmc / sq.
# Outputs land in gpurun_out/; copy what is to be kept into profiles/.
set -o pipefail
TAG=${1:?tag}
shift
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out
mkdir -p $O
CFG=${CFG:-3}
ONE="--steps 1 --warmup 0 --no-cpu --no-pcie --no-cliff --no-checks --no-exact --no-single --configs= --config $CFG ${RPS:+--rps $RPS}"
# a counter pass prints nothing for minutes: a ticker keeps the call visibly alive
( while sleep 50; do echo "tick $(date +%T)" >> $O/${TAG}_ticks.log; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
fail() { echo "$1 FAILED"; tail -${3:-20} "$2"; exit 1; }
for STEP in "$@"; do
  NAME=${STEP%%:*}
  ARGS=""
  [ "$STEP" != "$NAME" ] && ARGS=$(echo "${STEP#*:}" | tr '+' ' ')
  case $NAME in
  tests)
    L=$O/${TAG}_tests.log
    timeout -k 10 1000 python -u -m pytest ${ARGS:-tests -m gpu} -x -v --timeout 300 --timeout-method thread > $L 2>&1 \
      || fail TESTS $L 30
    tail -1 $L ;;
  smoke)
    L=$O/${TAG}_smoke.log
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $L 2>&1 || fail SMOKE $L
    tail -1 $L ;;
  bench)
    L=$O/${TAG}_bench.log
    timeout -k 10 900 python -u bench.py ${ARGS:---steps 20 --warmup 5} > $L 2>&1 || fail BENCH $L
    tail -c 400 $L; echo ;;
  quick)
    L=$O/${TAG}_quick.log
    timeout -k 10 300 python -u bench.py --no-cpu --no-single --no-pcie --no-cliff --configs= --steps 2 $ARGS > $L 2>&1 \
      || fail QUICK $L
    tail -c 300 $L; echo ;;
  single)
    L=$O/${TAG}_single.log
    timeout -k 10 300 python -u bench.py --rps 0 --no-cpu --no-single --no-pcie --no-cliff --configs= --steps 1 $ARGS > $L 2>&1 \
      || fail SINGLE $L
    tail -c 300 $L; echo ;;
  ktrace)
    L=$O/${TAG}_ks.log
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_ks -o ks --output-format csv \
      -- python3 $R/bench.py $ONE $ARGS) > $L 2>&1 || fail KTRACE $L
    F=$(find $O/${TAG}_ks -name '*kernel_stats.csv' | head -1)
    python3 $R/tools/ks_top.py "$F" 2>/dev/null | head -25
    find $O/${TAG}_ks -name '*kernel_trace.csv' -exec gzip -f {} \; ;;
  pmc)
    for C in FETCH_SIZE WRITE_SIZE; do
      L=$O/${TAG}_pmc_${C}.log
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $C -d $O/${TAG}_pmc_$C -o p --output-format csv \
        -- python3 $R/bench.py $ONE $ARGS) > $L 2>&1 || fail "PMC $C" $L
    done
    F=$(find $O/${TAG}_pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)
    W=$(find $O/${TAG}_pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)
    REC=$(python3 -c "from pixiu_amd import synth; print(synth.FULL_SIZES[$CFG])")
    RPSV=${RPS:-$(python3 -c "import bench; print(bench.DEFAULT_RPS[$CFG])")}
    python3 tools/pmc_summary.py "$F" "$W" $O/${TAG}_pmc.json \
      "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), python3 bench.py $ONE $ARGS ($TAG)" $CFG $RPSV $REC > /dev/null \
      || { echo "PMC SUMMARY FAILED"; exit 1; }
    gzip -f "$F" "$W"
    echo "pmc -> $O/${TAG}_pmc.json" ;;
  sq)
    L=$O/${TAG}_sq.log
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR -d $O/${TAG}_sq -o sq --output-format csv -- python3 $R/bench.py $ONE $ARGS) \
      > $L 2>&1 || fail SQ $L
    F=$(find $O/${TAG}_sq -name '*counter_collection.csv' | head -1)
    python3 tools/sq_summary.py "$F" > $O/${TAG}_sq_summary.txt && gzip -f "$F"
    head -12 $O/${TAG}_sq_summary.txt ;;
  phases)
    L=$O/${TAG}_phases.log
    PX_SET_VERBOSE=1 PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py $ONE --steps 2 $ARGS > $L 2>&1 || fail PHASES $L
    tail -3 $L ;;
  *)
    echo "unknown step $NAME"; exit 2 ;;
  esac
done
echo DONE
