#!/bin/bash
# Counters of the getitem gather (one launch: PX_GET_HEAD64=63), separate passes
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/${TAG}_counters.txt 2>&1 || true
P="$R/bench.py --no-cpu --no-single --no-pcie --no-cliff --configs= --no-checks --no-exact --steps 1 --warmup 0"
export PX_GET_HEAD64=63
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C -d $O/${TAG}_p$i -o p --output-format csv -- python3 $P > $O/${TAG}_p$i.log 2>&1 \
    || { echo "PMC pass $i FAILED"; tail -5 $O/${TAG}_p$i.log; exit 1; }
  F=$(find $O/${TAG}_p$i -name '*counter_collection.csv' | head -1)
  python3 $R/tools/pmc_kernel.py "::k_gather(" $F
  gzip -f $F
done
