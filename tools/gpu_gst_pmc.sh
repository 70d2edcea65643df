#!/bin/bash
# k_gst_encode counter passes (one rocprofv3 run each) on one setitem batch.
#   gpurun -- 'bash tools/gpu_gst_pmc.sh TAG N RPS'
set -o pipefail
TAG=${1:?tag}; N=${2:-10000}; RPS=${3:-2}
export TMPDIR=/tmp
O=gpurun_out/${TAG}; mkdir -p $O
i=0
for P in "SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES" \
         "TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o p$i --output-format csv -- python3 tools/gst_run.py 3 $N $RPS > $O/p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 $O/p$i.log; exit 1; }
  grep "kernel" $O/p$i.log
done
python3 tools/pmc_kernel.py k_gst_encode $O/p*/p*_counter_collection.csv
