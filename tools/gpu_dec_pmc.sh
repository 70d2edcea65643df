#!/bin/bash
# k_decode counter passes (one rocprofv3 run each) on a config-3 getitem batch.
#   gpurun -- 'bash tools/gpu_dec_pmc.sh TAG'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=gpurun_out/${TAG}; mkdir -p $O
i=0
for P in "SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES" \
         "TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o p$i --output-format csv -- python3 tools/decode_run.py 3 10000 2 > $O/p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 $O/p$i.log; exit 1; }
done
grep "waves" $O/p1.log
python3 tools/pmc_kernel.py "k_decode(" $O/p*/p*_counter_collection.csv
