#!/bin/bash
# k_decode investigation: prof-build counters (flag reasons, lane steps) and SQ counter passes.
#   gpurun -- 'bash tools/gpu_dec_prof.sh TAG'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=gpurun_out/${TAG}; mkdir -p $O
timeout -k 10 180 python -u tools/decode_profile.py 3 10000 2 > $O/decprof.log 2>&1 || { echo PROF FAILED; tail -20 $O/decprof.log; exit 1; }
cat $O/decprof.log
i=0
for P in "SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES" \
         "TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/p$i -o p$i --output-format csv -- python3 tools/decode_run.py 3 10000 2 > $O/p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_kernel.py "k_decode(" $O/p*/p*_counter_collection.csv
