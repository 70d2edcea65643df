#!/bin/bash
# decoder counters of config 3's set batch (prof build), then SQ counters of one bench step
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/decode_profile.py 3 10000 139 > $O/r05p_decprof.log 2>&1 || { echo DECPROF FAILED; tail -5 $O/r05p_decprof.log; exit 1; }
cat $O/r05p_decprof.log
bash tools/gpu_sq.sh r05p
