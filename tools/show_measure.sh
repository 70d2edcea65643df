#!/bin/bash
# summary of tools/gpu_measure.sh outputs: show_measure.sh r03f [top]
T=${1:?tag}
O=gpurun_out
grep "psa: step\|psa: N=" $O/${T}_bench.log | tail -4 | cut -c1-400
grep -o '"setitem_MBps": [0-9.]*\|"getitem_MBps": [0-9.]*\|"psa_split_ms": {[^}]*}\|"parity_counts": {[^}]*}' $O/${T}_bench.log
echo "single instance:"; grep -o '"setitem_MBps": [0-9.]*\|"compression_ratio": [0-9.]*\|"psa_split_ms": {[^}]*}\|"psa_rounds": [0-9]*' $O/${T}_single.log
tail -2 $O/${T}_tests.log
python tools/prof_db.py $O/${T}_prof/prof_results.db ${2:-24}
