#!/bin/bash
# single instance (one shard, chunks rotated by the MemPool rule): kernel trace of one set batch,
# to split its 53 rounds into kernel time and the gaps between kernels
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r05s6_ks -o ks --output-format csv \
  -- python3 bench.py --steps 1 --warmup 0 --configs= --no-cpu --no-pcie --no-cliff --no-checks --no-exact --no-single --config 3 --rps 0 > $O/r05s6_ks.log 2>&1 || { echo KTRACE FAILED; tail -20 $O/r05s6_ks.log; exit 1; }
tail -1 $O/r05s6_ks.log
find $O/r05s6_ks -name '*kernel_trace.csv' | head -1 | xargs gzip -f
