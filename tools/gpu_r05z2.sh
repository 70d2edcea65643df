#!/bin/bash
# round-5 final, part 2: kernel-trace summary and the two PMC passes of a config-3 step
# (tools/gpu_profile.sh without its tests and bench)
SKIP_TESTS=1 SKIP_BENCH=1 bash tools/gpu_profile.sh r05final
