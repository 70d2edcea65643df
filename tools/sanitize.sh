#!/bin/bash
# Every CPU test of the restatement under ASan + UBSan, and the host-only runtime code
# (tests/cpp/host_test.cpp); ~12 minutes.  Log: profiles/<tag>_sanitize.log
set -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan || exit 1
ASAN=$(gcc -print-file-name=libasan.so) UBSAN=$(gcc -print-file-name=libubsan.so)
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer \
  -I pixiu_amd/csrc tests/cpp/host_test.cpp -o /tmp/px_host_test -lpthread && /tmp/px_host_test || exit 1
LD_PRELOAD=$ASAN:$UBSAN ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  PXO_LIB=$PWD/oracle/_build/libpxo_asan.so python -m pytest -q -p no:cacheprovider \
  tests/test_oracle_golden.py tests/test_oracle_iter.py tests/test_reinsert.py tests/test_oracle_vs_ref.py
