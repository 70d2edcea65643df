mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
timeout -k 10 120 python -u tools/gst_profile.py 3 1024 1 > gpurun_out/gstprof_hint.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_hint.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_imix -o imix --output-format csv -- python3 tools/gst_run.py 3 1024 1 > gpurun_out/pmc_imix.log 2>&1 || exit 1
