T="timeout -k 10 150 python -u -m pytest tests/test_gpu_psa.py -k outgrows -x -q --timeout 120 --timeout-method thread"
mkdir -p gpurun_out
export PX_POOL_HASH=1 PX_PIN_COPY=1
$T > gpurun_out/bis2.log 2>&1 && echo "+win split ok" &&
unset PX_PIN_COPY && $T > gpurun_out/bis3.log 2>&1 && echo "+pin write ok" &&
unset PX_POOL_HASH && $T > gpurun_out/bis4.log 2>&1 && echo "+pool sort ok" &&
bash tools/gpu_run.sh r06y tests:tests/test_gpu_psa.py+tests/test_gpu_pools.py+tests/test_gpu_rounds.py+tests/test_gpu_refdig.py &&
RPS=0 bash tools/gpu_run.sh r06y_single ktrace &&
PIXIU_AMD_LIB=$PWD/pixiu_amd/libpixiu_amd_sortlce32.so PX_WIN_SPLIT=1 PX_POOL_HASH=1 PX_PIN_COPY=1 PX_SORT_PASS_MEMSET=1 RPS=0 bash tools/gpu_run.sh r06y_single1 ktrace
