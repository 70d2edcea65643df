set -o pipefail
export TMPDIR=/tmp
cd pixiu_amd && cp libpixiu_amd.so /tmp/keep.so && cd ..
timeout -k 10 200 python -u tools/decode_run.py 3 10000 2 4096,6144,8192,12288,16384 > gpurun_out/var_waves.log 2>&1 || exit 1
for v in am16 am40 lc128 lc2k; do
  cp pixiu_amd/libpixiu_amd_v$v.so pixiu_amd/libpixiu_amd.so
  timeout -k 10 120 python -u tools/decode_run.py 3 10000 2 0 > gpurun_out/var_$v.log 2>&1 || { cp /tmp/keep.so pixiu_amd/libpixiu_amd.so; exit 1; }
done
cp /tmp/keep.so pixiu_amd/libpixiu_amd.so
grep -h "waves" gpurun_out/var_*.log
