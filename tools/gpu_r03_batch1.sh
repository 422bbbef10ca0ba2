# round-3 batch: reference app cases, ILU / split tests, cylinder ILU timing, J.v kernel A/B
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r03_apps.sh cylinder_gls taylor-green-vortex_gls_sdirk3 taylor-green-vortex_gls_sdirk2 || exit 1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ilu.py tests/test_gpu_dist.py > gpurun_out/tests1.log 2>&1
rc=$?; echo "tests rc $rc"; [ $rc -gt 1 ] && exit $rc
bash tools/gpu_r03_cyl.sh 0.1 || exit 1
O=gpurun_out/jvab.log; rm -f $O
for L in softx_2020_200_amd/libgls_native.so tools/libgls_pf3.so tools/libgls_w3.so softx_2020_200_amd/libgls_native.so; do
  echo "== $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O 2>&1 || exit 1
done
