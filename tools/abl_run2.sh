set -o pipefail
O=gpurun_out/abl2.log; rm -f $O
for L in softx_2020_200_amd/libgls_native.so tools/libgls_abl_w6.so tools/libgls_abl_w7.so; do
  echo "== $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_app.py -m gpu >> $O 2>&1 || exit 1
