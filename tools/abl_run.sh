# J.v timings of the timing-only ablation builds (GLS_ABL bits: 1 no gather, 2 no scatter, 4 no sweeps, 8 no qd loads)
set -o pipefail
O=gpurun_out/abl.log; rm -f $O
for L in softx_2020_200_amd/libgls_native.so tools/libgls_abl1.so tools/libgls_abl2.so tools/libgls_abl4.so tools/libgls_abl8.so; do
  echo "== $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_app.py -m gpu >> $O 2>&1 || exit 1
