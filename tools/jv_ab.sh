# A/B timing of J.v kernel builds at Q2 128^3 (tools/jv_bench.py): default library vs tools/libgls_*.so
set -o pipefail
O=gpurun_out/jvab.log; rm -f $O
for L in softx_2020_200_amd/libgls_native.so tools/libgls_r0.so; do
  echo "== $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O 2>&1 || exit 1
done
