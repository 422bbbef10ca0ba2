set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
GLS_CELL_CACHE=$v timeout -k 10 200 python -u -m pytest tests/test_kelly.py -m gpu -x -q -k "mms2d_pipeline" --timeout 150 --timeout-method thread > gpurun_out/dbg_kelly_$v.log 2>&1; echo "cache=$v rc $?"; tail -2 gpurun_out/dbg_kelly_$v.log
done
