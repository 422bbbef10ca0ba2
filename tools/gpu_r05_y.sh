# round-5 box Y: forest J.v with the bricks' pencil launch overlapped with the leaves' per-cell launch (side stream)
# and C v in one pass; parity tests of the forest / hanging paths, then the octree line A/B (GLS_OCT_OVERLAP=0/1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_forest_bricks.py tests/test_gpu_octree_mg.py tests/test_gpu_uforest.py tests/test_gpu_umesh_mg.py tests/test_gpu_dist_mg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05y_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r05y_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/r05y_oct.txt
for ov in 0 1 0 1 0 1; do
  GLS_OCT_OVERLAP=$ov timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05y_tmp.json 2> gpurun_out/r05y_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05y_tmp.err; exit $rc; }
  echo "GLS_OCT_OVERLAP=$ov: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05y_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its', round(d['value'],2), 'it/s')")" >> gpurun_out/r05y_oct.txt
done
cat gpurun_out/r05y_oct.txt
