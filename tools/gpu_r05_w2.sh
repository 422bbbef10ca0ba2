# round-5 box W2: hanging-row condensation and C v line interpolation with all indices / weights loaded up front (in-tree
# library) against the gather-only state (tools/ab/libgls_native_gevonly.so): octree line A/B, then the per-cell,
# forest, multigrid and distributed GPU tests on the in-tree library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r05w2_ab.txt
for v in gevonly all gevonly all; do
  if [ $v = gevonly ]; then export GLS_NATIVE_LIB=$GRAFT_REPO_ROOT/tools/ab/libgls_native_gevonly.so; else unset GLS_NATIVE_LIB; fi
  timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05w2_tmp.json 2> gpurun_out/r05w2_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05w2_tmp.err; exit $rc; }
  echo "octree $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05w2_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its')")" >> gpurun_out/r05w2_ab.txt
done
unset GLS_NATIVE_LIB
cat gpurun_out/r05w2_ab.txt
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mapped.py tests/test_gpu_uforest.py tests/test_gpu_forest_bricks.py tests/test_gpu_umesh_mg.py tests/test_gpu_octree_mg.py tests/test_gpu_dist_general.py tests/test_gpu_ilu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r05w2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05w2_tests.log; exit $rc
