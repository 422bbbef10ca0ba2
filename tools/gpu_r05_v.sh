# round-5 box V: k_gather_ev with all slots, then all values, loaded up front (tools/ab/libgls_native_gev.so) against
# HEAD: octree line and cylinder3d (per-cell paths)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r05v_ab.txt
for v in base gev base gev; do
  if [ $v = gev ]; then export GLS_NATIVE_LIB=$GRAFT_REPO_ROOT/tools/ab/libgls_native_gev.so; else unset GLS_NATIVE_LIB; fi
  timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05v_tmp.json 2> gpurun_out/r05v_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05v_tmp.err; exit $rc; }
  echo "octree $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05v_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its')")" >> gpurun_out/r05v_ab.txt
  timeout -k 10 300 python3 bench.py --workload cylinder3d --no-pmc --no-cpu --steps 3 --warmup 1 > gpurun_out/r05v_tmp.json 2> gpurun_out/r05v_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05v_tmp.err; exit $rc; }
  echo "cylinder3d $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05v_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its')")" >> gpurun_out/r05v_ab.txt
done
cat gpurun_out/r05v_ab.txt
