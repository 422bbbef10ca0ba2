# round-5 box U: the per-cell kernel's integrate loops unrolled by 3 (tools/ab/libgls_native_unr.so, same VGPRs and
# occupancy) against HEAD: octree line (small leaf launches, latency) and cylinder3d (mapped per-cell throughput)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r05u_ab.txt
for v in base unr base unr; do
  if [ $v = unr ]; then export GLS_NATIVE_LIB=$GRAFT_REPO_ROOT/tools/ab/libgls_native_unr.so; else unset GLS_NATIVE_LIB; fi
  timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05u_tmp.json 2> gpurun_out/r05u_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05u_tmp.err; exit $rc; }
  echo "octree $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05u_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its')")" >> gpurun_out/r05u_ab.txt
  timeout -k 10 300 python3 bench.py --workload cylinder3d --no-pmc --no-cpu --steps 3 --warmup 1 > gpurun_out/r05u_tmp.json 2> gpurun_out/r05u_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05u_tmp.err; exit $rc; }
  echo "cylinder3d $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05u_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its')")" >> gpurun_out/r05u_ab.txt
done
cat gpurun_out/r05u_ab.txt
