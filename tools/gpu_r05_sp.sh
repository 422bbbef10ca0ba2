# round-5 box SP: the multigrid transfers' CSR-vector SpMV unrolled by 4 (a: tools/ab/libgls_native_spmv.so) against HEAD (base):
# octree line, cylinder3d and taylorcouette3d r3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r05sp_ab.txt
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" --no-pmc --no-cpu > gpurun_out/r05sp_tmp.json 2> gpurun_out/r05sp_tmp.err
  local rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05sp_tmp.err; return $rc; }
  echo "$name $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05sp_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its')")" >> gpurun_out/r05sp_ab.txt
}
for v in base a base a; do
  case $v in a) export GLS_NATIVE_LIB=$GRAFT_REPO_ROOT/tools/ab/libgls_native_spmv.so;;  *) unset GLS_NATIVE_LIB;; esac
  run octree --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 || exit 1

  run tc3 --workload taylorcouette3d --cyl-refine 3 --cyl-precond hmg --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r05sp_ab.txt
