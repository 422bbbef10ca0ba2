# round-5 box PC: listed batched probe blocks reading the linearization cache (cache) against re-deriving it from the
# state (state, GLS_ILU_PROBE_CACHE=0): ILU parity tests, then taylorcouette3d r3 and cylinder3d A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05pc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05pc_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/r05pc_ab.txt
run() {
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" --no-pmc --no-cpu > gpurun_out/r05pc_tmp.json 2> gpurun_out/r05pc_tmp.err
  local rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05pc_tmp.err; return $rc; }
  echo "$name $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05pc_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its')")" >> gpurun_out/r05pc_ab.txt
}
for v in state cache state cache; do
  if [ $v = state ]; then export GLS_ILU_PROBE_CACHE=0; else unset GLS_ILU_PROBE_CACHE; fi
  run tc3 --workload taylorcouette3d --cyl-refine 3 --cyl-precond hmg --steps 3 --warmup 1 || exit 1
  run cylinder3d --workload cylinder3d --steps 3 --warmup 1 || exit 1
done
cat gpurun_out/r05pc_ab.txt
