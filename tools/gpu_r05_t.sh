# round-5 box T: the octree line with multicolor ILU(0) smoothing below the finest level (smoother 2) against damped Jacobi
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r05t_oct.txt
for a in "--mg-smooth 2 2 --mg-omega 0.6" "--oct-smoother ilu-coarse --mg-smooth 2 2 --mg-omega 0.6" "--oct-smoother ilu-coarse --mg-smooth 1 1 --mg-omega 0.6" "--mg-smooth 2 2 --mg-omega 0.6" "--oct-smoother ilu-coarse --mg-smooth 2 2 --mg-omega 0.6" "--oct-smoother ilu-coarse --mg-smooth 1 1 --mg-omega 0.6"; do
  timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 $a --no-pmc --no-cpu > gpurun_out/r05t_tmp.json 2> gpurun_out/r05t_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05t_tmp.err; exit $rc; }
  echo "$a: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05t_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its', round(d['value'],2), 'it/s')")" >> gpurun_out/r05t_oct.txt
done
cat gpurun_out/r05t_oct.txt
