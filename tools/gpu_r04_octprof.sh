# rocprofv3 kernel stats of the octree GMG line (1.28M DoFs), then the app's forest-multigrid test and
# the app's Kelly / hanging tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_oct -o run --output-format csv -- \
  python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 \
  > gpurun_out/oct_prof.json 2> gpurun_out/oct_prof.err || { tail -20 gpurun_out/oct_prof.err; exit 1; }
f=$(find gpurun_out/prof_oct -name "run_kernel_stats.csv" | head -1); cp "$f" gpurun_out/oct_kernel_stats.csv
python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/oct_kernel_stats.csv')))
for x in r[:22]: print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])), x['Percentage'][:5])"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -s \
  tests/test_gpu_app.py -k "forest_multigrid or kelly or hanging or mms3d" > gpurun_out/app_forest.log 2>&1 || { tail -40 gpurun_out/app_forest.log; exit 1; }
grep -E "PASSED|FAILED|forest GMG" gpurun_out/app_forest.log
