# rocprofv3 kernel stats of the octree line with mixed-precision forest smoothing (1.28 M DoFs)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_octm -o run --output-format csv -- \
  python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 \
  > gpurun_out/prof_octm.json 2> gpurun_out/prof_octm.err || { tail -5 gpurun_out/prof_octm.err; exit 1; }
f=$(find gpurun_out/prof_octm -name "run_kernel_stats.csv" | head -1); cp "$f" gpurun_out/octm_kernel_stats.csv
python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/octm_kernel_stats.csv')))
for x in r[:14]: print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])), x['Percentage'][:5])"
