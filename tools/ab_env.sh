# A/B one environment setting on the bench: tools/ab_env.sh "VAR=value ..." -> gpurun_out/ab_{a,b}.json + traces
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --steps 3 --no-cpu > gpurun_out/ab_a.json 2>gpurun_out/ab_a.err || exit 1
env $1 timeout -k 10 200 python3 bench.py --steps 3 --no-cpu > gpurun_out/ab_b.json 2>gpurun_out/ab_b.err || exit 1
echo OK
