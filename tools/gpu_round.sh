#!/bin/bash
# One GPU session: parity tests, J.v microbench (cached vs recompute), bench line, rocprofv3
# kernel stats of the bench, PMC HBM traffic of the J.v kernel. Output under gpurun_out/.
# Each GPU step has its own time limit; a fault / abort / timeout ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
stop() { echo "step '$1' ended with $2" >> $O/round.log; exit $2; }
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/round.log
[ $rc -gt 1 ] && stop pytest $rc
timeout -k 10 120 python tools/jv_bench.py 128 20 > $O/jv.log 2>&1 || stop jv_bench $?
GLS_JV_RECOMPUTE=1 timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O/jv.log 2>&1 || stop jv_bench_recompute $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || stop bench $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/prof_bench.log 2>&1 || stop rocprof_stats $?
tools/pmc_traffic.sh 128 $O/pmc_traffic > $O/pmc_traffic.txt 2>&1 || stop pmc $?
echo done >> $O/round.log
