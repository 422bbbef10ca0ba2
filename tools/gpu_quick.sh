#!/bin/bash
# GPU tests + default bench + MG sweep (MG_SWEEP) in one session; outputs under gpurun_out/.
O=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -q > $O/gputests.log 2>&1; rc=$?
echo "pytest rc=$rc" > $O/quick.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_quick.json 2> $O/bench_quick.err || exit $?
if [ -n "$MG_SWEEP" ]; then bash tools/mg_sweep.sh || exit $?; fi
echo done >> $O/quick.log
