# round-5 box V: kernel stats of the configs[4] bench line at the reference's ILU fill 1 (Cuthill-McKee order)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05v_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload cylinder3d --ilu-fill 1 --steps 2 --warmup 1 --no-pmc --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r05v.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05v.err
rc=$?; echo "prof rc $rc"; exit $rc
