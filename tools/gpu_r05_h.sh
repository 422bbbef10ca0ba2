# round-5 box H: octree / two-level replica multigrid across ranks; configs[4] bench at the reference's ILU fill 1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_mg.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r05h_dist_mg.log 2>&1
rc=$?; echo "dist mg rc $rc"; tail -3 gpurun_out/r05h_dist_mg.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --workload cylinder3d --ilu-fill 1 --no-pmc > gpurun_out/r05h_cyl_fill1.json 2> gpurun_out/r05h_cyl_fill1.err
rc=$?; echo "cyl fill1 rc $rc"; tail -c 600 gpurun_out/r05h_cyl_fill1.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --workload cylinder3d --no-pmc > gpurun_out/r05h_cyl_fill0.json 2> gpurun_out/r05h_cyl_fill0.err
rc=$?; echo "cyl fill0 rc $rc"; exit $rc
