# round-3 final check at HEAD: full -m gpu suite, configs[2] bench under rocprofv3 --stats, the bench
# line, the cylinder3d (configs[4] problem) line, the configs[1] line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -2 gpurun_out/gpu_tests_final.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_prof_final.json 2> gpurun_out/bench_prof_final.err
rc=$?; echo "prof rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
rc=$?; echo "bench rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python3 bench.py --workload cylinder3d --steps 5 --warmup 1 > gpurun_out/bench_cyl3d_final.json 2> gpurun_out/bench_cyl3d_final.err
rc=$?; echo "cyl3d rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python3 bench.py --cells 64 --k 1 --kp 1 --nu 1 --scheme steady --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_q1_final.json 2> gpurun_out/bench_q1_final.err
rc=$?; echo "q1 rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cyl3d_final -o run --output-format csv -- python3 bench.py --workload cylinder3d --steps 3 --warmup 1 > gpurun_out/bench_cyl3d_prof_final.json 2> gpurun_out/bench_cyl3d_prof_final.err
rc=$?; echo "cyl3d prof rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
rc=$?; echo "smoke rc $rc"; exit $rc
