# round-3 batch 5: e2 tests + app --np pipelines, then the cylinder3d bench line and its kernel profile
set -o pipefail
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 python -u bench.py --workload cylinder3d --steps 3 --warmup 1 > gpurun_out/bench_cyl3d.log 2>&1
rc=$?; echo "cyl3d bench rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_app.py -k curved_wall > gpurun_out/tests_b5slip.log 2>&1
rc=$?; echo "curved slip rc $rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_dist_general.py > gpurun_out/tests_b4a.log 2>&1
rc=$?; echo "dist general rc $rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_app_configs.py > gpurun_out/tests_b4b.log 2>&1
rc=$?; echo "configs rc $rc"; exit $rc
