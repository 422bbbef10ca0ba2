# quick re-run of bench.py after host-side edits: N=1 line (with roofline traffic / lds) and N=2 on one GPU (gloo)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 2 --dist-backend gloo --cells 64 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_quick_np2.json 2> gpurun_out/bench_quick_np2.err
rc=$?; echo "np2 rc $rc"; exit $rc
