# bench.py's N>1 path on one GPU: 2 and 4 ranks sharing the card over the gloo/torch transport (the
# native RCCL transport needs one GPU per rank: the driver's 8-GPU node), 32^3 and 64^3 cubes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for NP in 2 4; do
  timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus $NP --dist-backend gloo --cells 64 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_np$NP.json 2> gpurun_out/bench_np$NP.err
  rc=$?; echo "np$NP rc $rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
