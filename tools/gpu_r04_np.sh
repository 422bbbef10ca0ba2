# bench.py's N>1 path at HEAD on one GPU: 2 and 4 ranks sharing the card over the gloo transport, 64^3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for NP in 1 2 4; do
  if [ $NP -eq 1 ]; then
    timeout -k 10 240 python3 bench.py --cells 64 --steps 2 --warmup 1 --no-cpu > gpurun_out/r04np_$NP.json 2> gpurun_out/r04np_$NP.err
  else
    timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 --master-port 29511 \
      bench.py --gpus $NP --dist-backend gloo --cells 64 --steps 2 --warmup 1 --no-cpu > gpurun_out/r04np_$NP.json 2> gpurun_out/r04np_$NP.err
  fi
  rc=$?; echo "np$NP rc $rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04np_$NP.err; exit $rc; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('N=%d ms/step %.1f its %.1f solver %s' % (d['n_gpus'], d['ms_per_step'], d['linear_iterations_per_step'], d['config'].get('linear_solver')))" gpurun_out/r04np_$NP.json
done
