# round-5 box Z: bench's transport fallback (the in-library RCCL pre-flight forced to fail on every rank -> the
# torch.distributed transport, labelled in the line), 2 ranks on the box's one GPU over gloo
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
GLS_BENCH_FAIL_NATIVE_PREFLIGHT=1 timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --cells 64 --steps 3 --warmup 1 --no-pmc --no-cpu > gpurun_out/r05z_np2_fallback.json 2> gpurun_out/r05z_np2_fallback.err
rc=$?; echo "np2 fallback rc $rc"; grep -a "fallback\|raised" gpurun_out/r05z_np2_fallback.err | head -5
python3 -c "import json;d=json.loads(open('gpurun_out/r05z_np2_fallback.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ('n_gpus','dist_impl','dist_impl_fallback','preflight_relerr','linear_iterations_per_step','ms_per_step')})"
exit $rc
