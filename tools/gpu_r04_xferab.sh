# A/B of the transfer kernels' planes per block (GLS_XFER_ZB) on the configs[2] bench line, one box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/xferab.log; rm -f $O
run() {  # TAG ENV -- bench args
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python3 bench.py "$@" > gpurun_out/xab_$tag.json 2> gpurun_out/xab_$tag.err || { echo "FAIL $tag" >> $O; return 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-8s ms/step %7.2f  its %5.1f' % (sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step']))" gpurun_out/xab_$tag.json $tag >> $O
}
B="--steps 8 --warmup 2 --no-cpu"
for v in "base X=1" "zb4 GLS_XFER_ZB=4" "zb2 GLS_XFER_ZB=2" "zb1 GLS_XFER_ZB=1" "base2 X=1" "zb2b GLS_XFER_ZB=2"; do
  set -- $v
  run $1 $2 $B || exit 1
done
cat $O
