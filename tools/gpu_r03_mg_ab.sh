# V-cycle smoothing on the finest level: GMRES iterations and step time per variant (configs[2] bench)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/mg_ab.log; rm -f $O
for V in "1 1" "0 1" "0 2" "1 0" "2 0"; do
  echo "== fine sweeps $V" >> $O
  timeout -k 10 150 python3 bench.py --no-cpu --steps 6 --warmup 2 --mg-fine-sweeps $V >> $O 2>&1 || exit 1
done
for W in 1.0 0.8; do
  echo "== fine sweeps 0 1, omega $W" >> $O
  timeout -k 10 150 python3 bench.py --no-cpu --steps 6 --warmup 2 --mg-fine-sweeps 0 1 --mg-omega $W >> $O 2>&1 || exit 1
done
