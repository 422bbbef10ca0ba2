set -e
B="timeout -k 10 200 python3 bench.py --steps 3 --no-cpu"
$B --mg-coarsest 2 > gpurun_out/cs_a.json 2>&1
GLS_MG_COARSE_SOLVER=lu_npvt $B --mg-coarsest 2 > gpurun_out/cs_b.json 2>&1
GLS_MG_COARSE_SOLVER=lu_npvt $B --mg-coarse-direct 1 > gpurun_out/cs_c.json 2>&1
GLS_MG_VERBOSE=1 timeout -k 10 200 python3 bench.py --steps 1 --no-cpu --mg-coarsest 2 > gpurun_out/cs_av.log 2>&1
