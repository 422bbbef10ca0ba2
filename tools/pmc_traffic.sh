#!/bin/bash
# HBM traffic of the J.v kernel from PMC (MI355X_MICROARCH.md "HBM" section): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes over tools/jv_bench.py, plus the same counters on
# k_copy (8 B/lane loads + stores of a known byte count: 2 x 8 x n_dofs) as this access width's
# calibration. Usage: tools/pmc_traffic.sh N OUTDIR
N=${1:-128}; OUT=${2:-gpurun_out/pmc_traffic}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for CTR in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-include-regex "gls_brick_kernel|gls_pencil_kernel|k_copy|k_slab_sum" -d $OUT/p$i -o run \
      --output-format csv -- python3 tools/jv_bench.py $N 4 > $OUT/p$i.log 2>&1 || exit 1
done
python3 - "$OUT" << 'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    print(k)
    for c, v in sorted(d.items()):
        print("   %-12s %14.4e KB per dispatch (mean of %d)" % (c, sum(v) / len(v), len(v)))
PY
