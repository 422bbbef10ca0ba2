#!/bin/bash
# LDS counters of the Q2 brick kernels for library variants (one rocprofv3 --pmc pass per library):
# default (padded-line stage arrays), tools/ab/libgls_r0.so (round-2 baseline), tools/ab/libgls_r2.so (padded, 3 waves/SIMD)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lds; mkdir -p $OUT
for v in main r0 r2; do
  L=$PWD/tools/ab/libgls_$v.so; [ $v = main ] && L=$PWD/softx_2020_200_amd/libgls_native.so
  GLS_NATIVE_LIB=$L timeout -k 10 120 python tools/jv_bench.py 128 20 >> $OUT/jv.log 2>&1 || exit 1
  GLS_NATIVE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM --kernel-include-regex "gls_brick_kernel" -d $OUT/$v -o run --output-format csv -- python3 tools/jv_bench.py 128 4 > $OUT/$v.log 2>&1 || exit 1
done
python3 - $OUT << 'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for v in ("main", "r0", "r2"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(out + "/%s/**/*counter_collection.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in sorted(agg.items()):
        print(v, k, " ".join("%s=%.3e" % (c, sum(x) / len(x)) for c, x in sorted(d.items())))
PY
