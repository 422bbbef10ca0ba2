#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02lds2; mkdir -p $OUT
for v in A C; do
  GLS_NATIVE_LIB=tools/exp_libgls_$v.so timeout -k 10 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "gls_brick_kernel" -d $OUT/$v -o run --output-format csv -- python3 tools/jv_bench.py 128 4 > $OUT/$v.log 2>&1 || exit 1
done
python3 - $OUT << 'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for v in "AC":
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(out + "/%s/**/*counter_collection.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in sorted(agg.items()):
        print(v, k, " ".join("%s=%.3e" % (c, sum(x) / len(x)) for c, x in sorted(d.items())))
PY
