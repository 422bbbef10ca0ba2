#!/bin/bash
# Separate rocprofv3 --pmc passes over tools/jv_bench.py (J.v kernel counters). Usage: tools/pmc_jv.sh N OUTDIR
N=${1:-64}; OUT=${2:-gpurun_out/pmc}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for CTRS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_UNALIGNED_STALL" \
            "SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FLOPS_FP64" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-include-regex "gls_brick_kernel" -d $OUT/p$i -o run --output-format csv -- python tools/jv_bench.py $N 4 > $OUT/p$i.log 2>&1 || exit 1
done
python - "$OUT" << 'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %16.4e  (n=%d per-dispatch mean)" % (c, sum(v) / len(v), len(v)))
PY
