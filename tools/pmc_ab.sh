# PMC counters of the Q2 J.v kernel variants (one rocprofv3 --pmc pass per counter set and variant)
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab; mkdir -p $OUT
i=0
for V in "X=1" "GLS_BRICK_V1=1"; do
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT"; do
  i=$((i+1))
  env $V timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-include-regex "brick" -d $OUT/p$i -o run --output-format csv -- python3 tools/jv_bench.py 128 3 > $OUT/p$i.log 2>&1 || exit 1
done
done
python3 - "$OUT" << 'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-24s %14.4e (n=%d)" % (c, sum(v) / len(v), len(v)))
PY
