#!/bin/bash
# VALU / MFMA / LDS counters of the Q2 brick kernels at HEAD (one rocprofv3 --pmc pass, 8 SQ + 1 GRBM
# counters) over tools/jv_bench.py 128: backs the design choice of VALU sum factorization over FP64
# MFMA (MFMA busy = 0) and shows the LDS issue share of the wave cycles
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_valu; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --kernel-include-regex "gls_brick_kernel" -d $OUT/p -o run --output-format csv -- python3 tools/jv_bench.py 128 4 > $OUT/p.log 2>&1 || exit 1
python3 - $OUT << 'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    m = {c: sum(x) / len(x) for c, x in d.items()}
    print(k, " ".join("%s=%.3e" % (c, v) for c, v in sorted(m.items())))
    wc = m.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print("    VALU-active / wave cycles %.3f, LDS-active / wave cycles %.3f, LDS wait / wave cycles %.3f, "
              "MFMA busy cycles %.3e" % (m.get("SQ_ACTIVE_INST_VALU", 0) / wc, m.get("SQ_ACTIVE_INST_LDS", 0) / wc,
                                         m.get("SQ_WAIT_INST_LDS", 0) / wc, m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)))
PY
