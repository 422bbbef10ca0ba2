#!/bin/bash
# Round-4 counters of the Q2 pencil + brick kernels over tools/jv_bench.py 128 (one rocprofv3 --pmc pass per
# counter group): wave-state split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY, disjoint,
# MI355X_MICROARCH.md PMC slots), VALU / LDS activity, LDS array cycles and bank conflicts, instruction
# counts incl. VMEM; then HBM traffic (tools/pmc_traffic.sh). Counters absent from `rocprofv3 -L` are skipped.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_r04}; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
have() { grep -q -w "$1" $OUT/avail.txt; }
pass() {  # pass NAME counters...
  local name=$1; shift; local list=""
  for c in "$@"; do if have $c; then list="$list $c"; else echo "skip $c (not listed)" >> $OUT/skipped.txt; fi; done
  [ -z "$list" ] && return 0
  timeout -s KILL 120 rocprofv3 --pmc $list --kernel-include-regex "gls_pencil_kernel|gls_brick_kernel|k_slab_sum" -d $OUT/$name -o run \
      --output-format csv -- python3 tools/jv_bench.py 128 4 > $OUT/$name.log 2>&1
}
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT || exit 1
pass b SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS || exit 1
python3 - $OUT << 'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:52]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    m = {c: sum(x) / len(x) for c, x in d.items()}
    print(k)
    print("   " + " ".join("%s=%.3e" % (c, v) for c, v in sorted(m.items())))
    wc = m.get("SQ_WAVE_CYCLES", 0)
    if wc:
        print("   per wave cycle: WAIT_ANY %.3f  WAIT_INST_ANY %.3f  ACTIVE_INST_ANY %.3f  VALU %.3f  LDS %.3f"
              % tuple(m.get(c, 0) / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                 "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS")))
    if m.get("SQ_LDS_IDX_ACTIVE"):
        print("   LDS bank-conflict share of LDS array cycles %.3f" % (m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]))
    if m.get("SQ_WAVES"):
        print("   per wave: VALU %.0f  LDS %.0f  SALU %.0f  VMEM rd %.0f  wr %.0f" % tuple(
            m.get(c, 0) / m["SQ_WAVES"] for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                                                  "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")))
PY
