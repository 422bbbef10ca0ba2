"""Summarize tools/ab_bench.sh outputs: ms/step and per-kernel ms of each bench line."""
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
for f in sorted(os.listdir(d)):
    if not f.endswith(".json"):
        continue
    try:
        j = json.loads(open(os.path.join(d, f)).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "no result:", e)
        continue
    k = j["kernel_ms"]
    print(f, "ms/step %.1f" % j["ms_per_step"], "jv %.3f f32 %.3f slab %.3f res %.3f diag %.3f" % (
        k["jacobian_apply"], k["smoother_jv_f32"], k["slab_sum"], k["residual"], k["diagonal"]))
