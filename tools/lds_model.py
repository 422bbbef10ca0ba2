"""Static LDS / VALU model of the brick J.v kernels from the CURRENT source (tooling, not product code).

Compiles softx_2020_200_amd/csrc/gls_brick_pencil.hip to gfx950 assembly, counts per kernel the LDS
instructions priced with MI355X_MICROARCH.md §LDS (ds_read_b64 2, ds_read_b128 4, ds_read2_b64 8,
ds_write_b64 ~6, ds_write2_b64 13, ...), the FP64 / FP32 VALU instructions and the VGPR count, and
writes profiles/<out>.json with the git commit of the source. bench.py reads it for its
roofline["lds"] block and labels that block a static model (conflict-free, straight-line count).
Usage: python tools/lds_model.py [out_name]   (default r05_lds_model)"""
import collections
import hashlib
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "softx_2020_200_amd", "csrc", "gls_brick_pencil.hip")
LDS_CYCLES = {'ds_read_b32': 2, 'ds_read_b64': 2, 'ds_read_b128': 4, 'ds_read_b96': 8, 'ds_read2_b32': 4,
              'ds_read2_b64': 8, 'ds_read2st64_b32': 4, 'ds_read2st64_b64': 8, 'ds_write_b32': 4,
              'ds_write_b64': 6, 'ds_write2_b32': 6, 'ds_write2st64_b32': 6, 'ds_write_b96': 10,
              'ds_write_b128': 13, 'ds_write2_b64': 13, 'ds_write2st64_b64': 13}


def main():
    out_name = sys.argv[1] if len(sys.argv) > 1 else "r05_lds_model"
    asm = "/tmp/gls_brick_pencil_model.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                           "-fno-slp-vectorize", "--cuda-device-only", "-S", SRC, "-o", asm],
                          cwd=os.path.dirname(SRC), stderr=subprocess.DEVNULL)
    lines = open(asm).read().split("\n")
    meta = {}
    cur = None
    for l in lines:
        m = re.match(r"\s+\.name:\s+(\S+)", l)
        if m:
            cur = m.group(1)
            meta[cur] = {}
        m = re.match(r"\s+\.(vgpr_count|sgpr_count|vgpr_spill_count):\s+(\d+)", l)
        if m and cur:
            meta[cur][m.group(1)] = int(m.group(2))
    kernels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if not m or "pencil_kernel" not in m.group(1):
            continue
        name = m.group(1)
        c = collections.Counter()
        lds = 0
        j = i
        while "s_endpgm" not in lines[j]:
            t = lines[j].strip().split()
            j += 1
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            op = t[0]
            if op.startswith("ds_"):
                lds += LDS_CYCLES.get(op, 4)
                c["lds_instructions"] += 1
            elif re.match(r"v_(fma|fmac|mul|add)_f64", op):
                c["valu_f64"] += 1
            elif re.match(r"v_(fma|fmac|mul|add)_f32", op):
                c["valu_f32"] += 1
            elif op.startswith("v_"):
                c["valu_other"] += 1
        kernels[name] = dict(lds_cycles_per_wave=lds, **c, **meta.get(name, {}))
    commit = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=ROOT, capture_output=True,
                            text=True).stdout.strip()
    dirty = subprocess.run(["git", "status", "--porcelain", SRC], cwd=ROOT, capture_output=True, text=True).stdout
    res = {"model": "static: straight-line instruction count of the compiled kernel, LDS instructions priced "
                    "conflict-free by MI355X_MICROARCH.md §LDS; every wave of the pencil kernel runs the whole "
                    "stream once (no loops except the diagonal's qy loop, x3)",
           "source": os.path.relpath(SRC, ROOT), "commit": commit + ("+dirty" if dirty else ""),
           "source_sha256": hashlib.sha256(open(SRC, "rb").read()).hexdigest(),
           "cells_per_wave": 6, "kernels": kernels}
    path = os.path.join(ROOT, "profiles", out_name + ".json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
