"""Build the in-tree HIP extension libgls_native.so for gfx950 (hipcc; no JIT cache)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgls_native.so")


def build(verbose=False, jobs=4):
    cmd = ["make", "-C", CSRC, "-j%d" % jobs]
    if not verbose:
        cmd.append("-s")
    subprocess.check_call(cmd)
    if not os.path.exists(LIB):
        raise RuntimeError("build did not produce %s" % LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
