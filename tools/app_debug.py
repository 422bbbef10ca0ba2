"""Run the C++ app on a generated MMS parameter file with verbose GMRES (debug helper)."""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_app import APP, G, mms_prm  # noqa: E402

pre = sys.argv[1] if len(sys.argv) > 1 else "mg"
d = tempfile.mkdtemp()
open(os.path.join(d, "c.prm"), "w").write(mms_prm(G["mms3d_gls"], 3, 2, 1))
env = dict(os.environ, GLS_GMRES_VERBOSE="1")
r = subprocess.run([APP, "--dim", "3", "--precond", pre, os.path.join(d, "c.prm")], cwd=d, env=env,
                   capture_output=True, text=True, timeout=300)
print(r.stdout[:8000])
print(r.stderr[-3000:])
