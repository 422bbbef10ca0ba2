# round-5 box K: reference application cases (error tables printed for the pressure-column study)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_app_reference.py -m gpu -v -s -k "test_reference_application_case" --timeout 300 --timeout-method thread > gpurun_out/r05k_ref.log 2>&1
rc=$?; echo "ref rc $rc"; grep -a "ours" gpurun_out/r05k_ref.log | cut -c1-600; exit $rc
