#!/bin/bash
# Product build: full GPU suite + smoke; DIAG build (libia_diag.so): the rotated-DB variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out/diagcheck
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/diagcheck/pytest_product.log 2>&1 || { echo "product pytest failed"; tail -30 gpurun_out/diagcheck/pytest_product.log; exit 1; }
tail -1 gpurun_out/diagcheck/pytest_product.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/diagcheck/smoke.log 2>&1 || { echo "smoke failed"; tail -10 gpurun_out/diagcheck/smoke.log; exit 1; }
cat gpurun_out/diagcheck/smoke.log | tail -1
IA_LIBIA=$R/image-analogies-python_amd/libia_diag.so timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -k "16 or 17" > gpurun_out/diagcheck/pytest_diag.log 2>&1 || { echo "diag pytest failed"; tail -30 gpurun_out/diagcheck/pytest_diag.log; exit 1; }
tail -1 gpurun_out/diagcheck/pytest_diag.log
echo ALL-OK
