#!/bin/bash
# Pruned-scan kernel versions: exactness (prune test, every k3p_variant) then one profiled cfg3
# job per variant (per-level kernel breakdown under gpurun_out/k3p_v*/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_prune.txt 2>&1 || { echo "prune test failed"; tail -40 gpurun_out/pytest_prune.txt; exit 1; }
grep -E "pairs left|passed|failed" gpurun_out/pytest_prune.txt
for v in ${VARIANTS:-0 1 2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k3p_v$v -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --k3p-variant $v > gpurun_out/k3p_v$v.json 2> gpurun_out/k3p_v$v.err || { echo "variant $v failed"; tail -20 gpurun_out/k3p_v$v.err; exit 1; }
  python3 tools/trace_breakdown.py gpurun_out/k3p_v$v/run_kernel_trace.csv 1 > gpurun_out/k3p_v$v.txt 2>&1 || true
  echo "== variant $v"; tail -3 gpurun_out/k3p_v$v.txt
done
echo ALL-OK
