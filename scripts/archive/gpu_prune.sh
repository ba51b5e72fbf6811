#!/bin/bash
# Pruned-scan check: the prune parity test, then cfg3 bench with pruning on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_prune.txt 2>&1 || { echo "prune test failed"; tail -40 gpurun_out/pytest_prune.txt; exit 1; }
tail -8 gpurun_out/pytest_prune.txt
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prune.json 2> gpurun_out/bench_prune.err || { echo "bench failed"; tail -20 gpurun_out/bench_prune.err; exit 1; }
cat gpurun_out/bench_prune.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_prune -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_prune.txt 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_prune.txt; exit 1; }
python3 tools/trace_breakdown.py $(ls gpurun_out/prof_prune/*/run_kernel_trace.csv 2>/dev/null || find gpurun_out/prof_prune -name '*kernel_trace.csv' | head -1) 1 > gpurun_out/breakdown_prune.txt 2>&1 || true
tail -4 gpurun_out/breakdown_prune.txt
echo ALL-OK
