#!/bin/bash
# Rotated DB + head filter (k3p_variant 16/17): focused parity tests, then the cfg3 bench line
# and its per-level kernel breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "16 or 17 or pruned or default" > gpurun_out/pytest_hf.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_hf.log; exit 1; }
tail -1 gpurun_out/pytest_hf.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_hf.json 2> gpurun_out/bench_hf.err || { echo "bench failed"; tail -20 gpurun_out/bench_hf.err; exit 1; }
cat gpurun_out/bench_hf.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hf -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_hf.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/prof_hf/run_kernel_trace.csv 1 > gpurun_out/breakdown_hf.txt 2>&1 || true
tail -5 gpurun_out/breakdown_hf.txt
echo ALL-OK
