#!/bin/bash
# One GPU-box session: parity tests, the bench line for both matchers, a rocprofv3 kernel trace.
# usage (from this container): gpurun --timeout 1100 -- bash scripts/gpu_check.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-seconds 15 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --matcher f32 --no-cpu-baseline > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err || { echo "bench f32 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo ALL-OK
