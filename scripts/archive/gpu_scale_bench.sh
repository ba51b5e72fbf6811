#!/bin/bash
# Scale parity (teacher forcing cfg2 / cfg3), the cfg3 state dump for offline teacher forcing,
# the bench line and its rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_scale.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_scale.log; exit 1; }
tail -2 gpurun_out/pytest_scale.log
timeout -k 10 200 python -u tools/dump_state.py gpurun_out/cfg3_state.npz 1024 1 2 3 4 5 6 7 8 9 > gpurun_out/dump.log 2>&1 || { echo "dump failed"; tail gpurun_out/dump.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 15 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/prof/run_kernel_trace.csv 1 > gpurun_out/breakdown.txt 2>&1 || true
echo ALL-OK
