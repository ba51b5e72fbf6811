#!/bin/bash
# One GPU-box session for the round's evidence: parity tests, smoke, the bench line, the
# rocprofv3 kernel trace of the same command, and the PMC passes of the dominant kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 200 bash tools/pmc_k3p.sh gpurun_out/pmc_k3p || exit 1
python3 tools/k3p_traffic.py gpurun_out/pmc_k3p profiles/k3p_traffic_cfg3.json cfg3 4093 > gpurun_out/k3p_traffic.txt 2>&1 || { echo "traffic failed"; tail gpurun_out/k3p_traffic.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 15 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/prof/run_kernel_trace.csv 1 > gpurun_out/breakdown.txt 2>&1 || true
echo ALL-OK
