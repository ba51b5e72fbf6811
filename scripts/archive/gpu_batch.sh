#!/bin/bash
# Batched levels / sweeps / cfg4: GPU parity tests, then bench lines for cfg3, cfg5 (batched and
# one job at a time) and cfg4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err || { echo "bench cfg3 failed"; tail -20 gpurun_out/bench_cfg3.err; exit 1; }
cat gpurun_out/bench_cfg3.json
timeout -k 10 300 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { echo "bench cfg5 failed"; tail -20 gpurun_out/bench_cfg5.err; exit 1; }
cat gpurun_out/bench_cfg5.json
timeout -k 10 300 python -u bench.py --config cfg5 --sequential --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg5_seq.json 2> gpurun_out/bench_cfg5_seq.err || { echo "bench cfg5 seq failed"; tail -20 gpurun_out/bench_cfg5_seq.err; exit 1; }
cat gpurun_out/bench_cfg5_seq.json
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { echo "bench cfg4 failed"; tail -20 gpurun_out/bench_cfg4.err; exit 1; }
cat gpurun_out/bench_cfg4.json
echo ALL-OK
