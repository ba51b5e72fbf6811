#!/bin/bash
# Round-2 check: GPU suite (batch, shard emulation, presorted K3p), bench lines for cfg3 (v7 and
# v11), cfg4, cfg5, and rocprofv3 kernel traces of the W-way shard emulation (cost model).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
$B --steps 3 --warmup 1 > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err || { echo "bench cfg3 failed"; tail -20 gpurun_out/bench_cfg3.err; exit 1; }
$B --steps 3 --warmup 1 --k3p-variant 11 > gpurun_out/bench_cfg3_v11.json 2> gpurun_out/bench_cfg3_v11.err || { echo "bench cfg3 v11 failed"; tail -20 gpurun_out/bench_cfg3_v11.err; exit 1; }
$B --steps 3 --warmup 1 --row-source 1 > gpurun_out/bench_cfg3_row1.json 2> gpurun_out/bench_cfg3_row1.err || { echo "bench cfg3 row1 failed"; tail -20 gpurun_out/bench_cfg3_row1.err; exit 1; }
$B --steps 3 --warmup 1 --row-source 1 --k3p-variant 11 > gpurun_out/bench_cfg3_row1_v11.json 2> gpurun_out/bench_cfg3_row1_v11.err || { echo "bench cfg3 row1 v11 failed"; tail -20 gpurun_out/bench_cfg3_row1_v11.err; exit 1; }
$B --config cfg4 --steps 2 --warmup 1 > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { echo "bench cfg4 failed"; tail -20 gpurun_out/bench_cfg4.err; exit 1; }
$B --config cfg5 --steps 1 --warmup 1 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { echo "bench cfg5 failed"; tail -20 gpurun_out/bench_cfg5.err; exit 1; }
for W in 2 4 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shard$W -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --shard-emulate $W > gpurun_out/bench_shard$W.json 2> gpurun_out/bench_shard$W.err || { echo "shard $W failed"; tail -20 gpurun_out/bench_shard$W.err; exit 1; }
  python3 tools/trace_breakdown.py gpurun_out/shard$W/run_kernel_trace.csv 1 > gpurun_out/breakdown_shard$W.txt 2>&1 || true
done
# timing-only diagnostic: K3p with one f16 product per 16 k instead of three (a single-pass
# prefilter's MFMA cost); its decisions are not certified, only the kernel time is read
IA_LIBIA=image-analogies-python_amd/libia_probe32.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/bench_probe32.json 2> gpurun_out/bench_probe32.err || echo "probe32 failed (diagnostic only)"
for f in cfg3 cfg3_v11 cfg3_row1 cfg3_row1_v11 cfg4 cfg5 shard2 shard4 shard8 probe32; do echo "$f $(cut -c1-200 gpurun_out/bench_$f.json)"; done
echo ALL-OK
