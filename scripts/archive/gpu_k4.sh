#!/bin/bash
# K4 / K3p iteration on the default path: pruned-scan parity tests, the cfg3 bench line under
# rocprofv3 and its per-level breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_shard.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "14 or 15 or pruned or default or shard" > gpurun_out/pytest_k4.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_k4.log; exit 1; }
tail -1 gpurun_out/pytest_k4.log
for i in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_k4_$i -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k4_$i.json 2> gpurun_out/bench_k4_$i.err || { echo "bench failed"; tail -5 gpurun_out/bench_k4_$i.err; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/prof_k4_$i/run_kernel_trace.csv 1 > gpurun_out/breakdown_k4_$i.txt 2>&1 || true
python3 -c "import json; d=json.load(open('gpurun_out/bench_k4_$i.json')); print(round(d['value']), round(d['ms_per_step'],1), d['stats']['fallbacks'])"
grep -E "finest" gpurun_out/breakdown_k4_$i.txt
done
echo ALL-OK
