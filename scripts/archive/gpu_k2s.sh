#!/bin/bash
# K2s over one workgroup per sorted query tile: presorted-scan parity (variants 11 / 15, wide
# batched steps, cfg4 teacher forcing), then the cfg4 line and its breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/k2s
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_batch.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "11 or 15 or wide or cfg4" > gpurun_out/k2s/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/k2s/pytest.log; exit 1; }
tail -1 gpurun_out/k2s/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k2s/prof -o run -- python3 -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/k2s/cfg4.json 2> gpurun_out/k2s/cfg4.err || { echo "cfg4 failed"; tail -5 gpurun_out/k2s/cfg4.err; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/k2s/prof/run_kernel_trace.csv 1 > gpurun_out/k2s/breakdown.txt 2>&1
python3 -c "import json; d=json.load(open('gpurun_out/k2s/cfg4.json')); print('cfg4', round(d['value']), round(d['ms_per_step'],1))"
grep "^level 9" gpurun_out/k2s/breakdown.txt | cut -c1-300
echo ALL-OK
