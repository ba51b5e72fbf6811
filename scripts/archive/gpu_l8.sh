#!/bin/bash
# Full GPU suite, then the cfg3 bench line with the default prune threshold (1024^2 level) and
# with the 512^2 level pruned too, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for pm in 524288 262144 524288 262144; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --prune-min-rows $pm > gpurun_out/b_pm$pm.json 2> gpurun_out/b_pm$pm.err || { echo "bench $pm failed"; tail -5 gpurun_out/b_pm$pm.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_pm$pm.json')); print($pm, round(d['value']), round(d['ms_per_step'],1))"
done
echo ALL-OK1
# K4 cost of the certification rescans: level-9 merge time unpruned (about 105 rescans per job)
# vs pruned (about 7,500)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p0 -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --prune 0 > gpurun_out/b_p0.json 2> gpurun_out/b_p0.err || { echo "prune0 failed"; exit 1; }
python3 tools/trace_breakdown.py gpurun_out/prof_p0/run_kernel_trace.csv 1 > gpurun_out/breakdown_p0.txt 2>&1 || true
grep -E "finest" gpurun_out/breakdown_p0.txt
echo ALL-OK2
