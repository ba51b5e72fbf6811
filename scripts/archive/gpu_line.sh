#!/bin/bash
# The round's measurement set for the current default kernels: GPU suite + smoke, the bench line
# (with the CPU baseline), a rocprofv3 kernel profile of the same command, the PMC passes of the
# pruned scan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/line
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
TAG=line_prof bash scripts/gpu_prof.sh || exit 1
bash tools/pmc_k3p.sh $OUT/pmc || exit 1
python3 tools/k3p_traffic.py $OUT/pmc $OUT/k3p_traffic.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$OUT/k3p_traffic.json')); print({k: d[k] for k in ('hbm_bytes_per_launch', 'plateau_hbm_bytes_per_launch')})"
rm -rf $OUT/pmc
echo ALL-OK
