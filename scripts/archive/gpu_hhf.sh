#!/bin/bash
# hi x hi block filter (k3p_variant 14/15): exactness tests, then a same-box A/B against v7 and
# a kernel profile of cfg3 with it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/hhf
timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/hhf/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/hhf/pytest.log; exit 1; }
tail -2 gpurun_out/hhf/pytest.log
grep -h "corrected pairs" gpurun_out/hhf/pytest.log | head -8
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/hhf/v7_$i.json 2> gpurun_out/hhf/v7_$i.err || { echo "v7 bench failed"; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --k3p-variant 14 > gpurun_out/hhf/v14_$i.json 2> gpurun_out/hhf/v14_$i.err || { echo "v14 bench failed"; tail -5 gpurun_out/hhf/v14_$i.err; exit 1; }
done
for f in gpurun_out/hhf/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); r=d['roofline']; print(round(d['value']), round(d['ms_per_step'],1), round(r.get('k3_us_per_launch',0),1), round(r.get('pairs_corrected_frac',0),3), d['stats']['bound_violations'])")"; done
TAG=cfg3_v14 bash scripts/gpu_prof.sh --k3p-variant 14 || exit 1
TAG=cfg4_v14 bash scripts/gpu_prof.sh --config cfg4 --k3p-variant 14 || exit 1
echo ALL-OK
