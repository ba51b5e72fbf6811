#!/bin/bash
# round 3, session X: the fused merge + gather on presorted wide steps too: parity tests, cfg4 / cfg3 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/x
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_debug.py tests/test_gpu_prune.py tests/test_gpu_scale.py tests/test_gpu_batch.py tests/test_gpu_parity.py > gpurun_out/x/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/x/pytest.log; exit 1; }
tail -3 gpurun_out/x/pytest.log
for pass in 1 2; do
  for cfg in cfg4 cfg3; do
    for fg in 1 0; do
      f=gpurun_out/x/${cfg}_f${fg}_$pass
      timeout -k 10 200 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --fuse-gather $fg > $f.json 2> $f.err || { echo "bench $cfg $fg failed"; tail -20 $f.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1), d['config']['level_pipeline'])"
    done
  done
done
echo R3X-OK
