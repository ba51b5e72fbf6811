#!/bin/bash
# round 3, session AC: fused merge + gather restricted to pruned levels again (unpruned opt-in):
# batch / pipeline / prune / debug parity, then cfg3 / cfg5 A/B of fuse_unpruned
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ac
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_debug.py tests/test_gpu_pipeline.py tests/test_gpu_prune.py tests/test_gpu_shard.py > gpurun_out/ac/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ac/pytest.log; exit 1; }
tail -1 gpurun_out/ac/pytest.log
for pass in 1 2; do
  for cfg in cfg3 cfg5; do
    for fu in 0 1; do
      f=gpurun_out/ac/${cfg}_u${fu}_$pass
      st=3; [ $cfg = cfg5 ] && st=1
      timeout -k 10 200 python -u bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline --fuse-unpruned $fu > $f.json 2> $f.err || { echo "bench $cfg $fu failed"; tail -20 $f.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
    done
  done
done
echo R3AC-OK
