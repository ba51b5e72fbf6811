#!/bin/bash
# round 3, session AB: the fused merge + gather on unpruned levels and batched jobs too: the
# GPU parity suite, then cfg3 / cfg5 / cfg4 A/B (fuse_gather 1 vs 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
for pass in 1 2; do
  for cfg in cfg3 cfg5; do
    for fg in 1 0; do
      f=gpurun_out/ab/${cfg}_f${fg}_$pass
      st=3; [ $cfg = cfg5 ] && st=1
      timeout -k 10 200 python -u bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline --fuse-gather $fg > $f.json 2> $f.err || { echo "bench $cfg $fg failed"; tail -20 $f.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
    done
  done
done
echo R3AB-OK
