#!/bin/bash
# round 3, session AE: pipelining overheads: skip waits on completed events, no per-step events on
# the finest level (nothing depends on it) - same box against the previous build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ae
for pass in 1 2; do
  f=gpurun_out/ae/old_$pass
  IA_PIPE_RECORD_ALL=1 IA_LIBIA=$PWD/diag/libia_head3.so timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $f.json 2> $f.err || { echo "old failed"; tail -20 $f.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
  f=gpurun_out/ae/new_$pass
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $f.json 2> $f.err || { echo "new failed"; tail -20 $f.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/ae/pytest.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/ae/pytest.log; exit 1; }
tail -1 gpurun_out/ae/pytest.log
echo R3AE-OK
