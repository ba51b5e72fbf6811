#!/bin/bash
# round 3, session Q: level pipelining (two contexts, per-step event waits): tests, then the
# cfg3 / cfg4 lines with and without it on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/q/pytest.log; exit 1; }
tail -1 gpurun_out/q/pytest.log
b() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/q/$tag.json 2> gpurun_out/q/$tag.err || { echo "$tag failed"; tail -8 gpurun_out/q/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/q/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'], 1), round(d['roofline'].get('k3_us_per_launch'), 2))"
}
b seq1 --steps 3 --warmup 1 && b pipe1 --steps 3 --warmup 1 --pipeline 1 && b seq2 --steps 3 --warmup 1 && b pipe2 --steps 3 --warmup 1 --pipeline 1 &&
b cfg4_seq --config cfg4 --steps 2 --warmup 1 && b cfg4_pipe --config cfg4 --steps 2 --warmup 1 --pipeline 1 || exit 1
echo R3Q-OK
