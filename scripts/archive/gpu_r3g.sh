#!/bin/bash
# round 3, session G: the one-launch multi-block pruned scan (k3p_blocks) and batched jobs on
# sharded levels: affected GPU tests, then cfg4 A/B (k3p_blocks 1 vs 0) and the cfg3 line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/g
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_prune.py -x -v --timeout 300 --timeout-method thread > gpurun_out/g/pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/g/pytest.log; exit 1; }
tail -3 gpurun_out/g/pytest.log
b() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/g/$tag.json 2> gpurun_out/g/$tag.err || { echo "$tag failed"; tail -8 gpurun_out/g/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/g/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'], 1), d['roofline'].get('k3_us_per_launch'), d['stats']['fallbacks'])"
}
b cfg4_blk --config cfg4 --steps 2 --warmup 1 &&
b cfg4_seq --config cfg4 --steps 2 --warmup 1 --k3p-blocks 0 &&
b cfg3 --steps 3 --warmup 1 &&
b cfg3_j8w8 --steps 1 --warmup 1 --shard-jobs 8 --shard-emulate 8 &&
b cfg3_j8 --steps 1 --warmup 1 --shard-jobs 8 || exit 1
echo R3G-OK
