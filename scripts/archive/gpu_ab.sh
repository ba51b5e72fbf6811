#!/bin/bash
# GPU suite, then an A/B profile on one box: cfg3 default, row_source 1, variant 11, shard
# emulation 2/4/8, the single-product diagnostic build; cfg5 batched with the 512^2 level pruned.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
# same-box A/B of the bench line: this tree vs round-2 start (ab_base = commit 982ab14 worktree)
mkdir -p gpurun_out/ab
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/head_$i.json 2> gpurun_out/ab/head_$i.err || { echo "head bench failed"; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --k3p-variant 12 > gpurun_out/ab/v12_$i.json 2> gpurun_out/ab/v12_$i.err || { echo "v12 bench failed"; tail -5 gpurun_out/ab/v12_$i.err; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --k3p-variant 13 > gpurun_out/ab/v13_$i.json 2> gpurun_out/ab/v13_$i.err || { echo "v13 bench failed"; tail -5 gpurun_out/ab/v13_$i.err; exit 1; }
  if [ -d ab_base ]; then (cd ab_base && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > ../gpurun_out/ab/base_$i.json 2> ../gpurun_out/ab/base_$i.err) || echo "base bench failed"; fi
done
for f in gpurun_out/ab/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(round(d['value']), round(d['ms_per_step'],1), round(d['roofline'].get('k3_us_per_launch',0),1))")"; done
TAG=cfg3 bash scripts/gpu_prof.sh || exit 1
TAG=cfg3_v12 bash scripts/gpu_prof.sh --k3p-variant 12 || exit 1
TAG=cfg3_v13 bash scripts/gpu_prof.sh --k3p-variant 13 || exit 1
TAG=cfg4_v13 bash scripts/gpu_prof.sh --config cfg4 --k3p-variant 13 || exit 1
TAG=cfg4 bash scripts/gpu_prof.sh --config cfg4 || exit 1
TAG=cfg5 bash scripts/gpu_prof.sh --config cfg5 || exit 1
echo ALL-OK
