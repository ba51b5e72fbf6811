#!/bin/bash
# GPU suite, then an A/B profile on one box: cfg3 default, row_source 1, variant 11, shard
# emulation 2/4/8, the single-product diagnostic build; cfg5 batched with the 512^2 level pruned.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
TAG=cfg3 bash scripts/gpu_prof.sh || exit 1
TAG=cfg3_row1 bash scripts/gpu_prof.sh --row-source 1 || exit 1
TAG=cfg3_v11 bash scripts/gpu_prof.sh --k3p-variant 11 || exit 1
for W in 2 4 8; do TAG=shard$W bash scripts/gpu_prof.sh --shard-emulate $W || exit 1; done
TAG=cfg5_prune bash scripts/gpu_prof.sh --config cfg5 --prune-min-rows 262144 || exit 1
IA_LIBIA=image-analogies-python_amd/libia_probe32.so TAG=probe32 bash scripts/gpu_prof.sh || echo "probe32 failed (diagnostic only)"
echo ALL-OK
