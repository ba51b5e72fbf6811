#!/bin/bash
# A/B profile on one box: cfg3 default, row_source 1, variant 11, shard emulation 2/4/8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=cfg3 bash scripts/gpu_prof.sh || exit 1
TAG=cfg3_row1 bash scripts/gpu_prof.sh --row-source 1 || exit 1
TAG=cfg3_v11 bash scripts/gpu_prof.sh --k3p-variant 11 || exit 1
for W in 2 4 8; do TAG=shard$W bash scripts/gpu_prof.sh --shard-emulate $W || exit 1; done
IA_LIBIA=image-analogies-python_amd/libia_probe32.so TAG=probe32 bash scripts/gpu_prof.sh || echo "probe32 failed (diagnostic only)"
echo ALL-OK
