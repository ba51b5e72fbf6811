#!/bin/bash
# prune exactness + variant benches + (optional) probe of one variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
VARIANTS="${VARIANTS:-4 5}" bash scripts/gpu_k3p.sh || exit 1
PVARIANTS="${PVARIANTS:-5}" bash scripts/gpu_k3p_probe.sh || exit 1
