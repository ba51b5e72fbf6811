#!/bin/bash
# round 3, session B: the GPU parity suite + smoke, then the pruned-scan variant traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_tests.sh && bash scripts/gpu_variants.sh && echo R3B-OK
