#!/bin/bash
# work stealing: the stealing exactness test, then the bench A/B against the round's base library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-steal}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prune.py -k "stealing" -s > $O/t_steal.log 2>&1 || { echo "steal test failed"; tail -30 $O/t_steal.log; exit 1; }
grep -E "stolen|passed|failed" $O/t_steal.log | tail -3
bash scripts/r6/ab_runs.sh ${1:-steal}/ab "head|libia_head.so|" "s0|libia.so|--steal 0" "s1|libia.so|--steal 1" "s1seq|libia.so|--steal 1 --pipeline 0"
