#!/bin/bash
# round 6: the new tests (slim reference fixtures; the two-rank cfg5 sweep rehearsed on one GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k slim -x -v --timeout 250 --timeout-method thread > $O/slim.log 2>&1 || { echo "slim failed"; tail -30 $O/slim.log; exit 1; }
tail -3 $O/slim.log
IA_TEST_SHARE_GPU=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -k cfg5 -x -v --timeout 850 --timeout-method thread > $O/mr.log 2>&1 || { echo "multirank failed"; tail -40 $O/mr.log; exit 1; }
tail -3 $O/mr.log
