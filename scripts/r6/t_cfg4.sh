#!/bin/bash
# wide-step changes: the wide-step / presorted tests, cfg4 teacher forcing, then the cfg4 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-t_cfg4}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py > $O/t_suites.log 2>&1 || { echo "suites failed"; tail -30 $O/t_suites.log; exit 1; }
tail -1 $O/t_suites.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 500 --timeout-method thread -k "cfg4" > $O/t_cfg4.log 2>&1 || { echo "cfg4 tests failed"; tail -30 $O/t_cfg4.log; exit 1; }
tail -1 $O/t_cfg4.log
bash scripts/r6/ab_cfg4.sh ${1:-t_cfg4}/ab "def|"
