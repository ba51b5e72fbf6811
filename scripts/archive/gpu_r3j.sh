#!/bin/bash
# round 3, session J: owner-computes hand-offs with store-completion waits instead of system
# fences: shard tests, the IPC rehearsal, the emulated model at W = 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/j
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -v -k "owner or batched" --timeout 300 --timeout-method thread > gpurun_out/j/pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/j/pytest.log; exit 1; }
tail -1 gpurun_out/j/pytest.log
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/xchg_rehearsal.py > gpurun_out/j/xchg_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/j/xchg_rehearsal.log; exit 1; }
grep -E "XCHG" gpurun_out/j/xchg_rehearsal.log
WS="${WS:-8}" bash scripts/gpu_shardmodel.sh || exit 1
echo R3J-OK
