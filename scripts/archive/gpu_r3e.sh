#!/bin/bash
# round 3, session E: parity suite + smoke (refactored exchange merge), the two-process
# exchange rehearsal, then the emulated-shard cost model (only pruned levels sharded)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/xchg_rehearsal.py > gpurun_out/xchg_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/xchg_rehearsal.log; exit 1; }
grep -E "XCHG" gpurun_out/xchg_rehearsal.log
bash scripts/gpu_shardmodel.sh && echo R3E-OK
