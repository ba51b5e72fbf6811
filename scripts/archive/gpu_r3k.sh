#!/bin/bash
# round 3, session K: full GPU suite + smoke after the exchange changes, the IPC rehearsal, the
# emulated owner-computes model at W = 2, 4 (W = 8 in session J) and the cfg3 / cfg4 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/k
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/xchg_rehearsal.py > gpurun_out/k/xchg_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/k/xchg_rehearsal.log; exit 1; }
grep -E "XCHG" gpurun_out/k/xchg_rehearsal.log
WS="2 4" bash scripts/gpu_shardmodel.sh > gpurun_out/k/model.log 2>&1 || { echo "model failed"; tail gpurun_out/k/model.log; exit 1; }
grep -E "weak|job:" gpurun_out/k/model.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 15 > gpurun_out/k/bench.json 2> gpurun_out/k/bench.err || { echo "bench failed"; tail -20 gpurun_out/k/bench.err; exit 1; }
cut -c1-200 gpurun_out/k/bench.json
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/k/cfg4.json 2> gpurun_out/k/cfg4.err || { echo "cfg4 failed"; tail -20 gpurun_out/k/cfg4.err; exit 1; }
cut -c1-200 gpurun_out/k/cfg4.json
echo R3K-OK
