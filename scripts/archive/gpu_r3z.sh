#!/bin/bash
# round 3, session Z: the fused merge + gather in owner-computes steps: shard / pipeline / prune
# parity tests, the N = 2 owner path on one GPU (IPC, ranks on CU halves), then the emulated
# per-rank model (tools/shard_model.py) for W = 1 2 4 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/z
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_pipeline.py tests/test_gpu_prune.py > gpurun_out/z/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/z/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/z/pytest.log
bash scripts/gpu_r3l.sh || exit 1
mkdir -p gpurun_out/z/l && cp gpurun_out/l/* gpurun_out/z/l/
bash scripts/gpu_shardmodel.sh > gpurun_out/z/shardmodel.txt 2>&1 || { echo "shard model failed"; tail -20 gpurun_out/z/shardmodel.txt; exit 1; }
grep -E "^job|weak|speedup" gpurun_out/z/shardmodel.txt
mkdir -p gpurun_out/z/shard && cp gpurun_out/shard/* gpurun_out/z/shard/
echo R3Z-OK
