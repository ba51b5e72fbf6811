#!/bin/bash
# round 3, session H: cost model of bench.py's N > 1 shard mode (W jobs over W emulated shards)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_shardmodel.sh || exit 1
echo R3H-OK
