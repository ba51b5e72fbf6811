#!/bin/bash
# round 3, session C: emulated-shard cost model traces (W = 1, 2, 4, 8), then the cfg3 PMC
# traffic of the pruned scan (profiles/k3p_traffic_cfg3.json) and the cfg3 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_shardmodel.sh || exit 1
timeout -k 10 400 bash tools/pmc_k3p.sh gpurun_out/pmc_cfg3 cfg3 k3h_prune3 || exit 1
python3 tools/k3p_traffic.py gpurun_out/pmc_cfg3 gpurun_out/k3p_traffic_cfg3.json cfg3 4093 > gpurun_out/k3p_traffic_cfg3.txt 2>&1 || { echo "traffic failed"; tail gpurun_out/k3p_traffic_cfg3.txt; exit 1; }
cp gpurun_out/k3p_traffic_cfg3.json profiles/k3p_traffic_cfg3.json
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.json | cut -c1-300
echo R3C-OK
