#!/bin/bash
# round 3, session M: fallback rehearsal of the N = 2 bench (session L), the v20 phase probe at
# the cfg3 plateau, and cfg4's PMC traffic with the one-launch two-block scan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_r3l.sh || exit 1
PVARIANTS=20 bash scripts/gpu_k3p_probe.sh || exit 1
timeout -k 10 500 bash tools/pmc_k3p.sh gpurun_out/pmc_cfg4 cfg4 k3h_prune3 || exit 1
python3 tools/k3p_traffic.py gpurun_out/pmc_cfg4 gpurun_out/k3p_traffic_cfg4.json cfg4 8189 > gpurun_out/k3p_traffic_cfg4.txt 2>&1 || { echo "traffic failed"; tail gpurun_out/k3p_traffic_cfg4.txt; exit 1; }
tail -4 gpurun_out/k3p_traffic_cfg4.txt
echo R3M-OK
