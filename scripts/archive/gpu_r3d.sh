#!/bin/bash
# round 3, session D: cfg5 pruning thresholds (bench lines), cfg4 bench line, then the cfg4 PMC
# traffic of the pruned scan (profiles/k3p_traffic_cfg4.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/d
b() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/d/$tag.json 2> gpurun_out/d/$tag.err || { echo "$tag failed"; tail -8 gpurun_out/d/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/d/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'], 1), d['roofline'].get('k3_us_per_launch'), d['stats']['pruned_levels'])"
}
b cfg5_def --config cfg5 --steps 1 --warmup 1 &&
b cfg5_p262k --config cfg5 --steps 1 --warmup 1 --prune-min-rows 262144 &&
b cfg5_p65k --config cfg5 --steps 1 --warmup 1 --prune-min-rows 65536 &&
b cfg4 --config cfg4 --steps 2 --warmup 1 &&
b cfg3_p262k --steps 3 --warmup 1 --prune-min-rows 262144 || exit 1
timeout -k 10 500 bash tools/pmc_k3p.sh gpurun_out/pmc_cfg4 cfg4 k3h_prune3 || exit 1
python3 tools/k3p_traffic.py gpurun_out/pmc_cfg4 gpurun_out/k3p_traffic_cfg4.json cfg4 16378 > gpurun_out/k3p_traffic_cfg4.txt 2>&1 || { echo "traffic failed"; tail gpurun_out/k3p_traffic_cfg4.txt; exit 1; }
echo R3D-OK
