#!/bin/bash
# round 3, session O: v20 tail split probe; cfg4 line with its own (one-launch) traffic; cfg5 line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/o
PVARIANTS=20 bash scripts/gpu_k3p_probe.sh > gpurun_out/o/probe.log 2>&1 || { echo probe failed; tail gpurun_out/o/probe.log; exit 1; }
grep K3P_PROBE gpurun_out/o/probe.log
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/o/cfg4.json 2> gpurun_out/o/cfg4.err || { echo "cfg4 failed"; tail -20 gpurun_out/o/cfg4.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/o/cfg4.json').read().strip().splitlines()[-1]); r=d['roofline']; print('cfg4', round(d['value']), r['frac'], r['traffic'], r['algorithmic_bytes_per_launch'], r['k3_us_per_launch'])"
timeout -k 10 300 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/o/cfg5.json 2> gpurun_out/o/cfg5.err || { echo "cfg5 failed"; tail -20 gpurun_out/o/cfg5.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/o/cfg5.json').read().strip().splitlines()[-1]); print('cfg5', round(d['value']), round(d['ms_per_step'],1))"
echo R3O-OK
