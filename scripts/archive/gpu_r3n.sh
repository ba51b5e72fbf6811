#!/bin/bash
# round 3, session N: K3p tail (candidate rows looked up before the subset merge): parity tests,
# the v20 phase probe with the tail's barrier wait, same-box A/B against the late lookup
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/n
timeout -k 10 600 python -u -m pytest tests/test_gpu_debug.py tests/test_gpu_prune.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/n/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/n/pytest.log; exit 1; }
tail -1 gpurun_out/n/pytest.log
PVARIANTS=20 bash scripts/gpu_k3p_probe.sh > gpurun_out/n/probe.log 2>&1 || { echo probe failed; tail gpurun_out/n/probe.log; exit 1; }
grep K3P_PROBE gpurun_out/n/probe.log
b() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  IA_LIBIA=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/n/$tag.json 2> gpurun_out/n/$tag.err || { echo "$tag failed"; tail -8 gpurun_out/n/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/n/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']), round(d['ms_per_step'], 1), round(d['roofline'].get('k3_us_per_launch'), 2))"
}
P=$PWD/image-analogies-python_amd/libia.so; L=$PWD/diag/libia_late.so
b early1 $P --steps 3 --warmup 1 && b late1 $L --steps 3 --warmup 1 && b early2 $P --steps 3 --warmup 1 && b late2 $L --steps 3 --warmup 1 || exit 1
echo R3N-OK
