#!/bin/bash
# round 3, session F (re-entry): HEAD parity suite + smoke, then the cfg3 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 15 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo R3F-OK
