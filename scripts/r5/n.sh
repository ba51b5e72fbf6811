#!/bin/bash
# round 5: the phase probe of the current pruned scan (sequential cfg3, 8 sampled workgroups)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5n; mkdir -p $O
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -20 $O/probe.err; exit 1; }
grep K3P_PROBE $O/probe.err | tail -7
echo ALL-OK
