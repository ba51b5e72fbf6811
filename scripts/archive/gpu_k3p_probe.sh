#!/bin/bash
# Diagnostic: phase cycles of the pruned scan at the 1024^2 plateau (PROBE=16 build in diag/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${PVARIANTS:-4}; do
  IA_LIBIA=$PWD/diag/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --k3p-variant $v > gpurun_out/probe_v$v.json 2> gpurun_out/probe_v$v.err || { echo "probe $v failed"; tail -20 gpurun_out/probe_v$v.err; exit 1; }
  echo "== variant $v"; grep K3P_PROBE gpurun_out/probe_v$v.err || true
done
echo ALL-OK
