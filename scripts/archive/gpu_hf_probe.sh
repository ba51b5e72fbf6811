#!/bin/bash
# HF pruned scan: phase split of the plateau launch (PROBE=16 build, s_memtime stamps) for
# k3p_variant 16 and 14 on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
for v in 16 14; do
  IA_LIBIA=$R/image-analogies-python_amd/libia_probe16.so timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --k3p-variant $v > gpurun_out/probe_v$v.json 2> gpurun_out/probe_v$v.err || { echo "probe $v failed"; tail -5 gpurun_out/probe_v$v.err; exit 1; }
  echo "v$v"; grep K3P_PROBE gpurun_out/probe_v$v.err | tail -3
done
echo ALL-OK
