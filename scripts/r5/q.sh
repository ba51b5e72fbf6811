#!/bin/bash
# round 5: the fused merge + gather's phase stamps (make PROBE=8: one sampled wave every 256
# steps of each level, printf), sequential and pipelined cfg3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5q; mkdir -p $O
for p in 0 1; do
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe8.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline $p > $O/probe8_p$p.json 2> $O/probe8_p$p.err || { echo "probe failed"; tail -20 $O/probe8_p$p.err; exit 1; }
grep -c "STAMP" $O/probe8_p$p.err
done
echo ALL-OK
