#!/bin/bash
# round 3, session AD: same-box cfg3 A/B of three libia builds: the round-3 final2 state, the
# owner-mode fusion commit, and the current tree (generalised fused kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ad
for pass in 1 2; do
  for lib in diag/libia_f2.so diag/libia_own.so image-analogies-python_amd/libia.so; do
    n=$(basename $lib .so)
    f=gpurun_out/ad/${n}_$pass
    IA_LIBIA=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $f.json 2> $f.err || { echo "bench $lib failed"; tail -20 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1))"
  done
done
echo R3AD-OK
