#!/bin/bash
# Same-box A/B: this tree (rank-count sort for every in-kernel sorted step + 4-record fused
# merge) vs libia_noA.so (bitonic above 256 queries) vs libia_noC.so (8-record merge), after
# the parity tests of the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/ab3
timeout -k 10 300 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab3/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ab3/pytest.log; exit 1; }
tail -1 gpurun_out/ab3/pytest.log
for i in 1 2; do
  for v in head noA noC; do
    lib=$R/image-analogies-python_amd/libia.so
    [ $v != head ] && lib=$R/image-analogies-python_amd/libia_$v.so
    IA_LIBIA=$lib timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab3/${v}_$i.json 2> gpurun_out/ab3/${v}_$i.err || { echo "bench $v failed"; tail -3 gpurun_out/ab3/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab3/${v}_$i.json')); r=d['roofline']; print('$v', round(d['value']), round(d['ms_per_step'],1), round(r['k3_us_per_launch'],1))"
  done
done
echo ALL-OK
