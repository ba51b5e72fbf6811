#!/bin/bash
# Same-box A/B: waves per workgroup of the one-wave-per-query kernels (K2h, K2p, K4): 4 (this
# build) vs 1 and 2 (libia_wpb1.so, libia_wpb2.so), after the parity subset on the WPB=1 build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out/wpb
IA_LIBIA=$R/image-analogies-python_amd/libia_wpb1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_prune.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not 12 and not 13" > gpurun_out/wpb/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/wpb/pytest.log; exit 1; }
tail -1 gpurun_out/wpb/pytest.log
for i in 1 2; do
  for v in 4 1 2; do
    lib=$R/image-analogies-python_amd/libia.so
    [ $v != 4 ] && lib=$R/image-analogies-python_amd/libia_wpb$v.so
    IA_LIBIA=$lib timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/wpb/w${v}_$i.json 2> gpurun_out/wpb/w${v}_$i.err || { echo "bench $v failed"; tail -3 gpurun_out/wpb/w${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/wpb/w${v}_$i.json')); print('wpb $v', round(d['value']), round(d['ms_per_step'],1))"
  done
done
echo ALL-OK
