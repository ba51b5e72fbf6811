#!/bin/bash
# cfg5 over several libia contexts (HIP streams + host threads): parity test, then the bench line
# with 1, 2 and 3 streams on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/streams
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread -k "two_streams or sweep" > gpurun_out/streams/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/streams/pytest.log; exit 1; }
tail -1 gpurun_out/streams/pytest.log
for s in 1 2 3 2 1; do
  timeout -k 10 300 python -u bench.py --config cfg5 --streams $s --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/streams/s$s.json 2> gpurun_out/streams/s$s.err || { echo "bench $s failed"; tail -5 gpurun_out/streams/s$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/streams/s$s.json')); print($s, round(d['value']), round(d['ms_per_step'],1))"
done
echo ALL-OK
