#!/bin/bash
# round 3, session V: fused K4(t) + K2p(t + 1) (k_merge_gather): parity tests, then bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/v
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_debug.py tests/test_gpu_pipeline.py tests/test_gpu_prune.py > gpurun_out/v/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/v/pytest.log; exit 1; }
tail -3 gpurun_out/v/pytest.log
for pass in 1 2; do
  for v in "1 4" "0 4"; do
    set -- $v
    f=gpurun_out/v/f$1_c$2_$pass
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --fuse-gather $1 --pipe-ctx $2 --pipe-priority 1 > $f.json 2> $f.err || { echo "bench $v failed"; tail -20 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1), d['config']['level_pipeline'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pv -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipeline 0 > gpurun_out/v/seq.json 2> gpurun_out/v/seq.err || { echo "trace failed"; tail -5 gpurun_out/v/seq.err; exit 1; }
cp /tmp/pv/run_kernel_stats.csv gpurun_out/v/kernel_stats_seq.csv
python3 tools/trace_breakdown.py /tmp/pv/run_kernel_trace.csv 1 > gpurun_out/v/breakdown_seq.txt 2>&1
grep -E "^level 9|finest level|^total" gpurun_out/v/breakdown_seq.txt | cut -c1-300
echo R3V-OK
