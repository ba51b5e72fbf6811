#!/bin/bash
# round 3, session T: pipelining with 3/4/5 contexts (+ priority); kernel trace of the 3- and
# 2-context runs through tools/pipe_trace.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/t
for pass in 1 2; do
  for v in "3 1" "4 1" "5 1" "4 0"; do
    set -- $v
    f=gpurun_out/t/c$1_p$2_$pass
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pipe-ctx $1 --pipe-priority $2 > $f.json 2> $f.err || { echo "bench $v failed"; tail -20 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],1), d['config']['level_pipeline'])"
  done
done
for c in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt$c -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipe-ctx $c --pipe-priority 1 > gpurun_out/t/trace_c$c.json 2> gpurun_out/t/trace_c$c.err || { echo "trace $c failed"; tail -5 gpurun_out/t/trace_c$c.err; exit 1; }
  head -1 /tmp/pt$c/run_kernel_trace.csv > gpurun_out/t/trace_header.txt
  python3 tools/pipe_trace.py /tmp/pt$c/run_kernel_trace.csv > gpurun_out/t/pipe_c$c.txt 2>&1
  cat gpurun_out/t/pipe_c$c.txt
  rm -rf /tmp/pt$c
done
echo R3T-OK
