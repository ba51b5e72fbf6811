#!/bin/bash
# k3p_variant 22 / 23 (hi-only DB stream): parity tests, then same-box A/B against 20 / 21
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_debug.py -m gpu -x -q --timeout 300 --timeout-method thread -k "22 or 23" > $O/pytest_v22.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_v22.log; exit 1; }
tail -1 $O/pytest_v22.log
summ() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'frac_t', round(r.get('frac_timed',0),3), 'bytes/launch', round(r.get('algorithmic_bytes_per_launch_timed',0)/1e6,1), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'tiles_pass', round(r.get('tiles_passing_frac',0),3), 'fallbacks', d['stats']['fallbacks'])"; }
for i in 1 2; do
  for v in "v20:" "v22:--k3p-variant 22" "v20seq:--pipeline 0" "v22seq:--pipeline 0 --k3p-variant 22"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline $a > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -20 $O/${n}_$i.err; exit 1; }
    summ $O/${n}_$i.json $n
  done
done
for v in "c4v20:--config cfg4" "c4v22:--config cfg4 --k3p-variant 22"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $a > $O/${n}.json 2> $O/${n}.err || { echo "bench $n failed"; tail -20 $O/${n}.err; exit 1; }
  summ $O/${n}.json $n
done
echo ALL-OK
