#!/bin/bash
# round-6 final evidence, part A: the GPU suite + smoke, the PMC traffic of the cfg3 scan (bench's
# roofline.traffic), the default bench line, and the rocprofv3 kernel trace of the same command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 bash tools/pmc_k3p.sh $O/pmc3 cfg3 k3h_prune3 --pipeline 0 || exit 1
python3 tools/k3p_traffic.py $O/pmc3 profiles/k3p_traffic_cfg3.json cfg3 4093 > $O/traffic3.txt 2>&1 || { echo "traffic3 failed"; tail $O/traffic3.txt; exit 1; }
cp profiles/k3p_traffic_cfg3.json $O/ ; rm -rf $O/pmc3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { echo "bench cfg3 failed"; tail -20 $O/bench_cfg3.err; exit 1; }
cat $O/bench_cfg3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
python3 tools/trace_breakdown.py $O/prof/run_kernel_trace.csv 1 > $O/breakdown.txt 2>&1 || true
python3 tools/pipe_trace.py $O/prof/run_kernel_trace.csv > $O/pipe_trace.txt 2>&1 || true
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv; rm -rf $O/prof
echo ALL-OK
