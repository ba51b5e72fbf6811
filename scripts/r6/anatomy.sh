#!/bin/bash
# round 6: launch anatomy of cfg3's pruned levels from raw kernel stamps (tools/stamp_anatomy.py)
#   scripts/r6/anatomy.sh OUT [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
rm -f /tmp/ia_stamps.bin
IA_STAMP_DUMP=/tmp/ia_stamps.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 tools/stamp_anatomy.py /tmp/ia_stamps.bin > $O/anatomy.txt 2>&1 || { echo "anatomy failed"; tail $O/anatomy.txt; exit 1; }
cat $O/anatomy.txt
