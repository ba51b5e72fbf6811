#!/bin/bash
# round 3, session A: peer-write exchange checks + bench line, then the K3p product / probe /
# variant traces (cfg3, cfg4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_xchg.sh && bash scripts/gpu_probe32.sh && echo R3A-OK
