#!/bin/bash
# rocprofv3 kernel-trace + stats over a short bench run (no PMC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-rp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile > "$OUT/rocprof.log" 2>&1
rc=$?; grep '^{' "$OUT/rocprof.log" | cut -c1-200; exit $rc
