#!/bin/bash
# Kernel trace (timestamps) of a short default bench run, for the view-overlap timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-trace}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-aux --no-pmc --no-profile ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; grep '^{' "$OUT/bench.log" | cut -c1-200; exit $rc
