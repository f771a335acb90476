#!/bin/bash
# The default bench line (with CPU baselines) and a rocprofv3 kernel-trace + stats of the same bench,
# reading the committed profiles/pmc_*.json (refresh those with tools/refresh_profiles.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-benchprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-aux > "$OUT/rocprof.log" 2>&1
