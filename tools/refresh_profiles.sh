#!/bin/bash
# Round-end evidence in one GPU call: PMC passes (HBM traffic, LDS conflicts, VALU/wait counters),
# the default bench line (with CPU baselines), and a rocprofv3 kernel-trace of the same bench.
# Copy the results into profiles/ afterwards.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-refresh}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/profile_pmc.sh "$TAG/pmc" > "$OUT/pmc.log" 2>&1 || { tail -20 "$OUT/pmc.log"; exit 1; }
cp "gpurun_out/$TAG/pmc/pmc_traffic.json" "gpurun_out/$TAG/pmc/pmc_valu.json" profiles/
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-aux --no-pmc > "$OUT/rocprof.log" 2>&1
