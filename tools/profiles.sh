#!/bin/bash
# Round-end evidence: PMC passes over the 8-view step and the single view (tools/pmc_views.sh), then
# rocprofv3 --kernel-trace --stats (CSV) of the default bench step and of the single-view bench.
# Each GPU step under its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/pmc_views.sh "$TAG/pmc_step" > "$OUT/pmc_step.log" 2>&1 || { tail -20 "$OUT/pmc_step.log"; exit 1; }
BENCH_ARGS="--views-total 1 --per-view --no-deferred" bash tools/pmc_views.sh "$TAG/pmc_single" > "$OUT/pmc_single.log" 2>&1 \
    || { tail -20 "$OUT/pmc_single.log"; exit 1; }
echo "pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks_step" -o run -- python3 bench.py \
    --steps 20 --warmup 3 --no-cpu-baseline --no-aux --no-pmc --no-single-view > "$OUT/ks_step.log" 2>&1 \
    || { tail -20 "$OUT/ks_step.log"; exit 1; }
grep '^{' "$OUT/ks_step.log" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks_single" -o run -- python3 bench.py \
    --views-total 1 --per-view --no-deferred --steps 40 --warmup 5 --no-cpu-baseline --no-aux --no-pmc --no-single-view \
    > "$OUT/ks_single.log" 2>&1 || { tail -20 "$OUT/ks_single.log"; exit 1; }
grep '^{' "$OUT/ks_single.log" | cut -c1-200
