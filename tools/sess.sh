#!/bin/bash
# GPU-box session in steps, each under its own time limit; the first failing step ends it.
# Usage: tools/sess.sh <tag> <step>...   steps: test | testsel:<pytest selection> | bench | benchq |
#        trace | hits | pmc | uselib:<ab name> | ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sess}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
    local name=$1 tmo=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 4 "$OUT/$name.log" | cut -c1-600
    [ $rc -eq 0 ] || exit $rc
}
for st in "$@"; do
  case "$st" in
    test) run pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
          cp -f gpurun_out/parity_stats.json "$OUT/" 2>/dev/null ;;
    testall)  # every GPU test (no -x); plain test failures (pytest exit 1) do not end the session,
              # anything else (a fault, an abort, a time limit) does
          echo "=== pytest_all ($(date +%T))"
          timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/pytest_all.log" 2>&1
          rc=$?
          echo "=== pytest_all rc=$rc"
          grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/pytest_all.log" | tail -n 12 | cut -c1-300
          cp -f gpurun_out/parity_stats.json "$OUT/" 2>/dev/null
          [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    testsel:*) run pytest_sel 600 python -u -m pytest ${st#testsel:} -m gpu -x -v --timeout 300 --timeout-method thread
          cp -f gpurun_out/parity_stats.json "$OUT/" 2>/dev/null ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py
           cp -f gpurun_out/pmc_step.json gpurun_out/pmc_single.json "$OUT/" 2>/dev/null ;;
    benchq) run benchq 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-aux --no-pmc --no-single-view ;;
    trace) run trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-aux --no-single-view --no-pmc
           python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "at::" not in r["Name"]:
        print(f'{r["Name"][:72]:72s} {r["Calls"]:>4} {float(r["AverageNs"])/1000:8.1f}us')
PY
           ;;
    hits) run hits 200 python -u tools/dbg/hit_dump.py ;;
    pmc) run pmc 400 bash tools/profile_pmc.sh "$TAG/pmc" ;;
    dist) run dist 700 bash tools/dist_rehearsal.sh "$TAG/dist" ;;
    calib) run calib 500 bash tools/hbm_calib.sh "$TAG/calib" ;;
    uselib:*)  # ab/<name>.so becomes the in-tree library for the steps after this one
          cp -f "ab/${st#uselib:}.so" gaussian-splatting-npu_amd/diff_gaussian_rasterization/libgsr_hip.so && echo "=== using ab/${st#uselib:}.so" ;;
    ab:*) run ab 900 bash tools/ab.sh ${st#ab:} ;;
    ab1:*) BENCH_EXTRA="--views-total 1 --per-view --no-deferred" run ab1 900 bash tools/ab.sh ${st#ab1:} ;;
    ab1np:*) BENCH_EXTRA="--views-total 1 --per-view --no-deferred --no-prefix-stream" run ab1np 900 bash tools/ab.sh ${st#ab1np:} ;;
    pmcv) run pmcv 500 bash tools/pmc_views.sh "$TAG/pmcv" ;;
    pmc1) BENCH_ARGS="--views-total 1 --per-view --no-deferred" run pmc1 500 bash tools/pmc_views.sh "$TAG/pmc1" ;;
    trace1) run trace1 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof1" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-aux --no-single-view --no-pmc --views-total 1 --per-view --no-deferred ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "session done"
