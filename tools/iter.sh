#!/bin/bash
# One iteration on the GPU box: GPU parity tests, then a rocprofv3 kernel-trace of a short bench
# (per-kernel averages printed), each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-it}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-aux > "$OUT/rocprof.log" 2>&1
rc=$?; grep '^{' "$OUT/rocprof.log" | cut -c1-160; [ $rc -ne 0 ] && exit $rc
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "at::" not in r["Name"]:
        print(f'{r["Name"][:64]:64s} {r["Calls"]:>4} {float(r["AverageNs"])/1000:8.1f}us')
PY
