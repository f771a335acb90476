#!/bin/bash
# Full GPU suite, then the default bench line (each step under its own limit; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r05full}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; cp -f gpurun_out/parity_stats.json "$OUT/" 2>/dev/null
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; grep '^{' "$OUT/bench.log" | cut -c1-300; exit $rc
