#!/bin/bash
# GPU-box session: GPU parity tests (incl. the full-size config-2 case), then the default bench
# line.  Each GPU step under its own time limit; a crash, fault or timeout ends the session.
# Usage: tools/session.sh <tag> [pytest selection...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sess}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SEL=${*:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; cp -f gpurun_out/parity_stats.json "$OUT/" 2>/dev/null
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; grep '^{' "$OUT/bench.log" | cut -c1-400; exit $rc
