#!/bin/bash
# GPU-box A/B session: optional GPU test selection on the in-tree build, then tools/ab.sh over
# ab/*.so.  Usage: tools/ab_session.sh <rounds> <kernels> [pytest selection...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
R=${1:-2}; KS=${2:-render_bwd,preprocess_bwd}; shift 2 || true
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 1500 bash tools/ab.sh "$R" "$KS"
