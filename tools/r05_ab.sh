#!/bin/bash
# GPU tests named by $2 (default: depth sort + bit-exact key tests), then a same-box A/B of ab/*.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r05ab}
SEL=${2:-tests/test_depth_sort.py tests/test_gpu_parity.py}
ROUNDS=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab.sh "$ROUNDS" > "$OUT/ab.log" 2>&1
rc=$?; cat "$OUT/ab.log"; exit $rc
