#!/bin/bash
# Round-5 new GPU tests first (each step under its own limit), then the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r05new}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_config3_scale.py tests/test_chair_gpu.py tests/test_chair_train.py \
    "tests/test_gpu_parity.py::test_packed_rect_boundary_keys_bit_exact" -m gpu -x -v --timeout 300 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; cp -f gpurun_out/parity_stats.json "$OUT/" 2>/dev/null
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; grep '^{' "$OUT/bench.log" | cut -c1-600; exit $rc
