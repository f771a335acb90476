#!/bin/bash
# Separate-DC / sparse-Adam iteration: their GPU tests, then the bench's aux legs (no CPU baselines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-dc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_separate_sh.py tests/test_adam.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench.log" 2>&1
rc=$?; grep '^{' "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps({k: d['aux'][k] for k in ('separate_sh','sparse_adam')}))"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile > "$OUT/rocprof.log" 2>&1
