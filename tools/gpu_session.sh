#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench, a rocprofv3 kernel-trace.
# Each GPU step has its own time limit; a crash/fault/timeout (exit >= 124 or signal)
# ends the session.  Plain test failures (pytest exit 1) do not stop the later steps.
# Usage: tools/gpu_session.sh [tag] [pytest-args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>
    local name=$1 tmo=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 15 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then
        echo "stopping session after $name (rc=$rc)"
        exit $rc
    fi
    return 0
}

step build 600 python -c "import __graft_entry__ as g; g.build()"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q "$@"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 10 --warmup 3
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile
echo "session done"
