#!/bin/bash
# HBM-counter calibration passes: tools/hbm_calib (known access patterns and
# byte counts) under rocprofv3 --pmc, one pass per counter group, never combined with trace domains.
# Output: gpurun_out/<tag>/ CSVs, calib.jsonl (the program's known bytes), counters.txt.
# Summarise with tools/hbm_calib_summary.py <dir>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-calib}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 120 tools/hbm_calib > "$OUT/calib.jsonl" 2> "$OUT/calib.err" || { cat "$OUT/calib.err"; exit 1; }
run() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- tools/hbm_calib \
        > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
run wrreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
if grep -q "TCC_EA0_RDREQ_128B" "$OUT/counters.txt"; then run rdreq128 TCC_EA0_RDREQ_128B_sum; fi
python3 tools/hbm_calib_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
