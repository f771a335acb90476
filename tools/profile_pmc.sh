#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 process per pass, --pmc only,
# never combined with trace domains).  Output: gpurun_out/<tag>/pmc*/ CSVs; summarise with
# tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --pmc-child --steps 1 --warmup 1 ${BENCH_ARGS:-}"
run() {
    local name=$1; shift
    echo "=== $name: $*"
    timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $BENCH > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
run pmc_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run pmc_fetch FETCH_SIZE
run pmc_write WRITE_SIZE
run pmc_valu SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
