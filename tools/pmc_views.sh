#!/bin/bash
# PMC counter passes (one rocprofv3 process per pass, --pmc only) over the bench's own step
# workload (bench.py --pmc-child: the step's launches and nothing else); BENCH_ARGS selects the
# workload (default: the 8-view batch; "--views-total 1 --per-view --no-deferred" = one view).
# Usage: tools/pmc_views.sh <tag>   -> gpurun_out/<tag>/{pmc_*, summary.json}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmcv}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
    local name=$1; shift
    echo "=== $name: $*"
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 bench.py --pmc-child --steps 1 --warmup 1 ${BENCH_ARGS:-} > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run sq2 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
run wrreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && echo summary ok
