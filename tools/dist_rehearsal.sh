#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box exactly as the driver launches it
# (`python bench.py --gpus 2`: the PMC passes, then bench.py starts torch.distributed.run with
# 2 ranks as its child): 2 ranks on the same GPU over gloo (the driver's 8-GPU runs use RCCL).
# Checks the launch, barrier, all-reduce, max-over-ranks timing and the single JSON line of rank 0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-dist}
mkdir -p "$OUT"
export TMPDIR=/tmp
# BENCH_EXTRA: more bench.py flags (e.g. "--views-per-rank 4" for the weak-scaling mode)
GSR_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
    ${BENCH_EXTRA:-} > "$OUT/bench2.log" 2>&1
rc=$?; grep '^{' "$OUT/bench2.log" > "$OUT/bench2.json"; cut -c1-400 "$OUT/bench2.json"
[ $rc -ne 0 ] && tail -30 "$OUT/bench2.log"; exit $rc
