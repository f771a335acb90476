#!/bin/bash
# GPU-box bench session: the default bench line (in-run PMC traffic passes, CPU baseline, aux legs),
# then the N=2 path rehearsed with 2 gloo ranks on the one GPU.  Each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "bench start $(date +%T)"
timeout -k 10 900 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; grep '^{' "$OUT/bench.log" > "$OUT/bench.json"; cut -c1-600 "$OUT/bench.json"; echo "bench rc=$rc $(date +%T)"
[ $rc -ne 0 ] && { tail -30 "$OUT/bench.log"; exit $rc; }
[ "${2:-}" = "nodist" ] && exit 0
GSR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
    > "$OUT/bench2.log" 2>&1
rc=$?; grep '^{' "$OUT/bench2.log" | cut -c1-600; [ $rc -ne 0 ] && tail -30 "$OUT/bench2.log"; exit $rc
