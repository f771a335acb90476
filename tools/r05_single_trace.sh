#!/bin/bash
# rocprofv3 kernel trace of the single-view step (config2_single_view's workload) for every ab/*.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r05st}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIB=gaussian-splatting-npu_amd/diff_gaussian_rasterization/libgsr_hip.so
cp "$LIB" /tmp/lib_orig.so
for v in ab/*.so; do
  n=$(basename "$v" .so)
  cp "$v" "$LIB"
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$n" -o run -- python3 bench.py --views-total 1 --per-view \
      --no-deferred --steps 20 --warmup 3 --no-cpu-baseline --no-aux --no-pmc --no-single-view --no-profile \
      > "$OUT/$n.log" 2>&1 || { cp /tmp/lib_orig.so "$LIB"; tail -5 "$OUT/$n.log"; exit 1; }
  echo "== $n $(grep '^{' "$OUT/$n.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
cp /tmp/lib_orig.so "$LIB"
