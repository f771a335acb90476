#!/bin/bash
# Same-box A/B of ab/*.so on the single-view step (train.py's path) and the per-view 8-view mode;
# prints the median / mean ms per step of each (R rounds, ABAB order).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-3}
MODES=${2:-single perview}
LIB=gaussian-splatting-npu_amd/diff_gaussian_rasterization/libgsr_hip.so
cp "$LIB" /tmp/lib_orig.so
mkdir -p gpurun_out/svab
for r in $(seq "$R"); do
  for v in ab/*.so; do
    n=$(basename "$v" .so)
    cp "$v" "$LIB"
    for mode in $MODES; do
      if [ $mode = single ]; then A="--views-total 1 --per-view --no-deferred --steps 40 --warmup 5"; else A="--per-view --steps 20 --warmup 3"; fi
      timeout -k 10 200 python3 bench.py $A --no-cpu-baseline --no-aux --no-pmc --no-single-view --no-profile \
          > "gpurun_out/svab/$n.$mode.$r.log" 2>&1 || { cp /tmp/lib_orig.so "$LIB"; tail -5 "gpurun_out/svab/$n.$mode.$r.log"; exit 1; }
      echo "$n $mode $(grep '^{' "gpurun_out/svab/$n.$mode.$r.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_mean"])')"
    done
  done
done
cp /tmp/lib_orig.so "$LIB"
