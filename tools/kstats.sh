#!/bin/bash
# rocprofv3 --kernel-trace --stats of a short bench run for every ab/*.so (one run each; $2: extra bench
# flags, e.g. "--views-total 1 --per-view --no-deferred" for the single view);
# prints the radix / render kernels' average durations per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ks}
EXTRA=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIB=gaussian-splatting-npu_amd/diff_gaussian_rasterization/libgsr_hip.so
cp "$LIB" /tmp/lib_orig.so
for v in ab/*.so; do
  n=$(basename "$v" .so)
  cp "$v" "$LIB"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$n" -o run -- python3 bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline --no-aux --no-pmc --no-single-view --no-profile $EXTRA > "$OUT/$n.log" 2>&1 || { cp /tmp/lib_orig.so "$LIB"; tail -5 "$OUT/$n.log"; exit 1; }
  echo "== $n $(grep '^{' "$OUT/$n.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  python3 tools/kstats_db.py "$(find "$OUT/$n" -name '*.db' | head -1)" | head -30
done
cp /tmp/lib_orig.so "$LIB"
