#!/bin/bash
# A/B timing of library variants on ONE box: ab/<name>.so files are swapped into place in turn
# (ABAB... order, R rounds) and each runs a short bench; prints value and per-kernel averages.
# Usage (on the GPU box): bash tools/ab.sh [rounds] [kernel,kernel,...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-2}
KS=${2:-render_fwd,render_bwd,preprocess_bwd,preprocess_fwd,depth_sort,tile_sort}
LIB=gaussian-splatting-npu_amd/diff_gaussian_rasterization/libgsr_hip.so
cp "$LIB" /tmp/lib_orig.so
mkdir -p gpurun_out/ab
for r in $(seq "$R"); do
  for v in ab/*.so; do
    n=$(basename "$v" .so)
    cp "$v" "$LIB"
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-aux --no-pmc --no-single-view ${BENCH_EXTRA:-} > "gpurun_out/ab/$n.$r.log" 2>&1 || { cp /tmp/lib_orig.so "$LIB"; tail -5 "gpurun_out/ab/$n.$r.log"; exit 1; }
    python3 - "gpurun_out/ab/$n.$r.log" "$n" "$KS" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(f'{sys.argv[2]:>12s} {d["value"]:8.1f}', " ".join(f'{n}={k[n]["avg_ms"]*1e3:.1f}' for n in sys.argv[3].split(",") if n in k))
PY
  done
done
cp /tmp/lib_orig.so "$LIB"
