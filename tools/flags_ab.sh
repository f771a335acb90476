#!/bin/bash
# A/B of bench.py flag sets on one box (rounds x flag sets), value + per-kernel averages.
# Usage: tools/flags_ab.sh <rounds> "<flags A>" "<flags B>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fab
R=$1; shift
for r in $(seq "$R"); do
  i=0
  for f in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-aux --no-pmc $f > "gpurun_out/fab/$i.$r.log" 2>&1 || { tail -5 "gpurun_out/fab/$i.$r.log"; exit 1; }
    python3 - "gpurun_out/fab/$i.$r.log" "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["roofline"]["kernels"]
print(f'{sys.argv[2][:40]:>40s} {d["value"]:8.1f} {d["ms_per_step"]:7.3f}ms', " ".join(f'{n}={k[n]["avg_ms"]*1e3:.1f}' for n in ("render_bwd", "preprocess_bwd") if n in k))
PY
  done
done
