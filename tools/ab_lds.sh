#!/bin/bash
# LDS / wait counters of render_bwd for every ab/*.so (one --pmc pass each over the bench's step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIB=gaussian-splatting-npu_amd/diff_gaussian_rasterization/libgsr_hip.so
cp "$LIB" /tmp/lib_orig.so
for v in ab/*.so; do
  n=$(basename "$v" .so)
  cp "$v" "$LIB"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
      --output-format csv -d gpurun_out/ablds/$n -o run -- python3 bench.py --pmc-child --steps 1 --warmup 1 \
      > gpurun_out/ablds/$n.log 2>&1 || { cp /tmp/lib_orig.so "$LIB"; tail -5 gpurun_out/ablds/$n.log; exit 1; }
  python3 - "$(find gpurun_out/ablds/$n -name '*counter_collection.csv' | head -1)" "$n" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "render_bwd" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], {k: f"{v:.4g}" for k, v in sorted(acc.items())},
      "conflict/instr", round(acc["SQ_LDS_BANK_CONFLICT"] / max(acc["SQ_INSTS_LDS"], 1), 3))
PY
done
cp /tmp/lib_orig.so "$LIB"
