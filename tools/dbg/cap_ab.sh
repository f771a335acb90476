#!/bin/bash
# A/B: HEAD library vs the experimental one with GSR_BWD_WAVES caps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
LIB=gaussian-splatting-npu_amd/diff_gaussian_rasterization/libgsr_hip.so
for r in 1 2; do
  for cfg in head:0 exp:0 exp:3 exp:2; do
    v=${cfg%%:*}; c=${cfg##*:}
    cp ab/$v.so $LIB
    if [ "$c" = 0 ]; then unset GSR_BWD_WAVES; else export GSR_BWD_WAVES=$c; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-aux --no-pmc --no-profile > gpurun_out/cap.log 2>&1 || exit 1
    echo "$cfg $(grep '^{' gpurun_out/cap.log | cut -c60-100)"
  done
done
