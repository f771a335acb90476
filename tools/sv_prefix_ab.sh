#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
for r in 1 2 3; do
for f in "" "--no-prefix-stream"; do
  timeout -k 10 200 python3 bench.py --views-total 1 --per-view --no-deferred --steps 40 --warmup 5 --no-cpu-baseline --no-aux --no-pmc --no-single-view --no-profile $f > /tmp/sv.log 2>&1 || exit 1
  echo "[$f] $(grep '^{' /tmp/sv.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_mean"])')"
done; done
