#!/bin/bash
# Build libgsr_hip.so with extra compiler flags into ab/<name>.so (for tools/ab.sh A/B runs).
# Usage: tools/build_variant.sh <name> "<extra hipcc flags>"   (ONLY=<file.hip>: the flags for that file only)
set -eu
cd "$(dirname "$0")/.."
NAME=$1
EXTRA=${2:-}
B=/tmp/gsr_variant_$NAME
rm -rf "$B"; mkdir -p "$B" ab
cd gaussian-splatting-npu_amd
pids=""
for f in csrc/*.hip; do
  o=$B/$(basename "$f" .hip).o
  fl=""
  [ "$(basename "$f")" = render.hip ] && fl="-fno-slp-vectorize"
  ex=$EXTRA
  [ -n "${ONLY:-}" ] && [ "$(basename "$f")" != "$ONLY" ] && ex=""
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
      -I../include -Icsrc $fl $ex -c "$f" -o "$o" &
  pids="$pids $!"
done
for p in $pids; do wait "$p" || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../ab/$NAME.so $B/*.o
echo "built ab/$NAME.so"
