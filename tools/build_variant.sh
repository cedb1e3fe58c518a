#!/bin/bash
# Build libfsem from a source tree into fast_speech_enhancement_metrics_amd/lib/var/NAME.so for
# A/B runs (tools/ab_bench.sh).  Usage: bash tools/build_variant.sh NAME [GIT_REV]
# Without GIT_REV the working tree is built; with it, that commit's csrc/include.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
REV=$2
OUT=$R/fast_speech_enhancement_metrics_amd/lib/var
mkdir -p "$OUT"
SRC=$R
if [ -n "$REV" ]; then
  SRC=$(mktemp -d)
  git -C "$R" archive "$REV" fast_speech_enhancement_metrics_amd/csrc include | tar x -C "$SRC"
fi
C=$SRC/fast_speech_enhancement_metrics_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC -Wno-unused-result ${EXTRA:-} \
  -o "$OUT/$NAME.so" "$C/pesq.hip" "$C/stoi.hip" "$C/resample.hip" $([ -f "$C/align.hip" ] && echo "$C/align.hip")
[ -n "$REV" ] && rm -rf "$SRC"
echo "$OUT/$NAME.so"
