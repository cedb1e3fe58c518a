#!/bin/bash
# Build libfsem from a source tree into fast_speech_enhancement_metrics_amd/lib/var/NAME.so for
# A/B runs (tools/ab_joint.py).  Usage: bash tools/build_variant.sh NAME [GIT_REV]
# Without GIT_REV the working tree is built; with it, that commit's csrc/include.  Per-source
# flags as _build.SOURCE_FLAGS (stoi.hip: the max-ilp scheduler); EXTRA applies to every source,
# EXTRA_<name> (e.g. EXTRA_pesq) to one.
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
T=$(mktemp -d)
for f in pesq pesq_back stoi resample align; do
  [ -f "$C/$f.hip" ] || continue
  FL=""
  { [ "$f" = "stoi" ] || [ "$f" = "resample" ]; } && FL="-mllvm -amdgpu-sched-strategy=max-ilp"
  [ "$f" = "pesq" ] && [ -z "${SLP_PESQ:-}" ] && FL="-fno-slp-vectorize"
  FX=EXTRA_$f  # per-source extra flags: EXTRA_pesq, EXTRA_stoi, ...
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result $FL ${EXTRA:-} ${!FX:-} -c -o "$T/$f.o" "$C/$f.hip"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/$NAME.so" "$T"/*.o
rm -rf "$T"
[ -n "$REV" ] && rm -rf "$SRC"
echo "$OUT/$NAME.so"
