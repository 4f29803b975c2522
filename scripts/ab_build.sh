#!/bin/bash
# A/B build of the step kernel: evariants/libeng_<name>.so from zb_engine.hip of a git revision
# (or the working tree with REV=cur), linked with the product's other objects. Diagnostic only.
#   scripts/ab_build.sh <name> [REV | cur | file <path>] [extra hipcc flags]   (SCHED= for the default scheduler)      then on the GPU: python tests/diag_variants.py evariants/libeng_*.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/ksim-gym-zbot_amd/csrc
OUT=$ROOT/evariants
NAME=$1; REV=${2:-cur}; shift 2 || true
mkdir -p "$OUT"
make -C "$CSRC" -s
SRC=$CSRC/zb_engine.hip
if [ "$REV" = cur ] && [ $# -eq 0 ] && [ -z "${SLP+x}" ] && [ -z "${SCHED+x}" ]; then
  # the working tree with the product flags: the product library just built is that variant
  cp "$ROOT/ksim-gym-zbot_amd/zbot_amd/libzbot_hip.so" "$OUT/libeng_$NAME.so"
  echo "built $OUT/libeng_$NAME.so (the product build)"
  exit 0
fi
if [ "$REV" = file ]; then SRC=$1; shift;
elif [ "$REV" != cur ]; then SRC=$OUT/zb_engine_$NAME.hip; git -C "$ROOT" show "$REV:ksim-gym-zbot_amd/csrc/zb_engine.hip" > "$SRC"; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$CSRC" -fno-signed-zeros \
  -freciprocal-math -fno-math-errno -fapprox-func ${SLP--fno-slp-vectorize} ${SCHED--mllvm -amdgpu-sched-strategy=iterative-ilp} "$@" -c -o "$OUT/eng_$NAME.o" "$SRC"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libeng_$NAME.so" "$OUT/eng_$NAME.o" \
  "$CSRC/build/zb_capi.o" "$CSRC/build/zb_ppo.o" "$CSRC/build/zb_policy.o" "$CSRC/build/zb_host.o"
echo "built $OUT/libeng_$NAME.so"
