#!/bin/bash
# Offline view of the specialised search kernel (CPU only): dump the generated source for the
# bench FBAS, compile it to gfx950 assembly with hipcc and count the instructions between the
# fast-step loop's labels.  Usage: bash tools/isa_dump.sh <outdir> [extra -D flags]
set -euo pipefail
out=${1:-/tmp/isa}; shift || true
mkdir -p "$out"
cd "$(dirname "$0")/.."
QI_JIT_CACHE=$out/cache QI_JIT_DUMP=$out/spec.hip python3 - <<'PY'
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
fb = qa.FBAS(fbas_gen.two_tier(10, 256), device=0)
fb.jit_precompile()
PY
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -Wno-pragma-once-outside-header \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -Xclang -target-feature -Xclang -packed-fp32-ops "$@" \
  -o "$out/spec.s" "$out/spec.hip" 2> "$out/compile.err" || { tail -20 "$out/compile.err"; exit 1; }
grep -E "^\s+(v_|s_|ds_|global_|buffer_|flat_)" "$out/spec.s" | wc -l
grep -E "vgpr_count|sgpr_count|lds_size|scratch" "$out/spec.s" | head -8
