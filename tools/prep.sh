#!/bin/bash
# Build everything in-tree and pre-compile the bench's specialised kernel (CPU only).
# Fails loudly, so a broken build never reaches a GPU run.
set -euo pipefail
cd "$(dirname "$0")/.."
make -C oracle -j8 > /tmp/qi_build.log 2>&1 || { tail -30 /tmp/qi_build.log; exit 1; }
make -C quorum_intersection_amd/csrc -j8 >> /tmp/qi_build.log 2>&1 || { grep -A5 error /tmp/qi_build.log | head -40; exit 1; }
python3 -c "
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
for t in (fbas_gen.two_tier(10, 256), fbas_gen.planted_deep(8, 512), fbas_gen.planted_deep(8, 512, plant=False)):
    fb = qa.FBAS(t, device=0)
    print('jit precompile ms', round(fb.jit_precompile(), 1))
"
