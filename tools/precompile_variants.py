"""Compile the specialised kernels of tools/ab.py variants HERE (no GPU needed), into the
in-tree cache that travels to the GPU box.  The box's processes import torch first and then
compile with torch's bundled (older) compiler library, whose code for the same source ran 6 %
slower: variants must be built by the same compiler as the default kernel to be comparable.

    python tools/precompile_variants.py [--workloads two_tier,planted_deep] name1=DEFINES1 ...
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import quorum_intersection_amd as qa  # noqa: E402
from quorum_intersection_amd import fbas_gen  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workloads", default="two_tier")
ap.add_argument("variants", nargs="+")
args = ap.parse_args()
WL = {"two_tier": lambda: fbas_gen.two_tier(10, 256), "planted_deep": lambda: fbas_gen.planted_deep(8, 512),
      "two_tier_8_192": lambda: fbas_gen.two_tier(8, 192)}
base_env = dict(os.environ)
for v in args.variants:
    name, _, spec = v.partition("=")
    os.environ.clear()
    os.environ.update(base_env)
    defs = []
    for tok in [t for t in spec.split(",") if t]:
        if tok.startswith("ENV:"):
            k, _, val = tok[4:].partition("=")
            os.environ[k] = val
        else:
            defs.append(tok)
    if defs:
        os.environ["QI_JIT_DEFINES"] = ",".join(defs)
    for wl in args.workloads.split(","):
        fb = qa.FBAS(WL[wl](), device=0)
        print(name, wl, "jit precompile ms", round(fb.jit_precompile(), 1), flush=True)
