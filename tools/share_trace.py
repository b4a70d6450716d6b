"""Diagnostics: per-launch trace (QI_TRACE) of ONE rank's share of an N-rank search.

    python tools/share_trace.py [world] [seed_units_per_rank] [rank]
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
from quorum_intersection_amd.distributed import DeviceSearch

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
per_rank = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
r = int(sys.argv[3]) if len(sys.argv) > 3 else 0
fb = qa.FBAS(fbas_gen.two_tier(10, 256))
os.environ["QI_TRACE"] = "1"
be = DeviceSearch(fb, jit=2)
be.restart()
be.grow(per_rank * world)
n = be.frontier()
buf = torch.empty(n * be.unit_bytes, dtype=torch.uint8, device="cuda")
be.export(n, buf)
for rep in range(2):
    be.restart()
    be.clear()
    be.import_(n, buf)
    be.keep_strided(r, world)
    print(f"==== share {r}/{world}: {be.frontier()} units (rep {rep})", file=sys.stderr, flush=True)
    while be.frontier():
        be.step()
