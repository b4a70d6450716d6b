"""Diagnostics: per-launch input/output unit counts and durations of one bench search
(QI_TRACE lines on stderr), after one warm-up search."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
from quorum_intersection_amd.distributed import DeviceSearch, distributed_search

wl = sys.argv[1] if len(sys.argv) > 1 else "two_tier"
text = fbas_gen.planted_deep(8, 512) if wl == "planted_deep" else fbas_gen.two_tier(10, 256)
fb = qa.FBAS(text)
os.environ.pop("QI_TRACE", None)
be = DeviceSearch(fb, jit=2)
distributed_search(be, device="cuda")
be.close()
os.environ["QI_TRACE"] = "1"
be = DeviceSearch(fb, jit=2)
r = distributed_search(be, device="cuda")
print("nodes", r.nodes, "launches", be.launches, "kernel_ms", be.kernel_ms, flush=True)
