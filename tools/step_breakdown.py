"""Diagnostics: host-side time of one bench step by call (per-SCC batch, restart, chain, reduce)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
from quorum_intersection_amd.distributed import DeviceSearch

fb = qa.FBAS(fbas_gen.two_tier(10, 256))
be = DeviceSearch(fb, jit=2)
sccs = fb.sccs()
masks = qa.masks_from_sets(sccs, fb.n)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 30
acc = {}
def t(name, f):
    t0 = time.perf_counter()
    r = f()
    acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
    return r
for it in range(N + 3):
    if it == 3:
        acc.clear()
    t("gfp_batch", lambda: fb.gfp_batch(masks, masks))
    t("restart", be.restart)
    while t("frontier", be.frontier):
        t("step", be.step)
        t("local_best", be.local_best)
    t("local_best", be.local_best)
    t("reduce", lambda: be.reduce(None))
tot = sum(acc.values())
for k, v in acc.items():
    print(f"{k:12s} {1e6 * v / N:8.1f} us")
print(f"{'total':12s} {1e6 * tot / N:8.1f} us; chain kernels {1e3 * be.dispatch_ms:8.1f} us (last search)")
