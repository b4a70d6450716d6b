"""Diagnostics: time of the batched per-SCC quorum checks (one query per SCC) on a network."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen

for name, text in (("two_tier_10_256", fbas_gen.two_tier(10, 256)), ("planted_deep_8_512", fbas_gen.planted_deep(8, 512))):
    fb = qa.FBAS(text, device=0)
    sccs = fb.sccs()
    masks = qa.masks_from_sets(sccs, fb.n)
    for rep in range(2):  # the first call on a fresh handle (allocations, staging buffer)
        fb2 = qa.FBAS(text, device=0)
        t0 = time.perf_counter(); fb2.gfp_batch(masks, masks); first = time.perf_counter() - t0
        t0 = time.perf_counter(); fb2.gfp_batch(masks, masks); second = time.perf_counter() - t0
        print(name, "fresh handle: first call %.3f ms, second %.3f ms" % (first * 1e3, second * 1e3), flush=True)
    for rep in range(3):
        t0 = time.perf_counter()
        out = fb.gfp_batch(masks, masks)
        dt = time.perf_counter() - t0
        # single queries: the largest SCC alone, and a singleton
        big = max(range(len(sccs)), key=lambda i: len(sccs[i]))
        t1 = time.perf_counter(); fb.gfp_batch(masks[big:big + 1], masks[big:big + 1]); d1 = time.perf_counter() - t1
        small = min(range(len(sccs)), key=lambda i: len(sccs[i]))
        t2 = time.perf_counter(); fb.gfp_batch(masks[small:small + 1], masks[small:small + 1]); d2 = time.perf_counter() - t2
    sizes = sorted((len(s) for s in sccs), reverse=True)
    print(name, "n", fb.n, "sccs", len(sccs), "sizes", sizes[:5], "all %.3f ms" % (dt * 1e3), "largest alone %.3f ms" % (d1 * 1e3),
          "smallest alone %.3f ms" % (d2 * 1e3), flush=True)
