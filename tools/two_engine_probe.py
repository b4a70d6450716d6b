"""Diagnostics: one search through E engines on ONE GPU (own stream and host thread each,
max_blocks resident waves each) against the single engine: do the tails of one engine's
launches fill with the other's work?  Prints the solve's timing fields (median of N)."""
import os, sys, time, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen

text = fbas_gen.two_tier(10, 256)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 7
fb = qa.FBAS(text)
for engines, blocks in ((1, 0), (2, 1152), (2, 1408), (2, 2304), (3, 768), (4, 576)):
    rows = []
    for _ in range(N):
        t0 = time.perf_counter()
        d = fb.solve_stats(engines=engines, device_mask=1, max_blocks=blocks, jit=2)
        wall = 1e3 * (time.perf_counter() - t0)
        rows.append((wall, d))
    assert all(r[1]["nodes"] == 121164209 for r in rows)
    rows.sort(key=lambda r: r[0])
    wall, d = rows[len(rows) // 2]
    keys = [k for k in d if k.startswith("t_")]
    print(engines, blocks, "wall_ms", round(wall, 3), {k: round(d[k], 3) for k in keys}, "launches", d["launches"], flush=True)
