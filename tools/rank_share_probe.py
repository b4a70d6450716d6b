"""Diagnostic: per-rank work of an N-rank search, measured on one GPU.

Rank 0's frontier growth (qi_search_grow to `seed` units) is timed, then each rank's strided
share units[r::world] is run to completion on its own and timed.  max(share) + growth
approximates the N-GPU step time without exchanges (no rebalancing); the spread of the shares
shows the imbalance a strided deal leaves.

    python tools/rank_share_probe.py [world] [seed_units_per_rank] [batch] [workload]

workload: two_tier (default, BASELINE configs[3]) or planted_deep (configs[4]: the shares
are run with the witness key of the other shares unknown, i.e. the worst case for early
termination; nodes are the shares' processed nodes, not the preorder-exact count).
"""
import os, sys, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
from quorum_intersection_amd.distributed import DeviceSearch

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
per_rank = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 64
workload = sys.argv[4] if len(sys.argv) > 4 else "two_tier"
text = fbas_gen.planted_deep(8, 512) if workload == "planted_deep" else fbas_gen.two_tier(10, 256)
fb = qa.FBAS(text)
be = DeviceSearch(fb, jit=2, batch=batch)
dev = torch.device("cuda", 0)


def run_share(r, buf, n):
    be.restart()
    be.clear()
    be.import_(n, buf)
    be.keep_strided(r, world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 0
    while be.frontier():
        be.step()
        steps += 1
    dt = time.perf_counter() - t0
    return dt, be.reduce(None)["nodes"], steps


for rep in range(2):
    be.restart()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    be.grow(per_rank * world)
    t_grow = time.perf_counter() - t0
    n = be.frontier()
    grow_nodes = be.reduce(None)["nodes"]
    buf = torch.empty(n * be.unit_bytes, dtype=torch.uint8, device=dev)
    be.export(n, buf)
    shares = [run_share(r, buf, n) for r in range(world)]
    ms = [s[0] * 1e3 for s in shares]
    print(json.dumps({"rep": rep, "workload": workload, "world": world, "seed_units": n, "grow_ms": t_grow * 1e3, "grow_nodes": grow_nodes,
                      "share_ms": [round(x, 3) for x in ms], "share_nodes": [s[1] for s in shares],
                      "share_steps": [s[2] for s in shares],
                      "est_step_ms": t_grow * 1e3 + max(ms), "total_nodes": grow_nodes + sum(s[1] for s in shares)}),
          flush=True)
