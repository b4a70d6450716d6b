"""Diagnostic: section breakdown of the search loop (jit=3 stamp build) on the bench workload."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
from quorum_intersection_amd.distributed import DeviceSearch, distributed_search

k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
fb = qa.FBAS(fbas_gen.two_tier(k, 256))
be = DeviceSearch(fb, jit=3)
distributed_search(be, device="cuda")
loc = be.reduce(None)
st = loc["stamps"][:6]
tot = sum(st)
names = ["pop/close", "fetch+poll", "spill", "fixpoints", "best+push", "coop"]
print(json.dumps({"nodes": loc["nodes"], "wave_iters": loc["wave_iters"], "coop_phases": loc["coop_phases"],
                  "cycles_per_wave_iter": tot / max(loc["wave_iters"], 1),
                  "share": {n: round(v / tot, 4) for n, v in zip(names, st)},
                  "cycles_per_iter": {n: round(v / max(loc["wave_iters"], 1), 1) for n, v in zip(names, st)}}, indent=1))
