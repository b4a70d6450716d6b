"""Diagnostics of persistent launches (QI_DONATE=1): per-search wall/kernel time, launch
count and the kernel's queue counters (stamps words 8-13 of the running totals).

    QI_DONATE=1 python tools/dq_probe.py [steps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import quorum_intersection_amd as qa  # noqa: E402
from quorum_intersection_amd import fbas_gen  # noqa: E402
from quorum_intersection_amd.distributed import DeviceSearch, distributed_search  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
fb = qa.FBAS(fbas_gen.two_tier(10, 256), device=0)
be = DeviceSearch(fb, jit=2)
for i in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = distributed_search(be, device="cuda")
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0)
    st = be.reduce(None)["stamps"]
    print(json.dumps({"ms": round(ms, 3), "kernel_ms": round(be.kernel_ms, 3), "launches": be.launches,
                      "nodes": res.nodes, "evals": res.evals, "wave_iters": res.wave_iters, "units": res.units,
                      "idle_wave_iters": st[0], "wait_lane_iters": st[1], "evict_donations": st[2],
                      "voluntary_donations": st[3], "queue_atomics": st[4], "persistent_wave_iters": st[5]}),
          flush=True)
