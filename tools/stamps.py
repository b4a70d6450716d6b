"""Diagnostic: section breakdown of the search loop (jit=3 stamp build) on the bench workload.

Besides the per-section s_memtime shares it reports wave lifetimes (s_memrealtime,
100 MHz) against the launch durations (HIP events): waves that finish before the slowest
wave of their launch leave their slot idle until the launch ends.
"""
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
SETS = {0: ["pop+install", "poll", "spill", "fixpoints", "best+push+flush+claim", "leaf phases"],
        1: ["pop", "close+install", "dout/qd+best", "evict+push", "flush_record", "claim"],
        4: ["fast steps", "full iterations", "-", "-", "-", "-"],
        3: ["install: vmcnt(0) wait", "claim: wait for the queue head (atomic)", "pop: LDS refill wait", "-", "-", "-"],
        2: ["fastp (|D|<=qmin)", "fastmin (|D|=qmin+1)", "coop (|D|>=qmin+2)", "done+poll", "spill", "fixpoints"]}
sset = 0
for tok in os.environ.get("QI_JIT_DEFINES", "").split(","):
    if tok.startswith("QI_STAMP_SET="):
        sset = int(tok.split("=")[1])
names = SETS[sset]
waves = max(loc["stamps"][7], 1)
life_s = loc["stamps"][6] * 1e-8  # summed wave lifetimes
kernel_s = be.kernel_ms * 1e-3
cus = torch.cuda.get_device_properties(0).multi_processor_count
print(json.dumps({"stamp_set": sset, "nodes": loc["nodes"], "wave_iters": loc["wave_iters"], "coop_phases": loc["coop_phases"], "stamp_cycles": st,
                  "cycles_per_wave_iter": tot / max(loc["wave_iters"], 1),
                  "share": {n: round(v / tot, 4) for n, v in zip(names, st)},
                  "cycles_per_iter": {n: round(v / max(loc["wave_iters"], 1), 1) for n, v in zip(names, st)},
                  "waves": waves, "launches": be.launches, "kernel_ms": be.kernel_ms,
                  "avg_wave_life_us": 1e6 * life_s / waves,
                  "loop_clock_ghz": tot / max(life_s, 1e-12) / 1e9,
                  "wave_slot_use_7_per_cu": life_s / (kernel_s * 7 * cus)}, indent=1))
