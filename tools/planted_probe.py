"""Diagnostic: search size and time-to-verdict of planted(k, 512) (BASELINE configs[4])."""
import os, sys, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen

for k in [int(x) for x in sys.argv[1:]] or [8, 10, 12, 14]:
    text = fbas_gen.planted(k, 512)
    fb = qa.FBAS(text)
    fb.solve_stats(jit=2)  # compile + warm
    t0 = time.perf_counter()
    d = fb.solve_stats(jit=2)
    dt = time.perf_counter() - t0
    print(json.dumps({"k": k, "verdict": d["verdict"], "nodes": d["nodes"], "evals": d["evals"],
                      "front": len(d.get("front", [])) if isinstance(d.get("front"), list) else None,
                      "ms": dt * 1e3, "kernel_ms": d["t_kernel_ms"], "launches": d["launches"]}), flush=True)
