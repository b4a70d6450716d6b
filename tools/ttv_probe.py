"""Diagnostic: where time-to-verdict goes (bench workload, from JSON text in host memory)."""
import os, sys, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen

text = fbas_gen.two_tier(10, 256)
for rep in range(2):
    for jit in (0, 1, 2):
        t0 = time.perf_counter()
        fb = qa.FBAS(text)
        t1 = time.perf_counter()
        d = fb.solve_stats(jit=jit)
        t2 = time.perf_counter()
        fb.close()
        t3 = time.perf_counter()
        print(json.dumps({"rep": rep, "jit": jit, "parse_ms": (t1 - t0) * 1e3, "solve_ms": (t2 - t1) * 1e3,
                          "close_ms": (t3 - t2) * 1e3, "scc_ms": d["t_scc_ms"], "search_ms": d["t_search_ms"],
                          "kernel_ms": d["t_kernel_ms"], "launches": d["launches"],
                          "jit_launches": d.get("jit_launches")}), flush=True)
