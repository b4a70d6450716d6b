"""Diagnostics: one solve of planted(k, n) with QI_TRACE step lines (large-SCC path)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
k, n = int(sys.argv[1]), int(sys.argv[2])
t0 = time.time()
d = qa.FBAS(fbas_gen.planted(k, n)).solve_stats()
print(f"planted_{k}_{n}: verdict={d['verdict']} nodes={d['nodes']} launches={d['launches']} {time.time()-t0:.2f}s", flush=True)
