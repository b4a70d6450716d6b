"""Diagnostic: do two search chains on two HIP streams fill each other's launch tails?

Times one full search of the bench workload alone, then two independent searches of the
same workload run concurrently from two host threads (each engine has its own stream).
A ratio well under 2 means concurrent chains recover slot time that a single chain's
launch tails leave idle.
"""
import os, sys, json, threading, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import quorum_intersection_amd as qa
from quorum_intersection_amd import fbas_gen
from quorum_intersection_amd.distributed import DeviceSearch, distributed_search

text = fbas_gen.two_tier(10, 256)
engines = []
for _ in range(2):
    fb = qa.FBAS(text)
    be = DeviceSearch(fb, jit=2)
    engines.append((fb, be))
for _, be in engines:  # warm up
    distributed_search(be, device="cuda")


def run(be, out, i):
    r = distributed_search(be, device="cuda")
    out[i] = r.nodes


reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    distributed_search(engines[0][1], device="cuda")
single = (time.perf_counter() - t0) / reps
t0 = time.perf_counter()
for _ in range(reps):
    out = [0, 0]
    th = [threading.Thread(target=run, args=(engines[i][1], out, i)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
pair = (time.perf_counter() - t0) / reps
print(json.dumps({"single_ms": single * 1e3, "two_concurrent_ms": pair * 1e3, "ratio": pair / single,
                  "nodes": out}))
