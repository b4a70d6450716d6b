"""Full single-threaded CPU search of a bench workload with the oracle (the reference's
algorithm restated, oracle/qi_oracle.cpp -O3), pinned to one core: validates or replaces
bench.py's bounded-sample cpu_baseline extrapolation.  The search
runs in a child process; this parent prints a heartbeat every 30 s (a silent GPU-box
command is taken to be hung after 3 minutes).

    taskset -c 0 python tools/cpu_full.py [k_top] [validators] > profiles/r02/cpu_full.json
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
CHILD = r'''
import json, os, sys, time
sys.path.insert(0, %r); sys.path.insert(0, %r)
from qi_testlib import Oracle
from quorum_intersection_amd import fbas_gen
text = fbas_gen.two_tier(%d, %d)
t0 = time.perf_counter()
r = Oracle().load(text).solve()
r["wall_s"] = time.perf_counter() - t0
print(json.dumps(r))
''' % (ROOT, os.path.join(ROOT, "tests"), k, n)
model = "unknown"
for ln in open("/proc/cpuinfo"):
    if ln.startswith("model name"):
        model = ln.split(":", 1)[1].strip()
        break
p = subprocess.Popen([sys.executable, "-c", CHILD], stdout=subprocess.PIPE, text=True)
t0 = time.time()
while p.poll() is None:
    time.sleep(1)
    if int(time.time() - t0) % 30 == 0:
        print(f"# running {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
r = json.loads(p.stdout.read().strip().splitlines()[-1])
print(json.dumps({"workload": f"two_tier({k}, {n})", "nodes": r["nodes"], "evals": r["evals"], "verdict": r["verdict"],
                  "search_seconds": r["search_seconds"], "solve_seconds": r["seconds"], "wall_s": r["wall_s"],
                  "evals_per_s": r["evals"] / r["seconds"], "affinity": sorted(os.sched_getaffinity(0)), "cores": 1,
                  "host_cpu": model, "host_nproc": os.cpu_count(),
                  "build": "oracle/qi_oracle.cpp g++ -O3 (oracle/Makefile)"}), flush=True)
