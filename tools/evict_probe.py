"""Diagnostics: the deep multi-word searches of test_large_scc_multiword_masks under a given
QI_EVICT (per-lane stack evictions per launch), with QI_TRACE step logs on stderr.

    QI_EVICT=8 QI_TRACE=1 python tools/evict_probe.py [k n ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quorum_intersection_amd as qa  # noqa: E402
from quorum_intersection_amd import fbas_gen  # noqa: E402

args = [int(x) for x in sys.argv[1:]] or [11, 60, 20, 80, 28, 120]
for k, n in zip(args[::2], args[1::2]):
    for jit in (1, 2):
        t0 = time.time()
        d = qa.FBAS(fbas_gen.planted(k, n)).solve_stats(jit=jit)
        print(f"planted_{k}_{n} jit={jit}: verdict={d['verdict']} nodes={d['nodes']} launches={d['launches']} "
              f"{time.time() - t0:.2f}s", flush=True)
