"""A/B of specialised-kernel variants in one process, interleaved to expose box noise.

    python tools/ab.py [--rounds 2] [--steps 10] [--workloads two_tier,planted_deep] \
        name1=DEFINES1 name2=DEFINES2 ...

DEFINES is a QI_JIT_DEFINES string ("A=1,B=2", may be empty); a token ENV:K=V inside it
sets an environment variable for that variant instead (engine knobs such as QI_GRACE).
Every measured search is checked against the golden node / eval counts.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import quorum_intersection_amd as qa  # noqa: E402
from quorum_intersection_amd import fbas_gen  # noqa: E402
from quorum_intersection_amd.distributed import DeviceSearch, distributed_search  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--workloads", default="two_tier")
ap.add_argument("variants", nargs="+")
args = ap.parse_args()

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_big.json")))
WL = {"two_tier": (fbas_gen.two_tier(10, 256), GOLD["two_tier_10_256"], 0),
      "planted_deep": (fbas_gen.planted_deep(8, 512), GOLD["planted_deep_8_512"], GOLD["planted_deep_8_512"]["scc_evals"]),
      "two_tier_8_192": (fbas_gen.two_tier(8, 192), GOLD["two_tier_8_192"], GOLD["two_tier_8_192"]["scc_evals"])}
base_env = dict(os.environ)
results = {}
for rnd in range(args.rounds):
    for v in args.variants:
        name, _, spec = v.partition("=")
        os.environ.clear()
        os.environ.update(base_env)
        defs = []
        for tok in [t for t in spec.split(",") if t]:
            if tok.startswith("ENV:"):
                k, _, val = tok[4:].partition("=")
                os.environ[k] = val
            else:
                defs.append(tok)
        if defs:
            os.environ["QI_JIT_DEFINES"] = ",".join(defs)
        for wl in args.workloads.split(","):
            text, gold, scc_evals = WL[wl]
            fb = qa.FBAS(text, device=0)
            be = DeviceSearch(fb, jit=2)
            for _ in range(2):
                distributed_search(be, device="cuda")
            ms, kms = [], []
            res = None
            for _ in range(args.steps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = distributed_search(be, device="cuda")
                torch.cuda.synchronize()
                ms.append(1e3 * (time.perf_counter() - t0))
                kms.append(be.kernel_ms)
            ms.sort()
            kms.sort()
            evals_want = gold["evals"] - (scc_evals if scc_evals else (gold["evals"] - res.evals if wl == "two_tier" else 0))
            ok = (res.nodes == gold["nodes"] and res.minq == gold["minq"] and bool(res.verdict) == bool(gold["verdict"])
                  and (wl == "two_tier" or res.evals == evals_want))
            row = {"variant": name, "workload": wl, "round": rnd, "ms_median": round(ms[len(ms) // 2], 4),
                   "ms_min": round(ms[0], 4), "kernel_ms_median": round(kms[len(kms) // 2], 4), "launches": be.launches,
                   "units": res.units, "wave_iters": res.wave_iters, "coop_phases": res.coop_phases, "blocks": getattr(be, "blocks", 0), "golden": "match" if ok else "MISMATCH"}
            print(json.dumps(row), flush=True)
            results.setdefault((name, wl), []).append(row["ms_median"])
            be.close()
            del be, fb
print("---- summary (median ms per search, per round) ----")
for (name, wl), v in results.items():
    print(f"{name:24s} {wl:16s} " + " ".join(f"{x:8.4f}" for x in v), flush=True)
