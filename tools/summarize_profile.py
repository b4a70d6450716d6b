#!/usr/bin/env python
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/.

Writes:
  kernel_stats.csv     rocprofv3 --kernel-trace --stats summary (verbatim)
  counters.json        PMC totals per kernel + per-dispatch averages for search_kernel
  summary.md           human-readable digest
and, with --traffic, profiles/traffic.json: HBM bytes per search_kernel launch for bench.py.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reads half the bytes of 16-B-per-lane streaming loads on gfx950, so it is
doubled (the frontier refills are 16-B-per-lane loads); WRITE_SIZE is taken as is.
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "qi_search_spec"  # run-time specialised search kernel (bench default)


def agg_counters(path):
    rows = list(csv.DictReader(open(path)))
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in rows:
        key = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
        tot[key] += float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
    return tot, disp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=None)
    ap.add_argument("--traffic", action="store_true")
    ap.add_argument("--k-top", type=int, default=10)
    ap.add_argument("--validators", type=int, default=256)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    src = a.src or os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    dst = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))))
    counters = {}
    per_dispatch = {}
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not p.startswith("pmc") or not os.path.exists(f):
            continue
        tot, disp = agg_counters(f)
        for (k, c), v in tot.items():
            counters.setdefault(k, {})[c] = v
            if KERNEL in k or ("search_kernel" in k and not any(KERNEL in kk for kk, _ in tot)):
                per_dispatch[c] = v / max(len(disp[(k, c)]), 1)
    search = ([s for s in stats if KERNEL in s["Name"]] or [s for s in stats if "search_kernel" in s["Name"]])[0]
    out = {"kernel_stats_search": search, "search_kernel_per_dispatch": per_dispatch, "totals": counters}
    json.dump(out, open(os.path.join(dst, "counters.json"), "w"), indent=1)
    pdc = per_dispatch
    lines = [f"# Profile {a.tag}", "", a.note, "",
             "`tools/profile.sh` on one MI355X: `rocprofv3 --kernel-trace --stats` + separate `--pmc` passes "
             "(bench.py default workload two_tier(k_top=10, 256)).", "",
             f"## Kernel stats ({search['Name'][:60]})", "",
             f"- calls {search['Calls']}, average {float(search['AverageNs'])/1e3:.1f} us, "
             f"min {float(search['MinNs'])/1e3:.1f} us, max {float(search['MaxNs'])/1e3:.1f} us, "
             f"{float(search['Percentage']):.1f}% of GPU time", "",
             "## PMC per search_kernel dispatch (average)", ""]
    for k in sorted(pdc):
        lines.append(f"- {k}: {pdc[k]:.4g}")
    if "SQ_WAVE_CYCLES" in pdc:
        w = pdc["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in pdc:
                lines.append(f"- {k} / SQ_WAVE_CYCLES = {pdc[k] / w:.3f}")
    fetch = pdc.get("FETCH_SIZE")
    write = pdc.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        hbm = (2 * fetch + write) * 1024
        lines += ["", f"HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B): {hbm:.4g}"]
        if a.traffic:
            json.dump({"k_top": a.k_top, "validators": a.validators, "hbm_bytes_per_launch": hbm,
                       "source": f"profiles/{a.tag}/counters.json", "fetch_kib": fetch, "write_kib": write},
                      open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
