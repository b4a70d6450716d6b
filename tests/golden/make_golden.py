"""Regenerate tests/golden/golden.json from the CPU oracle (oracle/qi_oracle.cpp).

The only reference-held known answers are the four fixture verdicts (correct*.json ->
true, broken*.json -> false; /root/reference/README.md:25-28).  Everything else here
(search-node counts, fixpoint-eval counts, minimal quorums visited, witnesses, SCC
facts) is produced by the oracle under the deterministic "lowest index" tie-break of
findBestNode (cpp:203-250) and pinned so later rounds cannot drift.

    python tests/golden/make_golden.py
    python tests/golden/make_golden.py --big [name prefix ...]   # golden_big.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from qi_testlib import FIXTURES, Oracle, fixture_text, random_fbas  # noqa: E402
from quorum_intersection_amd import fbas_gen  # noqa: E402

KEYS = ["verdict", "n", "nscc", "scc_with_quorum", "scc_quorum_ids", "front", "searched", "nodes", "evals",
        "scc_evals", "minq", "zero_fallback", "q1", "q2"]


def instances():
    for name in FIXTURES:
        yield name, fixture_text(name).decode()
    for k in range(2, 8):
        yield f"tiered_{k}", fbas_gen.tiered(k)
    yield "two_tier_7_256", fbas_gen.two_tier(7, 256)
    yield "tiered_5_shuffled", fbas_gen.tiered(5, seed=3)
    for k, n in ((4, 64), (5, 96)):
        yield f"planted_{k}_{n}", fbas_gen.planted(k, n)
    for s in range(40):
        yield f"random_{s}", random_fbas(s)


def big_instances():
    # the "64 orgs x 3 validators" benchmark configuration: two_tier(k_top, 192)
    for k in (7, 8):
        yield f"two_tier_{k}_192", fbas_gen.two_tier(k, 192)
    for k in (9, 10):
        yield f"two_tier_{k}_256", fbas_gen.two_tier(k, 256)
    # BASELINE configs[4]: the planted pair lies past 40% of the tree; "_intact" is the same
    # FBAS without the pair (plant=False), whose full search sizes the tree
    yield "planted_deep_8_512", fbas_gen.planted_deep(8, 512)
    yield "planted_deep_8_512_intact", fbas_gen.planted_deep(8, 512, plant=False)
    # a 35-vertex tier (two-word masks): the first witness 14.96 M nodes into the tree (~100 s)
    yield "planted_deep_9_512", fbas_gen.planted_deep(9, 512)


def big(only):
    """Bench-size instances (minutes of single-threaded oracle time each); `only` = name
    prefixes to regenerate, the other entries are kept."""
    path = os.path.join(HERE, "golden_big.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    o = Oracle()
    for name, text in big_instances():
        if only and not any(name.startswith(p) for p in only):
            continue
        r = o.load(text).solve()
        out[name] = {k: r[k] for k in KEYS}
        out[name]["oracle_seconds"] = round(r["seconds"], 2)
        print(name, out[name]["nodes"], out[name]["oracle_seconds"], flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


def main():
    if "--big" in sys.argv:
        return big(sys.argv[sys.argv.index("--big") + 1:])
    o = Oracle()
    out = {}
    for name, text in instances():
        r = o.load(text).solve()
        out[name] = {k: r[k] for k in KEYS}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {len(out)} instances")


if __name__ == "__main__":
    main()
