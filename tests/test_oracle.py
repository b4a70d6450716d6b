"""The CPU oracle pinned against the reference's known answers and the golden vectors.

Reference-held known answers: correct*.json -> true, broken*.json -> false
(/root/reference/README.md:25-28).  The golden counts are the oracle's own output under
the lowest-index tie-break (tests/golden/make_golden.py) and pin it across rounds.
An independent pure-Python restatement of containsQuorumSlice / containsQuorum checks
the oracle's fixpoint on small random inputs.
"""
import json
import os
import random

import pytest

from qi_testlib import FIXTURES, GOLDEN, Oracle, fixture_text, random_fbas
from quorum_intersection_amd import fbas_gen

GOLD = json.load(open(os.path.join(GOLDEN, "golden.json")))


def test_fixture_verdicts_match_reference_readme():
    o = Oracle()
    for name in FIXTURES:
        r = o.load(fixture_text(name)).solve()
        assert r["verdict"] == name.startswith("correct"), name


@pytest.mark.parametrize("name", sorted(GOLD))
def test_oracle_matches_golden(name):
    o = Oracle()
    if name in FIXTURES:
        text = fixture_text(name)
    elif name.startswith("tiered_5_shuffled"):
        text = fbas_gen.tiered(5, seed=3)
    elif name.startswith("tiered_"):
        text = fbas_gen.tiered(int(name.split("_")[1]))
    elif name.startswith("two_tier_"):
        _, _, k, n = name.split("_")
        text = fbas_gen.two_tier(int(k), int(n))
    elif name.startswith("planted_"):
        _, k, n = name.split("_")
        text = fbas_gen.planted(int(k), int(n))
    else:
        text = random_fbas(int(name.split("_")[1]))
    if name in ("tiered_7", "two_tier_7_256"):
        pytest.skip("large: covered by the GPU parity suite")
    r = o.load(text).solve()
    for k, v in GOLD[name].items():
        assert r[k] == v, (name, k)


def test_independent_model_counts():
    # counts from an independent throwaway model of cpp:90-400 written before the oracle
    o = Oracle()
    assert (o.load(fixture_text("correct")).solve()["nodes"], o.load(fixture_text("correct")).solve()["evals"]) == (11, 80)
    assert (o.load(fixture_text("broken")).solve()["nodes"], o.load(fixture_text("broken")).solve()["evals"]) == (7, 70)
    r = o.load(fbas_gen.tiered(6)).solve()
    assert (r["nodes"], r["evals"], r["minq"]) == (111461, 220117, 1215)


def test_broken_witness_is_the_known_pair():
    g = Oracle().load(fixture_text("broken"))
    r = g.solve()
    ids = g.graph()["ids"]
    assert r["front"] == [3, 4, 6, 10]
    assert r["q1"] == [3, 10] and r["q2"] == [4, 6]
    assert ids[4] == "GCGB2S2KGYARPVIA37HYZXVRM2YZUEXA6S33ZU5BUDC6THSB62LZSTYH"  # SDF validator 1


@pytest.mark.parametrize("seed", range(6))
def test_verdict_invariant_under_random_tiebreak(seed):
    o = Oracle()
    for name in FIXTURES:
        g = o.load(fixture_text(name))
        assert g.solve(1, seed)["verdict"] == g.solve(0)["verdict"]
    g = o.load(fbas_gen.tiered(4))
    assert g.solve(1, seed)["verdict"] is True


# ---- independent restatement of cpp:90-177 (pure Python, small inputs only) ---------
def _py_slice(node, q, avail):
    if not avail[node]:
        return False
    if q is None:
        return False
    t = q["t"]
    entries = len(q["v"]) + len(q["i"])
    MASK = (1 << 64) - 1
    thr = t
    fail = (entries - t + 1) & MASK
    items = [("v", x) for x in q["v"]] + [("i", x) for x in q["i"]]
    for kind, x in items:
        ok = avail[x] if kind == "v" else _py_slice(node, x, avail)
        if ok:
            thr = (thr - 1) & MASK
        else:
            fail = (fail - 1) & MASK
        if thr == 0:
            return True
        if fail == 0:
            return False
    return False


def _py_graph(text):
    data = json.loads(text)
    idx = {}
    for i, d in enumerate(data):
        idx[d["publicKey"]] = i

    def conv(q):
        if not q:
            return None
        return {"t": int(q["threshold"]), "v": [idx.get(x, 0) for x in q["validators"]],
                "i": [c for c in (conv(z) for z in q["innerQuorumSets"])]}

    return [conv(d["quorumSet"]) for d in data]


def _py_gfp(qs, nodes, avail):
    avail = list(avail)
    removed = []
    cur = list(nodes)
    while True:
        count = len(cur)
        nxt = []
        for x in cur:
            if not _py_slice(x, qs[x], avail):
                if avail[x]:
                    avail[x] = False
                    removed.append(x)
            else:
                nxt.append(x)
        cur = nxt
        if count == len(cur):
            return cur


@pytest.mark.parametrize("seed", range(25))
def test_oracle_gfp_equals_python_restatement(seed):
    text = random_fbas(seed + 100, n=10)
    g = Oracle().load(text)
    # empty/null quorum sets become None; inner empty dicts never occur in the generator
    qs = _py_graph(text)
    rng = random.Random(seed)
    for _ in range(30):
        nodes = [v for v in range(g.n) if rng.random() < 0.7]
        rng.shuffle(nodes)
        avail = [rng.random() < 0.8 for _ in range(g.n)]
        assert g.contains_quorum(nodes, avail) == _py_gfp(qs, nodes, avail)


def test_threshold_zero_quirk():
    # t = 0: the size_t counters wrap, so the slice holds iff the FIRST entry is unavailable
    nodes = [
        {"publicKey": "A", "quorumSet": {"threshold": 0, "validators": ["B", "A"], "innerQuorumSets": []}},
        {"publicKey": "B", "quorumSet": {"threshold": 1, "validators": ["A"], "innerQuorumSets": []}},
    ]
    g = Oracle().load(json.dumps(nodes))
    assert g.slice(0, [True, False]) is True
    assert g.slice(0, [True, True]) is False


def test_planted_deep_construction():
    # BASELINE configs[4] generator: the golden witness (oracle, make_golden.py --big) is a
    # pair of disjoint quorums of the SCC, and plant=False breaks exactly that pair (HB
    # members then need b0, which lies in the A-side quorum)
    big = json.load(open(os.path.join(GOLDEN, "golden_big.json")))
    g = big["planted_deep_8_512"]
    assert (g["verdict"], g["nodes"]) == (False, 1895551)
    assert big["planted_deep_8_512_intact"]["verdict"] and big["planted_deep_8_512_intact"]["nodes"] == 4750447
    q1, q2, scc = set(g["q1"]), set(g["q2"]), set(g["front"])
    assert q1 and q2 and not (q1 & q2) and q1 <= scc and q2 <= scc and len(scc) == 32
    for plant in (True, False):
        o = Oracle().load(fbas_gen.planted_deep(8, 512, plant=plant))
        a1 = [v in q1 for v in range(o.n)]
        a2 = [v in q2 for v in range(o.n)]
        assert all(o.slice(v, a2) for v in q2)
        assert all(o.slice(v, a1) for v in q1) == plant


# ---- libstdc++ unordered_set order (toRemove, cpp:308/331) --------------------------------
def _oracle_lib():
    import ctypes
    L = Oracle().L
    L.qio_hash_order.restype = ctypes.c_uint64
    L.qio_hash_order.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    L.qio_hash_bucket_counts.restype = None
    L.qio_hash_bucket_counts.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    return L


def test_hash_bucket_growth_is_the_emulated_one():
    # the ordered search kernel assumes 13/29/59/127/257 buckets from the 1st/14th/30th/
    # 60th/128th distinct insertion on (qi_ordered_kernel.h, hash_grow_at)
    import ctypes
    out = (ctypes.c_uint64 * 300)()
    _oracle_lib().qio_hash_bucket_counts(300, out)
    want = [13] * 13 + [29] * 16 + [59] * 30 + [127] * 68 + [257] * 130 + [541] * 43
    assert list(out) == want


@pytest.mark.parametrize("seed", range(12))
def test_hash_iteration_order_matches_libstdcxx(seed):
    # the product's emulation (host build of the device code) against the real container
    import ctypes
    import quorum_intersection_amd as qa
    L, P = _oracle_lib(), qa.lib()
    rng = random.Random(seed)
    for trial in range(60):
        n = rng.choice([1, 2, 5, 13, 14, 15, 29, 30, 31, 59, 60, 61, 127, 128, 129, 200, 256, 257, 258, 300, 541, 542, 700])
        keys = rng.sample(range(max(n, rng.choice([n, 2 * n + 7, 600, 100000]))), n)
        seq = [rng.randrange(n) for _ in range(rng.randint(0, 2 * n))]
        if rng.random() < 0.5:
            seq = rng.sample(range(n), rng.randint(0, n))
        K = (ctypes.c_uint32 * n)(*keys)
        S = (ctypes.c_uint32 * max(len(seq), 1))(*seq)
        want = (ctypes.c_uint32 * n)()
        got = (ctypes.c_uint32 * n)()
        nw = L.qio_hash_order(K, n, S, len(seq), want)
        ng = ctypes.c_uint32()
        qa.check(P.qi_hash_iteration_order(K, n, S, len(seq), got, ctypes.byref(ng)))
        assert list(got)[: ng.value] == list(want)[:nw], (n, keys, seq)
