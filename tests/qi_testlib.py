"""Test helpers: the CPU oracle (oracle/qi_oracle.cpp via ctypes) and random FBAS inputs.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load the oracle.
"""
from __future__ import annotations

import ctypes
import json
import os
import random
import subprocess
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# QI_ORACLE_SO: another build of the same oracle source (bench.py times the -O0 build, the
# reference's documented CMake build having no build type)
ORACLE_SO = os.environ.get("QI_ORACLE_SO") or os.path.join(ORACLE_DIR, "_build", "libqi_oracle.so")
ORACLE_BIN = os.path.join(ORACLE_DIR, "_build", "qi_oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
FIXTURES = ["correct", "broken", "correct_trivial", "broken_trivial"]


def build_oracle() -> None:
    if not (os.path.exists(ORACLE_SO) and os.path.exists(ORACLE_BIN)):
        subprocess.run(["make", "-C", ORACLE_DIR, "-j4"], check=True, capture_output=True)


class Oracle:
    _lib = None

    def __init__(self):
        if Oracle._lib is None:
            build_oracle()
            L = ctypes.CDLL(ORACLE_SO)
            L.qio_load.restype = ctypes.c_void_p
            L.qio_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
            L.qio_last_error.restype = ctypes.c_char_p
            L.qio_free.argtypes = [ctypes.c_void_p]
            L.qio_free_str.argtypes = [ctypes.c_void_p]
            L.qio_num_vertices.restype = ctypes.c_uint64
            L.qio_num_vertices.argtypes = [ctypes.c_void_p]
            L.qio_contains_quorum.restype = ctypes.c_uint64
            L.qio_contains_quorum.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64,
                                              ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint32)]
            L.qio_slice.restype = ctypes.c_int
            L.qio_slice.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint8)]
            for fn in ("qio_graph_json", "qio_solve", "qio_solve_text", "qio_pagerank_text"):
                getattr(L, fn).restype = ctypes.c_void_p
            L.qio_graph_json.argtypes = [ctypes.c_void_p]
            L.qio_solve.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
            L.qio_solve_text.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            L.qio_pagerank_text.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_uint64]
            Oracle._lib = L
        self.L = Oracle._lib

    def _str(self, p) -> str:
        s = ctypes.cast(p, ctypes.c_char_p).value.decode(errors="surrogateescape")
        self.L.qio_free_str(p)
        return s

    def load(self, text) -> "OracleGraph":
        b = text.encode() if isinstance(text, str) else bytes(text)
        h = self.L.qio_load(b, len(b))
        if not h:
            raise ValueError(self.L.qio_last_error().decode())
        return OracleGraph(self, h)


class OracleGraph:
    def __init__(self, o: Oracle, h):
        self.o, self.h = o, h
        self.n = int(o.L.qio_num_vertices(h))

    def __del__(self):
        try:
            self.o.L.qio_free(self.h)
        except Exception:
            pass

    def graph(self) -> Dict:
        return json.loads(self.o._str(self.o.L.qio_graph_json(self.h)))

    def solve(self, tiebreak: int = 0, seed: int = 0, budget: int = 0) -> Dict:
        return json.loads(self.o._str(self.o.L.qio_solve(self.h, tiebreak, seed, budget)))

    def solve_text(self, verbose=False, graphviz=False) -> str:
        return self.o._str(self.o.L.qio_solve_text(self.h, int(verbose), int(graphviz)))

    def pagerank_text(self, m=0.0001, c=0.0001, iters=100000) -> str:
        return self.o._str(self.o.L.qio_pagerank_text(self.h, m, c, iters))

    def contains_quorum(self, nodes: List[int], avail: List[bool]) -> List[int]:
        xs = (ctypes.c_uint32 * max(len(nodes), 1))(*nodes)
        av = (ctypes.c_uint8 * max(self.n, 1))(*[1 if a else 0 for a in avail])
        out = (ctypes.c_uint32 * max(len(nodes), 1))()
        k = self.o.L.qio_contains_quorum(self.h, xs, len(nodes), av, out)
        return [int(out[i]) for i in range(k)]

    def slice(self, v: int, avail: List[bool]) -> bool:
        av = (ctypes.c_uint8 * max(self.n, 1))(*[1 if a else 0 for a in avail])
        return bool(self.o.L.qio_slice(self.h, v, av))


def fixture_text(name: str) -> bytes:
    with open(os.path.join(GOLDEN, name + ".json"), "rb") as f:
        return f.read()


# ------------------------------------------------------------------------------------
# Random stellarbeat-format FBAS with the quirks the reference's semantics expose:
# nested inner sets, duplicate validator refs, unknown ids (-> vertex 0), null quorum
# sets, threshold 0 and threshold > entries, self references.
# ------------------------------------------------------------------------------------
def random_fbas(seed: int, n: int = 12, depth: int = 2, quirks: bool = True, max_inner: int = 3, t0: bool = True) -> str:
    rng = random.Random(seed)
    keys = [f"V{seed}_{i}" for i in range(n)]

    def qset(level: int) -> Dict:
        nv = rng.randint(0, min(5, n))
        vals = [rng.choice(keys) for _ in range(nv)]
        if quirks and rng.random() < 0.1:
            vals.append("UNKNOWN_" + str(rng.randint(0, 3)))
        if quirks and vals and rng.random() < 0.15:
            vals.append(rng.choice(vals))  # duplicate reference
        inner = []
        if level < depth:
            for _ in range(rng.randint(0, max_inner)):
                inner.append(qset(level + 1))
        entries = len(vals) + len(inner)
        if entries == 0:
            vals = [rng.choice(keys)]
            entries = 1
        t = rng.randint(1, entries)
        if quirks:
            r = rng.random()
            if r < 0.05:
                t = 0 if t0 else t
            elif r < 0.08:
                t = entries + rng.randint(1, 2)
        return {"threshold": t, "validators": vals, "innerQuorumSets": inner}

    nodes = []
    for i, k in enumerate(keys):
        if quirks and rng.random() < 0.08:
            q = None
        else:
            q = qset(0)
        nodes.append({"publicKey": k, "name": f"node {i}", "quorumSet": q})
    return json.dumps(nodes)


def random_masks(rng: random.Random, n: int, count: int, p: float = 0.6) -> List[List[int]]:
    return [[v for v in range(n) if rng.random() < p] for _ in range(count)]


def random_org_fbas(seed: int, n_orgs: int = 6, quirks: bool = True, t0: bool = False) -> str:
    """Search-heavy random FBAS: organisations of 1-4 validators whose quorum sets are
    random threshold trees over organisations (so the main SCC is large), with
    occasional duplicate refs, outside/unknown refs and t > entries; threshold 0 only
    with t0=True (anti-monotone slices: the search then runs the order-exact kernel, whose
    counts and witnesses are compared with the oracle like any other)."""
    rng = random.Random(seed)
    orgs = []
    for o in range(n_orgs):
        orgs.append([f"O{seed}_{o}_{j}" for j in range(rng.randint(1, 4))])
    keys = [k for org in orgs for k in org]

    def org_set(org):
        t = rng.randint(1, len(org))
        vals = list(org)
        if quirks and rng.random() < 0.1:
            vals.append(rng.choice(org))
        return {"threshold": t, "validators": vals, "innerQuorumSets": []}

    nodes = []
    for o, org in enumerate(orgs):
        for k in org:
            picked = [x for x in range(n_orgs) if rng.random() < 0.75] or [o]
            inner = [org_set(orgs[x]) for x in picked]
            vals = []
            if rng.random() < 0.3:
                vals = rng.sample(keys, rng.randint(1, 3))
            if quirks and rng.random() < 0.1:
                vals.append("OUTSIDE_" + str(rng.randint(0, 2)))
            entries = len(inner) + len(vals)
            t = max(1, int(round(entries * rng.uniform(0.4, 0.8))))
            r0, r1 = rng.random(), rng.random()
            if quirks and t0 and r0 < 0.03:
                t = 0
            if quirks and r1 < 0.03:
                t = entries + 1
            nodes.append({"publicKey": k, "name": k.lower(), "quorumSet":
                          {"threshold": t, "validators": vals, "innerQuorumSets": inner}})
    return json.dumps(nodes)
