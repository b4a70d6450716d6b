"""The multi-rank driver (quorum_intersection_amd.distributed) on CPU: gloo, world size 2.

A synthetic search backend replays the device engine's contract -- budgeted preorder
walks of subtree units, stack spills, segment logs keyed by root path, pruning after the
best witness -- over an irregular deterministic binary tree with planted witnesses, so
the coordination (frontier growth + broadcast + strided shares, best-key exchange,
rebalancing by send/recv, exact preorder reduction) is checked against a sequential
preorder walk.
"""
import os
import socket
import struct
from typing import List, Optional, Tuple

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from quorum_intersection_amd.distributed import (SearchBackend, best_of, distributed_search, needs_rebalance,
                                                 plan_rebalance, slice_bounds)

DEPTH = 14


def _h(bits: int, depth: int, salt: int) -> int:
    x = (bits * 0x9E3779B97F4A7C15 + depth * 0xBF58476D1CE4E5B9 + salt) & ((1 << 64) - 1)
    x ^= x >> 31
    x = (x * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return x ^ (x >> 29)


class Tree:
    """Node = (bits, depth): path bits MSB-first in a 32-bit word (depth <= 31)."""

    def __init__(self, salt: int, witnesses: List[Tuple[int, int]]):
        self.salt = salt
        self.wit = set(witnesses)

    def internal(self, bits, depth):
        return depth < DEPTH and (bits, depth) not in self.wit and _h(bits, depth, self.salt) % 7 != 0

    def evals(self, bits, depth):
        return 2 if self.internal(bits, depth) else 1 + _h(bits, depth, self.salt + 1) % 3

    def child(self, bits, depth, inc):
        return (bits | ((0x80000000 >> depth) if inc else 0), depth + 1)

    def preorder(self):
        """Sequential reference: count nodes/evals up to and including the first witness."""
        nodes = evals = 0
        stack = [(0, 0)]
        while stack:
            b, d = stack.pop()
            nodes += 1
            evals += self.evals(b, d)
            if (b, d) in self.wit:
                return nodes, evals, (b, d)
            if self.internal(b, d):
                stack.append(self.child(b, d, True))
                stack.append(self.child(b, d, False))
        return nodes, evals, None


def _after(k, b):  # preorder "strictly after" on (bits, depth)
    return (k[0], k[1]) > (b[0], b[1])


class FakeSearch(SearchBackend):
    key_words = 1
    unit_bytes = 8

    def __init__(self, tree: Tree, budget: int = 5, max_units: int = 7):
        self.t = tree
        self.budget = budget
        self.max_units = max_units  # units processed per "launch"
        self.restart()

    def restart(self):
        self.units: List[Tuple[int, int]] = [(0, 0)]
        self.log: List[Tuple[Tuple[int, int], int, int]] = []
        self.best: Optional[Tuple[int, int]] = None
        self.gbest: Optional[Tuple[int, int]] = None

    def reset(self):
        self.units = [(0, 0)]

    def clear(self):
        self.units = []

    def drop_log(self):
        self.log = []
        self.best = None
        self.gbest = None

    def frontier(self):
        return len(self.units)

    def keep_slice(self, b, e):
        self.units = self.units[b:e]

    def keep_strided(self, offset, stride):  # rotating deal, as qi_search_keep_strided
        self.units = [u for i, u in enumerate(self.units) if (i // stride + i) % stride == offset]

    def grow(self, target):
        while self.units and len(self.units) < target:
            self.step()

    def _pruned(self, k):
        return self.gbest is not None and _after(k, self.gbest)

    def step(self):
        take, self.units = self.units[: self.max_units], self.units[self.max_units:]
        out = []
        for root in take:
            if self._pruned(root):
                continue
            stack = [root]
            nodes = evals = 0
            while stack:
                if nodes >= self.budget:
                    out.extend(reversed(stack))
                    break
                b, d = stack.pop()
                if self._pruned((b, d)):
                    stack = []
                    break
                nodes += 1
                evals += self.t.evals(b, d)
                if (b, d) in self.t.wit:
                    if self.best is None or _after(self.best, (b, d)):
                        self.best = (b, d)
                    if self.gbest is None or _after(self.gbest, (b, d)):
                        self.gbest = (b, d)
                    stack = []
                    break
                if self.t.internal(b, d):
                    stack.append(self.t.child(b, d, True))
                    stack.append(self.t.child(b, d, False))
            self.log.append((root, nodes, evals))
        self.units = out + self.units

    def export(self, count, dst):
        moved, self.units = self.units[len(self.units) - count:], self.units[: len(self.units) - count]
        dst.copy_(torch.tensor(list(struct.pack(f"<{2 * count}I", *[x for u in moved for x in u])), dtype=torch.uint8))

    def import_(self, count, src):
        vals = struct.unpack(f"<{2 * count}I", bytes(src.tolist()))
        self.units.extend((vals[2 * i], vals[2 * i + 1]) for i in range(count))

    def local_best(self):
        return ((self.best[0],), self.best[1]) if self.best else None

    def set_best(self, key):
        k = (key[0][0], key[1])
        if self.gbest is None or _after(self.gbest, k):
            self.gbest = k

    def reduce(self, key):
        n = e = 0
        for root, nodes, evals in self.log:
            if key is not None and _after(root, (key[0][0], key[1])):
                continue
            n += nodes
            e += evals
        return {"nodes": n, "evals": e, "minq": 0, "zero_fallback": 0, "rounds": 0}

    def witness(self):
        return [self.best[0]], [self.best[1]]


TREES = [
    (1, []),
    (2, []),
    (3, [(0b1010 << 28, 4)]),
    (4, [(0b0111 << 28, 4), (0b0011 << 28, 4)]),
    (5, [(0b11 << 30, 2)]),
    (6, [(0xFF000000, 8), (0x0F000000, 10)]),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = []
        for (salt, wit), seed in [(tw, sd) for tw in TREES for sd in (0, 3, 40)]:
            t = Tree(salt, wit)
            be = FakeSearch(t, budget=3 + rank, max_units=5 + 3 * rank)
            r = distributed_search(be, device="cpu", lanes=16, min_move=1, seed_units=seed)
            res.append((salt, seed, r.verdict, r.nodes, r.evals, r.q1, r.q2, r.moved_units))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_distributed_gloo_world2_exact_counts():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    moved = 0
    for i, ((salt, wit), seed) in enumerate([(tw, sd) for tw in TREES for sd in (0, 3, 40)]):
        nodes, evals, w = Tree(salt, wit).preorder()
        for rank in (0, 1):
            s, sd, verdict, n, e, q1, q2, mv = out[rank][i]
            assert (s, sd) == (salt, seed)
            assert verdict == (w is None)
            assert (n, e) == (nodes, evals), (salt, rank, n, e, nodes, evals)
            if w is not None:
                assert (q1, q2) == ([w[0]], [w[1]])
            moved += mv
    assert moved > 0  # the rebalancing path ran


def test_single_process_driver_matches_preorder():
    for salt, wit in TREES:
        t = Tree(salt, wit)
        r = distributed_search(FakeSearch(t, budget=4, max_units=3), device="cpu", lanes=8)
        nodes, evals, w = t.preorder()
        assert (r.nodes, r.evals, r.verdict) == (nodes, evals, w is None)


def test_planning_helpers():
    assert [slice_bounds(10, r, 3) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert plan_rebalance([10, 0]) == [(0, 1, 5)]
    moves = plan_rebalance([100, 0, 50, 10])
    sizes = [100, 0, 50, 10]
    for s, d, c in moves:
        sizes[s] -= c
        sizes[d] += c
    assert max(sizes) - min(sizes) <= 1
    assert best_of([None, ((5,), 3), ((5,), 2), ((4,), 9)]) == ((4,), 9)
    assert needs_rebalance([10, 1000], lanes=64) and not needs_rebalance([500, 510], lanes=64)
