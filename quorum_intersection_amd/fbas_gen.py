"""Deterministic synthetic stellarbeat-format FBAS generators (benchmark and test workloads).

The reference ships no generator; these produce JSON arrays in the exact input format
parsed by quorum_intersection.cpp:420-436 (``publicKey``, ``name``, ``quorumSet`` with
``threshold`` / ``validators`` / ``innerQuorumSets``).  No random values appear in
quorum sets; ``seed`` only permutes the order of the JSON entries (0 = identity).

G1 ``tiered(k)``      one SCC of k organisations x 3 validators; every validator trusts
                      ceil(2k/3) of the k organisations, each organisation 2-of-3.
G2 ``two_tier(k, N)`` G1(k) as the top tier (vertices 0..3k-1, so it is Tarjan component
                      #0, cpp:621/691) plus N-3k lower validators in organisations of 3
                      that each need 2-of-{top tier, own organisation}.
G3 ``planted(k, N)``  G2 with a planted pair of disjoint quorums inside the top tier:
                      two extra top-tier organisations A, B whose members trust only
                      their own organisation plus the tier, so that {A} and {B} are each
                      quorums on their own, reached deep in the exclusion-first search.
"""
from __future__ import annotations

import json
import math
import random
from typing import Dict, List


def _key(prefix: str, i: int, j: int) -> str:
    return f"G{prefix}{i:04d}X{j}"


def _qset(threshold: int, validators=None, inner=None) -> Dict:
    return {
        "threshold": threshold,
        "validators": list(validators or []),
        "innerQuorumSets": list(inner or []),
    }


def tiered_nodes(k: int, org_size: int = 3, inner_threshold: int = 2, prefix: str = "T") -> List[Dict]:
    orgs = [[_key(prefix, o, j) for j in range(org_size)] for o in range(k)]
    top = _qset(math.ceil(2 * k / 3), [], [_qset(inner_threshold, org) for org in orgs])
    nodes = []
    for o, org in enumerate(orgs):
        for j, pk in enumerate(org):
            nodes.append({"publicKey": pk, "name": f"top org {o} validator {j}", "quorumSet": top})
    return nodes


def two_tier_nodes(k_top: int, n_total: int) -> List[Dict]:
    top = tiered_nodes(k_top)
    top_qset = top[0]["quorumSet"]
    n_lower = n_total - len(top)
    if n_lower < 0:
        raise ValueError("n_total smaller than the top tier")
    nodes = list(top)
    o = 0
    while n_lower > 0:
        size = min(3, n_lower)
        org = [_key("L", o, j) for j in range(size)]
        qs = _qset(2, [], [top_qset, _qset(min(2, size), org)])
        for j, pk in enumerate(org):
            nodes.append({"publicKey": pk, "name": f"lower org {o} validator {j}", "quorumSet": qs})
        n_lower -= size
        o += 1
    return nodes


def planted_nodes(k_top: int, n_total: int) -> List[Dict]:
    """Top tier of k_top organisations plus two planted organisations A and B (3 each)
    whose validators accept 2-of-3 of their own organisation alone (as one inner set of a
    1-of-2 root: {own org, tier}); the tier members do not list A or B, so A and B
    trust the tier but not each other: {A} and {B} are disjoint quorums.  A and B are
    placed last in the top tier so the exclusion-first search reaches them late."""
    orgs = [[_key("T", o, j) for j in range(3)] for o in range(k_top)]
    tier = _qset(math.ceil(2 * k_top / 3), [], [_qset(2, org) for org in orgs])
    a = [_key("A", 0, j) for j in range(3)]
    b = [_key("B", 0, j) for j in range(3)]
    nodes = []
    for o, org in enumerate(orgs):
        for j, pk in enumerate(org):
            nodes.append({"publicKey": pk, "name": f"top org {o} validator {j}", "quorumSet": tier})
    for tag, org in (("A", a), ("B", b)):
        qs = _qset(1, [], [_qset(2, org), tier])
        for j, pk in enumerate(org):
            nodes.append({"publicKey": pk, "name": f"planted {tag} validator {j}", "quorumSet": qs})
    # tier members must reach A and B for one SCC: add them as a never-satisfiable-alone
    # extra inner set of the tier (threshold unchanged), keeping quorums inside the tier.
    tier["innerQuorumSets"].append(_qset(3, a + b))
    n_lower = n_total - len(nodes)
    top_qset = tier
    o = 0
    while n_lower > 0:
        size = min(3, n_lower)
        org = [_key("L", o, j) for j in range(size)]
        qs = _qset(2, [], [top_qset, _qset(min(2, size), org)])
        for j, pk in enumerate(org):
            nodes.append({"publicKey": pk, "name": f"lower org {o} validator {j}", "quorumSet": qs})
        n_lower -= size
        o += 1
    return nodes


def planted_deep_nodes(k: int = 8, n_total: int = 512, plant: bool = True) -> List[Dict]:
    """A tier of k organisations (k >= 8, 2-of-3 inside, ceil(2k/3)-of-k outside) whose
    members also accept an alternative slice, planting two disjoint quorums that the
    exclusion-first search (arXiv 1902.06493) can only pair up late in preorder:

    * A side: organisations 0-3 and hub HA (3, 2-of-3).  An A member also accepts
      {2 of its organisation, 2 of HA, b0} where b0 = member 0 of organisation 0; an HA
      member needs {2 of HA, b0, 2 of each of organisations 0-3}; b0 also accepts {2 of HA}.  QA = b0 + one more
      of organisation 0 + 2 of each of organisations 1-3 + 2 of HA (10 vertices) is a
      quorum, and every QA contains b0.
    * B side: organisations 4..k-1 and hub HB (5, 5-of-5).  A B member also accepts {all 3 of
      its organisation, all of HB}; an HB member accepts {all of HB, all of organisations
      4..k-1}.  QB = all of them (3(k-4) + 5 vertices, more than half the SCC): never a
      candidate set of the search (|D| <= m/2), only found by the visitor.
    * QA and QB each hold 2 members of enough organisations to meet every tier quorum, so
      every minimal quorum without b0 intersects every quorum: the root's exclusion
      subtree (b0 has the highest in-degree and is the root's branch vertex) is
      witness-free, and the first witness (D = a QA, complement containing QB) lies in the
      root's inclusion subtree.
    Lower validators (organisations of 3 trusting the tier) fill up to n_total.
    plant=False adds b0 to every HB slice, so every QB meets every QA: the same search tree
    without the witness (its full size is the yardstick for the witness's depth)."""
    assert k >= 8
    orgs = [[_key("T", o, j) for j in range(3)] for o in range(k)]
    tier = _qset(math.ceil(2 * k / 3), [], [_qset(2, org) for org in orgs])
    ha = [_key("HA", 0, j) for j in range(3)]
    hb = [_key("HB", 0, j) for j in range(5)]
    b0 = orgs[0][0]
    a_orgs, b_orgs = orgs[:4], orgs[4:]
    nodes = []
    for o, org in enumerate(orgs):
        for j, pk in enumerate(org):
            if o < 4:
                alt = _qset(3, [b0], [_qset(2, org), _qset(2, ha)])
                if pk == b0:
                    alt = _qset(1, [], [_qset(2, ha), alt])
            else:
                alt = _qset(2, [], [_qset(3, org), _qset(len(hb), hb)])
            nodes.append({"publicKey": pk, "name": f"tier org {o} validator {j}",
                          "quorumSet": _qset(1, [], [tier, alt])})
    a_block = _qset(4, [], [_qset(2, org) for org in a_orgs])  # 2 of each A organisation
    for j, pk in enumerate(ha):
        nodes.append({"publicKey": pk, "name": f"hub A {j}", "quorumSet": _qset(3, [b0], [_qset(2, ha), a_block])})
    hb_inner = [_qset(len(hb), hb)] + [_qset(3, org) for org in b_orgs]
    hb_vals = [] if plant else [b0]
    for j, pk in enumerate(hb):
        nodes.append({"publicKey": pk, "name": f"hub B {j}",
                      "quorumSet": _qset(len(hb_vals) + len(hb_inner), hb_vals, hb_inner)})
    n_lower = n_total - len(nodes)
    o = 0
    while n_lower > 0:
        size = min(3, n_lower)
        org = [_key("L", o, j) for j in range(size)]
        qs = _qset(2, [], [tier, _qset(min(2, size), org)])
        for j, pk in enumerate(org):
            nodes.append({"publicKey": pk, "name": f"lower org {o} validator {j}", "quorumSet": qs})
        n_lower -= size
        o += 1
    return nodes


def to_json(nodes: List[Dict], seed: int = 0) -> str:
    nodes = list(nodes)
    if seed:
        random.Random(seed).shuffle(nodes)
    return json.dumps(nodes, indent=1)


def tiered(k: int, seed: int = 0) -> str:
    return to_json(tiered_nodes(k), seed)


def two_tier(k_top: int, n_total: int, seed: int = 0) -> str:
    return to_json(two_tier_nodes(k_top, n_total), seed)


def planted(k_top: int, n_total: int, seed: int = 0) -> str:
    return to_json(planted_nodes(k_top, n_total), seed)


def planted_deep(k: int = 8, n_total: int = 512, seed: int = 0, plant: bool = True) -> str:
    return to_json(planted_deep_nodes(k, n_total, plant), seed)
