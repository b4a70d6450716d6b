"""Deterministic synthetic stellarbeat-format FBAS generators.

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
