"""Snapshot sanity filter: drop validators whose quorum set can never be satisfied.

Host-side mirror of the reference's offline scrubber ``fix_quorum_configurations.py``
(fix_quorum_configurations.py:11-15), kept interface-compatible so that a pipeline of the form

    python fix_quorum_configurations.py < snapshot.json > fixed.json

can become

    python -m quorum_intersection_amd.sanity < snapshot.json > fixed.json

Semantics (fix_quorum_configurations.py:11-15): a node is kept iff
``len(validators) + len(innerQuorumSets) >= threshold`` of its *top-level* quorum set
(inner sets are not inspected, duplicates count).  The reference indexes the quorum set
directly, so a ``null`` quorumSet raises ``TypeError`` and a missing key raises
``KeyError``; both are reproduced (``strict=False`` instead keeps such nodes, which is what
quorum_intersection.cpp:405-408 does with them: a never-satisfied empty set).  Output is
the stdlib ``json.dump`` text of the kept nodes in input order (py:8), byte-identical to
the reference's.  Not on the GPU path: the checker itself accepts insane sets
(containsQuorumSlice, cpp:99-138, simply never satisfies them).
"""
from __future__ import annotations

import json
import sys
from typing import Any, Iterable, List, TextIO


def is_quorum_config_sane(q_set: Any) -> bool:
    """fix_quorum_configurations.py:11-12: entry count >= threshold."""
    entries = len(q_set["validators"]) + len(q_set["innerQuorumSets"])
    return entries >= q_set["threshold"]


def fix_configuration(config: Iterable[Any], strict: bool = True) -> List[Any]:
    """fix_quorum_configurations.py:14-15: the nodes with a sane quorum set, in order."""
    kept = []
    for node in config:
        q_set = node["quorumSet"]
        if not strict and (not isinstance(q_set, dict) or "threshold" not in q_set):
            kept.append(node)
            continue
        if is_quorum_config_sane(q_set):
            kept.append(node)
    return kept


def load_quorum_definitions(stream: TextIO) -> Any:
    return json.load(stream)


def store_quorum_definitions(data: Any, stream: TextIO) -> None:
    json.dump(data, stream)


def main(argv: List[str] | None = None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description="drop validators whose top-level threshold exceeds their entries")
    ap.add_argument("--lenient", action="store_true",
                    help="keep null/incomplete quorum sets instead of failing like the reference script")
    args = ap.parse_args(argv)
    data = fix_configuration(load_quorum_definitions(sys.stdin), strict=not args.lenient)
    store_quorum_definitions(data, sys.stdout)
    return 0


if __name__ == "__main__":
    sys.exit(main())
