"""Sanity filter (quorum_intersection_amd/sanity.py) vs the semantics of the reference's
fix_quorum_configurations.py:11-15.  There are no reference outputs for this script (it
raises on every bundled snapshot: their null quorumSets, py:12), so the expected results
below are restated by hand from those lines; parity beyond them is unpinned."""
import io
import json
import subprocess
import sys

import pytest

from qi_testlib import ROOT, fixture_text
from quorum_intersection_amd import sanity


def node(key, thr, validators=(), inner=()):
    return {"publicKey": key, "name": key.lower(),
            "quorumSet": {"threshold": thr, "validators": list(validators), "innerQuorumSets": list(inner)}}


def test_keeps_sane_and_drops_over_threshold():
    inner = {"threshold": 9, "validators": [], "innerQuorumSets": []}  # inner sets are not inspected
    cfg = [node("A", 2, ["A", "B"]),            # 2 >= 2
           node("B", 3, ["A", "B"]),            # 2 < 3: dropped
           node("C", 2, ["A"], [inner]),        # 1 + 1 >= 2
           node("D", 0),                        # 0 >= 0
           node("E", 1),                        # 0 < 1: dropped
           node("F", 2, ["A", "A"])]            # duplicates count
    kept = sanity.fix_configuration(cfg)
    assert [n["publicKey"] for n in kept] == ["A", "C", "D", "F"]


def test_null_quorum_set_raises_like_the_reference():
    with pytest.raises(TypeError):
        sanity.fix_configuration(json.loads(fixture_text("correct")))
    with pytest.raises(KeyError):
        sanity.fix_configuration([{"publicKey": "X", "quorumSet": {"threshold": 1}}])


@pytest.mark.parametrize("name", ["correct", "broken"])
def test_lenient_keeps_null_sets_and_fixtures_are_sane(name):
    data = json.loads(fixture_text(name))
    assert sanity.fix_configuration(data, strict=False) == data


@pytest.mark.parametrize("name", ["correct_trivial", "broken_trivial"])
def test_cli_output_is_stdlib_json_dump(name):
    text = fixture_text(name).decode()
    out = subprocess.run([sys.executable, "-m", "quorum_intersection_amd.sanity"], input=text, capture_output=True,
                         text=True, cwd=ROOT, check=True).stdout
    buf = io.StringIO()
    json.dump(json.loads(text), buf)
    assert out == buf.getvalue()


def test_cli_fails_on_null_sets_unless_lenient():
    text = fixture_text("broken").decode()
    r = subprocess.run([sys.executable, "-m", "quorum_intersection_amd.sanity"], input=text, capture_output=True,
                       text=True, cwd=ROOT)
    assert r.returncode != 0 and "TypeError" in r.stderr
    r = subprocess.run([sys.executable, "-m", "quorum_intersection_amd.sanity", "--lenient"], input=text,
                       capture_output=True, text=True, cwd=ROOT, check=True)
    assert json.loads(r.stdout) == json.loads(text)
