"""CPU-only checks of the product library: it loads, exports every C-ABI symbol declared
in include/quorum_intersection.h, and its host stages (JSON ingestion with
property_tree semantics, graph build, boost-numbered SCCs) agree with the oracle.
No compute entry point is called here (no GPU)."""
import json
import os
import re
import subprocess

import pytest

from qi_testlib import FIXTURES, ROOT, Oracle, fixture_text, random_fbas
import quorum_intersection_amd as qa
from quorum_intersection_amd import _capi, fbas_gen

HEADER = os.path.join(ROOT, "include", "quorum_intersection.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(qi_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = qa.lib()
    names = header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
        assert n in _capi.SIGNATURES, f"{n} missing from the ctypes signature table"
    assert L.qi_abi_version() == 4


def test_library_has_gfx950_code_object():
    so = _capi.LIB_PATH
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", so], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(so, "rb").read()
    assert b"gfx950" in blob


def _product_graph(text):
    f = qa.FBAS(text, device=0)
    return f.adjacency(), f.scc_ids(), f.n_sccs, [f.vertex(v)[0] for v in range(f.n)]


def _oracle_graph(text):
    g = Oracle().load(text).graph()
    return g["adj"], g["comp"], g["nscc"], g["ids"]


@pytest.mark.parametrize("name", FIXTURES)
def test_graph_and_scc_parity_fixtures(name):
    t = fixture_text(name)
    assert _product_graph(t) == _oracle_graph(t)


@pytest.mark.parametrize("seed", range(30))
def test_graph_and_scc_parity_random(seed):
    t = random_fbas(seed, n=20)
    assert _product_graph(t) == _oracle_graph(t)


def test_graph_parity_generated():
    for t in (fbas_gen.tiered(4), fbas_gen.two_tier(5, 64), fbas_gen.planted(4, 40), fbas_gen.tiered(6, seed=7)):
        assert _product_graph(t) == _oracle_graph(t)


EDGE_CASES = {
    "empty_array": "[]",
    "top_level_object": json.dumps({"a": {"publicKey": "A", "quorumSet": {"threshold": 1, "validators": ["A"],
                                                                         "innerQuorumSets": []}}}),
    "threshold_as_string": json.dumps([{"publicKey": "A", "quorumSet": {"threshold": " 1 ", "validators": ["A"],
                                                                         "innerQuorumSets": []}}]),
    "threshold_negative": json.dumps([{"publicKey": "A", "quorumSet": {"threshold": -1, "validators": ["A"],
                                                                        "innerQuorumSets": []}}]),
    # property_tree keeps "-1" as text and get<size_t> wraps it to SIZE_MAX (libstdc++
    # num_get, no failbit): a never-satisfiable threshold, not a parse error
    "threshold_negative_string": json.dumps([{"publicKey": "A", "quorumSet": {"threshold": "-1", "validators": ["A"],
                                                                               "innerQuorumSets": []}}]),
    "threshold_minus_zero": json.dumps([{"publicKey": "A", "quorumSet": {"threshold": "-0", "validators": ["A"],
                                                                          "innerQuorumSets": []}}]),
    "threshold_float": json.dumps([{"publicKey": "A", "quorumSet": {"threshold": 1.0, "validators": ["A"],
                                                                     "innerQuorumSets": []}}]),
    "missing_validators": json.dumps([{"publicKey": "A", "quorumSet": {"threshold": 1, "innerQuorumSets": []}}]),
    "missing_quorumset": json.dumps([{"publicKey": "A"}]),
    "missing_publickey": json.dumps([{"name": "x", "quorumSet": None}]),
    "null_everything": json.dumps([{"publicKey": "A", "name": None, "quorumSet": None}]),
    "quorumset_scalar": json.dumps([{"publicKey": "A", "quorumSet": 7}]),
    "duplicate_keys": json.dumps([
        {"publicKey": "A", "quorumSet": {"threshold": 1, "validators": ["B"], "innerQuorumSets": []}},
        {"publicKey": "B", "quorumSet": {"threshold": 1, "validators": ["A"], "innerQuorumSets": []}},
        {"publicKey": "A", "quorumSet": {"threshold": 2, "validators": ["A", "C"], "innerQuorumSets": []}},
    ]),
    "unknown_ids": json.dumps([
        {"publicKey": "A", "quorumSet": {"threshold": 2, "validators": ["X", "Y", "A"], "innerQuorumSets": []}},
        {"publicKey": "B", "quorumSet": {"threshold": 1, "validators": ["Z"], "innerQuorumSets": []}},
    ]),
    "unicode_escapes": '[{"publicKey": "\\u00e9\\ud83d\\ude00", "name": "n\\n", "quorumSet": null}]',
    "bad_json": '[{"publicKey": "A", }]',
    "trailing_garbage": "[] x",
    "validators_null": json.dumps([{"publicKey": "A", "quorumSet": {"threshold": 1, "validators": None,
                                                                     "innerQuorumSets": None}}]),
    "number_key": json.dumps([{"publicKey": 12, "quorumSet": {"threshold": 1, "validators": [12],
                                                              "innerQuorumSets": []}}]),
}


@pytest.mark.parametrize("case", sorted(EDGE_CASES))
def test_json_edge_case_parity(case):
    text = EDGE_CASES[case]
    o_err = p_err = None
    try:
        o = _oracle_graph(text)
    except ValueError as e:
        o_err = str(e)
    try:
        p = _product_graph(text)
    except qa.QIError as e:
        p_err = e
    assert (o_err is None) == (p_err is None), (case, o_err, p_err)
    if p_err is not None:
        assert p_err.code == _capi.QI_ERR_PARSE
    else:
        assert p == o


def test_no_device_entry_points_fail_loudly_without_gpu():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    f = qa.FBAS(fixture_text("correct"))
    with pytest.raises(qa.QIError) as e:
        f.solve_stats()
    assert e.value.code == _capi.QI_ERR_DEVICE


def test_pagerank_text_matches_oracle():
    # -p is host code (float power iteration, cpp:532-613)
    for name in FIXTURES:
        t = fixture_text(name)
        assert qa.pagerank_text(t) == Oracle().load(t).pagerank_text()
    t = fixture_text("correct")
    assert qa.pagerank_text(t, 0.15, 1e-6, 50) == Oracle().load(t).pagerank_text(0.15, 1e-6, 50)


def test_cli_help_and_invalid_option():
    exe = os.path.join(ROOT, "bin", "quorum_intersection")
    r = subprocess.run([exe, "-h"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("Allowed options:\n") and r.stdout.endswith("algorithm\n\n")
    r = subprocess.run([exe, "--bogus"], capture_output=True, text=True)
    assert r.returncode == 1 and r.stdout.startswith("Invalid option!\nAllowed options:")
    r = subprocess.run([exe, "-p"], input=fixture_text("correct_trivial"), capture_output=True)
    assert r.returncode == 0
    assert r.stdout.decode() == Oracle().load(fixture_text("correct_trivial")).pagerank_text()


@pytest.mark.parametrize("case", ["broken", "two_tier_10", "planted_20_80", "org_multiplicity", "threshold0"])
def test_specialised_kernel_sources_compile(case):
    # hipRTC compiles the generated evaluator + the shared kernel header for gfx950 on the
    # CPU (no device needed); exercised at run time by the -m gpu parity suite.
    from qi_testlib import random_org_fbas
    texts = {
        "broken": fixture_text("broken"),
        "two_tier_10": fbas_gen.two_tier(10, 256),
        "planted_20_80": fbas_gen.planted(20, 80),
        "org_multiplicity": random_org_fbas(9, 7),
        "threshold0": random_org_fbas(3, 6, t0=True),
    }
    if case == "threshold0":  # threshold-0 SCCs run the ordered kernel, which has no specialised form
        with pytest.raises(qa.QIError) as e:
            qa.FBAS(texts[case]).jit_precompile()
        assert e.value.code == _capi.QI_ERR_UNSUPPORTED
        return
    ms = qa.FBAS(texts[case]).jit_precompile()
    assert ms >= 0


def test_bench_default_workloads_have_golden_counts():
    # bench.py checks every measured search against these (node count, verdict)
    import json
    big = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_big.json")))
    for key in ("two_tier_10_256", "planted_deep_8_512"):
        assert key in big and big[key]["nodes"] > 0 and "verdict" in big[key]
