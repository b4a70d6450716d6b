"""qi_gfp_batch_static (the entry point that allocates nothing) against qi_gfp_batch.

Both run containsQuorum (cpp:140-177) for a batch of (nodes, availableNodes) queries; the
static variant takes device masks and keeps its per-query state in the library's fixed
device scratch array.  Its results must equal the existing entry point's bit for bit, on
two calls in a row (the second smaller: the array keeps the first call's contents), and
the existing entry point's results are themselves checked against the oracle.
"""
import numpy as np
import pytest

import quorum_intersection_amd as qa
from quorum_intersection_amd import _capi
from qi_testlib import Oracle, fixture_text, random_fbas

pytestmark = pytest.mark.gpu


def _queries(n, count, seed):
    rng = np.random.default_rng(seed)
    w = max((n + 63) // 64, 1)
    nodes = rng.integers(0, 2**63, size=(count, w), dtype=np.uint64) | (rng.integers(0, 2, size=(count, w), dtype=np.uint64) << np.uint64(63))
    avail = nodes | rng.integers(0, 2**63, size=(count, w), dtype=np.uint64)
    tail = n % 64
    if tail:
        mask = np.uint64((1 << tail) - 1)
        nodes[:, -1] &= mask
        avail[:, -1] &= mask
    nodes[0] = avail[0]  # one query with every listed vertex available
    return nodes, avail


def _static(f, nodes, avail):
    import torch

    dev = torch.device("cuda", f.device)
    dn = torch.from_numpy(nodes.view(np.int64).copy()).to(dev)
    da = torch.from_numpy(avail.view(np.int64).copy()).to(dev)
    do = torch.full_like(dn, -1)
    torch.cuda.synchronize(dev)
    f.gfp_batch_static(dn.data_ptr(), da.data_ptr(), nodes.shape[0], do.data_ptr())
    return do.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("name,text", [
    ("broken.json", None),
    ("random_fbas(3, n=40)", None),
    ("threshold0", None),
])
def test_static_matches_gfp_batch_two_calls(name, text):
    if name == "broken.json":
        text = fixture_text("broken")
    elif name == "threshold0":  # threshold-0 sets: the kernel's exact ascending Gauss-Seidel sweep
        text = random_fbas(11, n=24, t0=True)
    else:
        text = random_fbas(3, n=40, t0=False)
    f = qa.FBAS(text, device=0)
    nodes, avail = _queries(f.n, 257, seed=5)
    want = f.gfp_batch(nodes, avail)  # existing entry point (also the set-up call)
    got = _static(f, nodes, avail)
    assert np.array_equal(got, want), name
    # second call, smaller input, different queries: stale state from the first call in the array
    nodes2, avail2 = _queries(f.n, 19, seed=6)
    want2 = f.gfp_batch(nodes2, avail2)
    got2 = _static(f, nodes2, avail2)
    assert np.array_equal(got2, want2), name
    # and the existing entry point agrees with the oracle on a sample of them
    o = Oracle().load(text)
    for i in range(0, 19, 6):
        ns = [v for v in range(f.n) if (int(nodes2[i, v >> 6]) >> (v & 63)) & 1]
        av = [bool((int(avail2[i, v >> 6]) >> (v & 63)) & 1) for v in range(f.n)]
        keep = set(o.contains_quorum(ns, av))
        gotset = {v for v in range(f.n) if (int(got2[i, v >> 6]) >> (v & 63)) & 1}
        assert gotset == keep, (name, i)


def test_static_needs_setup_and_rejects_oversize():
    import torch

    f = qa.FBAS(fixture_text("broken"), device=0)
    nodes, avail = _queries(f.n, 4, seed=1)
    dev = torch.device("cuda", 0)
    dn = torch.from_numpy(nodes.view(np.int64).copy()).to(dev)
    with pytest.raises(qa.QIError) as e:  # no set-up call yet
        f.gfp_batch_static(dn.data_ptr(), dn.data_ptr(), 4, dn.data_ptr())
    assert e.value.code == _capi.QI_ERR_STATE
    f.gfp_batch(nodes, avail)
    with pytest.raises(qa.QIError) as e:  # far more queries than the fixed array holds
        f.gfp_batch_static(dn.data_ptr(), dn.data_ptr(), 1 << 24, dn.data_ptr())
    assert e.value.code == _capi.QI_ERR_CAPACITY
    host = np.zeros((4, nodes.shape[1]), dtype=np.uint64)
    with pytest.raises(qa.QIError) as e:  # host memory is refused, not dereferenced on the GPU
        f.gfp_batch_static(host.ctypes.data, host.ctypes.data, 4, host.ctypes.data)
    assert e.value.code == _capi.QI_ERR_ARG


def test_static_on_caller_stream():
    import torch

    f = qa.FBAS(fixture_text("correct"), device=0)
    nodes, avail = _queries(f.n, 64, seed=9)
    want = f.gfp_batch(nodes, avail)
    dev = torch.device("cuda", 0)
    dn = torch.from_numpy(nodes.view(np.int64).copy()).to(dev)
    da = torch.from_numpy(avail.view(np.int64).copy()).to(dev)
    do = torch.zeros_like(dn)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(st):
        f.gfp_batch_static(dn.data_ptr(), da.data_ptr(), 64, do.data_ptr(), stream=st.cuda_stream)
    st.synchronize()
    assert np.array_equal(do.cpu().numpy().view(np.uint64), want)
