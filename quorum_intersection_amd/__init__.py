"""MI355X-native quorum-intersection checker (drop-in for fixxxedpoint/quorum_intersection).

Host mirror of the reference's interface over the C-ABI (include/quorum_intersection.h):

    solve(json_text, verbose=False, graphviz=False) -> bool       # solve(istream&,...) cpp:709
    FBAS(json_text).containsQuorum(nodes, availableNodes) -> list  # containsQuorum   cpp:140
    FBAS(json_text).checkMinimalQuorums() -> (bool, q1, q2)        # checkMinimalQuorums cpp:348
    FBAS(json_text).solve_stats() -> dict                          # solve(Graph) + counters

Everything that evaluates quorums runs in HIP kernels for gfx950; without a GPU these
calls raise QIError(QI_ERR_DEVICE).  JSON ingestion, graph building and the SCC
decomposition are host C++ (as in the reference) and work without a GPU.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _capi
from ._capi import QIError, check, lib

__all__ = ["FBAS", "QIError", "solve", "solve_text", "pagerank_text", "lib", "masks_from_sets"]


def _u32p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def masks_from_sets(sets: Sequence[Sequence[int]], n: int) -> np.ndarray:
    """Pack vertex sets into [len(sets), ceil(n/64)] uint64 masks (bit v%64 of word v//64)."""
    w = (n + 63) // 64
    out = np.zeros((len(sets), max(w, 1)), dtype=np.uint64)
    for i, s in enumerate(sets):
        for v in s:
            out[i, v >> 6] |= np.uint64(1) << np.uint64(v & 63)
    return out


def sets_from_masks(masks: np.ndarray, n: int) -> List[List[int]]:
    res = []
    for row in masks:
        bits = np.unpackbits(row.view(np.uint8), bitorder="little")[:n]
        res.append([int(v) for v in np.nonzero(bits)[0]])
    return res


class FBAS:
    """A parsed stellarbeat configuration (vertices, trust graph, SCCs) bound to a GPU."""

    def __init__(self, json_text, device: int = 0):
        data = json_text.encode() if isinstance(json_text, str) else bytes(json_text)
        h = ctypes.c_void_p()
        check(lib().qi_fbas_from_json(data, len(data), device, ctypes.byref(h)))
        self._h = h
        self.device = device
        self.n = int(lib().qi_fbas_num_vertices(h))

    def close(self):
        if getattr(self, "_h", None):
            lib().qi_fbas_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---- host-side structure ---------------------------------------------------------
    @property
    def n_sccs(self) -> int:
        return int(lib().qi_fbas_num_sccs(self._h))

    def scc_ids(self) -> List[int]:
        a = np.zeros(max(self.n, 1), dtype=np.uint32)
        check(lib().qi_fbas_scc_ids(self._h, _u32p(a)))
        return [int(x) for x in a[: self.n]]

    def sccs(self) -> List[List[int]]:
        ids = self.scc_ids()
        out: List[List[int]] = [[] for _ in range(self.n_sccs)]
        for v, c in enumerate(ids):
            out[c].append(v)
        return out

    def adjacency(self) -> List[List[int]]:
        ne = int(lib().qi_fbas_num_edges(self._h))
        off = np.zeros(self.n + 1, dtype=np.uint32)
        tgt = np.zeros(max(ne, 1), dtype=np.uint32)
        check(lib().qi_fbas_adjacency(self._h, _u32p(off), _u32p(tgt)))
        return [[int(x) for x in tgt[off[v]: off[v + 1]]] for v in range(self.n)]

    def vertex(self, v: int) -> Tuple[str, str]:
        pk, nm = ctypes.c_char_p(), ctypes.c_char_p()
        check(lib().qi_fbas_vertex(self._h, v, ctypes.byref(pk), ctypes.byref(nm)))
        return pk.value.decode(errors="surrogateescape"), nm.value.decode(errors="surrogateescape")

    # ---- device: containsQuorum ------------------------------------------------------
    def gfp_batch(self, nodes: np.ndarray, avail: np.ndarray) -> np.ndarray:
        """Batched containsQuorum on uint64 masks [B, ceil(n/64)]."""
        nodes = np.ascontiguousarray(nodes, dtype=np.uint64)
        avail = np.ascontiguousarray(avail, dtype=np.uint64)
        if nodes.shape != avail.shape or nodes.ndim != 2 or nodes.shape[1] != max((self.n + 63) // 64, 1):
            raise ValueError("masks must be [B, ceil(n/64)] and equal shapes")
        out = np.zeros_like(nodes)
        check(lib().qi_gfp_batch(self._h, _u64p(nodes), _u64p(avail), nodes.shape[0], _u64p(out)))
        return out

    def gfp_batch_static(self, d_nodes: int, d_avail: int, count: int, d_out: int, stream: int = 0) -> None:
        """qi_gfp_batch_static: the same fixpoints on DEVICE masks (raw device addresses of
        [count, ceil(n/64)] uint64 arrays on this FBAS's GPU) with no allocation; needs one
        earlier gfp_batch / solve on this FBAS (set-up)."""
        check(lib().qi_gfp_batch_static(self._h, ctypes.c_void_p(d_nodes), ctypes.c_void_p(d_avail), count,
                                        ctypes.c_void_p(d_out), ctypes.c_void_p(stream or None)))

    def containsQuorum(self, nodes: Sequence[int], availableNodes: Sequence[bool]) -> List[int]:
        """containsQuorum(nodes, availableNodes) (cpp:140-177): survivors in `nodes` order."""
        avail_set = [v for v, a in enumerate(availableNodes) if a]
        m = self.gfp_batch(masks_from_sets([list(nodes)], self.n), masks_from_sets([avail_set], self.n))
        keep = set(sets_from_masks(m, self.n)[0])
        return [v for v in nodes if v in keep]

    # ---- device: solve / search -------------------------------------------------------
    def solve_stats(self, grow_budget: int = 0, run_budget: int = 0, max_blocks: int = 0, jit: int = 0,
                    batch: int = 0, engines: int = 0, device_mask: int = 0, tiebreak: int = 0,
                    tie_seed: int = 0) -> Dict:
        """jit: 0 auto (specialised kernel compiled in the background for long searches),
        1 table-interpreting kernel only, 2 specialised kernel from the first launch.
        engines / device_mask: sharded search over several engines (one host thread and
        HIP stream each) on the devices of device_mask (0 = this FBAS's device)."""
        # tiebreak: 0 lowest vertex index, 1 the reference's uniform draw (seeded with tie_seed)
        opts = _capi.SolveOpts(tiebreak, grow_budget, run_budget, max_blocks, jit, batch, engines, device_mask, tie_seed)
        res = _capi.SolveResult()
        q1 = np.zeros(max(self.n, 1), dtype=np.uint32)
        q2 = np.zeros(max(self.n, 1), dtype=np.uint32)
        check(lib().qi_solve(self._h, ctypes.byref(opts), ctypes.byref(res), _u32p(q1), _u32p(q2)))
        d = {k: getattr(res, k) for k, _ in _capi.SolveResult._fields_}
        d["verdict"] = bool(res.verdict)
        d["searched"] = bool(res.searched)
        d["q1"] = [int(x) for x in q1[: res.q1_len]]
        d["q2"] = [int(x) for x in q2[: res.q2_len]]
        return d

    def jit_precompile(self) -> float:
        """Compile/cache the specialised search kernel for sccs.front() (no GPU needed); ms."""
        ms = ctypes.c_double()
        check(lib().qi_fbas_jit_precompile(self._h, ctypes.byref(ms)))
        return ms.value

    def checkMinimalQuorums(self) -> Tuple[bool, List[int], List[int]]:
        """checkMinimalQuorums(sccs.front(), ...) (cpp:348-400): (intersecting, q1, q2)."""
        d = self.solve_stats()
        if not d["searched"]:
            raise QIError(_capi.QI_ERR_STATE, "search not defined: exactly one SCC must contain a quorum")
        return d["verdict"], d["q1"], d["q2"]

    def solve_text(self, verbose: bool = False, graphviz: bool = False) -> Tuple[str, bool]:
        p = ctypes.c_void_p()
        verdict = ctypes.c_int()
        check(lib().qi_solve_text(self._h, int(verbose), int(graphviz), ctypes.byref(p), ctypes.byref(verdict)))
        try:
            text = ctypes.cast(p, ctypes.c_char_p).value.decode(errors="surrogateescape")
        finally:
            lib().qi_free(p)
        return text, bool(verdict.value)

    def pagerank_text(self, dangling: float = 0.0001, convergence: float = 0.0001,
                      max_iterations: int = 100000) -> str:
        p = ctypes.c_void_p()
        check(lib().qi_pagerank_text(self._h, dangling, convergence, max_iterations, ctypes.byref(p)))
        try:
            return ctypes.cast(p, ctypes.c_char_p).value.decode(errors="surrogateescape")
        finally:
            lib().qi_free(p)


def solve(json_text, verbose: bool = False, graphviz: bool = False, device: int = 0) -> bool:
    """solve(istream&, ostream&, verbose, graphviz) (cpp:709-716): the verdict."""
    return FBAS(json_text, device).solve_text(verbose, graphviz)[1]


def solve_text(json_text, verbose: bool = False, graphviz: bool = False, device: int = 0) -> Tuple[str, bool]:
    return FBAS(json_text, device).solve_text(verbose, graphviz)


def pagerank_text(json_text, dangling: float = 0.0001, convergence: float = 0.0001,
                  max_iterations: int = 100000) -> str:
    return FBAS(json_text, -1).pagerank_text(dangling, convergence, max_iterations)
