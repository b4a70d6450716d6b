"""ctypes binding of the C-ABI in include/quorum_intersection.h.

The shared library is built in-tree (quorum_intersection_amd/_lib/libqi_amd.so) by
``__graft_entry__.build()``; importing this module without it raises immediately --
there is no CPU fallback for the hot path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_size_t, c_uint32, c_uint64, c_void_p

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libqi_amd.so")

QI_OK = 0
QI_ERR_PARSE = 1
QI_ERR_DEVICE = 2
QI_ERR_ARG = 3
QI_ERR_UNSUPPORTED = 4
QI_ERR_CAPACITY = 5
QI_ERR_STATE = 6


class QIError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[qi error {code}] {msg}")
        self.code = code


class SolveOpts(ctypes.Structure):
    _fields_ = [("tiebreak", c_uint32), ("grow_budget", c_uint32), ("run_budget", c_uint32), ("max_blocks", c_uint32),
                ("jit", c_uint32), ("batch", c_uint32), ("engines", c_uint32), ("device_mask", c_uint32),
                ("tie_seed", c_uint32)]


class SolveResult(ctypes.Structure):
    _fields_ = [
        ("verdict", c_int32),
        ("searched", c_int32),
        ("n_vertices", c_uint32),
        ("n_sccs", c_uint32),
        ("sccs_with_quorum", c_uint32),
        ("front_size", c_uint32),
        ("nodes", c_uint64),
        ("evals", c_uint64),
        ("scc_evals", c_uint64),
        ("minq", c_uint64),
        ("zero_fallback", c_uint64),
        ("rounds", c_uint64),
        ("launches", c_uint64),
        ("q1_len", c_uint32),
        ("q2_len", c_uint32),
        ("t_scc_ms", c_double),
        ("t_search_ms", c_double),
        ("t_kernel_ms", c_double),
        ("nonmonotone", c_uint32),
        ("jit_launches", c_uint32),
        ("engines", c_uint32),
        ("devices", c_uint32),
        ("units_moved", c_uint64),
        ("t_device_init_ms", c_double),
        ("nodes_processed", c_uint64),
    ]


class SearchOpts(ctypes.Structure):
    _fields_ = [("grow_budget", c_uint32), ("run_budget", c_uint32), ("max_blocks", c_uint32), ("jit", c_uint32),
                ("batch", c_uint32)]


class StepInfo(ctypes.Structure):
    _fields_ = [
        ("frontier_in", c_uint64),
        ("frontier_out", c_uint64),
        ("processed", c_uint64),
        ("budget", c_uint32),
        ("blocks", c_uint32),
        ("new_witnesses", c_uint64),
        ("kernel_ms", c_double),
        ("specialized", c_uint32),
        ("launches", c_uint32),
        ("dispatches", c_uint32),
        ("pad", c_uint32),
        ("dispatch_ms", c_double),
    ]


class Shape(ctypes.Structure):
    _fields_ = [("m", c_uint32), ("mask_words", c_uint32), ("tns", c_uint32), ("tn_words", c_uint32),
                ("tns_with_children", c_uint32), ("roots", c_uint32), ("groups", c_uint32),
                ("extra_terms", c_uint32), ("qmin_inside", c_uint32), ("qmin_outside", c_uint32)]


class Totals(ctypes.Structure):
    _fields_ = [("nodes", c_uint64), ("evals", c_uint64), ("minq", c_uint64), ("zero_fallback", c_uint64),
                ("rounds", c_uint64), ("units", c_uint64), ("wave_iters", c_uint64), ("coop_phases", c_uint64),
                ("stamps", c_uint64 * 8)]


# name -> (restype, argtypes); must match include/quorum_intersection.h exactly
SIGNATURES = {
    "qi_last_error": (c_char_p, []),
    "qi_abi_version": (c_int, []),
    "qi_device_count": (c_int, []),
    "qi_device_warmup": (c_int, [c_int, POINTER(c_double)]),
    "qi_timing_json": (c_char_p, []),
    "qi_fbas_from_json": (c_int, [c_char_p, c_size_t, c_int, POINTER(c_void_p)]),
    "qi_fbas_destroy": (None, [c_void_p]),
    "qi_fbas_num_vertices": (c_uint32, [c_void_p]),
    "qi_fbas_num_edges": (c_uint32, [c_void_p]),
    "qi_fbas_num_sccs": (c_uint32, [c_void_p]),
    "qi_fbas_scc_ids": (c_int, [c_void_p, POINTER(c_uint32)]),
    "qi_fbas_adjacency": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32)]),
    "qi_fbas_vertex": (c_int, [c_void_p, c_uint32, POINTER(c_char_p), POINTER(c_char_p)]),
    "qi_gfp_batch": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), c_uint32, POINTER(c_uint64)]),
    "qi_gfp_batch_static": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p]),
    "qi_solve": (c_int, [c_void_p, POINTER(SolveOpts), POINTER(SolveResult), POINTER(c_uint32), POINTER(c_uint32)]),
    "qi_solve_text": (c_int, [c_void_p, c_int, c_int, POINTER(c_void_p), POINTER(c_int)]),
    "qi_solve_text_ex": (c_int, [c_void_p, c_int, c_int, POINTER(SolveOpts), POINTER(c_void_p), POINTER(c_int)]),
    "qi_pagerank_text": (c_int, [c_void_p, c_float, c_float, c_uint64, POINTER(c_void_p)]),
    "qi_free": (None, [c_void_p]),
    "qi_search_create": (c_int, [c_void_p, POINTER(SearchOpts), POINTER(c_void_p)]),
    "qi_search_destroy": (None, [c_void_p]),
    "qi_search_unit_bytes": (c_uint32, [c_void_p]),
    "qi_search_key_words": (c_uint32, [c_void_p]),
    "qi_search_reset": (c_int, [c_void_p]),
    "qi_search_clear": (c_int, [c_void_p]),
    "qi_search_step": (c_int, [c_void_p, POINTER(StepInfo)]),
    "qi_search_frontier": (c_uint64, [c_void_p]),
    "qi_search_keep_slice": (c_int, [c_void_p, c_uint64, c_uint64]),
    "qi_search_grow": (c_int, [c_void_p, c_uint64, POINTER(StepInfo)]),
    "qi_search_keep_strided": (c_int, [c_void_p, c_uint64, c_uint64]),
    "qi_search_export": (c_int, [c_void_p, c_uint64, c_void_p]),
    "qi_search_import": (c_int, [c_void_p, c_uint64, c_void_p]),
    "qi_search_local_best": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32)]),
    "qi_search_set_best": (c_int, [c_void_p, POINTER(c_uint32), c_uint32]),
    "qi_search_share_best": (c_int, [c_void_p, c_void_p]),
    "qi_search_reduce": (c_int, [c_void_p, POINTER(c_uint32), c_uint32, POINTER(Totals)]),
    "qi_search_witness": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32),
                                  POINTER(c_uint32)]),
    "qi_search_restart": (c_int, [c_void_p]),
    "qi_search_kernel_ms": (c_double, [c_void_p]),
    "qi_search_shape": (c_int, [c_void_p, POINTER(Shape)]),
    "qi_fbas_jit_precompile": (c_int, [c_void_p, POINTER(c_double)]),
    "qi_search_wait_jit": (c_int, [c_void_p]),
    "qi_hash_iteration_order": (c_int, [POINTER(c_uint32), c_uint32, POINTER(c_uint32), c_uint32, POINTER(c_uint32),
                                        POINTER(c_uint32)]),
}

_lib = None
torch_first = True  # False once the library was loaded in a process that had not imported torch


def lib() -> ctypes.CDLL:
    """Load the in-tree HIP library; raise if it is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950) first")
        # PyTorch-ROCm ships its own libamdhip64.so.7 (ROCm 7.0) with the same soname as
        # /opt/rocm's (7.2): whichever loads first serves the whole process, and torch
        # then refuses a runtime that is not its own ("No HIP GPUs are available").  A
        # process that uses torch beside this library (the multi-rank driver, tests moving
        # units through tensors) must therefore load torch FIRST: import torch before the
        # first call into this package, or set QI_TORCH_RUNTIME=1 and it is imported here.
        # Otherwise torch is not touched (no seconds of import, and the system runtime the
        # library was built against is used).
        import sys
        if os.environ.get("QI_TORCH_RUNTIME") == "1" and "torch" not in sys.modules:
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        global torch_first
        torch_first = "torch" in sys.modules
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.qi_abi_version() != 4:
            raise ImportError("libqi_amd.so ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != QI_OK:
        raise QIError(rc, lib().qi_last_error().decode(errors="replace"))
