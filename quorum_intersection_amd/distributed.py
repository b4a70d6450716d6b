"""Multi-GPU branch-and-bound search: one process per GPU, torch.distributed over RCCL.

The search tree of iterateMinimalQuorums (quorum_intersection.cpp:252-346) is sharded
by branch prefix:

  1. rank 0 grows the frontier from the root (cpp:393) with a short chain of device
     launches until it holds ``seed_units`` subtree units (branch prefixes);
  2. it broadcasts those units (one RCCL broadcast of packed unit bytes), and every rank
     keeps its dealt share (rounds of ``world`` units, offset rotating by one per round) --
     neighbouring prefixes have correlated subtree sizes, so a deal balances better than
     contiguous slices, and the rotation breaks periodic patterns in the frontier order;
  3. every rank runs chains of device launches on its own units; between chains the
     ranks exchange only frontier sizes + best-witness keys (one all_gather of a few
     int64s) and, when some rank would idle part of its GPU while another holds surplus,
     move units with send/recv (host-planned, deterministic on every rank).

The data path has no collective.  Counts stay preorder-exact because every processed
segment is logged with its root path key on the rank that processed it; at the end each
rank reduces its log against the globally preorder-first witness and the totals are
summed with one all_reduce.

The coordination logic is backend-agnostic (``SearchBackend``): ``DeviceSearch`` wraps
the C-ABI step-wise search on a HIP device; tests drive a synthetic CPU backend over the
gloo process group.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _capi

if not _capi.torch_first:
    raise ImportError("quorum_intersection_amd.distributed: the HIP library was loaded before torch, so the process "
                      "runs on another HIP runtime than torch's; import torch (or this module) before the first "
                      "call into the package, or set QI_TORCH_RUNTIME=1")

Key = Tuple[Tuple[int, ...], int]  # (path key words, depth); preorder = lexicographic


class SearchBackend:
    """What the multi-rank driver needs from one rank's search engine."""

    key_words: int
    unit_bytes: int

    def reset(self) -> None: ...
    def clear(self) -> None: ...
    def restart(self) -> None: ...
    def drop_log(self) -> None: ...
    def step(self) -> None: ...
    def grow(self, target: int) -> None: ...
    def frontier(self) -> int: ...
    def keep_slice(self, begin: int, end: int) -> None: ...
    def keep_strided(self, offset: int, stride: int) -> None: ...
    def export(self, count: int, dst: torch.Tensor) -> None: ...
    def import_(self, count: int, src: torch.Tensor) -> None: ...
    def local_best(self) -> Optional[Key]: ...
    def set_best(self, key: Key) -> None: ...
    def reduce(self, key: Optional[Key]) -> Dict[str, int]: ...
    def witness(self) -> Tuple[List[int], List[int]]: ...


class DeviceSearch(SearchBackend):
    """C-ABI step-wise search (include/quorum_intersection.h) on one HIP device."""

    def __init__(self, fbas, grow_budget: int = 0, run_budget: int = 0, max_blocks: int = 0, jit: int = 0,
                 batch: int = 0):
        from . import _capi
        self._c = _capi
        self.L = _capi.lib()
        self.fbas = fbas
        h = ctypes.c_void_p()
        opts = _capi.SearchOpts(grow_budget, run_budget, max_blocks, jit, batch)
        _capi.check(self.L.qi_search_create(fbas.handle, ctypes.byref(opts), ctypes.byref(h)))
        self.h = h
        self.key_words = int(self.L.qi_search_key_words(h))
        self.unit_bytes = int(self.L.qi_search_unit_bytes(h))
        self.kernel_ms = 0.0
        self.launches = 0
        self.dispatches = 0
        self.dispatch_ms = 0.0
        self.data_device = torch.device("cuda", fbas.device)  # where exported units live

    def close(self):
        if self.h:
            self.L.qi_search_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        self._c.check(self.L.qi_search_reset(self.h))

    def clear(self):
        self._c.check(self.L.qi_search_clear(self.h))

    def restart(self):
        self._c.check(self.L.qi_search_restart(self.h))
        self.kernel_ms = 0.0
        self.launches = 0
        self.dispatches = 0
        self.dispatch_ms = 0.0

    def drop_log(self):
        # forget processed segments and bests but keep the current frontier
        n = self.frontier()
        keep = None
        if n:
            keep = torch.empty(n * self.unit_bytes, dtype=torch.uint8, device=self.data_device)
            _settle(keep)
            self.export(n, keep)
        self._c.check(self.L.qi_search_restart(self.h))
        self.clear()
        if n:
            self.import_(n, keep)

    def step(self):
        info = self._c.StepInfo()
        self._c.check(self.L.qi_search_step(self.h, ctypes.byref(info)))
        self.kernel_ms += info.kernel_ms
        self.launches += int(info.launches)
        self.dispatches += int(info.dispatches)
        self.dispatch_ms += info.dispatch_ms
        self.spec_launches = getattr(self, "spec_launches", 0) + int(info.specialized)
        self.blocks = int(info.blocks)

    def grow(self, target):
        info = self._c.StepInfo()
        self._c.check(self.L.qi_search_grow(self.h, target, ctypes.byref(info)))
        self.kernel_ms += info.kernel_ms
        self.launches += int(info.launches)
        self.dispatches += int(info.dispatches)
        self.dispatch_ms += info.dispatch_ms

    def frontier(self) -> int:
        return int(self.L.qi_search_frontier(self.h))

    def keep_slice(self, begin, end):
        self._c.check(self.L.qi_search_keep_slice(self.h, begin, end))

    def keep_strided(self, offset, stride):
        self._c.check(self.L.qi_search_keep_strided(self.h, offset, stride))

    def export(self, count, dst):
        self._c.check(self.L.qi_search_export(self.h, count, ctypes.c_void_p(dst.data_ptr())))

    def import_(self, count, src):
        self._c.check(self.L.qi_search_import(self.h, count, ctypes.c_void_p(src.data_ptr())))

    def local_best(self):
        k = (ctypes.c_uint32 * self.key_words)()
        d = ctypes.c_uint32()
        if self.L.qi_search_local_best(self.h, k, ctypes.byref(d)) == 1:
            return tuple(int(x) for x in k), int(d.value)
        return None

    def set_best(self, key):
        k = (ctypes.c_uint32 * self.key_words)(*key[0])
        self._c.check(self.L.qi_search_set_best(self.h, k, key[1]))

    def share_best(self, shared: Optional["SharedBest"]):
        """Fold this engine's best key into `shared` after every launch and let its kernels
        poll it (qi_search_share_best); None ends the sharing."""
        self._c.check(self.L.qi_search_share_best(self.h, ctypes.c_void_p(shared.address if shared else None)))
        self._shared = shared  # keeps the mapping alive while the engine uses it

    def reduce(self, key):
        t = self._c.Totals()
        if key is None:
            self._c.check(self.L.qi_search_reduce(self.h, None, 0, ctypes.byref(t)))
        else:
            k = (ctypes.c_uint32 * self.key_words)(*key[0])
            self._c.check(self.L.qi_search_reduce(self.h, k, key[1], ctypes.byref(t)))
        return {"nodes": t.nodes, "evals": t.evals, "minq": t.minq, "zero_fallback": t.zero_fallback,
                "rounds": t.rounds, "units": t.units, "wave_iters": t.wave_iters, "coop_phases": t.coop_phases,
                "stamps": [int(x) for x in t.stamps]}

    def wait_jit(self) -> bool:
        return self.L.qi_search_wait_jit(self.h) == 1

    def shape(self) -> Dict[str, int]:
        sh = self._c.Shape()
        self._c.check(self.L.qi_search_shape(self.h, ctypes.byref(sh)))
        return {k: int(getattr(sh, k)) for k, _ in self._c.Shape._fields_}

    def witness(self):
        n = self.fbas.n
        q1 = (ctypes.c_uint32 * max(n, 1))()
        q2 = (ctypes.c_uint32 * max(n, 1))()
        l1, l2 = ctypes.c_uint32(), ctypes.c_uint32()
        self._c.check(self.L.qi_search_witness(self.h, q1, ctypes.byref(l1), q2, ctypes.byref(l2)))
        return list(q1)[: l1.value], list(q2)[: l2.value]


class SharedBest:
    """The ranks' shared best-witness key: one 64-bit word in a POSIX shared-memory page that
    every rank of the node maps (the search runs on the GPUs of ONE node).  Each rank's
    engine folds its launches' best keys into it and its kernels poll it, so a witness found
    on one GPU prunes the others inside their chains of launches; the exact result still
    comes from the all_gather of keys and the preorder-filtered reduction."""

    def __init__(self, name: str, create: bool):
        self.path = os.path.join("/dev/shm", name)
        flags = os.O_RDWR | (os.O_CREAT if create else 0)
        fd = os.open(self.path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, mmap.PAGESIZE)
            self.mm = mmap.mmap(fd, mmap.PAGESIZE)
        finally:
            os.close(fd)
        self.created = create
        self._word = ctypes.c_uint64.from_buffer(self.mm)
        self.address = ctypes.addressof(self._word)
        if create:
            self.reset()

    def reset(self) -> None:
        self._word.value = 0xFFFFFFFFFFFFFFFF

    @property
    def value(self) -> int:
        return int(self._word.value)

    def close(self) -> None:
        if getattr(self, "mm", None) is not None:
            del self._word
            try:
                self.mm.close()
            except BufferError:
                pass
            self.mm = None
            if self.created:
                try:
                    os.unlink(self.path)
                except OSError:
                    pass

    @staticmethod
    def for_group(group=None, tag: str = "") -> "SharedBest":
        """Collective: group rank 0 creates the page, the others map it."""
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        name = [f"qi_best_{os.getpid()}_{tag}_{time.time_ns()}" if rank == 0 else None]
        sb = SharedBest(name[0], True) if rank == 0 else None
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(name, src=src, group=group)
        if sb is None:
            sb = SharedBest(name[0], False)
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.barrier(group=group)  # every rank has mapped it before rank 0 may unlink
        return sb


# ------------------------------------------------------------------------------------
# Host-side planning (pure functions, unit-tested)
# ------------------------------------------------------------------------------------
def slice_bounds(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous preorder-respecting slice of the initial frontier for `rank`."""
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def plan_rebalance(sizes: Sequence[int], min_move: int = 1) -> List[Tuple[int, int, int]]:
    """Moves (src, dst, count) that bring every rank to within one unit of the mean.
    Deterministic: every rank computes the same plan from the same gathered sizes."""
    world = len(sizes)
    total = sum(sizes)
    target = [total // world + (1 if r < total % world else 0) for r in range(world)]
    excess = [(s - t, r) for r, (s, t) in enumerate(zip(sizes, target))]
    donors = sorted([(e, r) for e, r in excess if e > 0], reverse=True)
    takers = sorted([(-e, r) for e, r in excess if e < 0], reverse=True)
    moves = []
    i = j = 0
    donors = [list(x) for x in donors]
    takers = [list(x) for x in takers]
    while i < len(donors) and j < len(takers):
        c = min(donors[i][0], takers[j][0])
        if c >= min_move:
            moves.append((donors[i][1], takers[j][1], c))
        donors[i][0] -= c
        takers[j][0] -= c
        if donors[i][0] == 0:
            i += 1
        if takers[j][0] == 0:
            j += 1
    return moves


def best_of(keys: Sequence[Optional[Key]]) -> Optional[Key]:
    ks = [k for k in keys if k is not None]
    return min(ks) if ks else None


def needs_rebalance(sizes: Sequence[int], lanes: int) -> bool:
    """Rebalance when some rank would idle part of its GPU while another holds surplus."""
    if max(sizes) == 0:
        return False
    lo, hi = min(sizes), max(sizes)
    return lo < lanes and hi > 2 * max(lo, 1)


# ------------------------------------------------------------------------------------
# The multi-rank driver
# ------------------------------------------------------------------------------------
@dataclass
class DistResult:
    verdict: bool
    nodes: int
    evals: int
    minq: int
    zero_fallback: int
    rounds: int
    q1: List[int] = field(default_factory=list)
    q2: List[int] = field(default_factory=list)
    launches: int = 0
    moved_units: int = 0
    wall_s: float = 0.0
    units: int = 0
    wave_iters: int = 0
    coop_phases: int = 0


def _gather_state(be: SearchBackend, device, group) -> Tuple[List[int], List[Optional[Key]]]:
    kw = be.key_words
    best = be.local_best()
    row = [be.frontier(), 1 if best else 0, best[1] if best else 0] + (list(best[0]) if best else [0] * kw)
    t = torch.tensor(row, dtype=torch.int64, device=device)
    world = dist.get_world_size(group)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    sizes, keys = [], []
    for v in torch.stack(out).tolist():  # one device-to-host copy for all ranks' rows
        v = [int(x) for x in v]
        sizes.append(v[0])
        keys.append((tuple(v[3:3 + kw]), v[2]) if v[1] else None)
    return sizes, keys


def _unit_buf(be: SearchBackend, count: int, device) -> torch.Tensor:
    return torch.empty(count * be.unit_bytes, dtype=torch.uint8, device=getattr(be, "data_device", device))


def _to_comm(t: torch.Tensor, device) -> torch.Tensor:
    """Unit bytes live on the backend's device; a CPU (gloo) group stages them on the host."""
    return t if t.device == torch.device(device) else t.to(device)


def _settle(t: torch.Tensor) -> None:
    """The engine copies units on its own non-blocking HIP stream, which is not ordered
    after torch's current stream: a blocking RCCL collective only makes the *current
    stream* wait for its result, and a fresh caching-allocator block may still be in use
    by work queued there.  Drain the current stream before the engine touches `t`."""
    if t.is_cuda:
        torch.cuda.current_stream(t.device).synchronize()


def distributed_search(be: SearchBackend, group=None, device="cpu", lanes: int = 1 << 17,
                       rebalance: bool = True, min_move: int = 64, seed_units: int = 0,
                       shared: Optional[SharedBest] = None) -> DistResult:
    """Run one full search across the ranks of `group`; every rank returns the result.
    shared: the ranks' SharedBest page (already given to every rank's engine with
    share_best): rank 0 resets it here, before the frontier broadcast that starts the
    other ranks."""
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(group), dist.get_world_size(group)
    else:
        rank, world = 0, 1
    t0 = time.perf_counter()
    if shared is not None and rank == 0:
        shared.reset()
    be.restart()
    launches = 0
    moved = 0
    if world > 1:
        # (1) rank 0 grows the frontier from the root (cpp:393) ...
        target = seed_units or 2048 * world
        if rank == 0:
            be.grow(target)
        n = torch.tensor([be.frontier() if rank == 0 else 0], dtype=torch.int64, device=device)
        # group rank 0 as a global rank (broadcast takes global ranks, also with a sub-group)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(n, src, group=group)
        n = int(n.item())
        # (2) ... hands it to every rank; each keeps its dealt share (rotating offset)
        if rank != 0:
            be.clear()
        if n:
            buf = _unit_buf(be, n, device)
            _settle(buf)
            if rank == 0:
                be.export(n, buf)
            cbuf = _to_comm(buf, device)
            dist.broadcast(cbuf, src, group=group)
            if cbuf is not buf:
                buf.copy_(cbuf)
            _settle(buf)
            be.import_(n, buf)
            be.keep_strided(rank, world)
    # (3) independent chains of launches; exchange sizes/best keys; rebalance surplus
    while True:
        if be.frontier():
            be.step()
            launches += 1
        sizes, keys = _gather_state(be, device, group) if world > 1 else ([be.frontier()], [be.local_best()])
        best = best_of(keys)
        if best is not None:
            be.set_best(best)
        if sum(sizes) == 0:
            break
        if world > 1 and rebalance and needs_rebalance(sizes, lanes):
            for src, dst, cnt in plan_rebalance(sizes, min_move=min_move):
                gsrc = dist.get_global_rank(group, src) if group is not None else src
                gdst = dist.get_global_rank(group, dst) if group is not None else dst
                if rank == src:
                    buf = _unit_buf(be, cnt, device)
                    _settle(buf)
                    be.export(cnt, buf)
                    dist.send(_to_comm(buf, device), gdst, group=group)
                elif rank == dst:
                    buf = _unit_buf(be, cnt, device)
                    cbuf = _to_comm(buf, device)
                    dist.recv(cbuf, gsrc, group=group)
                    if cbuf is not buf:
                        buf.copy_(cbuf)
                    _settle(buf)
                    be.import_(cnt, buf)
                moved += cnt
    # (4) preorder-exact totals against the global best witness: the loop's last exchange
    # (every frontier empty, no launch since) already holds every rank's final best key
    loc = be.reduce(best)
    tot = [int(loc["nodes"]), int(loc["evals"]), int(loc["minq"]), int(loc["zero_fallback"]), int(loc["rounds"]),
           launches, int(loc.get("units", 0)), int(loc.get("wave_iters", 0)), int(loc.get("coop_phases", 0))]
    if world > 1:  # one process: no device round trip for the totals
        vec = torch.tensor(tot, dtype=torch.int64, device=device)
        dist.all_reduce(vec, group=group)
        tot = [int(x) for x in vec.tolist()]
    q1: List[int] = []
    q2: List[int] = []
    if best is not None:
        owner = keys.index(best)
        if world > 1:
            n = be.fbas.n if hasattr(be, "fbas") else 0
            w = torch.full((2, max(n, 1) + 1), -1, dtype=torch.int64, device=device)
            if rank == owner:
                a, b = be.witness()
                w[0, 0], w[1, 0] = len(a), len(b)
                if a:
                    w[0, 1:1 + len(a)] = torch.tensor(a, dtype=torch.int64, device=device)
                if b:
                    w[1, 1:1 + len(b)] = torch.tensor(b, dtype=torch.int64, device=device)
            # `owner` indexes the group's ranks; broadcast takes a global rank
            src = dist.get_global_rank(group, owner) if group is not None else owner
            dist.broadcast(w, src, group=group)
            wl = w.tolist()
            q1 = [int(x) for x in wl[0][1:1 + int(wl[0][0])]]
            q2 = [int(x) for x in wl[1][1:1 + int(wl[1][0])]]
        else:
            q1, q2 = be.witness()
    return DistResult(verdict=best is None, nodes=tot[0], evals=tot[1], minq=tot[2], zero_fallback=tot[3],
                      rounds=tot[4], q1=q1, q2=q2, launches=tot[5], moved_units=moved,
                      wall_s=time.perf_counter() - t0, units=tot[6], wave_iters=tot[7], coop_phases=tot[8])
