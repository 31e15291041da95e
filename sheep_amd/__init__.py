"""sheep_amd — MI355X implementation of Sheep's map/reduce partitioning path.

Python mirror of the reference's lib/ interfaces (chan150/sheep) over the C ABI of
``sheep_amd/lib/libsheep_hip.so`` (declared in ``include/sheep_hip.h``):

=========================  ======================================================
reference (file:line)      here
=========================  ======================================================
mpiSequence / degreeSeq.   :func:`degree_sequence`  (sequence.h:52-93)
fileSequence               :func:`degree_sequence` ``mode='dat'|'net'``  (:95-128)
JTree(graph, seq)          :func:`build_tree`  (jtree.h:111-122, jtree.cpp:66-145)
JNodeTable::merge          :func:`merge_trees`  (jnode.cpp:174-201)
JNodeTable::makeKids       :class:`KidTable`  (jnode.h:190-204)
Partition(seq,jnodes,k..)  :func:`partition`  (partition.cpp:50-157)
Partition::print           :meth:`PartitionResult.print_text`  (partition.h:135-143)
Partition::evaluate        :func:`evaluate`  (partition.cpp:428-521)
JNodeTable::Facts          :func:`facts`  (jnode.cpp:256-290)
=========================  ======================================================

Device memory is torch-allocated (``torch.cuda``), streams are torch's current
stream; every computation runs in the HIP kernels of libsheep_hip.so.  There is NO
CPU fallback: importing this package without the built library, or calling it without
a GPU, raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SHEEP_HIP_LIB: another build of the same library (A/B measurements of kernel variants,
# e.g. sheep_amd/lib/variants/*.so); the default is the in-tree build
LIB_PATH = os.environ.get("SHEEP_HIP_LIB") or os.path.join(_HERE, "lib", "libsheep_hip.so")

INVALID_ID = 0xFFFFFFFF
INVALID_PART = -1
DEGREE_MODES = {"llama": 0, "dat": 1, "net": 2}
EVAL_GRAPH, EVAL_DOWN, EVAL_UP = 1, 2, 4

ABI_VERSION = 6   # include/sheep_hip.h SHEEP_ABI_VERSION
_ERRORS = {-1: ValueError, -2: RuntimeError, -3: IndexError, -4: RuntimeError, -5: MemoryError}


class SheepError(RuntimeError):
    pass


class _PartInfo(ctypes.Structure):
    _fields_ = [("created", ctypes.c_int32), ("first_size", ctypes.c_uint64), ("second_size", ctypes.c_uint64),
                ("max_component", ctypes.c_uint64), ("total_weight", ctypes.c_uint64),
                ("packing_nodes", ctypes.c_uint64), ("heavy_nodes", ctypes.c_uint64),
                ("event_launches", ctypes.c_uint64)]


class _Eval(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in (
        "edges_cut", "vcom_vol", "max_vertex_bal", "ecv_hash", "max_hash_bal", "ecv_down", "max_down_bal",
        "ecv_up", "max_up_bal", "edges", "nodes")]


class _Facts(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in (
        "width", "root_cnt", "vert_height", "edge_height", "vert_cnt", "edge_cnt", "halo_id", "core_id", "fill")]


class Tuning(ctypes.Structure):
    """sheep_tuning (include/sheep_hip.h): the algorithm variants of one context; -1 keeps
    a field's default.  Every variant gives the same bit-exact result."""
    _fields_ = [("fin_map_bits", ctypes.c_int32), ("fin_merge_bits", ctypes.c_int32), ("fin_dc", ctypes.c_int32),
                ("top_bits", ctypes.c_int32), ("top_blocks", ctypes.c_int32), ("big_bits", ctypes.c_int32),
                ("big_dense", ctypes.c_int64), ("big_hot_bits", ctypes.c_int32), ("big_hot16", ctypes.c_int32),
                ("relabel_planes", ctypes.c_int32), ("relabel_per", ctypes.c_int32),
                ("cross_win_levels", ctypes.c_int32), ("hook_batch", ctypes.c_int32),
                ("merge_cut_bits", ctypes.c_int32), ("event_loop", ctypes.c_int32),
                ("hook_up", ctypes.c_int32)]

    @classmethod
    def of(cls, **kw):
        """The defaults (-1 everywhere) with the named fields set; unknown names raise."""
        t = cls(*([-1] * len(cls._fields_)))
        names = {f for f, _ in cls._fields_}
        for k, v in kw.items():
            if k not in names:
                raise KeyError(f"no tuning field {k!r} (fields: {sorted(names)})")
            setattr(t, k, int(v))
        return t

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def lib() -> ctypes.CDLL:
    """Load libsheep_hip.so (fails loudly: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run `make hip` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, U64, I32, I16, D = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int16, ctypes.c_double
    sig = {
        "sheep_last_error": ([], ctypes.c_char_p),
        "sheep_abi_version": ([], I32),
        "sheep_ctx_create": ([I32, P, ctypes.POINTER(P)], I32),
        "sheep_ctx_destroy": ([P], I32),
        "sheep_ctx_trim": ([P], I32),
        "sheep_ctx_workspace": ([P, ctypes.c_char_p, ctypes.c_size_t], I32),
        "sheep_ctx_sync": ([P], I32),
        "sheep_ctx_stream": ([P], P),
        "sheep_malloc": ([P, ctypes.c_size_t, ctypes.POINTER(P)], I32),
        "sheep_free": ([P, P], I32),
        "sheep_memcpy_h2d": ([P, P, P, ctypes.c_size_t], I32),
        "sheep_memcpy_d2h": ([P, P, P, ctypes.c_size_t], I32),
        "sheep_timer_enable": ([P, I32], I32),
        "sheep_timer_get": ([P, ctypes.c_char_p, ctypes.POINTER(D), ctypes.POINTER(U64), ctypes.POINTER(U64)], I32),
        "sheep_timer_reset": ([P], I32),
        "sheep_timer_names": ([P, ctypes.c_char_p, ctypes.c_size_t], I32),
        "sheep_tuning_default": ([ctypes.POINTER(Tuning)], I32),
        "sheep_ctx_set_tuning": ([P, ctypes.POINTER(Tuning)], I32),
        "sheep_ctx_get_tuning": ([P, ctypes.POINTER(Tuning)], I32),
        "sheep_group_set_tuning": ([P, ctypes.POINTER(Tuning)], I32),
        "sheep_degree_count": ([P, P, U64, I32, P, U64, ctypes.POINTER(U64)], I32),
        "sheep_sequence_from_degrees": ([P, P, U64, P, P, ctypes.POINTER(U64)], I32),
        "sheep_positions": ([P, P, U64, P, U64], I32),
        "sheep_build_tree": ([P, P, U64, P, U64, U64, P], I32),
        "sheep_merge_trees": ([P, P, P, U64, P], I32),
        "sheep_merge_trees_many": ([P, P, ctypes.c_uint32, U64, P], I32),
        "sheep_merge_trees_part": ([P, P, ctypes.c_uint32, U64, ctypes.c_uint32, ctypes.c_uint32, P,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], I32),
        "sheep_kids_create": ([P, P, U64, ctypes.POINTER(P)], I32),
        "sheep_kids_destroy": ([P], I32),
        "sheep_partition": ([P, P, U64, P, U64, U64, P, I16, D, I32, I32, P, ctypes.POINTER(_PartInfo)], I32),
        "sheep_partition_pos": ([P, P, U64, P, U64, P, U64, P, I16, D, I32, I32, P, ctypes.POINTER(_PartInfo)], I32),
        "sheep_evaluate": ([P, P, U64, P, U64, P, I32, ctypes.POINTER(_Eval)], I32),
        "sheep_evaluate_step": ([P, P, U64, P, U64, P, U64, P, I32, ctypes.POINTER(_Eval)], I32),
        "sheep_facts": ([P, P, U64, ctypes.POINTER(_Facts)], I32),
        "sheep_eval_sizes": ([I32, I32, U64, ctypes.POINTER(U64), ctypes.POINTER(U64)], I32),
        "sheep_eval_num_parts": ([P, P, U64, ctypes.POINTER(ctypes.c_int32)], I32),
        "sheep_eval_shard": ([P, P, U64, P, U64, P, I32, I32, P, P], I32),
        "sheep_eval_combine": ([P, P, P, U64, P, P, U64], I32),
        "sheep_eval_finish": ([P, P, P, U64, P, I32, I32, ctypes.POINTER(_Eval)], I32),
        "sheep_edge_parts": ([P, P, U64, P, U64, P, P], I32),
        "sheep_group_create": ([P, I32, ctypes.POINTER(P)], I32),
        "sheep_group_join": ([I32, I32, I32, ctypes.c_char_p, I32, I32, ctypes.POINTER(P)], I32),
        "sheep_group_destroy": ([P], I32),
        "sheep_group_size": ([P], I32),
        "sheep_group_local_count": ([P], I32),
        "sheep_group_rank": ([P, I32], I32),
        "sheep_group_ctx": ([P, I32], P),
        "sheep_group_uses_rccl": ([P], I32),
        "sheep_group_abort": ([P, ctypes.c_char_p], I32),
        "sheep_group_failed": ([P], I32),
        "sheep_group_barrier": ([P], I32),
        "sheep_group_allreduce_max_u64": ([P, ctypes.POINTER(U64)], I32),
        "sheep_group_reduce_trees": ([P, P, U64, I32], I32),
        "sheep_group_sequence": ([P, P, P, P, U64, P, P, ctypes.POINTER(U64), ctypes.POINTER(U64)], I32),
        "sheep_group_build_tree": ([P, P, P, P, U64, U64, P, I32], I32),
        "sheep_group_broadcast_parts": ([P, P, U64], I32),
        "sheep_group_transfer": ([P, I32, I32, P, P, U64], I32),
        "sheep_group_evaluate": ([P, P, P, P, U64, P, I32, ctypes.POINTER(_Eval)], I32),
        "sheep_parse_net": ([P, P, U64, I32, P, U64, ctypes.POINTER(U64)], I32),
        "sheep_powerlaw_generate": ([P, U64, U64, D, U64, P, U64, ctypes.POINTER(U64)], I32),
        "sheep_rmat_generate": ([P, I32, I32, U64, P, U64, ctypes.POINTER(U64)], I32),
        "sheep_rmat_generate_host": ([I32, I32, U64, P, U64, ctypes.POINTER(U64)], I32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.sheep_abi_version() != ABI_VERSION:   # (struct layouts below are this header's)
        raise ImportError(f"{LIB_PATH}: ABI version {L.sheep_abi_version()}, this binding expects {ABI_VERSION}")
    _lib = L
    return L


def _check(rc: int) -> None:
    if rc != 0:
        msg = lib().sheep_last_error().decode(errors="replace")
        raise _ERRORS.get(rc, SheepError)(f"sheep_hip error {rc}: {msg}")


def _ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


class Context:
    """One device + the torch current stream (so torch and sheep kernels stay ordered)."""

    def __init__(self, device: int = 0, stream=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("sheep_amd needs a HIP device (torch.cuda.is_available() is False)")
        self.device = device
        torch.cuda.set_device(device)
        s = stream if stream is not None else torch.cuda.current_stream(device)
        self._stream = s
        h = ctypes.c_void_p()
        _check(lib().sheep_ctx_create(device, ctypes.c_void_p(s.cuda_stream), ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            lib().sheep_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        _check(lib().sheep_ctx_sync(self.handle))

    def trim(self):
        """Free the context's device workspace (sheep_ctx_trim)."""
        _check(lib().sheep_ctx_trim(self.handle))

    def workspace(self) -> dict:
        """The device workspaces the context holds, name -> bytes (largest first)."""
        buf = ctypes.create_string_buffer(1 << 16)
        _check(lib().sheep_ctx_workspace(self.handle, buf, 1 << 16))
        return {k: int(v) for k, v in (x.split("=") for x in buf.value.decode().split(",") if x)}

    # device-side kernel timers (HIP events on the context stream)
    def timing(self, on: bool = True):
        _check(lib().sheep_timer_enable(self.handle, int(on)))

    def timer(self, name: str):
        """(ms, launches, algorithmic bytes) accumulated for one instrumented region."""
        ms, n, b = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().sheep_timer_get(self.handle, name.encode(), ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b)))
        return ms.value, n.value, b.value

    def timer_names(self) -> list:
        buf = ctypes.create_string_buffer(4096)
        _check(lib().sheep_timer_names(self.handle, buf, 4096))
        return [x for x in buf.value.decode().split(",") if x]

    def timer_reset(self):
        _check(lib().sheep_timer_reset(self.handle))

    def set_tuning(self, **kw):
        """sheep_ctx_set_tuning: the named fields of Tuning set, the rest at their defaults
        (no arguments: every default)."""
        _check(lib().sheep_ctx_set_tuning(self.handle, ctypes.byref(Tuning.of(**kw))))

    def tuning(self) -> dict:
        t = Tuning()
        _check(lib().sheep_ctx_get_tuning(self.handle, ctypes.byref(t)))
        return t.as_dict()


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def _torch():
    import torch
    return torch


def _dev(ctx: "Context") -> str:
    return f"cuda:{ctx.device}"


def _dev_u32(n: int, ctx: "Context"):
    t = _torch()
    return t.empty(max(int(n), 1), dtype=t.int32, device=_dev(ctx))


def records_to_device(tail: np.ndarray, head: np.ndarray, weight: np.ndarray | None = None):
    """XS1 records (12 bytes: u32 tail, u32 head, f32 weight) as a [R,3] int32 device tensor."""
    t = _torch()
    R = len(tail)
    host = np.empty((R, 3), dtype=np.uint32)
    host[:, 0] = tail
    host[:, 1] = head
    host[:, 2] = (np.ones(R, np.float32) if weight is None else np.asarray(weight, np.float32)).view(np.uint32)
    return t.from_numpy(host.view(np.int32)).to("cuda")


def to_numpy_u32(x) -> np.ndarray:
    return x.detach().cpu().numpy().view(np.uint32)


# ---------------------------------------------------------------------------------
# sequence.h
# ---------------------------------------------------------------------------------
@dataclass
class Sequence:
    seq: object          # device int32 tensor [n] (u32 vids)
    pos: object          # device int32 tensor [pos_size] (u32 jnids, INVALID elsewhere)
    n: int
    pos_size: int        # max(seq) + 1 (jtree.h:113) for readSequence; max_nodes for degree seqs

    def numpy(self) -> np.ndarray:
        return to_numpy_u32(self.seq[: self.n])


def degree_count(records, nrec: int | None = None, mode: str = "llama", deg=None, vs_cap: int | None = None,
                 ctx: Context | None = None):
    """Accumulate one shard's degrees into `deg` (device u32); returns (deg, max_slot)."""
    ctx = ctx or default_context()
    t = _torch()
    nrec = records.shape[0] if nrec is None else nrec
    if deg is None:
        raise ValueError("pass a zeroed degree tensor `deg` of the vertex-slot capacity")
    ms = ctypes.c_uint64()
    _check(lib().sheep_degree_count(ctx.handle, _ptr(records), nrec, DEGREE_MODES[mode], _ptr(deg), deg.numel(),
                                    ctypes.byref(ms)))
    return deg, ms.value


def sequence_from_degrees(deg, vs: int, ctx: Context | None = None) -> Sequence:
    ctx = ctx or default_context()
    seq, pos = _dev_u32(vs, ctx), _dev_u32(vs, ctx)
    n = ctypes.c_uint64()
    _check(lib().sheep_sequence_from_degrees(ctx.handle, _ptr(deg), vs, _ptr(seq), _ptr(pos), ctypes.byref(n)))
    return Sequence(seq, pos, n.value, vs)


def degree_sequence(records, mode: str = "llama", vs_cap: int | None = None, ctx: Context | None = None) -> Sequence:
    """degreeSequence / mpiSequence (mode 'llama') or fileSequence ('dat' / 'net')."""
    ctx = ctx or default_context()
    t = _torch()
    nrec = records.shape[0]
    if vs_cap is None:   # 1 + max vid, the ids read as u32 (an int32 tensor holds them); no wide copies
        if nrec:
            ends = records[:, :2]
            lo, hi = int(ends.min().item()), int(ends.max().item())
            # ids >= 2^31 read negative: the u32 maximum is then the largest negative one
            # (only those are copied out), not 2^32 - 1
            vs_cap = ((int(ends[ends < 0].max().item()) & 0xFFFFFFFF) if lo < 0 else hi) + 1
        else:
            vs_cap = 1
    deg = t.zeros(max(vs_cap, 1), dtype=t.int32, device=_dev(ctx))
    _, vs = degree_count(records, nrec, mode, deg, ctx=ctx)
    return sequence_from_degrees(deg, vs, ctx)


def sequence_from_host(seq: np.ndarray, ctx: Context | None = None) -> Sequence:
    """readSequence path (sequence.h:159-168): an arbitrary sequence -> seq/pos on device."""
    ctx = ctx or default_context()
    t = _torch()
    seq = np.asarray(seq, dtype=np.uint32)
    n = len(seq)
    pos_size = int(seq.max()) + 1 if n else 0
    d_seq = t.from_numpy(seq.view(np.int32).copy()).to(_dev(ctx)) if n else _dev_u32(1, ctx)
    pos = _dev_u32(pos_size, ctx)
    _check(lib().sheep_positions(ctx.handle, _ptr(d_seq), n, _ptr(pos), pos_size))
    return Sequence(d_seq, pos, n, pos_size)


# ---------------------------------------------------------------------------------
# jtree / jnode
# ---------------------------------------------------------------------------------
def build_tree(records, seq: Sequence, nrec: int | None = None, ctx: Context | None = None, out=None):
    """JTree(graph, seq): device tensor [n, 2] int32 = JNode {parent, pst_weight}
    (written into `out`, an [n, 2] int32 tensor, when given)."""
    ctx = ctx or default_context()
    t = _torch()
    nrec = records.shape[0] if nrec is None else nrec
    tree = out if out is not None else t.empty((max(seq.n, 1), 2), dtype=t.int32, device=_dev(ctx))
    _check(lib().sheep_build_tree(ctx.handle, _ptr(records), nrec, _ptr(seq.pos), seq.pos_size, seq.n, _ptr(tree)))
    return tree[: seq.n]


def merge_trees(a, b, ctx: Context | None = None):
    """JNodeTable::merge(lhs, rhs): Liu over the union of both parent-edge sets."""
    ctx = ctx or default_context()
    t = _torch()
    n = a.shape[0]
    if b.shape[0] != n:
        raise ValueError("trees of different sizes")
    out = t.empty((max(n, 1), 2), dtype=t.int32, device=_dev(ctx))
    _check(lib().sheep_merge_trees(ctx.handle, _ptr(a), _ptr(b), n, _ptr(out)))
    return out[:n]


def merge_trees_many(trees, ctx: Context | None = None):
    """The whole mpi_merge reduction (jnode.cpp:203-250) in one pass: `trees` is a
    (k, n, 2) int32 tensor of k partial trees; returns their merged tree."""
    ctx = ctx or default_context()
    t = _torch()
    k, n = trees.shape[0], trees.shape[1]
    trees = trees.contiguous()
    out = t.empty((max(n, 1), 2), dtype=t.int32, device=_dev(ctx))
    _check(lib().sheep_merge_trees_many(ctx.handle, _ptr(trees), k, n, _ptr(out)))
    return out[:n]


def merge_trees_part(trees, part: int, nparts: int, ctx: Context | None = None):
    """One part of a split K-way merge (sheep_merge_trees_part): returns (tree, lo, hi) —
    every node's pst and the parents of nodes [lo, hi) are the merged tree's."""
    ctx = ctx or default_context()
    t = _torch()
    k, n = trees.shape[0], trees.shape[1]
    trees = trees.contiguous()
    out = t.empty((max(n, 1), 2), dtype=t.int32, device=_dev(ctx))
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().sheep_merge_trees_part(ctx.handle, _ptr(trees), k, n, part, nparts, _ptr(out), ctypes.byref(lo),
                                        ctypes.byref(hi)))
    return out[:n], lo.value, hi.value


def tree_to_device(parent: np.ndarray, pst: np.ndarray):
    t = _torch()
    host = np.stack([np.asarray(parent, np.uint32), np.asarray(pst, np.uint32)], axis=1)
    return t.from_numpy(host.view(np.int32).copy()).to("cuda")


def tree_to_numpy(tree):
    a = to_numpy_u32(tree).reshape(-1, 2)
    return a[:, 0].copy(), a[:, 1].copy()


class KidTable:
    """makeKids (jnode.h:190-204): kid lists kept on the device; forwardPartition's
    in-place std::sort of a packing node's kids persists across k (partition.cpp:104-106)."""

    def __init__(self, tree, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.n = tree.shape[0]
        h = ctypes.c_void_p()
        _check(lib().sheep_kids_create(self.ctx.handle, _ptr(tree), self.n, ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            lib().sheep_kids_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class PartitionResult:
    parts: object            # device int16 tensor, vid-indexed, size max(seq)+1
    num_parts: int           # the k asked for
    created: int
    first_size: int
    second_size: int
    max_component: int
    total_weight: int
    packing_nodes: int
    heavy_nodes: int
    event_launches: int = 0   # packing-event kernel launches (sheep_tuning event_loop)

    def print_text(self) -> str:   # partition.h:135-143
        return (f"Actually created {self.created} partitions.\n"
                f"First two partition sizes: {self.first_size} and {self.second_size}\n")

    def numpy(self) -> np.ndarray:
        return self.parts.detach().cpu().numpy()


def partition(seq: Sequence, tree, k: int, balance: float = 1.03, vtx_weight: bool = False,
              pst_weight: bool = True, kids: KidTable | None = None, ctx: Context | None = None,
              use_pos: bool = True) -> PartitionResult:
    """Partition(seq, jnodes, k, balance, vtx, pst, pre=false) + forwardPartition.
    use_pos: the parts reach their vid slots through the sequence's index (sheep_partition_pos);
    False: by the per-jnid scatter of sheep_partition (the same result)."""
    ctx = ctx or default_context()
    t = _torch()
    kids = kids or KidTable(tree, ctx)
    pos_size = seq.pos_size
    parts = t.empty(max(pos_size, 1), dtype=t.int16, device=_dev(ctx))
    info = _PartInfo()
    if use_pos:
        _check(lib().sheep_partition_pos(ctx.handle, _ptr(tree), tree.shape[0], _ptr(seq.seq), seq.n, _ptr(seq.pos),
                                         pos_size, kids.handle, int(k), float(balance), int(vtx_weight),
                                         int(pst_weight), _ptr(parts), ctypes.byref(info)))
    else:
        _check(lib().sheep_partition(ctx.handle, _ptr(tree), tree.shape[0], _ptr(seq.seq), seq.n, pos_size,
                                     kids.handle, int(k), float(balance), int(vtx_weight), int(pst_weight),
                                     _ptr(parts), ctypes.byref(info)))
    return PartitionResult(parts[:pos_size], int(k), info.created, info.first_size, info.second_size,
                           info.max_component, info.total_weight, info.packing_nodes, info.heavy_nodes,
                           info.event_launches)


@dataclass
class EvalResult:
    edges_cut: int
    vcom_vol: int
    max_vertex_bal: int
    ecv_hash: int
    max_hash_bal: int
    ecv_down: int
    max_down_bal: int
    ecv_up: int
    max_up_bal: int
    edges: int
    nodes: int

    def text(self, num_parts: int, with_seq: bool = True) -> str:
        """The reference's printf lines (partition.cpp:468-472, 517-520), byte for byte."""
        E, N = self.edges, self.nodes
        Ek, Nk = E // num_parts, N // num_parts
        f = lambda a, b: _cfmt(a, b)
        s = (f"edges cut: {self.edges_cut} ({f(self.edges_cut, E)}%)\n"
             f"Vcom. vol: {self.vcom_vol} ({f(self.vcom_vol, E)}%)\n"
             f"  balance: {self.max_vertex_bal} ({f(self.max_vertex_bal, Nk)}%)\n"
             f"ECV(hash): {self.ecv_hash} ({f(self.ecv_hash, E)}%)\n"
             f"  balance: {self.max_hash_bal} ({f(self.max_hash_bal, Ek)}%)\n")
        if with_seq:
            s += (f"ECV(down): {self.ecv_down} ({f(self.ecv_down, E)}%)\n"
                  f"  balance: {self.max_down_bal} ({f(self.max_down_bal, Ek)}%)\n"
                  f"ECV(up)  : {self.ecv_up} ({f(self.ecv_up, E)}%)\n"
                  f"  balance: {self.max_up_bal} ({f(self.max_up_bal, Ek)}%)\n")
        return s


def _cfmt(a: int, b: int) -> str:
    """C printf("%f", (double)a / b) including inf/nan spellings."""
    if b == 0:
        return "inf" if a > 0 else "-nan"
    return "%f" % (a / b)


def evaluate(records, seq: Sequence, parts, what: int = 0, nrec: int | None = None,
             ctx: Context | None = None, from_step: bool = False) -> EvalResult:
    """Partition::evaluate(graph, seq) / evaluate(graph).  from_step: the same counts from the
    position-space edges the context's last build_tree over these records and this sequence
    left in HBM (sheep_evaluate_step; an error if it ran on anything else)."""
    ctx = ctx or default_context()
    nrec = records.shape[0] if nrec is None else nrec
    out = _Eval()
    if from_step:
        _check(lib().sheep_evaluate_step(ctx.handle, _ptr(records), nrec, _ptr(seq.seq), seq.n, _ptr(seq.pos),
                                         seq.pos_size, _ptr(parts), what, ctypes.byref(out)))
    else:
        _check(lib().sheep_evaluate(ctx.handle, _ptr(records), nrec, _ptr(seq.pos), seq.pos_size, _ptr(parts), what,
                                    ctypes.byref(out)))
    return EvalResult(*[getattr(out, f) for f, _ in _Eval._fields_])


class ShardedEvaluator:
    """Partition::evaluate over edge shards: each shard's records ORed
    into per-vertex part bitsets and summed counts, states of other devices combined with
    :meth:`combine`, one node pass in :meth:`finish`."""

    def __init__(self, seq: Sequence, parts, what: int = 0, nparts: int | None = None,
                 ctx: Context | None = None):
        self.ctx = ctx or default_context()
        t = _torch()
        self.seq, self.parts, self.what = seq, parts, what
        if nparts is None:
            n = ctypes.c_int32()
            _check(lib().sheep_eval_num_parts(self.ctx.handle, _ptr(parts), seq.pos_size, ctypes.byref(n)))
            nparts = n.value
        self.nparts = nparts
        bw, aw = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().sheep_eval_sizes(what, nparts, seq.pos_size, ctypes.byref(bw), ctypes.byref(aw)))
        self.bits = t.zeros(max(bw.value, 1), dtype=t.int64, device=f"cuda:{self.ctx.device}")
        self.acc = t.zeros(aw.value, dtype=t.int64, device=f"cuda:{self.ctx.device}")
        self.bits_words, self.acc_words = bw.value, aw.value

    @staticmethod
    def num_parts(parts, seq: Sequence, ctx: Context | None = None) -> int:
        """max part + 1 over the vid-indexed parts (partition.cpp:433-435)."""
        ctx = ctx or default_context()
        n = ctypes.c_int32()
        _check(lib().sheep_eval_num_parts(ctx.handle, _ptr(parts), seq.pos_size, ctypes.byref(n)))
        return n.value

    def add(self, records, nrec: int | None = None):
        nrec = records.shape[0] if nrec is None else nrec
        _check(lib().sheep_eval_shard(self.ctx.handle, _ptr(records), nrec, _ptr(self.seq.pos), self.seq.pos_size,
                                      _ptr(self.parts), self.what, self.nparts, _ptr(self.bits), _ptr(self.acc)))

    def combine(self, bits, acc):
        """OR another state's bits (same layout, on this device) and add its counts."""
        _check(lib().sheep_eval_combine(self.ctx.handle, _ptr(self.bits), _ptr(bits), self.bits_words,
                                        _ptr(self.acc), _ptr(acc), self.acc_words))

    def finish(self) -> "EvalResult":
        out = _Eval()
        _check(lib().sheep_eval_finish(self.ctx.handle, _ptr(self.bits), _ptr(self.acc), self.seq.pos_size,
                                       _ptr(self.parts), self.what, self.nparts, ctypes.byref(out)))
        return EvalResult(*[getattr(out, f) for f, _ in _Eval._fields_])


def edge_parts(records, seq: Sequence, parts, nrec: int | None = None, ctx: Context | None = None):
    """Part each record is written to by writePartitionedGraph (partition.cpp:588-670):
    the part of its earlier-positioned endpoint (device int16 per record)."""
    ctx = ctx or default_context()
    nrec = records.shape[0] if nrec is None else nrec
    t = _torch()
    out = t.empty(max(int(nrec), 1), dtype=t.int16, device=_dev(ctx))
    _check(lib().sheep_edge_parts(ctx.handle, _ptr(records), nrec, _ptr(seq.pos), seq.pos_size, _ptr(parts),
                                  _ptr(out)))
    return out[:nrec]


@dataclass
class Facts:
    width: int
    root_cnt: int
    vert_height: int
    edge_height: int
    vert_cnt: int
    edge_cnt: int
    halo_id: int
    core_id: int
    fill: int

    def text(self) -> str:   # jnode.h:285-291
        return (f"TREEFAQS: width:{self.width}\troots:{self.root_cnt}\n"
                f"\tvheight:{self.vert_height}\teheight:{self.edge_height}\n"
                f"\tverts:{self.vert_cnt}\tedges:{self.edge_cnt}\n"
                f"\thalo:{self.halo_id}\tcore:{self.core_id}\n"
                f"\tfill:{self.fill}\n")


def facts(tree, ctx: Context | None = None) -> Facts:
    ctx = ctx or default_context()
    out = _Facts()
    _check(lib().sheep_facts(ctx.handle, _ptr(tree), tree.shape[0], ctypes.byref(out)))
    return Facts(*[getattr(out, f) for f, _ in _Facts._fields_])


# ---------------------------------------------------------------------------------
# several GPUs in one process (graph2tree -i / -r without MPI)
# ---------------------------------------------------------------------------------
def _ptr_array(ts):
    return (ctypes.c_void_p * len(ts))(*[_ptr(t) for t in ts])


class _BorrowedContext(Context):
    """A rank's context inside a Group (owned by the group)."""

    def __init__(self, device: int, handle):
        self.device = device
        self.handle = handle

    def close(self):
        self.handle = None


class Group:
    """The ranks of graph2tree's MPI world (sheep_group_* in include/sheep_hip.h).

    ``Group(devices)`` — this process drives every rank (rank r on devices[r]): RCCL
    between distinct devices, device copies when a device is listed more than once.
    ``Group.join(device, rank, world, host, port)`` — one process per rank (mpiexec /
    torch.distributed ranks): this process holds one rank; RCCL when every rank has a
    device of its own, host memory over TCP when ranks share one (``link``).

    Per-rank arguments and results are lists over the ranks THIS process holds
    (``self.local`` of them, global ranks ``self.ranks``)."""

    REDUCE = {"none": 0, "kway": 1, "binomial": 2}
    LINK = {"auto": 0, "rccl": 1, "host": 2}

    def __init__(self, devices=None, _handle=None):
        if _handle is None:
            self.devices = list(devices)
            arr = (ctypes.c_int * len(self.devices))(*self.devices)
            h = ctypes.c_void_p()
            _check(lib().sheep_group_create(arr, len(self.devices), ctypes.byref(h)))
        else:
            h = _handle
            self.devices = list(devices)
        self.handle = h
        self.size = lib().sheep_group_size(h)
        self.local = lib().sheep_group_local_count(h)
        self.ranks = [lib().sheep_group_rank(h, i) for i in range(self.local)]
        self.ctx = [_BorrowedContext(d, ctypes.c_void_p(lib().sheep_group_ctx(h, i)))
                    for i, d in enumerate(self.devices)]

    @classmethod
    def join(cls, device: int, rank: int, world: int, host: str = "127.0.0.1", port: int = 29650,
             link: str = "auto") -> "Group":
        h = ctypes.c_void_p()
        _check(lib().sheep_group_join(int(device), int(rank), int(world), host.encode(), int(port), cls.LINK[link],
                                      ctypes.byref(h)))
        return cls([device], _handle=h)

    @property
    def rccl(self) -> bool:
        return bool(lib().sheep_group_uses_rccl(self.handle))

    @property
    def failed(self) -> bool:
        """A collective failed or timed out (SHEEP_JOIN_TIMEOUT), or abort() ran: the
        communicators are aborted and every later collective raises."""
        return bool(lib().sheep_group_failed(self.handle))

    def abort(self, reason: str = "requested by the caller"):
        """sheep_group_abort: end the world (ncclCommAbort), one stderr line per local rank."""
        _check(lib().sheep_group_abort(self.handle, reason.encode()))

    def close(self):
        if getattr(self, "handle", None):
            lib().sheep_group_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, i):
        return f"cuda:{self.devices[i]}"

    def _ready(self):
        """The ranks run on streams of their own: finish torch's work on every device
        (inputs, zero-filled outputs) before a group call reads it."""
        t = _torch()
        for d in sorted(set(self.devices)):
            t.cuda.synchronize(d)

    def barrier(self):
        _check(lib().sheep_group_barrier(self.handle))

    def set_tuning(self, **kw):
        """sheep_group_set_tuning: Context.set_tuning on every local rank's context."""
        _check(lib().sheep_group_set_tuning(self.handle, ctypes.byref(Tuning.of(**kw))))

    def allreduce_max(self, v: int) -> int:
        x = ctypes.c_uint64(int(v))
        _check(lib().sheep_group_allreduce_max_u64(self.handle, ctypes.byref(x)))
        return x.value

    def sequence(self, shards, vs_cap: int, deg=None, seq=None, pos=None):
        """mpiSequence over the ranks' record shards: a Sequence per local rank (all
        equal).  deg / seq / pos: optional per-rank buffers (deg zeroed) to reuse."""
        t = _torch()
        L = self.local
        deg = deg or [t.zeros(max(vs_cap, 1), dtype=t.int32, device=self._dev(i)) for i in range(L)]
        seq = seq or [t.empty(max(vs_cap, 1), dtype=t.int32, device=self._dev(i)) for i in range(L)]
        pos = pos or [t.empty(max(vs_cap, 1), dtype=t.int32, device=self._dev(i)) for i in range(L)]
        nrec = (ctypes.c_uint64 * L)(*[s.shape[0] for s in shards])
        n, vs = ctypes.c_uint64(), ctypes.c_uint64()
        self._ready()
        _check(lib().sheep_group_sequence(self.handle, _ptr_array(shards), nrec, _ptr_array(deg), vs_cap,
                                          _ptr_array(seq), _ptr_array(pos), ctypes.byref(n), ctypes.byref(vs)))
        return [Sequence(seq[i], pos[i], n.value, vs.value) for i in range(L)]

    def build_tree(self, shards, seqs, reduce: str = "kway", trees=None):
        """JTree per shard + mpi_merge: per local rank its tree — rank 0's is the merged
        tree for kway / binomial, every tree is the rank's partial tree for "none"."""
        t = _torch()
        L = self.local
        n = seqs[0].n
        trees = trees or [t.empty((max(n, 1), 2), dtype=t.int32, device=self._dev(i)) for i in range(L)]
        nrec = (ctypes.c_uint64 * L)(*[s.shape[0] for s in shards])
        self._ready()
        _check(lib().sheep_group_build_tree(self.handle, _ptr_array(shards), nrec, _ptr_array([s.pos for s in seqs]),
                                            seqs[0].pos_size, n, _ptr_array(trees), self.REDUCE[reduce]))
        return [x[:n] for x in trees]

    def reduce_trees(self, trees, reduce: str = "kway"):
        """The reduction step alone over the local ranks' partial trees (in place)."""
        self._ready()
        _check(lib().sheep_group_reduce_trees(self.handle, _ptr_array(trees), trees[0].shape[0], self.REDUCE[reduce]))
        return trees

    def broadcast_parts(self, parts, pos_size: int):
        """Partition::mpi_sync: rank 0's parts to every rank.  `parts` lists one int16
        tensor (pos_size entries) per local rank; rank 0's holds the parts."""
        self._ready()
        _check(lib().sheep_group_broadcast_parts(self.handle, _ptr_array(parts), pos_size))
        return [p[:pos_size] for p in parts]

    def transfer(self, src_rank: int, dst_rank: int, src=None, dst=None, nbytes: int | None = None):
        """One point-to-point move (ncclSend/ncclRecv under RCCL) of src_rank's tensor
        `src` into dst_rank's tensor `dst`; every rank of the world calls it."""
        if nbytes is None:
            t = src if src is not None else dst
            nbytes = t.numel() * t.element_size()
        self._ready()
        _check(lib().sheep_group_transfer(self.handle, int(src_rank), int(dst_rank),
                                          ctypes.c_void_p(_ptr(src) if src is not None else 0),
                                          ctypes.c_void_p(_ptr(dst) if dst is not None else 0), int(nbytes)))
        return dst

    def evaluate(self, shards, seqs, parts, what: int = 0) -> "EvalResult":
        """The evaluator over the shards; the counts are rank 0's (zero elsewhere)."""
        L = self.local
        nrec = (ctypes.c_uint64 * L)(*[s.shape[0] for s in shards])
        out = _Eval()
        self._ready()
        _check(lib().sheep_group_evaluate(self.handle, _ptr_array(shards), nrec, _ptr_array([s.pos for s in seqs]),
                                          seqs[0].pos_size, _ptr_array(parts), what, ctypes.byref(out)))
        return EvalResult(*[getattr(out, f) for f, _ in _Eval._fields_])


# ---------------------------------------------------------------------------------
# synthetic input
# ---------------------------------------------------------------------------------
def rmat(scale: int, edgefactor: int = 16, seed: int = 1, ctx: Context | None = None):
    """Graph500-parameter RMAT records generated in HBM: [R, 3] int32 device tensor."""
    ctx = ctx or default_context()
    t = _torch()
    cap = edgefactor << scale
    out = t.empty((cap, 3), dtype=t.int32, device=_dev(ctx))
    n = ctypes.c_uint64()
    _check(lib().sheep_rmat_generate(ctx.handle, scale, edgefactor, seed, _ptr(out), cap, ctypes.byref(n)))
    return out[: n.value]


TWITTER_VERTICES = 41_652_230      # twitter-2010 (slurm-fen-twitter.out:2)


def powerlaw(nverts: int = TWITTER_VERTICES, draws: int = 2_222_000_000, gamma: float = 1.9, seed: int = 2010,
             ctx: Context | None = None):
    """Chung-Lu power-law records generated in HBM (BASELINE config C4): [R, 3] int32."""
    ctx = ctx or default_context()
    t = _torch()
    out = t.empty((draws, 3), dtype=t.int32, device=_dev(ctx))
    n = ctypes.c_uint64()
    _check(lib().sheep_powerlaw_generate(ctx.handle, nverts, draws, float(gamma), seed, _ptr(out), draws,
                                         ctypes.byref(n)))
    return out[: n.value]


def rmat_host(scale: int, edgefactor: int = 16, seed: int = 1) -> np.ndarray:
    """The same generator on the CPU: structured array of XS1 records (for .dat files)."""
    cap = edgefactor << scale
    buf = np.empty(cap * 3, dtype=np.uint32)
    n = ctypes.c_uint64()
    _check(lib().sheep_rmat_generate_host(scale, edgefactor, seed, buf.ctypes.data, cap, ctypes.byref(n)))
    return buf[: 3 * n.value].reshape(-1, 3)


def parse_net(text: bytes, skip_comments: bool = False, ctx: Context | None = None):
    """A SNAP text edge list parsed on the GPU (sheep_parse_net): [R, 3] int32 device
    records, SNAPReader semantics (skip_comments: the graph loader's '#'/'%' lines)."""
    ctx = ctx or default_context()
    t = _torch()
    raw = t.frombuffer(bytearray(text), dtype=t.uint8).to(_dev(ctx)) if text else t.empty(1, dtype=t.uint8,
                                                                                            device=_dev(ctx))
    cap = len(text) // 4 + 1
    out = t.empty((cap, 3), dtype=t.int32, device=_dev(ctx))
    n = ctypes.c_uint64()
    _check(lib().sheep_parse_net(ctx.handle, _ptr(raw), len(text), int(skip_comments), _ptr(out), cap,
                                 ctypes.byref(n)))
    return out[: n.value]


XS1 = np.dtype([("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])


def read_dat(path: str) -> np.ndarray:
    return np.fromfile(path, dtype=XS1)
