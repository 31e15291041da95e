"""ctypes wrapper of oracle/lib/libsheep_oracle.so — the CPU restatement of the
reference path.  TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, never by sheep_amd/.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SHEEP_ORACLE_LIB: another build of the same restatement (`make asan`: AddressSanitizer +
# UBSan, oracle/lib/asan/)
LIB_PATH = os.environ.get("SHEEP_ORACLE_LIB") or os.path.join(_HERE, "lib", "libsheep_oracle.so")
INVALID = 0xFFFFFFFF
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built; run `make oracle`")
        L = ctypes.CDLL(LIB_PATH)
        P, U64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.or_last_error.restype = ctypes.c_char_p
        L.or_sequence.argtypes = [P, P, U64, I32, P, U64, ctypes.POINTER(U64)]
        L.or_build_tree.argtypes = [P, P, U64, U64, U64, P, U64, P, P]
        L.or_build_tree_mr.argtypes = [P, P, U64, P, U64, U64, P, P]
        L.or_merge.argtypes = [P, P, P, P, U64, P, P]
        L.or_facts.argtypes = [P, P, U64, P]
        L.or_kids_create.argtypes = [P, U64]
        L.or_kids_create.restype = P
        L.or_kids_free.argtypes = [P]
        L.or_partition.argtypes = [P, P, U64, P, U64, P, ctypes.c_int16, ctypes.c_double, I32, I32, P, U64,
                                   ctypes.POINTER(U64), P]
        L.or_set_threads.argtypes = [I32]
        L.or_evaluate.argtypes = [P, P, U64, P, U64, P, U64, P]
        L.or_facts_text.argtypes = [P, P, U64, P, U64]
        L.or_eval_text.argtypes = [P, ctypes.c_int16, P, U64]
        L.or_fnv1a.argtypes = [P, U64]
        L.or_fnv1a.restype = U64
        _lib = L
    return _lib


def _chk(rc):
    if rc != 0:
        raise RuntimeError("oracle: " + lib().or_last_error().decode())


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _p(a):
    return a.ctypes.data


def fnv1a(a) -> str:
    """FNV-1a of an array's bytes as 16 hex digits (oracle/ref/ref_harness's digests)."""
    a = np.ascontiguousarray(a)
    return "%016x" % lib().or_fnv1a(_p(a), a.nbytes)


def set_threads(n: int):
    """OpenMP threads of the graph build and evaluators (default 1)."""
    lib().or_set_threads(int(n))


def sequence(tail, head, mode="llama"):
    """mode 'llama' (degreeSequence over the LLAMA graph), 'records' (the same degrees
    counted straight from the records, no adjacency build), 'dat' / 'net' (fileSequence)."""
    tail, head = _u32(tail), _u32(head)
    cap = 2 * len(tail) + 2
    out = np.empty(cap, np.uint32)
    n = ctypes.c_uint64()
    _chk(lib().or_sequence(_p(tail), _p(head), len(tail), {"llama": 0, "dat": 1, "net": 2, "records": 3}[mode],
                           _p(out), cap, ctypes.byref(n)))
    return out[: n.value].copy()


def build_tree(tail, head, seq, part=0, num_parts=0):
    tail, head, seq = _u32(tail), _u32(head), _u32(seq)
    n = len(seq)
    parent, pst = np.empty(n, np.uint32), np.empty(n, np.uint32)
    _chk(lib().or_build_tree(_p(tail), _p(head), len(tail), part, num_parts, _p(seq), n, _p(parent), _p(pst)))
    return parent, pst


def build_tree_mr(tail, head, seq, shards=16):
    """The same tree in graph2tree -r's map/reduce form: `shards` contiguous record
    shards' partial trees (OpenMP threads) merged in binomial rounds (mpi_merge).  Linear
    memory in the records, for the BASELINE-size checks (C3-C5)."""
    tail, head, seq = _u32(tail), _u32(head), _u32(seq)
    n = len(seq)
    parent, pst = np.empty(n, np.uint32), np.empty(n, np.uint32)
    _chk(lib().or_build_tree_mr(_p(tail), _p(head), len(tail), _p(seq), n, int(shards), _p(parent), _p(pst)))
    return parent, pst


def merge(pa, wa, pb, wb):
    pa, wa, pb, wb = map(_u32, (pa, wa, pb, wb))
    n = len(pa)
    po, wo = np.empty(n, np.uint32), np.empty(n, np.uint32)
    _chk(lib().or_merge(_p(pa), _p(wa), _p(pb), _p(wb), n, _p(po), _p(wo)))
    return po, wo


FACT_FIELDS = ("width", "root_cnt", "vert_height", "edge_height", "vert_cnt", "edge_cnt", "halo_id", "core_id", "fill")


def facts(parent, pst):
    parent, pst = _u32(parent), _u32(pst)
    out = np.zeros(9, np.uint64)
    _chk(lib().or_facts(_p(parent), _p(pst), len(parent), _p(out)))
    return dict(zip(FACT_FIELDS, map(int, out)))


def facts_text(parent, pst):
    parent, pst = _u32(parent), _u32(pst)
    buf = ctypes.create_string_buffer(1024)
    _chk(lib().or_facts_text(_p(parent), _p(pst), len(parent), buf, 1024))
    return buf.value.decode()


def print_text(parent, pst, seq):
    """JTree::print (jtree.h:60-66) -> JNodeTable::print(id) (jnode.h:263-267) on the
    default path: jnid -> vid through the sequence (get_sequence, jtree.h:50-57), width =
    1 + pst (jnode.h:258-260, no junction data), pre_weight 0 (USE_PRE_WEIGHT off,
    defs.h:62).  Pure Python: small trees only."""
    out = []
    for i, (par, w) in enumerate(zip(np.asarray(parent, np.uint32).tolist(), np.asarray(pst, np.uint32).tolist())):
        out.append("%4d:%-8d%6d:w%6d:pre%6d:pst        ->[%4d]\n" % (i, int(seq[i]), 1 + w, 0, w, par))
    return "".join(out)


class Kids:
    """Persistent kid table for one tree (partition_tree keeps it across k)."""

    def __init__(self, parent):
        self.parent = _u32(parent)
        self.h = lib().or_kids_create(_p(self.parent), len(self.parent))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_kids_free(self.h)
            self.h = None


def partition(parent, pst, seq, k, balance=1.03, vtx=False, pstw=True, kids=None):
    parent, pst, seq = _u32(parent), _u32(pst), _u32(seq)
    kids = kids or Kids(parent)
    cap = int(seq.max()) + 1 if len(seq) else 1
    parts = np.empty(cap, np.int16)
    vs = ctypes.c_uint64()
    info = np.zeros(3, np.int64)
    _chk(lib().or_partition(_p(parent), _p(pst), len(parent), _p(seq), len(seq), kids.h, int(k), float(balance), int(vtx),
                            int(pstw), _p(parts), cap, ctypes.byref(vs), _p(info)))
    return parts[: vs.value].copy(), {"created": int(info[0]), "max_component": int(info[1]),
                                      "packing_nodes": int(info[2])}


EVAL_FIELDS = ("edges_cut", "vcom_vol", "max_vertex_bal", "ecv_hash", "max_hash_bal", "ecv_down", "max_down_bal",
               "ecv_up", "max_up_bal", "edges", "nodes")


def evaluate(tail, head, seq, parts):
    tail, head, seq = _u32(tail), _u32(head), _u32(seq)
    parts = np.ascontiguousarray(parts, np.int16)
    out = np.zeros(11, np.uint64)
    _chk(lib().or_evaluate(_p(tail), _p(head), len(tail), _p(seq), len(seq), _p(parts), len(parts), _p(out)))
    return dict(zip(EVAL_FIELDS, map(int, out)))


def eval_text(ev: dict, num_parts: int) -> str:
    v = np.array([ev[f] for f in EVAL_FIELDS], np.uint64)
    buf = ctypes.create_string_buffer(2048)
    _chk(lib().or_eval_text(_p(v), int(num_parts), buf, 2048))
    return buf.value.decode()
