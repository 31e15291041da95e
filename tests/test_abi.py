"""The drop-in boundary on the CPU: libsheep_hip.so loads without a GPU and exports every
entry point include/sheep_hip.h declares; the host-only generator matches the committed
golden inputs; errors come back as status codes (no compute calls need a device)."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

from conftest import ROOT, manifest

HEADER = os.path.join(ROOT, "include", "sheep_hip.h")
LIB = os.path.join(ROOT, "sheep_amd", "lib", "libsheep_hip.so")


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(sheep_\w+)\s*\(", text, re.M)))


def lib():
    if not os.path.exists(LIB):
        pytest.skip("libsheep_hip.so not built (make hip)")
    return ctypes.CDLL(LIB)


def test_header_declares_the_path():
    names = declared()
    for must in ("sheep_degree_count", "sheep_sequence_from_degrees", "sheep_positions", "sheep_build_tree",
                 "sheep_merge_trees", "sheep_merge_trees_many", "sheep_kids_create", "sheep_partition", "sheep_evaluate", "sheep_facts"):
        assert must in names


def test_every_declared_symbol_is_exported():
    L = lib()
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_errors_are_status_codes_without_a_device():
    L = lib()
    L.sheep_last_error.restype = ctypes.c_char_p
    h = ctypes.c_void_p()
    rc = L.sheep_ctx_create(0, None, ctypes.byref(h))
    if rc == 0:
        L.sheep_ctx_destroy(h)
        pytest.skip("a HIP device is visible")
    assert rc in (-1, -2)   # SHEEP_ERR_ARG (no such device) or SHEEP_ERR_HIP
    assert L.sheep_last_error()
    n = ctypes.c_uint64()
    assert L.sheep_rmat_generate_host(40, 16, 1, None, 0, ctypes.byref(n)) == -1


@pytest.mark.parametrize("name", ["rmat10", "rmat12", "rmat14"])
def test_host_generator_matches_golden_inputs(name):
    import sheep_amd
    lib()
    scale, ef, seed = manifest()["_rmat"][name]
    r = sheep_amd.rmat_host(scale, ef, seed)
    rec = np.zeros(len(r), dtype=[("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])
    rec["tail"], rec["head"], rec["weight"] = r[:, 0], r[:, 1], 1.0
    assert hashlib.md5(rec.tobytes()).hexdigest() == manifest()[f"{name}.dat"]
    # generator contract: simple graph, tail > head, sorted by (tail, head)
    assert np.all(rec["tail"] > rec["head"])
    key = rec["tail"].astype(np.uint64) << 32 | rec["head"]
    assert np.all(np.diff(key.astype(np.int64)) > 0)


def test_tuning_defaults_without_a_device():
    """sheep_tuning_default needs no device; the defaults are the documented ones."""
    import sheep_amd
    lib()
    t = sheep_amd.Tuning()
    assert sheep_amd.lib().sheep_tuning_default(ctypes.byref(t)) == 0
    assert t.as_dict() == {"fin_map_bits": 13, "fin_merge_bits": 12, "fin_dc": 1, "top_bits": 16, "top_blocks": 4,
                           "big_bits": 21, "big_dense": 256, "big_hot_bits": 15, "big_hot16": 0, "relabel_planes": 1,
                           "relabel_per": 8, "cross_win_levels": 2, "hook_batch": 0,
                           "merge_cut_bits": 0, "event_loop": 4096, "hook_up": 0}
    with pytest.raises(KeyError):
        sheep_amd.Tuning.of(no_such_field=1)


def test_library_reads_one_debug_variable():
    """The algorithm variants are per-context options (sheep_tuning), not environment
    variables: the sources read SHEEP_DEBUG (debugging) and SHEEP_JOIN_TIMEOUT (how long
    joined ranks wait for each other) and nothing else."""
    csrc = os.path.join(ROOT, "sheep_amd", "csrc")
    names = set()
    for f in os.listdir(csrc):
        names |= set(re.findall(r'getenv\("(\w+)"\)', open(os.path.join(csrc, f)).read()))
    assert names == {"SHEEP_DEBUG", "SHEEP_JOIN_TIMEOUT"}, names
