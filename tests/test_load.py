"""Partial loads (graph2tree -l p/k, and rank r of an -i -r world): LLAMAGraph(filename, part,
num_parts) hands lc_partial_load_part / num_parts to the loader (graph_wrapper.h:43-63), so a
rank reads only its records.  sheep_dat_range / sheep_read_dat (host-only, used by the façade's
loadRecords and the CLIs) must read exactly part p's byte range [(p-1)R/k, pR/k) x 12 of a .dat
file and nothing else: checked here with the process's read-byte counter (/proc/self/io
rchar counts every byte read() / pread() return)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "sheep_amd", "lib", "libsheep_hip.so")
XS1 = np.dtype([("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])


def _lib():
    if not os.path.exists(LIB):
        pytest.skip("libsheep_hip.so not built")
    L = ctypes.CDLL(LIB)
    U64P = ctypes.POINTER(ctypes.c_uint64)
    L.sheep_dat_range.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, U64P, U64P]
    L.sheep_read_dat.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, U64P]
    L.sheep_last_error.restype = ctypes.c_char_p
    return L


def _rchar():
    with open("/proc/self/io") as f:
        for line in f:
            if line.startswith("rchar:"):
                return int(line.split()[1])
    raise RuntimeError("no rchar")


@pytest.fixture
def dat(tmp_path):
    rng = np.random.default_rng(7)
    R = 300_001   # not a multiple of any part count used below
    rec = np.zeros(R, XS1)
    rec["tail"] = rng.integers(0, 1 << 20, R)
    rec["head"] = rng.integers(0, 1 << 20, R)
    rec["weight"] = 1.0
    path = tmp_path / "g.dat"
    rec.tofile(path)
    with open(path, "ab") as f:
        f.write(b"\x01\x02\x03")   # a trailing partial record is not a record (size // 12)
    return str(path).encode(), rec


def _read_part(L, path, part, k):
    first, count, got = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    assert L.sheep_dat_range(path, part, k, ctypes.byref(first), ctypes.byref(count)) == 0
    out = np.empty(count.value, XS1)
    base = _rchar()
    calib = _rchar() - base   # (reading the counter itself)
    base = _rchar()
    assert L.sheep_read_dat(path, first.value, count.value, out.ctypes.data, ctypes.byref(got)) == 0
    read = _rchar() - base - calib
    assert got.value == count.value
    return first.value, out, read


@pytest.mark.parametrize("k", [1, 2, 3, 4, 7])
def test_partial_load_reads_only_its_range(dat, k):
    L = _lib()
    path, rec = dat
    R = len(rec)
    parts = []
    for p in range(1, k + 1):
        first, out, read = _read_part(L, path, p, k)
        assert first == (p - 1) * R // k and len(out) == p * R // k - first
        assert np.array_equal(out, rec[first:first + len(out)])
        assert len(out) * 12 <= read <= len(out) * 12 + 256, (p, read)   # its bytes, none of the others'
        parts.append(out)
    assert np.array_equal(np.concatenate(parts), rec)


def test_whole_file_and_errors(dat, tmp_path):
    L = _lib()
    path, rec = dat
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.sheep_dat_range(path, 0, 0, ctypes.byref(first), ctypes.byref(count)) == 0
    assert (first.value, count.value) == (0, len(rec))
    assert L.sheep_dat_range(path, 3, 2, ctypes.byref(first), ctypes.byref(count)) == -1    # part > num_parts
    assert L.sheep_dat_range(path, 0, 2, ctypes.byref(first), ctypes.byref(count)) == -1    # parts are 1-indexed
    missing = str(tmp_path / "none.dat").encode()
    assert L.sheep_dat_range(missing, 1, 2, ctypes.byref(first), ctypes.byref(count)) == -1
    assert b"cannot open" in L.sheep_last_error()
    got = ctypes.c_uint64()
    out = np.empty(10, XS1)
    assert L.sheep_read_dat(missing, 0, 10, out.ctypes.data, ctypes.byref(got)) == -1
    # past the end: only what is there
    assert L.sheep_read_dat(path, len(rec) - 4, 10, np.empty(10, XS1).ctypes.data, ctypes.byref(got)) == 0
    assert got.value == 4
