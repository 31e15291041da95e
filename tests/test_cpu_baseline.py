"""The CPU baseline's reference runs (oracle/_ref/ref_harness, built from /root/reference by
oracle/ref/Makefile; test infrastructure): the literal -i sequence (mpiSequence, whose
comparator captures the degree vector by value, sequence.h:85) and the by-reference form
that bench.py's cpu_baseline times produce the same sequence, merged tree and parts at every
rank count, and those equal the reference-built golden files."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
MPIEXEC = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
pytestmark = pytest.mark.skipif(not (os.path.exists(HARNESS) and MPIEXEC),
                                reason="oracle/_ref/ref_harness or mpiexec not built here")


def _fnv(b: bytes) -> str:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def _run(mode, path, k, p):
    r = subprocess.run([MPIEXEC, "-n", str(p), HARNESS, mode, path, str(k)], capture_output=True, text=True,
                       timeout=120, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-500:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("name,k", [("hep", 2), ("edge", 2)])
def test_literal_ir_matches_by_reference_and_golden(name, k):
    path = os.path.join(GOLDEN, f"{name}.dat")
    tre = open(os.path.join(GOLDEN, f"{name}.tre"), "rb").read()[4:]   # [u32 end_id][JNode ...]
    parts = os.path.join(GOLDEN, f"{name}.k{k}.parts")
    seq = np.loadtxt(os.path.join(GOLDEN, f"{name}.seq"), dtype=np.uint32).reshape(-1)
    want = {"seq": _fnv(seq.tobytes()), "tree": _fnv(tre)}
    if os.path.exists(parts):
        want["parts"] = _fnv(open(parts, "rb").read())
    for p in (1, 2, 3):
        for mode in ("mpi", "mpi_ir"):
            got = _run(mode, path, k, p)["fnv"]
            for key, v in want.items():
                assert got[key] == v, (mode, p, key)


def test_reference_flow_on_rmat_matches_the_restatement(tmp_path):
    """The reference flow (2 MPI ranks) on an RMAT-14 graph gives the oracle restatement's
    sequence, tree and parts (k = 8), compared through the harness's FNV-1a digests — the
    digests bench.py's cpu_baseline compares with the GPU's results (`matches_gpu`); and
    oracle.fnv1a is that digest."""
    import oracle
    import sheep_amd
    b = np.random.default_rng(3).integers(0, 256, 1000, dtype=np.uint8)
    assert oracle.fnv1a(b) == _fnv(b.tobytes())
    r = sheep_amd.rmat_host(14, 16, 14).astype(np.uint32)
    path = str(tmp_path / "r14.dat")
    r.tofile(path)
    got = _run("mpi", path, 8, 2)["fnv"]
    t, h = r[:, 0], r[:, 1]
    seq = oracle.sequence(t, h)
    p, w = oracle.build_tree(t, h, seq)
    tw = np.empty(2 * len(p), np.uint32)
    tw[0::2], tw[1::2] = p, w
    parts, _ = oracle.partition(p, w, seq, 8)
    assert got == {"seq": oracle.fnv1a(seq.astype(np.uint32)), "tree": oracle.fnv1a(tw),
                   "parts": oracle.fnv1a(np.asarray(parts, np.int16))}
