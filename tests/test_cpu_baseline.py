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
