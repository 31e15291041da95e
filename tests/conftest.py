import hashlib
import json
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

XS1 = np.dtype([("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])
GRAPHS = ["hep", "rmat10", "rmat12", "rmat14", "edge"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def manifest():
    return json.load(open(os.path.join(GOLDEN, "MANIFEST.json")))


def golden_records(name):
    """Input records of a golden graph (regenerating the rmat inputs that are not
    committed, md5-checked against the manifest)."""
    path = os.path.join(GOLDEN, f"{name}.dat")
    if os.path.exists(path):
        rec = np.fromfile(path, dtype=XS1)
    else:
        import sheep_amd
        scale, ef, seed = manifest()["_rmat"][name]
        r = sheep_amd.rmat_host(scale, ef, seed)
        rec = np.zeros(len(r), dtype=XS1)
        rec["tail"], rec["head"], rec["weight"] = r[:, 0], r[:, 1], 1.0
    assert hashlib.md5(rec.tobytes()).hexdigest() == manifest()[f"{name}.dat"], f"{name}.dat input drifted"
    return rec


def golden_seq(name, kind="seq"):
    return np.loadtxt(os.path.join(GOLDEN, f"{name}.{kind}"), dtype=np.uint32, ndmin=1)


def read_tre(path):
    raw = np.fromfile(path, dtype=np.uint32)
    end_id = int(raw[0])
    nodes = raw[1:].reshape(-1, 2)
    return end_id, nodes[:, 0].copy(), nodes[:, 1].copy()


def golden_tree(name, which="tre"):
    end_id, parent, pst = read_tre(os.path.join(GOLDEN, f"{name}.{which}"))
    assert end_id == len(parent)
    return parent, pst


def golden_parts(name, k):
    return np.fromfile(os.path.join(GOLDEN, f"{name}.k{k}.parts"), dtype=np.int16)


def golden_part_text(name):
    """Split the reference's partition_tree -f -g output into (facts, [per-k blocks])."""
    txt = open(os.path.join(GOLDEN, f"{name}.part.txt")).read()
    lines = txt.splitlines(keepends=True)
    facts = "".join(lines[:5])
    blocks, cur = [], []
    for ln in lines[5:]:
        if ln.startswith("Actually created") and cur:
            blocks.append("".join(cur))
            cur = []
        cur.append(ln)
    if cur:
        blocks.append("".join(cur))
    return facts, blocks


PRINT_GRAPHS = ["hep", "rmat10", "rmat12", "edge"]


def check_print(text, name, tag="print"):
    """graph2tree -t output against the reference's JTree::print run (make_golden.py):
    the committed file where there is one, else its md5 and line count."""
    entry = manifest()["_print"][f"{name}.{tag}.txt"]
    path = os.path.join(GOLDEN, f"{name}.{tag}.txt")
    if os.path.exists(path):
        assert text == open(path).read(), f"{name}.{tag}"
    assert text.count("\n") == entry["lines"], f"{name}.{tag}"
    assert hashlib.md5(text.encode()).hexdigest() == entry["md5"], f"{name}.{tag}"


def ks(name):
    return manifest()["_ks"][name]


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_ctx():
    if not gpu_available():
        pytest.skip("no HIP device")
    import sheep_amd
    return sheep_amd.default_context()
