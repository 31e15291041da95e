"""The drop-in CLIs (sheep_amd/cli/*.cpp over libsheep_hip.so) against the reference's
golden outputs: same files byte for byte, same stdout lines (timing lines aside)."""
import filecmp
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT, golden_records, ks

BIN = os.path.join(ROOT, "sheep_amd", "bin")
CLIS = ("graph2tree", "partition_tree", "merge_trees", "degree_sequence")
TIMING = ("Loaded graph in:", "Sorted in:", "Mapped in:", "Reduced in:", "Loaded tree in:", "Partitioning took:",
          "Finished in:", "Built in:", "Loaded in:")


def run(*args, check=True):
    p = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=120)
    if check:
        assert p.returncode == 0, p.stdout + p.stderr
    return p


def dat_path(name, tmp_path):
    """The golden input as a .dat file (the larger RMAT inputs are regenerated, md5-checked)."""
    path = os.path.join(GOLDEN, f"{name}.dat")
    if os.path.exists(path):
        return path
    path = str(tmp_path / f"{name}.dat")
    golden_records(name).tofile(path)
    return path


def strip_timing(text):
    return "".join(ln for ln in text.splitlines(keepends=True) if not ln.startswith(TIMING))


@pytest.mark.parametrize("cli", CLIS)
def test_usage_without_gpu(cli):
    """Argument errors are reported like the reference's, before any device is touched."""
    exe = os.path.join(BIN, cli)
    if not os.path.exists(exe):
        pytest.skip("CLIs not built (make cli)")
    p = run(exe, check=False)
    assert p.returncode == 1
    assert p.stdout.startswith("USAGE:")


def test_unknown_option_without_gpu():
    exe = os.path.join(BIN, "graph2tree")
    if not os.path.exists(exe):
        pytest.skip("CLIs not built (make cli)")
    p = run(exe, "-Q", "x.dat", check=False)
    assert p.returncode == 1 and p.stdout == "Unknown option character '\\x51'.\n"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hep", "rmat12", "edge"])
def test_graph2tree_tree_and_facts(gpu_ctx, tmp_path, name):
    dat = dat_path(name, tmp_path)
    out = tmp_path / "t.tre"
    p = run(os.path.join(BIN, "graph2tree"), dat, "-o", out, "-f")
    assert filecmp.cmp(out, os.path.join(GOLDEN, f"{name}.tre"), shallow=False)
    assert strip_timing(p.stdout) == open(os.path.join(GOLDEN, f"{name}.facts")).read()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hep", "edge"])
def test_graph2tree_partial_loads_and_merge_trees(gpu_ctx, tmp_path, name):
    """graph2tree -l 1/2, 2/2 with the sequence file, then merge_trees (the script path)."""
    dat = dat_path(name, tmp_path)
    seq = os.path.join(GOLDEN, f"{name}.seq")
    halves = []
    for part, which in ((1, "h1"), (2, "h2")):
        out = tmp_path / f"{which}.tre"
        run(os.path.join(BIN, "graph2tree"), dat, "-l", f"{part}/2", "-s", seq, "-o", out)
        assert filecmp.cmp(out, os.path.join(GOLDEN, f"{name}.{which}.tre"), shallow=False), which
        halves.append(out)
    merged = tmp_path / "m.tre"
    p = run(os.path.join(BIN, "merge_trees"), halves[0], halves[1], "-o", merged, "-f")
    assert filecmp.cmp(merged, os.path.join(GOLDEN, f"{name}.merge.tre"), shallow=False)
    assert p.stdout == open(os.path.join(GOLDEN, f"{name}.facts")).read()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hep", "rmat12", "edge"])
def test_degree_sequence_cli(gpu_ctx, tmp_path, name):
    dat = dat_path(name, tmp_path)
    out = tmp_path / "s.seq"
    p = run(os.path.join(BIN, "degree_sequence"), dat, out)
    assert p.stdout.startswith("Sorted in: ")
    assert filecmp.cmp(out, os.path.join(GOLDEN, f"{name}.fileseq"), shallow=False)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hep", "rmat12", "edge"])
def test_partition_tree_cli(gpu_ctx, tmp_path, name):
    """partition_tree -v -f -g G SEQ TREE k1 k2 ... (-v turns the timing lines off):
    TREEFAQS + per-k print + both evaluators, byte-exact with the reference's run."""
    dat = dat_path(name, tmp_path)
    p = run(os.path.join(BIN, "partition_tree"), "-v", "-f", "-g", dat, os.path.join(GOLDEN, f"{name}.seq"),
            os.path.join(GOLDEN, f"{name}.tre"), *ks(name))
    assert p.stdout == open(os.path.join(GOLDEN, f"{name}.part.txt")).read()
