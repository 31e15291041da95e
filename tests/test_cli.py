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


# ---- graph2tree -i / -r: the MPI world as one process over several GPUs ----------------
def _world_env(ranks):
    """SHEEP_DEVICES lists device 0 `ranks` times: the world's ranks rehearsed on one GPU
    (device copies stand in for RCCL, which needs distinct devices)."""
    return dict(os.environ, SHEEP_DEVICES=",".join(["0"] * ranks))


def run_env(env, *args, check=True):
    p = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=120, env=env)
    if check:
        assert p.returncode == 0, p.stdout + p.stderr
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 3])
@pytest.mark.parametrize("name", ["hep", "edge"])
def test_graph2tree_world_ir(gpu_ctx, tmp_path, name, ranks):
    """mpirun -n P graph2tree G -s SEQ -o OUT -ir (graph2tree.cpp:134-218): rank 0 writes
    the all-reduced degree sequence and the merged tree, both equal to the serial ones."""
    dat = dat_path(name, tmp_path)
    seq, out = tmp_path / "w.seq", tmp_path / "w.tre"
    p = run_env(_world_env(ranks), os.path.join(BIN, "graph2tree"), dat, "-s", seq, "-o", out, "-i", "-r", "-f")
    assert filecmp.cmp(seq, os.path.join(GOLDEN, f"{name}.seq"), shallow=False)
    assert filecmp.cmp(out, os.path.join(GOLDEN, f"{name}.tre"), shallow=False)
    assert strip_timing(p.stdout) == open(os.path.join(GOLDEN, f"{name}.facts")).read()
    assert "Reduced in:" in p.stdout and "Mapped in:" in p.stdout


@pytest.mark.gpu
def test_graph2tree_world_i_partial_trees(gpu_ctx, tmp_path):
    """-i without -r: every rank saves its shard's tree as OUTrr r0.tre (graph2tree.cpp:
    144-149), the map-worker files; their merge is the whole tree."""
    import numpy as np
    import oracle
    from conftest import golden_seq, read_tre
    dat = dat_path("hep", tmp_path)
    out = tmp_path / "m"
    run_env(_world_env(3), os.path.join(BIN, "graph2tree"), dat, "-s", os.path.join(GOLDEN, "hep.seq"), "-o", out, "-i")
    r = golden_records("hep")
    seq = golden_seq("hep")
    for rank in range(3):
        _, p, w = read_tre(str(out) + f"{rank:02d}r0.tre")
        op, ow = oracle.build_tree(r["tail"], r["head"], seq, rank + 1, 3)
        assert np.array_equal(p, op) and np.array_equal(w, ow), rank


@pytest.mark.gpu
def test_graph2tree_world_fast_partition_path(gpu_ctx, tmp_path):
    """graph2tree G -s SEQ -o OUT -p K -ir (the "fast partition path", horizontal-dist.sh:
    30-37): parts broadcast (mpi_sync), every rank writes its shard's edges into
    OUT-wRRRR-pPPPP.  Per part, the union of the ranks' lines is the serial writer's."""
    dat = dat_path("hep", tmp_path)
    out = tmp_path / "P"
    p = run_env(_world_env(3), os.path.join(BIN, "graph2tree"), dat, "-s", os.path.join(GOLDEN, "hep.seq"), "-o", out,
                "-p", "4", "-i", "-r")
    assert p.returncode == 0
    for part in range(4):
        lines = []
        for rank in range(3):
            lines += open(f"{out}-w{rank:04d}-p{part:04d}").read().splitlines()
        want = open(os.path.join(GOLDEN, f"hep.k4.g{part:04d}")).read().splitlines()
        assert sorted(lines) == sorted(want), part


@pytest.mark.gpu
def test_graph2tree_world_prints_partition(gpu_ctx, tmp_path):
    """graph2tree G -p K -ir without -o: rank 0 prints Partition::print (graph2tree.cpp:214-215)."""
    import numpy as np
    import oracle
    from conftest import golden_seq, golden_tree
    dat = dat_path("hep", tmp_path)
    p = run_env(_world_env(2), os.path.join(BIN, "graph2tree"), dat, "-p", "4", "-i", "-r")
    gp, gw = golden_tree("hep")
    parts, info = oracle.partition(gp, gw, golden_seq("hep"), 4)
    want = (f"Actually created {info['created']} partitions.\n"
            f"First two partition sizes: {np.count_nonzero(parts == 0)} and {np.count_nonzero(parts == 1)}\n")
    assert strip_timing(p.stdout) == want


# ---- f3: the out-of-core map/reduce of scripts/horizontal-dist.sh on the drop-ins --------
@pytest.mark.gpu
@pytest.mark.parametrize("workers", [4, 5])
def test_horizontal_dist_flow(gpu_ctx, tmp_path, workers):
    """scripts/horizontal-dist.sh without MPI (sort-worker.sh -> map-worker.sh x W ->
    reduce-worker.sh rounds with REDUCTION=2 -> part-worker.sh), run with the drop-in
    binaries and the scripts' own file names: the final tree, TREEFAQS and partition_tree
    output equal the serial path on the file sequence (the oracle's)."""
    import oracle
    from conftest import golden_seq
    dat = dat_path("hep", tmp_path)
    prefix = str(tmp_path / "hep")
    seq_file = prefix + ".seq"
    run(os.path.join(BIN, "degree_sequence"), dat, seq_file + ".tmp")          # sort-worker.sh:22
    os.rename(seq_file + ".tmp", seq_file)
    for i in range(workers):                                                    # map-worker.sh:32-34
        out = f"{prefix}{i:02d}"
        run(os.path.join(BIN, "graph2tree"), dat, "-l", f"{i + 1}/{workers}", "-s", seq_file, "-o", out)
        os.rename(out, out + "r0.tre")
    step, step_size, w = 0, workers, (workers + 1) // 2                         # horizontal-dist.sh:47-60
    while step_size != 1:
        for i in range(w):                                                      # reduce-worker.sh:24-40
            inputs = [f"{prefix}{j:02d}r{step}.tre" for j in range(i, step_size, w)]
            outf = f"{prefix}{i:02d}r{step + 1}.tre"
            if len(inputs) == 1:
                os.rename(inputs[0], outf)
            else:
                run(os.path.join(BIN, "merge_trees"), *inputs, "-o", outf + ".tmp")
                os.rename(outf + ".tmp", outf)
        step, step_size, w = step + 1, w, (w + 1) // 2
    os.rename(f"{prefix}00r{step}.tre", prefix + ".tre")
    p = run(os.path.join(BIN, "partition_tree"), "-v", "-f", "-g", dat, seq_file, prefix + ".tre", 2, 4)  # part-worker.sh:25
    r = golden_records("hep")
    fseq = golden_seq("hep", "fileseq")
    op, ow = oracle.build_tree(r["tail"], r["head"], fseq)
    want = oracle.facts_text(op, ow)
    kids = oracle.Kids(op)
    for k in (2, 4):
        parts, info = oracle.partition(op, ow, fseq, k, kids=kids)
        import numpy as np
        want += (f"Actually created {info['created']} partitions.\n"
                 f"First two partition sizes: {np.count_nonzero(parts == 0)} and {np.count_nonzero(parts == 1)}\n")
        want += oracle.eval_text(oracle.evaluate(r["tail"], r["head"], fseq, parts), k)
    assert p.stdout == want


# ---- f4: .net (SNAP text) input ---------------------------------------------------------
def _write_net(path, rec, header=""):
    with open(path, "w") as f:
        f.write(header)
        for t, h in zip(rec["tail"], rec["head"]):
            f.write(f"{t}\t{h}\n")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hep", "edge"])
def test_net_input(gpu_ctx, tmp_path, name):
    """The same graph as SNAP text: graph2tree's tree equals the .dat one; degree_sequence
    follows SNAPReader (readerwriter.h:78-90: whitespace-separated pairs, no repeated last
    record), i.e. the oracle's 'net' file sequence; partition_tree -g on the .net graph
    prints the golden lines."""
    import numpy as np
    import oracle
    from conftest import golden_seq
    r = golden_records(name)
    net = str(tmp_path / f"{name}.net")
    _write_net(net, r)
    out = tmp_path / "t.tre"
    run(os.path.join(BIN, "graph2tree"), net, "-o", out)
    assert filecmp.cmp(out, os.path.join(GOLDEN, f"{name}.tre"), shallow=False)
    sq = tmp_path / "n.seq"
    run(os.path.join(BIN, "degree_sequence"), net, sq)
    assert np.array_equal(np.loadtxt(sq, dtype=np.uint32, ndmin=1), oracle.sequence(r["tail"], r["head"], "net"))
    p = run(os.path.join(BIN, "partition_tree"), "-v", "-f", "-g", net, os.path.join(GOLDEN, f"{name}.seq"),
            os.path.join(GOLDEN, f"{name}.tre"), *ks(name))
    assert p.stdout == open(os.path.join(GOLDEN, f"{name}.part.txt")).read()


@pytest.mark.gpu
def test_net_reader_stops_like_snapreader(gpu_ctx, tmp_path):
    """SNAPReader stops at the first pair that does not parse: degree_sequence over a file
    whose 100th line is garbage sees the first 99 records only.  (LLAMA's own text loader is
    un-vendored; graph2tree's loader skips '#' comment lines, parity unpinned.)"""
    import numpy as np
    import oracle
    r = golden_records("hep")
    net = str(tmp_path / "bad.net")
    with open(net, "w") as f:
        for i, (t, h) in enumerate(zip(r["tail"], r["head"])):
            f.write("x y\n" if i == 99 else f"{t} {h}\n")
    sq = tmp_path / "n.seq"
    run(os.path.join(BIN, "degree_sequence"), net, sq)
    assert np.array_equal(np.loadtxt(sq, dtype=np.uint32, ndmin=1),
                          oracle.sequence(r["tail"][:99], r["head"][:99], "net"))
    hdr = str(tmp_path / "hdr.net")
    _write_net(hdr, r, header="# Directed graph: hep\n# FromNodeId\tToNodeId\n")
    out = tmp_path / "t.tre"
    run(os.path.join(BIN, "graph2tree"), hdr, "-o", out)
    assert filecmp.cmp(out, os.path.join(GOLDEN, "hep.tre"), shallow=False)


@pytest.mark.gpu
def test_partition_tree_sequence_longer_than_tree(gpu_ctx, tmp_path):
    """partition_tree with a sequence longer than the tree: the reference's parts.at(i)
    throws std::out_of_range (partition.cpp:65) and the process aborts."""
    from conftest import golden_seq
    seq = golden_seq("edge")
    longer = tmp_path / "long.seq"
    open(longer, "w").write("".join(f"{v}\n" for v in list(seq) + [int(seq.max()) + 1]))
    p = run(os.path.join(BIN, "partition_tree"), longer, os.path.join(GOLDEN, "edge.tre"), 2, check=False)
    assert p.returncode == 134 and "out_of_range" in p.stderr
