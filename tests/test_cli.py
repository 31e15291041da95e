"""The drop-in CLIs (sheep_amd/cli/*.cpp over libsheep_hip.so) against the reference's
golden outputs: same files byte for byte, same stdout lines (timing lines aside)."""
import filecmp
import os
import shutil
import socket
import subprocess

import pytest

from conftest import GOLDEN, ROOT, check_print, golden_records, ks, manifest

BIN = os.environ.get("SHEEP_BIN_DIR") or os.path.join(ROOT, "sheep_amd", "bin")   # (make asan: sheep_amd/bin/asan)
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
@pytest.mark.parametrize("name", ["hep", "rmat10", "rmat12", "edge"])
def test_graph2tree_print(gpu_ctx, tmp_path, name):
    """graph2tree G -f -t (graph2tree.cpp:107-108, 227-230): TREEFAQS, then JTree::print
    (jtree.h:60-66) of every node, byte-exact with the reference's print; and the partial
    trees of -l 1/2 and 2/2 with the sequence file."""
    dat = dat_path(name, tmp_path)
    p = run(os.path.join(BIN, "graph2tree"), dat, "-f", "-t")
    facts = open(os.path.join(GOLDEN, f"{name}.facts")).read()
    text = strip_timing(p.stdout)
    assert text.startswith(facts)
    check_print(text[len(facts):], name, "print")
    for part, tag in ((1, "h1.print"), (2, "h2.print")):
        p = run(os.path.join(BIN, "graph2tree"), dat, "-l", f"{part}/2", "-s", os.path.join(GOLDEN, f"{name}.seq"), "-t")
        check_print(strip_timing(p.stdout), name, tag)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hep", "rmat12", "edge"])
def test_partition_tree_cli(gpu_ctx, tmp_path, name):
    """partition_tree -v -f -g G SEQ TREE k1 k2 ... (-v turns the timing lines off):
    TREEFAQS + per-k print + both evaluators, byte-exact with the reference's run."""
    dat = dat_path(name, tmp_path)
    p = run(os.path.join(BIN, "partition_tree"), "-v", "-f", "-g", dat, os.path.join(GOLDEN, f"{name}.seq"),
            os.path.join(GOLDEN, f"{name}.tre"), *ks(name))
    assert p.stdout == open(os.path.join(GOLDEN, f"{name}.part.txt")).read()


# ---- graph2tree -i / -r: the MPI world over several GPUs ---------------------------------
# Two launches (sheep/world.hpp): "devices" — ONE process drives the ranks listed in
# SHEEP_DEVICES (device 0 listed `ranks` times: device copies stand in for RCCL, which needs
# distinct devices); "mpiexec" — the reference's own launch, `mpiexec -n P graph2tree ...`,
# one process per rank (they share device 0, so the host link over TCP carries the data).
MPIEXEC = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
LAUNCHES = ["devices", "mpiexec"]


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def seq_copy(tmp_path, name="hep"):
    """A copy of the golden sequence: with -i, rank 0 WRITES the all-reduced sequence to
    the -s file (graph2tree.cpp:174-175)."""
    dst = tmp_path / f"{name}.in.seq"
    shutil.copy(os.path.join(GOLDEN, f"{name}.seq"), dst)
    return dst


def world_run(launch, ranks, *args, check=True):
    env = dict(os.environ)
    for k in ("SHEEP_DEVICES", "RANK", "WORLD_SIZE", "LOCAL_RANK", "PMI_RANK", "PMI_SIZE"):
        env.pop(k, None)
    if launch == "devices":
        env["SHEEP_DEVICES"] = ",".join(["0"] * ranks)
        cmd = [os.path.join(BIN, "graph2tree"), *args]
    else:
        if not MPIEXEC:
            pytest.skip("no mpiexec on this host")
        env["SHEEP_MASTER_PORT"] = str(_free_port())
        cmd = [MPIEXEC, "-n", str(ranks), os.path.join(BIN, "graph2tree"), *args]
    p = subprocess.run([str(a) for a in cmd], capture_output=True, text=True, timeout=180, env=env)
    if check:
        assert p.returncode == 0, p.stdout + p.stderr
    return p


def test_graph2tree_single_rank_without_launcher(tmp_path):
    """No SHEEP_DEVICES and no launcher: `graph2tree -i` is a world of ONE rank, as an MPI
    program started without mpiexec (MPI_Comm_size 1), whatever the number of GPUs."""
    import sys
    sys.path.insert(0, ROOT)
    src = open(os.path.join(ROOT, "sheep_amd", "include", "sheep", "world.hpp")).read()
    assert "if (devs.empty()) devs.push_back(0);" in src


@pytest.mark.gpu
@pytest.mark.parametrize("launch", LAUNCHES)
@pytest.mark.parametrize("ranks", [2, 3])
@pytest.mark.parametrize("name", ["hep", "edge"])
def test_graph2tree_world_ir(gpu_ctx, tmp_path, name, ranks, launch):
    """mpirun -n P graph2tree G -s SEQ -o OUT -ir -f (graph2tree.cpp:134-218): rank 0 writes
    the all-reduced degree sequence and the merged tree, both equal to the serial ones, and
    prints the merged tree's TREEFAQS (under mpiexec every rank prints its own tree's)."""
    dat = dat_path(name, tmp_path)
    seq, out = tmp_path / "w.seq", tmp_path / "w.tre"
    p = world_run(launch, ranks, dat, "-s", seq, "-o", out, "-i", "-r", "-f")
    assert filecmp.cmp(seq, os.path.join(GOLDEN, f"{name}.seq"), shallow=False)
    assert filecmp.cmp(out, os.path.join(GOLDEN, f"{name}.tre"), shallow=False)
    facts = open(os.path.join(GOLDEN, f"{name}.facts")).read()
    if launch == "devices":   # the ranks print one after another, rank 0 (the merged tree) first
        assert strip_timing(p.stdout).startswith(facts)
    else:
        assert facts in strip_timing(p.stdout)
    assert strip_timing(p.stdout).count("TREEFAQS") == ranks
    assert p.stdout.count("Reduced in:") == 1 and p.stdout.count("Mapped in:") == 1


def _print_blocks(text, name, tags):
    """Split a world's -t output into one block per rank (each the tree's line count)."""
    lines = text.splitlines(keepends=True)
    blocks, at = [], 0
    for tag in tags:
        n = manifest()["_print"][f"{name}.{tag}.txt"]["lines"]
        blocks.append("".join(lines[at:at + n]))
        at += n
    assert at == len(lines)
    return blocks


@pytest.mark.gpu
@pytest.mark.parametrize("name,launch", [("edge", "devices"), ("edge", "mpiexec"), ("rmat10", "devices"),
                                         ("hep", "devices")])
def test_graph2tree_world_print(gpu_ctx, tmp_path, name, launch):
    """graph2tree G -s SEQ -ir -t over 2 ranks: tree.print() is not leader-gated
    (graph2tree.cpp:229-230), so rank 0 prints the merged tree (== the whole graph's) and
    rank 1 its own shard's partial tree (mpi_merge leaves the senders' nodes as they were,
    jnode.cpp:241); with -i alone both ranks print their partial trees (-l 1/2, 2/2)."""
    dat = dat_path(name, tmp_path)
    for flags, tags in ((("-i", "-r"), ("print", "h2.print")), (("-i",), ("h1.print", "h2.print"))):
        p = world_run(launch, 2, dat, "-s", seq_copy(tmp_path, name), *flags, "-t")
        text = strip_timing(p.stdout)
        if launch == "mpiexec":   # two processes: either may flush first (each < one pipe write)
            first = manifest()["_print"][f"{name}.{tags[0]}.txt"]["md5"]
            import hashlib
            head = "".join(text.splitlines(keepends=True)[:manifest()["_print"][f"{name}.{tags[0]}.txt"]["lines"]])
            if hashlib.md5(head.encode()).hexdigest() != first:
                tags = tags[::-1]
        for block, tag in zip(_print_blocks(text, name, tags), tags):
            check_print(block, name, tag)


@pytest.mark.gpu
@pytest.mark.parametrize("launch", LAUNCHES)
def test_graph2tree_world_i_partial_trees(gpu_ctx, tmp_path, launch):
    """-i without -r: every rank saves its shard's tree as OUTrr r0.tre (graph2tree.cpp:
    144-149), the map-worker files; their merge is the whole tree."""
    import numpy as np
    import oracle
    from conftest import golden_seq, read_tre
    dat = dat_path("hep", tmp_path)
    out = tmp_path / "m"
    world_run(launch, 3, dat, "-s", seq_copy(tmp_path), "-o", out, "-i")
    r = golden_records("hep")
    seq = golden_seq("hep")
    for rank in range(3):
        _, p, w = read_tre(str(out) + f"{rank:02d}r0.tre")
        op, ow = oracle.build_tree(r["tail"], r["head"], seq, rank + 1, 3)
        assert np.array_equal(p, op) and np.array_equal(w, ow), rank


@pytest.mark.gpu
@pytest.mark.parametrize("launch", LAUNCHES)
def test_graph2tree_world_i_partitions_each_partial_tree(gpu_ctx, tmp_path, launch):
    """-i -p K without -r (graph2tree.cpp:144-149, 203-213): every rank partitions ITS
    partial tree and writes its shard's edges under OUTrr r0.tre%04d; rank 0 alone prints
    when there is no -o."""
    import numpy as np
    import oracle
    from conftest import golden_seq
    dat = dat_path("hep", tmp_path)
    out = tmp_path / "q"
    r = golden_records("hep")
    seq = golden_seq("hep")
    world_run(launch, 2, dat, "-s", seq_copy(tmp_path), "-o", out, "-p", "4", "-i")
    R = len(r)
    pos = np.full(int(seq.max()) + 1, -1, np.int64)
    pos[seq] = np.arange(len(seq))
    for rank in range(2):
        op, ow = oracle.build_tree(r["tail"], r["head"], seq, rank + 1, 2)
        parts, info = oracle.partition(op, ow, seq, 4)
        want = {}
        for t, h in zip(r["tail"][rank * R // 2:(rank + 1) * R // 2], r["head"][rank * R // 2:(rank + 1) * R // 2]):
            x, y = min(t, h), max(t, h)
            if x == y:
                continue
            owner = x if pos[x] < pos[y] else y
            want.setdefault(int(parts[owner]), []).append(f"{x} {y}")
        for part in range(info["created"]):
            got = open(f"{out}{rank:02d}r0.tre{part:04d}").read().splitlines()
            assert sorted(got) == sorted(want.get(part, [])), (rank, part)
    p = world_run(launch, 2, dat, "-s", seq_copy(tmp_path), "-p", "4", "-i")
    op, ow = oracle.build_tree(r["tail"], r["head"], seq, 1, 2)
    parts, info = oracle.partition(op, ow, seq, 4)
    assert strip_timing(p.stdout) == (f"Actually created {info['created']} partitions.\n"
                                      f"First two partition sizes: {np.count_nonzero(parts == 0)} and "
                                      f"{np.count_nonzero(parts == 1)}\n")


@pytest.mark.gpu
@pytest.mark.parametrize("launch", LAUNCHES)
def test_graph2tree_world_fast_partition_path(gpu_ctx, tmp_path, launch):
    """graph2tree G -s SEQ -o OUT -p K -ir (the "fast partition path", horizontal-dist.sh:
    30-37): parts broadcast (mpi_sync), every rank writes its shard's edges into
    OUT-wRRRR-pPPPP.  Per part, the union of the ranks' lines is the serial writer's."""
    dat = dat_path("hep", tmp_path)
    out = tmp_path / "P"
    world_run(launch, 3, dat, "-s", seq_copy(tmp_path), "-o", out, "-p", "4", "-i", "-r")
    for part in range(4):
        lines = []
        for rank in range(3):
            lines += open(f"{out}-w{rank:04d}-p{part:04d}").read().splitlines()
        want = open(os.path.join(GOLDEN, f"hep.k4.g{part:04d}")).read().splitlines()
        assert sorted(lines) == sorted(want), part


@pytest.mark.gpu
@pytest.mark.parametrize("launch", LAUNCHES)
def test_graph2tree_world_prints_partition(gpu_ctx, tmp_path, launch):
    """graph2tree G -p K -ir without -o: rank 0 prints Partition::print (graph2tree.cpp:214-215)."""
    import numpy as np
    import oracle
    from conftest import golden_seq, golden_tree
    dat = dat_path("hep", tmp_path)
    p = world_run(launch, 2, dat, "-p", "4", "-i", "-r")
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
