#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Runs in the build container only (it needs /root/reference and oracle/_ref, built by
`make ref`).  Every expected output here is produced by oracle/_ref — the reference's
lib/ (JTree, JNodeTable, Partition, sequence.h) and its degree_sequence / merge_trees
CLIs compiled from /root/reference — never by our restatement or by the GPU code.

Inputs:
  hep     data/hep-th.dat (the reference's own fixture; copied as input data)
  rmat10  / rmat12 / rmat14  our seeded RMAT generator (sheep_rmat_generate_host)
  edge    a hand-made multigraph with self-loops, duplicates, isolated slots and
          several components (LLAMA semantics: self-loop stored once)
Outputs per graph G (see MANIFEST.json for md5s):
  G.dat            input records (XS1, 12 B each)
  G.seq            ref_harness seq      (degreeSequence, LLAMA degrees)
  G.fileseq        degree_sequence CLI  (fileSequence: last record twice)
  G.tre            ref_harness tree     (JTree + save)
  G.facts          TREEFAQS printed by the reference
  G.h1.tre/G.h2.tre  partial trees over halves 1/2 and 2/2 (graph2tree -l semantics)
  G.merge.tre      merge_trees CLI over the two halves
  G.part.txt       partition_tree -f -g flow (TREEFAQS, per-k print + both evaluators)
  G.k<K>.parts     vid-indexed int16 parts per k (same run, so kid order persists)
  G.k<K>.g%04d     writePartitionedGraph(graph, seq, prefix) files (graph2tree -p K -o)
  G.k<K>.f%04d     writePartitionedGraph(filename, seq, prefix) files (partition_tree -o)
  G.print.txt, G.h1.print.txt, G.h2.print.txt
                   ref_harness print: JTree::print (graph2tree -t) of the whole tree and of
                   the halves' partial trees; committed for PRINT_FILES, md5 only (in
                   MANIFEST.json "_print") for the others

`make_golden.py --print` regenerates only the print fixtures (and their manifest entries).
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")
sys.path.insert(0, ROOT)

KS = {"hep": [2, 3, 4, 16, 64], "rmat10": [2, 16], "rmat12": [4, 16, 64], "rmat14": [16, 64], "edge": [1, 2, 3]}
# partition files (writePartitionedGraph): graph order (graph2tree -p -o) -> G.k<K>.g%04d,
# input-file order (partition_tree -g G -o) -> G.k<K>.f%04d
WRITE_K = {"hep": 4, "rmat10": 16, "edge": 2}
# graph2tree -t dumps: committed as files for these, md5 + line count only for the rest
PRINT_FILES = ("edge", "rmat10")
PRINT_GRAPHS = ("hep", "rmat10", "rmat12", "edge")


def run(*args, **kw):
    return subprocess.run([str(a) for a in args], check=True, capture_output=True, text=True, **kw).stdout


def write_dat(path, tail, head):
    rec = np.zeros(len(tail), dtype=[("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])
    rec["tail"], rec["head"], rec["weight"] = tail, head, 1.0
    rec.tofile(path)


def edge_graph():
    # self-loops (5,5) (9,9); duplicate (3,1) x3; slot 6 and 8 isolated; two components
    pairs = [(3, 1), (3, 1), (4, 3), (5, 5), (5, 2), (3, 1), (7, 4), (9, 9), (9, 7), (2, 0), (10, 0),
             (12, 11), (13, 12), (13, 11), (14, 14), (15, 13), (7, 5), (10, 7)]
    t = np.array([p[0] for p in pairs], np.uint32)
    h = np.array([p[1] for p in pairs], np.uint32)
    return t, h


def make_prints(manifest):
    """JTree::print of the whole tree and of the two halves' partial trees (graph2tree -t,
    -l 1/2 and 2/2 with the golden sequence)."""
    sys.path.insert(0, os.path.dirname(HERE))
    from conftest import golden_records   # the committed input, or the md5-checked regenerated one
    H = os.path.join(REF, "ref_harness")
    out = {}
    tmp = os.path.join(HERE, "_tmp_print")
    os.makedirs(tmp, exist_ok=True)
    for name in PRINT_GRAPHS:
        dat = os.path.join(HERE, f"{name}.dat")
        if not os.path.exists(dat):
            dat = os.path.join(tmp, f"{name}.dat")
            golden_records(name).tofile(dat)
        seq = os.path.join(HERE, f"{name}.seq")
        for tag, extra in (("print", ()), ("h1.print", ("1/2",)), ("h2.print", ("2/2",))):
            text = run(H, "print", dat, seq, *extra)
            fname = f"{name}.{tag}.txt"
            out[fname] = {"md5": hashlib.md5(text.encode()).hexdigest(), "lines": text.count("\n")}
            if name in PRINT_FILES:
                open(os.path.join(HERE, fname), "w").write(text)
    shutil.rmtree(tmp)
    manifest["_print"] = out


def main():
    if not os.path.exists(os.path.join(REF, "ref_harness")):
        sys.exit("build oracle/_ref first: make ref")
    if sys.argv[1:] == ["--print"]:
        path = os.path.join(HERE, "MANIFEST.json")
        manifest = json.load(open(path))
        make_prints(manifest)
        for f in sorted(os.listdir(HERE)):
            if f.endswith(".print.txt"):
                manifest[f] = hashlib.md5(open(os.path.join(HERE, f), "rb").read()).hexdigest()
        json.dump(manifest, open(path, "w"), indent=1, sort_keys=True)
        print(f"wrote {len(manifest['_print'])} print digests")
        return
    import sheep_amd
    graphs = {}
    hep = np.fromfile("/root/reference/data/hep-th.dat", dtype=[("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])
    graphs["hep"] = None   # copied verbatim below
    for name, scale, seed in (("rmat10", 10, 10), ("rmat12", 12, 12), ("rmat14", 14, 14)):
        r = sheep_amd.rmat_host(scale, 16, seed)
        graphs[name] = (r[:, 0], r[:, 1])
    graphs["edge"] = edge_graph()

    manifest = {}
    tmp = os.path.join(HERE, "_tmp")
    os.makedirs(tmp, exist_ok=True)
    for name, th in graphs.items():
        dat = os.path.join(HERE, f"{name}.dat")
        if th is None:
            shutil.copyfile("/root/reference/data/hep-th.dat", dat)
        else:
            write_dat(dat, *th)
        H = os.path.join(REF, "ref_harness")
        run(H, "seq", dat, os.path.join(HERE, f"{name}.seq"))
        run(os.path.join(REF, "degree_sequence"), dat, os.path.join(HERE, f"{name}.fileseq"))
        facts = run(H, "tree", dat, os.path.join(HERE, f"{name}.seq"), os.path.join(HERE, f"{name}.tre"))
        open(os.path.join(HERE, f"{name}.facts"), "w").write(facts)
        run(H, "tree", dat, os.path.join(HERE, f"{name}.seq"), os.path.join(HERE, f"{name}.h1.tre"), "1/2")
        run(H, "tree", dat, os.path.join(HERE, f"{name}.seq"), os.path.join(HERE, f"{name}.h2.tre"), "2/2")
        # merge_trees maps its inputs O_RDWR and rewrites their headers: work on copies
        a, b = os.path.join(tmp, "a.tre"), os.path.join(tmp, "b.tre")
        shutil.copyfile(os.path.join(HERE, f"{name}.h1.tre"), a)
        shutil.copyfile(os.path.join(HERE, f"{name}.h2.tre"), b)
        run(os.path.join(REF, "merge_trees"), a, b, "-o", os.path.join(HERE, f"{name}.merge.tre"))
        shutil.copyfile(os.path.join(HERE, f"{name}.tre"), a)
        out = run(H, "part", dat, os.path.join(HERE, f"{name}.seq"), a, os.path.join(HERE, f"{name}."),
                  *KS[name])
        open(os.path.join(HERE, f"{name}.part.txt"), "w").write(out)
        if name in WRITE_K:
            k = WRITE_K[name]
            for cmd, tag in (("write", "g"), ("writefile", "f")):
                shutil.copyfile(os.path.join(HERE, f"{name}.tre"), a)
                run(H, cmd, dat, os.path.join(HERE, f"{name}.seq"), a, k, os.path.join(HERE, f"{name}.k{k}.{tag}"))
    shutil.rmtree(tmp)
    for f in sorted(os.listdir(HERE)):
        if f.endswith((".py", ".json")) or f.startswith("_"):
            continue
        manifest[f] = hashlib.md5(open(os.path.join(HERE, f), "rb").read()).hexdigest()
    # rmat12/rmat14 inputs are regenerated by the tests from the generator (md5-checked
    # against this manifest) instead of being committed
    for big in ("rmat12.dat", "rmat14.dat"):
        os.remove(os.path.join(HERE, big))
    make_prints(manifest)
    manifest["_ks"] = KS
    manifest["_write_k"] = WRITE_K
    manifest["_rmat"] = {"rmat10": [10, 16, 10], "rmat12": [12, 16, 12], "rmat14": [14, 16, 14]}
    json.dump(manifest, open(os.path.join(HERE, "MANIFEST.json"), "w"), indent=1, sort_keys=True)
    print(f"wrote {len(manifest)} entries")


if __name__ == "__main__":
    main()
