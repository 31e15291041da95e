"""One rank of a joined sheep_group (test_gpu_parity.py::test_group_join_processes_match_
single_gpu): python group_worker.py RANK WORLD PORT OUTDIR.  Every rank generates the same
RMAT-16 graph on device 0, keeps its contiguous edge shard, and runs the world's
collective calls; ranks write what they hold to OUTDIR/rankR.npz.

python group_worker.py RANK WORLD PORT OUTDIR stall (test_group_join_rank_stalls): the last
rank joins and then takes no part; every other rank's first collective must fail within
SHEEP_JOIN_TIMEOUT, after which the world refuses every call."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import torch
    import sheep_amd
    d = sheep_amd.rmat(16, 16, 16)
    s1 = sheep_amd.degree_sequence(d)
    res = sheep_amd.partition(s1, sheep_amd.build_tree(d, s1), 32) if rank == 0 else None
    R = d.shape[0]
    shard = d[rank * R // world:(rank + 1) * R // world].contiguous()
    g = sheep_amd.Group.join(0, rank, world, "127.0.0.1", port, link="auto")
    print(f"rank {rank}: link={'rccl' if g.rccl else 'host'}", flush=True)
    if len(sys.argv) > 5 and sys.argv[5] == "stall":
        timeout = int(os.environ["SHEEP_JOIN_TIMEOUT"])
        if rank == world - 1:
            time.sleep(timeout + 4)   # alive, links open, never enters a collective
            g.close()
            return
        t0 = time.time()
        try:
            g.sequence([shard], 1 << 16)
            raise SystemExit("the collective returned although a rank never took part")
        except RuntimeError as e:
            print(f"rank {rank}: failed after {time.time() - t0:.2f} s: {e}", flush=True)
        assert g.failed
        t0 = time.time()
        try:
            g.barrier()
            raise SystemExit("a failed world accepted another collective")
        except RuntimeError as e:
            print(f"rank {rank}: refused after {time.time() - t0:.2f} s: {e}", flush=True)
        g.close()
        return
    seq = g.sequence([shard], 1 << 16)
    keep = {"seq": seq[0].numpy()}
    for mode in ("kway", "binomial"):
        tree = g.build_tree([shard], seq, mode)[0]
        p, w = sheep_amd.tree_to_numpy(tree)
        keep[f"parent_{mode}"], keep[f"pst_{mode}"] = p, w
    parts = res.parts.clone() if rank == 0 else torch.full((seq[0].pos_size,), 7, dtype=torch.int16, device="cuda")
    parts = g.broadcast_parts([parts], seq[0].pos_size)[0]
    keep["parts"] = parts.cpu().numpy()
    ev = g.evaluate([shard], seq, [parts])
    keep["ecv"] = np.array([ev.ecv_down, ev.max_down_bal, ev.edges_cut, ev.ecv_hash, ev.ecv_up], np.uint64)
    g.barrier()
    np.savez(os.path.join(out, f"rank{rank}.npz"), **keep)
    g.close()


if __name__ == "__main__":
    main()
