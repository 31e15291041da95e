/*
 * sheep_hip.h — C ABI of libsheep_hip.so, the MI355X (gfx950) implementation of Sheep's
 * map/reduce partitioning path:
 *
 *   degree sequence -> relabel -> per-shard elimination tree (map) -> tree merge
 *   (reduce) -> partition_tree downward assignment + ECV(down)/balance evaluator.
 *
 * Plain pointers and sizes only.  "_dev" pointers are device (HBM) pointers on the
 * context's device; every call is asynchronous on the context's stream unless it
 * returns a host-side value (documented per call), in which case it synchronises.
 *
 * Every entry point returns SHEEP_OK (0) or a negative status; sheep_last_error()
 * returns the message of the calling thread's last failure.  The reference throws
 * (std::bad_alloc / std::out_of_range) or asserts in the corresponding places; the
 * façade in sheep_amd/include/sheep/sheep.hpp maps these codes back to the same
 * behaviour.
 *
 * Reference interfaces replaced (chan150/sheep, file:line):
 *   sheep_degree_count            sequence.h:65-78  (mpiSequence local degrees; LLAMA
 *                                 out_degree, graph_wrapper.h:87-89) and
 *                                 sequence.h:95-107 (fileSequence degree loop)
 *   sheep_sequence_from_degrees   sequence.h:80-92 / :109-121 (compact + (deg,vid) sort)
 *   sheep_positions               jtree.h:113,142-143 (vid -> jnid index)
 *   sheep_build_tree              jtree.h:111-122 + jtree.cpp:66-145 (JTree map step)
 *   sheep_merge_trees             jnode.cpp:174-201 (JNodeTable::merge) and the
 *                                 per-hop op of mpi_merge, jnode.cpp:203-250
 *   sheep_kids_create/_destroy    jnode.h:190-204 (makeKids; the persistent kid table)
 *   sheep_partition               partition.cpp:50-67 + :86-157 (Partition ctor,
 *                                 forwardPartition) and partition.h:135-143 (print counts)
 *   sheep_evaluate                partition.cpp:428-473 + :475-521 (both evaluators)
 *   sheep_facts                   jnode.cpp:256-290 (JNodeTable::Facts)
 *   sheep_rmat_generate           (new) synthetic Graph500-style RMAT .dat records
 */
#ifndef SHEEP_HIP_H
#define SHEEP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version: raised whenever a public struct changes size or layout or an entry point its
 * signature (INTEGRATION.md "ABI versions" lists the changes).  sheep_abi_version() returns the
 * library's; a caller built against another header should refuse to run. */
#define SHEEP_ABI_VERSION 6
int sheep_abi_version(void);

#define SHEEP_OK 0
#define SHEEP_ERR_ARG (-1)     /* bad argument (null pointer, size mismatch)          */
#define SHEEP_ERR_HIP (-2)     /* HIP runtime error (no device, launch failure, ...)  */
#define SHEEP_ERR_RANGE (-3)   /* reference would throw std::out_of_range (.at())    */
#define SHEEP_ERR_PACK (-4)    /* forwardPartition would never terminate             */
#define SHEEP_ERR_ALLOC (-5)   /* device allocation failed (reference: bad_alloc)     */

#define SHEEP_INVALID_ID 0xFFFFFFFFu /* INVALID_VID / INVALID_JNID, defs.h:82 jnode.h:43 */
#define SHEEP_INVALID_PART ((int16_t)-1) /* INVALID_PART, partition.h:44 */

/* .dat record, 12 bytes: struct xs1 (readerwriter.h:36-40). */
typedef struct {
  uint32_t tail;
  uint32_t head;
  float weight;
} sheep_xs1;

/* One tree node, 8 bytes: JNodeTable::JNode (jnode.h:56-69); .tre = u32 end_id + these. */
typedef struct {
  uint32_t parent;
  uint32_t pst_weight;
} sheep_jnode;

/* Degree-count semantics. */
enum {
  SHEEP_DEGREE_LLAMA = 0,    /* LLAMA out_degree: self-loop counted once            */
  SHEEP_DEGREE_FILE_DAT = 1, /* fileSequence over XS1: +1 per endpoint, self-loop +2,
                                last record counted twice (readerwriter.h:138-146)  */
  SHEEP_DEGREE_FILE_NET = 2  /* fileSequence over SNAP text: +1 per endpoint         */
};

typedef struct sheep_ctx sheep_ctx;
typedef struct sheep_kids sheep_kids;

typedef struct {
  int32_t created;          /* max part + 1 ("Actually created %d partitions.")     */
  uint64_t first_size;      /* count of part 0 over the vid-indexed vector          */
  uint64_t second_size;     /* count of part 1                                      */
  uint64_t max_component;   /* (size_t)((total / k) * balance)                      */
  uint64_t total_weight;
  uint64_t packing_nodes;   /* nodes where first-fit-decreasing packing ran         */
  uint64_t heavy_nodes;     /* |{v : subtree weight > max_component}|               */
  uint64_t event_launches;  /* packing-event kernel launches (sheep_tuning event_loop) */
} sheep_partition_info;

typedef struct {
  uint64_t edges_cut, vcom_vol, max_vertex_bal, ecv_hash, max_hash_bal;
  uint64_t ecv_down, max_down_bal, ecv_up, max_up_bal;
  uint64_t edges;  /* getEdges() = adjacency entries / 2 (graph_wrapper.h:79-81) */
  uint64_t nodes;  /* getNodes() = slots with degree != 0                       */
} sheep_eval;

typedef struct {
  uint64_t width, root_cnt, vert_height, edge_height, vert_cnt, edge_cnt, halo_id, core_id, fill;
} sheep_facts_t;

/* ---- context ------------------------------------------------------------------- */
const char *sheep_last_error(void);
/* Every call of the context is issued on `hip_stream` as given — NULL is the device's
 * null stream (PyTorch's default stream), so callers that share buffers with other
 * work order it simply by passing the stream that work runs on.  SHEEP_OWN_STREAM makes
 * the context create (and destroy) a non-blocking stream of its own. */
#define SHEEP_OWN_STREAM ((void *)(intptr_t)-1)
int sheep_ctx_create(int device, void *hip_stream, sheep_ctx **out);
int sheep_ctx_destroy(sheep_ctx *ctx);
/* Frees the context's device workspace (the scratch arrays kernels keep between calls,
 * sized by the largest graph seen, and the spare kid-table buffers); the next call
 * allocates again.  Synchronises the context's stream. */
int sheep_ctx_trim(sheep_ctx *ctx);
/* The context's device workspaces as "name=bytes" pairs, comma-separated, largest first,
 * into buf[cap] (what sheep_ctx_trim would free; for memory reports). */
int sheep_ctx_workspace(sheep_ctx *ctx, char *buf, size_t cap);
int sheep_ctx_sync(sheep_ctx *ctx);
void *sheep_ctx_stream(sheep_ctx *ctx);
int sheep_malloc(sheep_ctx *ctx, size_t bytes, void **dev_out);
int sheep_free(sheep_ctx *ctx, void *dev);
int sheep_memcpy_h2d(sheep_ctx *ctx, void *dst_dev, const void *src_host, size_t bytes);
int sheep_memcpy_d2h(sheep_ctx *ctx, void *dst_host, const void *src_dev, size_t bytes);
/* device to device on the context's stream (asynchronous) */
int sheep_memcpy_d2d(sheep_ctx *ctx, void *dst_dev, const void *src_dev, size_t bytes);
/* Device-side timing per instrumented region (HIP events on the context stream; see
 * DESIGN.md §Measurement): name = "degree" | "relabel" | "etree" | ...; returns the
 * accumulated ms, launch count and algorithmic bytes since the last reset. */
int sheep_timer_enable(sheep_ctx *ctx, int on);
int sheep_timer_get(sheep_ctx *ctx, const char *name, double *ms, uint64_t *launches,
                    uint64_t *alg_bytes);
int sheep_timer_reset(sheep_ctx *ctx);
/* Names of every region timed since the last reset, comma-separated, into buf[cap]. */
int sheep_timer_names(sheep_ctx *ctx, char *buf, size_t cap);

/* ---- tuning -----------------------------------------------------------------------
 * The algorithm's variants, one options struct per context (no reference analogue: the
 * reference has one sequential algorithm).  Every variant computes the same bit-exact
 * result; only time and device memory differ.  The defaults are the measured best
 * (DESIGN.md §3); A/B runs (bench.py --tune) and the branch-forcing parity tests set the
 * others.  A field equal to SHEEP_TUNE_DEFAULT keeps its default.  sheep_ctx_set_tuning
 * checks every field's range (SHEEP_ERR_ARG) and NULL restores the defaults. */
#define SHEEP_TUNE_DEFAULT (-1)
typedef struct sheep_tuning {
  int32_t fin_map_bits;    /* map: levels below this many position bits finish per block, 8..13 */
  int32_t fin_merge_bits;  /* merge: the same, 8..13 */
  int32_t fin_dc;          /* 1: per-block divide and conquer (k_fin_dc), 0: Liu's sweep per block */
  int32_t top_bits;        /* dense top-block MSF cut: 0 off, else its size in position bits, 9..16 */
  int32_t top_blocks;      /* blocks cut there (the top one included), 1..9 */
  int32_t big_bits;        /* early MSF cut of the top subproblem: 0 off, else 17..30 position bits */
  int64_t big_dense;       /* the early cut needs >= this many group edges per vertex, >= 1 */
  int32_t big_hot_bits;    /* early cut: LDS window of picks, 10..15 position bits */
  int32_t big_hot16;       /* early cut: 1 = u16-distance window over 2^16 positions */
  int32_t relabel_planes;  /* relabel scatter: 1 = stage pairs as two u32 planes, 0 = one u64 array */
  int32_t relabel_per;     /* relabel scatter: records per thread per staged sub-tile, 4, 8, 12 or 15 */
  int32_t cross_win_levels;/* etree: levels (from the first) whose cross pass keeps minima in an LDS window, 0..8
                            * (maps too sparse for the early cut: one more) */
  int32_t hook_batch;      /* etree hook rounds find all of a thread's roots at once: 0 never, 1 merges, 2 all */
  int32_t merge_cut_bits;  /* merges: the early MSF cut of the top 2^bits positions, whatever the density: 0 off, 14..30 */
  int32_t event_loop;      /* partition packing events: 0 one launch per event, else one persistent launch while the
                              event table fits this many entries (in LDS), 1..4096 */
  int32_t hook_up;         /* etree hook rounds hook the smaller root under the larger (root = top, no light-top
                              pass): 0 never, 1 merges, 2 all */
} sheep_tuning;
int sheep_tuning_default(sheep_tuning *out);
int sheep_ctx_set_tuning(sheep_ctx *ctx, const sheep_tuning *t);
int sheep_ctx_get_tuning(sheep_ctx *ctx, sheep_tuning *out);

/* ---- degree sequence --------------------------------------------------------------
 * Adds this shard's degrees into deg_dev[0, deg_cap) (caller zeroes it once; shards
 * accumulate, or are summed with an all-reduce).  *max_slot_out (host, synchronises)
 * = 1 + max vid seen (LLAMA max_nodes()).  Fails with SHEEP_ERR_RANGE if a vid >= deg_cap. */
int sheep_degree_count(sheep_ctx *ctx, const sheep_xs1 *rec_dev, uint64_t nrec, int mode,
                       uint32_t *deg_dev, uint64_t deg_cap, uint64_t *max_slot_out);

/* seq_dev[0,n) = slots with deg != 0 sorted by (degree, vid); pos_dev[0, vs) = jnid of
 * each slot or SHEEP_INVALID_ID.  *n_out (host, synchronises). */
int sheep_sequence_from_degrees(sheep_ctx *ctx, const uint32_t *deg_dev, uint64_t vs,
                                uint32_t *seq_dev, uint32_t *pos_dev, uint64_t *n_out);

/* pos_dev[0, pos_size) from an arbitrary sequence (readSequence path); pos_size must be
 * max(seq)+1.  Duplicate vids: SHEEP_ERR_ARG (the reference asserts, jtree.h:166). */
int sheep_positions(sheep_ctx *ctx, const uint32_t *seq_dev, uint64_t n, uint32_t *pos_dev,
                    uint64_t pos_size);

/* ---- map: per-shard elimination tree ---------------------------------------------
 * tree_dev[0,n): Liu's elimination tree of this shard's records under the order pos
 * (parent INVALID = root) and pst_weight = #later neighbours.  Records whose endpoint
 * is >= pos_size while the other endpoint is sequenced -> SHEEP_ERR_RANGE
 * (jtree.cpp:75 index.at).  When the context's last sheep_degree_count (LLAMA mode) saw
 * the same rec_dev/nrec with max_slot == pos_size, its head-bucket layout is reused for
 * the relabel; records changed in place since are detected on the device and recounted,
 * so reuse never changes the result. */
int sheep_build_tree(sheep_ctx *ctx, const sheep_xs1 *rec_dev, uint64_t nrec,
                     const uint32_t *pos_dev, uint64_t pos_size, uint64_t n,
                     sheep_jnode *tree_dev);

/* ---- reduce: merge two trees over the same n ------------------------------------ */
int sheep_merge_trees(sheep_ctx *ctx, const sheep_jnode *a_dev, const sheep_jnode *b_dev,
                      uint64_t n, sheep_jnode *out_dev);
/* k trees over the same n, stored one after another (trees_dev[j * n + i]): the whole
 * reduction mpi_merge performs over k ranks (jnode.cpp:203-250, MPI_Reduce with
 * mpi_merge_reduction) in one pass — the elimination tree of the union of all k
 * parent-edge sets, pst summed.  Equal to any order of k - 1 sheep_merge_trees calls. */
int sheep_merge_trees_many(sheep_ctx *ctx, const sheep_jnode *trees_dev, uint32_t k,
                           uint64_t n, sheep_jnode *out_dev);
/* The same merge split over nparts = 2^l GPUs (the log-depth reduce of mpi_merge,
 * jnode.cpp:203-250, without its serial tail): every part runs the first l levels of the
 * merge over all k trees, then only its own subproblem.  out_dev holds every node's pst
 * and a correct parent for every node in [*v_lo, *v_hi); the nparts ranges tile [0, n),
 * so the parts' slices together are sheep_merge_trees_many's tree.  k <= 64. */
int sheep_merge_trees_part(sheep_ctx *ctx, const sheep_jnode *trees_dev, uint32_t k,
                           uint64_t n, uint32_t part, uint32_t nparts, sheep_jnode *out_dev,
                           uint64_t *v_lo, uint64_t *v_hi);

/* ---- partition ------------------------------------------------------------------ */
int sheep_kids_create(sheep_ctx *ctx, const sheep_jnode *tree_dev, uint64_t n,
                      sheep_kids **out);
/* The context keeps a destroyed table's device buffers (3 x 4 B x n) for the next
   sheep_kids_create on it, or frees them in sheep_ctx_destroy; the context must outlive
   its kid tables. */
int sheep_kids_destroy(sheep_kids *kids);
/* parts_vid_dev[0, pos_size) (pos_size = max(seq)+1) receives the vid-indexed parts
 * (SHEEP_INVALID_PART for unsequenced slots): parts of jnids 0 .. seq_n-1 go to
 * seq[0 .. seq_n-1] (partition.cpp:62-66).  seq_n > n fails with SHEEP_ERR_RANGE, the
 * reference's parts.at(i) throw; a shorter sequence converts only its own entries.
 * info->created / first_size / second_size are counted over the vid-indexed vector
 * (partition.h:135-143).  info is host (synchronises). */
int sheep_partition(sheep_ctx *ctx, const sheep_jnode *tree_dev, uint64_t n,
                    const uint32_t *seq_dev, uint64_t seq_n, uint64_t pos_size, sheep_kids *kids, int16_t k,
                    double balance, int vtx_weight, int pst_weight, int16_t *parts_vid_dev,
                    sheep_partition_info *info);
/* The same with the sequence's vid -> jnid index pos_dev[0, pos_size) (sheep_positions /
 * sheep_sequence_from_degrees; pos[seq[j]] = j, SHEEP_INVALID_ID elsewhere): the parts
 * reach their vid slots by one streaming gather over pos instead of a scattered 2-B store
 * per jnid.  Same results as sheep_partition for the same sequence. */
int sheep_partition_pos(sheep_ctx *ctx, const sheep_jnode *tree_dev, uint64_t n,
                        const uint32_t *seq_dev, uint64_t seq_n, const uint32_t *pos_dev, uint64_t pos_size,
                        sheep_kids *kids, int16_t k, double balance, int vtx_weight, int pst_weight,
                        int16_t *parts_vid_dev, sheep_partition_info *info);

/* ---- evaluators: both partition.cpp evaluators over one graph (all records) -------
 * what: bitmask SHEEP_EVAL_GRAPH (edges cut, Vcom vol, vertex balance, ECV(hash) +
 * balance), SHEEP_EVAL_DOWN (ECV(down) + balance), SHEEP_EVAL_UP; 0 = all.
 * Ratios are printed by the caller from these counts and getEdges()/getNodes(). */
#define SHEEP_EVAL_GRAPH 1
#define SHEEP_EVAL_DOWN 2
#define SHEEP_EVAL_UP 4
int sheep_evaluate(sheep_ctx *ctx, const sheep_xs1 *rec_dev, uint64_t nrec,
                   const uint32_t *pos_dev, uint64_t pos_size, const int16_t *parts_vid_dev,
                   int what, sheep_eval *out);
/* The same counts from the position-space edges the context's last map
 * (sheep_build_tree over rec_dev[0, nrec) with this sequence: seq_dev[0, seq_n) and its
 * index pos_dev[0, pos_size)) left grouped in HBM: no pass over the records unless they
 * hold self-loops, and the random side of every edge reads jnid-indexed state (parts: 2 B
 * per node, owner bits: 8 B per node per metric for k <= 64) instead of vid-indexed rows.
 * SHEEP_ERR_ARG when the context's last map ran on other records or another index (or the
 * context was trimmed since), or when seq_dev is not the sequence pos_dev indexes
 * (pos[seq[j]] != j, checked on the device); the records must be unchanged since that map.
 * An edge endpoint without a part is SHEEP_ERR_RANGE, as in sheep_evaluate; a sequenced
 * vertex that is no endpoint may have none. */
int sheep_evaluate_step(sheep_ctx *ctx, const sheep_xs1 *rec_dev, uint64_t nrec,
                        const uint32_t *seq_dev, uint64_t seq_n, const uint32_t *pos_dev, uint64_t pos_size,
                        const int16_t *parts_vid_dev, int what, sheep_eval *out);
/* The same evaluators over edge shards (the records of one graph
 * split over devices or passes):
 *   sheep_eval_sizes      u64 words of the bitset and accumulator state for (what,
 *                         nparts, pos_size); nparts = max part + 1
 *                         (sheep_eval_num_parts).  The bitset state holds one row per
 *                         vertex slot: (pos << 16 | part), then the owner bit words;
 *                         every shard writes the same row heads, so OR-combining keeps them;
 *   sheep_eval_shard      ORs one shard's owner bits into bits_dev and adds its counts into
 *                         acc_dev (both zeroed by the caller before the first shard);
 *   sheep_eval_combine    bits_dev |= bits_src, acc_dev += acc_src (state of another
 *                         device's shards, copied over: the reduction step);
 *   sheep_eval_finish     the per-vertex pass over the combined state and the result
 *                         (host, synchronises).
 * shard + finish over all records == sheep_evaluate. */
int sheep_eval_sizes(int what, int32_t nparts, uint64_t pos_size, uint64_t *bits_words, uint64_t *acc_words);
int sheep_eval_num_parts(sheep_ctx *ctx, const int16_t *parts_vid_dev, uint64_t pos_size, int32_t *nparts_out);
int sheep_eval_shard(sheep_ctx *ctx, const sheep_xs1 *rec_dev, uint64_t nrec, const uint32_t *pos_dev,
                     uint64_t pos_size, const int16_t *parts_vid_dev, int what, int32_t nparts,
                     uint64_t *bits_dev, uint64_t *acc_dev);
int sheep_eval_combine(sheep_ctx *ctx, uint64_t *bits_dev, const uint64_t *bits_src_dev, uint64_t bits_words,
                       uint64_t *acc_dev, const uint64_t *acc_src_dev, uint64_t acc_words);
int sheep_eval_finish(sheep_ctx *ctx, const uint64_t *bits_dev, const uint64_t *acc_dev, uint64_t pos_size,
                      const int16_t *parts_vid_dev, int what, int32_t nparts, sheep_eval *out);

/* ---- partition files ----------------------------------------------------------------
 * edge_part_dev[i] = the part record i is written to by writePartitionedGraph
 * (partition.cpp:588-670): the part of its earlier-positioned endpoint.  An endpoint
 * without a position or a part -> SHEEP_ERR_RANGE (the reference's pos.at() / assert).
 * The host writes the per-part text files (sheep.hpp Partition::writePartitionedGraph). */
int sheep_edge_parts(sheep_ctx *ctx, const sheep_xs1 *rec_dev, uint64_t nrec, const uint32_t *pos_dev,
                     uint64_t pos_size, const int16_t *parts_vid_dev, int16_t *edge_part_dev);

/* ---- several GPUs of one node: the MPI world of graph2tree -i / -r -------------------
 * A world of `world` ranks; rank r holds edge shard r on one device.  Two ways to form it:
 *   sheep_group_create  ONE process drives every rank: rank r on devices[r], a context of its
 *                       own each (graph2tree -i / -r without mpiexec, SHEEP_DEVICES);
 *   sheep_group_join    ONE PROCESS PER RANK (replaces MPI_Init / MPI_Comm_rank / _size,
 *                       graph2tree.cpp:134-143): every rank calls it with its device, rank and
 *                       the world size; they meet over TCP at host:port (rank 0 listens there).
 *                       This is how `mpiexec -n W graph2tree ... -ir` and bench.py's
 *                       torch.distributed ranks run.
 * Data moves by RCCL when every rank has a device of its own (ncclCommInitAll, or
 * ncclCommInitRank with rank 0's id sent over the TCP links; xGMI), by device copies when
 * one process lists a device twice, and through host memory over the TCP links when
 * processes share a device (a one-GPU rehearsal).  `link` forces the choice for a joined
 * world (SHEEP_LINK_RCCL fails when two ranks share a device; a world of ONE with
 * SHEEP_LINK_RCCL opens a one-rank communicator, so every collective below and a self
 * send/recv run through RCCL on one GPU).
 * Per-rank array arguments (rec_dev[i], deg_dev[i], ...) are indexed by the LOCAL ranks of
 * the calling process (sheep_group_local_count of them; local i is global rank
 * sheep_group_rank(g, i)) and live on that rank's device.  Every call is collective: all
 * processes of a joined world make it, with the same scalars.  The ranks run on streams of
 * their own: inputs written on other streams must be complete before a call (synchronise
 * them first); every call is complete on return.  Replaces (chan150/sheep):
 *   sheep_group_sequence        mpiSequence (sequence.h:65-93): per-shard LLAMA degrees
 *                               into deg_dev[i] (zeroed by the caller, capacity cap), the
 *                               MPI_Allreduce(MAX) of max_slot and MPI_Allreduce(SUM) of the
 *                               degrees, then the same seq/pos on every rank
 *   sheep_group_build_tree      JTree per shard (graph2tree.cpp:185-189) + mpi_merge
 *                               (jnode.cpp:203-250): reduce 0 = partial trees only (tree_dev[i]
 *                               = the local rank's tree), 1 = gather + one K-way merge on
 *                               rank 0, 2 = binomial rounds of pairwise merges on disjoint rank
 *                               pairs; with 1 / 2 the merged tree is rank 0's tree_dev
 *   sheep_group_broadcast_parts Partition::mpi_sync (partition.cpp:69-79): rank 0's parts
 *   sheep_group_evaluate        Partition::evaluate over the shards: per-rank part bitsets,
 *                               binomial OR-reduction, the node pass on rank 0 (*out is
 *                               zero on the other ranks)
 *   sheep_group_barrier / sheep_group_allreduce_max_u64   MPI_Barrier / MPI_Allreduce(MAX)
 *   sheep_group_transfer        one point-to-point move of `bytes` from rank `from`'s src to
 *                               rank `to`'s dst (ncclSend/ncclRecv in one group under RCCL; the
 *                               hop of mpi_merge's MPI_Reduce, jnode.cpp:238-241); src / dst
 *                               matter only where that rank is local
 * Failure (the job-ending behaviour of MPI's default error handler, graph2tree.cpp:134-157):
 * no call waits on another rank for longer than SHEEP_JOIN_TIMEOUT seconds (default 300).
 * A joined world's communicator is non-blocking (ncclConfig_t.blocking = 0); every collective
 * polls ncclCommGetAsyncError and its streams against that deadline, and the TCP links poll
 * their sockets.  On an RCCL error, a dead peer or an expired deadline the call aborts the
 * communicators (ncclCommAbort), prints one line per local rank to stderr ("sheep: rank R of
 * W (bus B): COLLECTIVE of N bytes failed: CAUSE") and returns SHEEP_ERR_HIP; every later
 * collective of that world fails at once (sheep_group_failed = 1), and destroying it is safe.
 *   sheep_group_abort           the same on request (reason: the text of the stderr line) */
typedef struct sheep_group sheep_group;
#define SHEEP_LINK_AUTO 0
#define SHEEP_LINK_RCCL 1
#define SHEEP_LINK_HOST 2
int sheep_group_create(const int *devices, int ndev, sheep_group **out);
int sheep_group_join(int device, int rank, int world, const char *host, int port, int link, sheep_group **out);
int sheep_group_destroy(sheep_group *g);
int sheep_group_size(const sheep_group *g);                /* world size */
int sheep_group_local_count(const sheep_group *g);         /* ranks held by this process */
int sheep_group_rank(const sheep_group *g, int local);     /* global rank of local rank i */
sheep_ctx *sheep_group_ctx(sheep_group *g, int local);
int sheep_group_uses_rccl(const sheep_group *g);
int sheep_group_abort(sheep_group *g, const char *reason);
int sheep_group_failed(const sheep_group *g);               /* 1 after a failed collective or an abort */
int sheep_group_barrier(sheep_group *g);
int sheep_group_allreduce_max_u64(sheep_group *g, uint64_t *value);
/* sheep_ctx_set_tuning on every context of this process's ranks */
int sheep_group_set_tuning(sheep_group *g, const sheep_tuning *t);
int sheep_group_sequence(sheep_group *g, const sheep_xs1 *const *rec_dev, const uint64_t *nrec,
                         uint32_t *const *deg_dev, uint64_t cap, uint32_t *const *seq_dev,
                         uint32_t *const *pos_dev, uint64_t *n_out, uint64_t *vs_out);
int sheep_group_build_tree(sheep_group *g, const sheep_xs1 *const *rec_dev, const uint64_t *nrec,
                           const uint32_t *const *pos_dev, uint64_t pos_size, uint64_t n,
                           sheep_jnode *const *tree_dev, int reduce);
/* the reduction step alone (tree_dev[r] = rank r's partial tree; reduce 1 or 2 as above) */
int sheep_group_reduce_trees(sheep_group *g, sheep_jnode *const *tree_dev, uint64_t n, int reduce);
int sheep_group_broadcast_parts(sheep_group *g, int16_t *const *parts_vid_dev, uint64_t pos_size);
int sheep_group_transfer(sheep_group *g, int from, int to, const void *src_dev, void *dst_dev, uint64_t bytes);
int sheep_device_count(int *out);
int sheep_group_evaluate(sheep_group *g, const sheep_xs1 *const *rec_dev, const uint64_t *nrec,
                         const uint32_t *const *pos_dev, uint64_t pos_size,
                         const int16_t *const *parts_vid_dev, int what, sheep_eval *out);
/* Host-only self-test of a joined world's TCP links (no device touched): rank 0's bytes to
 * every rank, a ring shift, a gather to rank 0, all-reduce max / sum.  *checksum_out = the
 * world's sum of FNV-1a hashes of every received buffer, *max_out = the max of the ranks'
 * own buffer hashes (tests/test_dist.py checks both on CPUs). */
int sheep_mesh_selftest(int rank, int world, const char *host, int port, uint64_t bytes, uint64_t *checksum_out,
                        uint64_t *max_out);
/* Host-only check of the links' deadline: rank stall_rank joins and then takes no part; every
 * other rank's barrier must fail (SHEEP_ERR_HIP, sheep_last_error naming the peer) within
 * timeout_s.  *waited_s_out = the barrier's wait (0 on the stalled rank, which returns
 * SHEEP_OK after sleeping past the deadline). */
int sheep_mesh_selftest_stall(int rank, int world, const char *host, int port, int stall_rank, int timeout_s,
                              double *waited_s_out);

/* ---- tree facts (TREEFAQS) -------------------------------------------------------- */
int sheep_facts(sheep_ctx *ctx, const sheep_jnode *tree_dev, uint64_t n, sheep_facts_t *out);

/* ---- .dat partial loads (LLAMAGraph(filename, part, num_parts), graph_wrapper.h:43-63) ----
 * Host-only.  sheep_dat_range: records [*first_out, *first_out + *count_out) of a .dat file
 * (R = file size / 12 records) form part `part` of `num_parts` (1-indexed, contiguous:
 * [(part-1)R/num_parts, part R/num_parts); num_parts = 0: the whole file).
 * sheep_read_dat: preads exactly records [first, first + count) into out_host (no other byte
 * of the file is read); *got_out = records read.  An unreadable file is SHEEP_ERR_ARG.
 * sheep_record_stats (device; synchronises): *max_slot_out = 1 + the largest vid of
 * rec_dev[0, nrec) (LLAMA max_nodes, 0 for no records), *loops_out = self-loop records. */
int sheep_dat_range(const char *filename, uint64_t part, uint64_t num_parts, uint64_t *first_out, uint64_t *count_out);
int sheep_read_dat(const char *filename, uint64_t first, uint64_t count, sheep_xs1 *out_host, uint64_t *got_out);
int sheep_record_stats(sheep_ctx *ctx, const sheep_xs1 *rec_dev, uint64_t nrec, uint64_t *max_slot_out,
                       uint64_t *loops_out);

/* ---- .net (SNAP text) ingest ---------------------------------------------------------
 * text_dev[0, bytes): a SNAP text edge list in HBM.  Whitespace-separated unsigned decimal
 * pairs become records {tail, head, 1.0f} in out_dev (capacity cap records) the way
 * SNAPReader reads them (readerwriter.h:78-90): the input ends at the first token that is
 * not a 32-bit unsigned decimal, an incomplete last pair is dropped.  skip_comments = 1
 * drops lines whose first token starts with '#' or '%' first (the graph loader's
 * handling of SNAP headers; LLAMA's own loader is un-vendored, so parity-unpinned).
 * *nrec_out (host, synchronises) = records written. */
int sheep_parse_net(sheep_ctx *ctx, const char *text_dev, uint64_t bytes, int skip_comments, sheep_xs1 *out_dev,
                    uint64_t cap, uint64_t *nrec_out);

/* ---- synthetic input ---------------------------------------------------------------
 * Graph500-parameter RMAT (A,B,C,D = .57,.19,.19,.05, no per-level noise), vertex
 * labels permuted by a seeded Feistel bijection, self-loops and duplicate pairs
 * removed, orientation tail > head, records sorted by (tail, head), weight 1.0f.
 * out_dev needs capacity (ef << scale) records; *nrec_out (host) = records kept.
 * sheep_rmat_generate_host is the identical generator on the CPU (for .dat files). */
int sheep_rmat_generate(sheep_ctx *ctx, int scale, int edgefactor, uint64_t seed,
                        sheep_xs1 *out_dev, uint64_t cap, uint64_t *nrec_out);
int sheep_rmat_generate_host(int scale, int edgefactor, uint64_t seed, sheep_xs1 *out_host,
                             uint64_t cap, uint64_t *nrec_out);
/* Chung-Lu power law (BASELINE config C4, twitter-2010 scale): `draws` edges whose two
 * endpoints are drawn independently with probability ~ (rank + x0)^-1/(gamma-1) over
 * `nverts` vertices (x0: the top vertex takes 0.1% of the draws), labels permuted,
 * self-loops and duplicates removed, tail > head, sorted by (tail, head), weight 1.0f.
 * out_dev needs capacity `draws` records; *nrec_out (host) = records kept. */
int sheep_powerlaw_generate(sheep_ctx *ctx, uint64_t nverts, uint64_t draws, double gamma, uint64_t seed,
                            sheep_xs1 *out_dev, uint64_t cap, uint64_t *nrec_out);

#ifdef __cplusplus
}
#endif
#endif /* SHEEP_HIP_H */
