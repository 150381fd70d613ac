/*
 * nas.h -- C ABI of the MI355X network-aware placement engine.
 *
 * Drop-in boundary for the placement decision of
 * pablojara/kubernetesNetAwareScheduler (scheduler/scheduler.go):
 *
 *   func (s *CustomScheduler) findNodesThatFit(pod *v1.Pod) (string, error)   :239
 *     -> prioritize(nodes, pod) map[string]int                                :248
 *     -> findBestNode(priorities) string                                      :384
 *
 * The Go host (or the C++ host mirror in kubernetesnetawarescheduler_amd/host)
 * keeps the node-name table, the informer loop and Bind; this library deals in
 * node INDICES only.  INTEGRATION.md shows the cgo binding.
 *
 * Conventions
 *  - Every entry returns int: NAS_OK (0) or a negative NAS_ERR_*; on error
 *    nas_last_error(ctx) holds a message.  No C++ exception crosses the ABI.
 *  - All pointers are HOST pointers owned by the caller and are not retained
 *    after the call returns (cgo pointer rules).  Device memory is owned by
 *    the context.  Every call is blocking: it synchronises the context's HIP
 *    stream before returning, like the Go function it replaces.
 *  - A context is NOT thread-safe (one per goroutine / OS thread); each entry
 *    re-binds the context's HIP device, so a cgo call may land on any thread.
 *  - Node codes in outputs: >= 0 node index, NAS_NONE (-2) the "none"
 *    pseudo-node (scheduler.go:267-272, :364; Bind to it fails at :207),
 *    NAS_EMPTY (-1) the empty string findBestNode returns when no score is
 *    positive (:386) -- and, in extended mode, "no node fits".
 */
#ifndef NAS_H_
#define NAS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NAS_ABI_VERSION 2

/* status codes */
#define NAS_OK 0
#define NAS_ERR_ARG (-1)         /* bad argument (null, size, not a permutation, ...) */
#define NAS_ERR_HIP (-2)         /* HIP runtime error (also: no GPU / extension missing) */
#define NAS_ERR_STATE (-3)       /* call out of order (e.g. nas_place before uploads) */
#define NAS_ERR_NOMEM (-4)       /* device allocation failed */
#define NAS_ERR_COMM (-5)        /* RCCL error */
#define NAS_ERR_UNSUPPORTED (-6) /* size or dtype outside what the kernels support */

/* node codes */
#define NAS_NONE (-2)
#define NAS_EMPTY (-1)

/* element types of the traffic (WA) and latency (L) matrices */
#define NAS_DT_I8 1   /* int8, int32 accumulation: exact integer scores */
#define NAS_DT_BF16 2 /* bf16 bits (uint16), fp32 accumulation */
#define NAS_DT_I32 3  /* traffic only, with NAS_DT_I8 latency: int32 traffic, exact integer
                       * scores (see nas_upload_traffic_dense) */
#define NAS_DT_F32 4  /* fp32 latency and traffic as measured (no quantisation): each
                       * operand split into three bf16 planes (x = h + m + l), the
                       * products to 2^-24 relative on the bf16 MFMA (six terms),
                       * fp32 accumulation -- costs within 1e-5 relative of an fp64
                       * sum */

/* winner slots returned by nas_score_reference (order of scheduler.go:360-365) */
#define NAS_W_CPU 0
#define NAS_W_MEM 1
#define NAS_W_NETSENT 2
#define NAS_W_NETREC 3
#define NAS_W_BANDWIDTH 4 /* always NAS_NONE: the :353 bug */
#define NAS_W_DISK 5

/* candidates kept per pod between scoring and commit: the 8 smallest
 * (cost, node) among fitting nodes, of which the first `count` are
 * guaranteed to be the exact global ranking (see nas_get_candidates) */
#define NAS_K_CANDIDATES 8

typedef struct nas_ctx nas_ctx;

typedef struct nas_config {
    int32_t device;   /* HIP device ordinal */
    int32_t flags;    /* reserved, 0 */
    int32_t reserved0;
    int32_t reserved1;
} nas_config;

/* Per-context options (nas_set_option); every option has a production
 * default, and nothing is read from the environment. */
#define NAS_OPT_STAGE_TIMINGS 1  /* 1 (default): per-stage HIP events (nas_get_timings
                                  * fit/cost/merge/commit); 0: only the events a call
                                  * synchronises on (total_ms stays valid) */
#define NAS_OPT_COMM_TIMEOUT_MS 2 /* deadline of every wait of a call that issued RCCL
                                   * collectives, in ms (default 120000; 0 = no deadline).
                                   * On expiry the communicators are aborted
                                   * (ncclCommAbort), the call returns NAS_ERR_COMM and the
                                   * context is poisoned: every later call except
                                   * nas_last_error / nas_destroy returns NAS_ERR_COMM.
                                   * It also bounds nas_comm_init: communicators not built
                                   * by then (a rank never joined) -> NAS_ERR_COMM */
#define NAS_OPT_REHEARSE_WORLD 3 /* DIAGNOSTIC, default 0.  G > 1, set before nas_comm_init
                                  * with world 1: the context takes rank 0's shard geometry
                                  * of a G-rank node shard and stands the other ranks' lists
                                  * in with shifted copies of its own -- times one rank of a
                                  * G-GPU pass on one GPU.  Placements are NOT meaningful. */
#define NAS_OPT_INJECT_STALL_MS 4 /* TEST ONLY, default 0: the next call with a
                                   * communicator enqueues a device-side delay of this many
                                   * ms behind its collectives, on the stream it waits on
                                   * last (exercises NAS_OPT_COMM_TIMEOUT_MS); cleared when
                                   * used */
#define NAS_OPT_COMMIT_WAIT_MS 5  /* bound of the device-side wait that orders a pipelined
                                   * nas_place's last commit behind the commit stream's
                                   * earlier ones, in ms; default 0 = automatic: the
                                   * NAS_OPT_COMM_TIMEOUT_MS deadline when the pass issues
                                   * collectives (10 min when that is 0), else 2000.  On
                                   * expiry the pass fails: NAS_ERR_COMM with communicators
                                   * aborted and the context poisoned, or NAS_ERR_HIP without
                                   * a communicator (the context stays usable) */
#define NAS_OPT_INJECT_COMMIT_STALL_MS 6 /* TEST ONLY, default 0: the next pipelined
                                   * nas_place enqueues a device-side delay of this many ms
                                   * on its commit stream ahead of the last commit there
                                   * (exercises NAS_OPT_COMMIT_WAIT_MS); cleared when used */
#define NAS_OPT_SYNTH_PROFILE 7 /* generator of the next nas_synth_cluster / nas_synth_batch
                                 * (benchmarks): 0 (default) racks of 32 in zones of 16 racks,
                                 * latency by distance class, dense background traffic 0..2
                                 * plus bound peers in the home rack / zone; 1 SURVEY.md
                                 * §8(d)'s C3 operand distribution over the full int8 range:
                                 * latency U{1..127} (symmetric, zero diagonal), traffic
                                 * U{0..127} to every node, no peer structure */
#define NAS_OPT_COMMIT_CUS 8     /* CUs per XCD kept for the commit stream of a world-1
                                  * context's nas_place (0..4, default 0: none); the scoring
                                  * streams then run on the other CUs (CU-masked streams from
                                  * the process-wide pool).  Node shards keep their own
                                  * reservation (nas_comm_init). */
#define NAS_OPT_COST_CACHE 9      /* cost-row cache of nas_place (one cluster): the pass's
                                   * cost launches also store every (pod, node) cost, P x N
                                   * x 4 B (4 GB at 10k x 100k), and its gathered rescores
                                   * read a pod's row instead of recomputing the contraction
                                   * (herds: every pod ranking the same nodes first).
                                   * 0 off, 1 on, 2 (default) auto: on when the previous
                                   * nas_place of the same shape needed >= 4 rescore rounds
                                   * and the cache takes <= 16 GB.  Placements are the same
                                   * either way. */
#define NAS_OPT_HERD_PLAN 10      /* nas_place's chunk plan (one cluster, no communicator):
                                   * 0 pipelined (chunks scored on two streams while the
                                   * commit stream walks earlier ones; each chunk's fit sees
                                   * the capacity two or more chunks back), 1 the herd plan
                                   * (fit + cost, merge and commit chunk after chunk on one
                                   * stream: every chunk's fit sees its predecessors'
                                   * commits), 2 (default) auto: pipelined until a pass of
                                   * the shape needs >= 8 rescore rounds, then the herd plan
                                   * for that shape.  Placements are the same either way. */
int nas_set_option(nas_ctx *ctx, int32_t key, int64_t value);

/* per-stage device times of the last nas_place / nas_score_reference call,
 * measured with HIP events on the context's stream */
typedef struct nas_timings {
    float fit_ms;      /* resource-fit filter kernel */
    float cost_ms;     /* MFMA contraction + fused top-k epilogue (all launches) */
    float merge_ms;    /* per-pod merge of node-tile candidate lists (+ comm) */
    float commit_ms;   /* greedy commit kernel(s) */
    float vote_ms;     /* reference-mode vote kernel */
    float total_ms;    /* whole call, device side */
    int32_t cost_launches;   /* launches of the contraction kernel */
    int32_t rescore_rounds;  /* commit stops that needed a rescore */
    int32_t unschedulable;   /* pods with no fitting node */
    int32_t commit_rounds;   /* rounds of the parallel commit walk (all windows) */
    int32_t rescored_pods;   /* pods re-scored by host-side gathered rescores */
} nas_timings;

/* ---- lifecycle --------------------------------------------------------- */
int nas_version(void);

/* Process-wide debug counters (any thread, no context): out[i] for
 * i < min(n, NAS_DBG_COUNT).  CU-masked streams (node-shard contexts reserve
 * CUs for their commit stream) come from a process-wide pool: contexts borrow
 * them and return them on nas_destroy, so CREATED stays bounded by the most
 * masked streams ever in use at once, however many contexts come and go. */
#define NAS_DBG_MASKED_STREAMS_CREATED 0 /* masked streams the pool ever created (all live) */
#define NAS_DBG_MASKED_STREAMS_LENT 1    /* of them, held by contexts now */
#define NAS_DBG_MASKED_STREAMS_IDLE 2    /* of them, idle in the pool */
#define NAS_DBG_LIVE_CONTEXTS 3          /* contexts created and not yet destroyed */
#define NAS_DBG_COUNT 4
int nas_debug_counters(int64_t *out, int32_t n);
int nas_create(nas_ctx **out, const nas_config *cfg);
void nas_destroy(nas_ctx *ctx);
const char *nas_last_error(nas_ctx *ctx);
int nas_get_timings(nas_ctx *ctx, nas_timings *out);

/* ---- reference mode: the vote scorer of scheduler.go:248-394 ---------------
 *
 * Snapshot = one PrometheusNodeMetrics record per node (scheduler.go:24-32),
 * SoA, n_snapshots blocks of n_nodes: field[s * n_nodes + node].  Go `int` is
 * int64 (rx, tx, disk).  The reference scrapes a fresh snapshot per pod
 * (:275-279); here pod p scores against snapshot pod_snapshot[p].
 */
int nas_upload_snapshot(nas_ctx *ctx, const double *cpu, const double *mem, const int64_t *rx,
                        const int64_t *tx, const double *bw, const int64_t *disk,
                        int32_t n_nodes, int32_t n_snapshots);

/* Go map iteration orders, made explicit: order1[n_nodes] is the order of
 * `range nodeMetricsMap` (:334); order2[n_nodes+1] the order of
 * `range priorities` (:387), where value n_nodes is the "none" key.
 * n_orders == 1: one order set for every snapshot; n_orders == n_snapshots:
 * one per snapshot.  Both must be permutations (NAS_ERR_ARG otherwise). */
int nas_upload_orders(nas_ctx *ctx, const int32_t *order1, const int32_t *order2,
                      int32_t n_orders);

/* One order set per POD instead (n_pods sets): pod p of the next
 * nas_score_reference (which must score exactly n_pods pods) walks order set
 * p on snapshot pod_snapshot[p] -- e.g. a batch of pods scored against ONE
 * scraped snapshot, each pod with the map orders of its own prioritize call
 * (scheduler.go:334, :387), without a snapshot copy per pod. */
int nas_upload_pod_orders(nas_ctx *ctx, const int32_t *order1, const int32_t *order2,
                          int32_t n_pods);

/* Score P pods.  order1/order2 non-NULL: one shared order set for this call;
 * NULL: the sets from nas_upload_orders.  pod_snapshot NULL: pod p uses
 * snapshot p.  best_out[P]: node index / NAS_NONE / NAS_EMPTY (the
 * findNodesThatFit result, :245).  winners_out[P*6] optional (NAS_W_*). */
int nas_score_reference(nas_ctx *ctx, const int32_t *order1, const int32_t *order2,
                        const int32_t *pod_snapshot, int32_t P, int32_t *best_out,
                        int32_t *winners_out);

/* ---- reference mode, node axis sharded (vote row) --------
 * Each of the six loops of scheduler.go:334-359 is a first-occurrence
 * arg-extremum in order1, i.e. a lexicographic (value, pos1) reduction that
 * splits over node slices.  A shard reduces its slice to one partial record
 * per snapshot; records of all slices merge in any order into the same six
 * extrema, from which the net-sent rule (:347-354), the votes (:360-365) and
 * findBestNode (:384-394) follow.
 *
 * Record of one snapshot: six (value, pos1) extrema in the order below;
 * value = the IEEE-754 bits of the double (cpu, mem, bw) or the int64
 * (rx, tx, disk) of the first node in order1 holding the extremum among the
 * slice's nodes that beat the sentinel (:258-265; disk also != 0, :355);
 * pos1 = that node's position in order1, NAS_VOTE_NOPOS if no node of the
 * slice qualifies (value then 0). */
#define NAS_VOTE_NOPOS 0x7fffffff
#define NAS_VP_CPU 0
#define NAS_VP_MEM 1
#define NAS_VP_BW 2
#define NAS_VP_RX 3
#define NAS_VP_TX 4
#define NAS_VP_DISK 5
typedef struct nas_vote_extremum {
    int64_t value;
    int32_t pos1;
    int32_t reserved; /* 0 */
} nas_vote_extremum;
typedef struct nas_vote_partial {
    nas_vote_extremum m[6]; /* NAS_VP_* */
} nas_vote_partial;         /* 96 bytes */

/* Upload nodes [node_lo, node_lo + n_local) of n_snapshots snapshots of an
 * n_nodes-node cluster: field[s * n_local + i] is node node_lo + i.  Orders
 * (nas_upload_orders / the order arguments) stay over all n_nodes nodes.
 * With a communicator (nas_comm_init), nas_score_reference on a shard
 * reduces the slice, all-gathers the partial records over RCCL and merges
 * them: every rank returns the full result (the ranks' slices must tile
 * [0, n_nodes) and every rank must make the same call).  Without one, use
 * nas_vote_partials + nas_vote_merge and move the records yourself. */
int nas_upload_snapshot_shard(nas_ctx *ctx, const double *cpu, const double *mem,
                              const int64_t *rx, const int64_t *tx, const double *bw,
                              const int64_t *disk, int32_t n_nodes, int32_t node_lo,
                              int32_t n_local, int32_t n_snapshots);

/* Partial records of snapshots [0, S) over this context's node slice (a
 * whole-cluster snapshot is one slice): out[S].  order1/order2 as in
 * nas_score_reference (only order1's positions are used here). */
int nas_vote_partials(nas_ctx *ctx, const int32_t *order1, const int32_t *order2, int32_t S,
                      nas_vote_partial *out);

/* Merge parts[n_parts * S] (slice-major: parts[k * S + s]) into the decision
 * of snapshots [0, S) with this context's orders (as nas_score_reference with
 * pod_snapshot NULL and P = S): best_out[S], winners_out[S * 6] optional. */
int nas_vote_merge(nas_ctx *ctx, const nas_vote_partial *parts, int32_t n_parts, int32_t S,
                   int32_t *best_out, int32_t *winners_out);

/* ---- extended mode: fit -> network cost -> top-k -> greedy commit ---------
 *
 * Resources are int32: cpu in millicores, memory in KiB, pod slots.
 */

/* Dense latency matrix L[m * n + j] = latency from node m to node j,
 * uploaded once (dtype NAS_DT_I8, NAS_DT_BF16 or NAS_DT_F32).  Integer scores are exact
 * int32: nas_place / nas_score return NAS_ERR_UNSUPPORTED when some pod's
 * sum_m |WA[p,m]| * max|L| exceeds INT32_MAX. */
int nas_upload_latency(nas_ctx *ctx, const void *L, int32_t dtype, int32_t n);

/* Free capacity per node; also resets the working capacity nas_place uses. */
int nas_upload_capacity(nas_ctx *ctx, const int32_t *cpu_milli, const int32_t *mem_kib,
                        const int32_t *pods, int32_t n);

/* Reset the working capacity to the last uploaded capacity.  Stream-ordered:
 * returns without waiting; every later call on this context sees the reset. */
int nas_reset_capacity(nas_ctx *ctx);

/* Read back the working (remaining) capacity. */
int nas_get_capacity(nas_ctx *ctx, int32_t *cpu_milli, int32_t *mem_kib, int32_t *pods,
                     int32_t n);

/* Pending pods in placement order: resource requests (>= 0). */
int nas_upload_pods(nas_ctx *ctx, const int32_t *req_cpu_milli, const int32_t *req_mem_kib,
                    const int32_t *req_pods, int32_t P);

/* Traffic of each pending pod to each node, WA[p * n + m] = sum of
 * W[p,q] over already-bound peers q with node(q) == m (dense).  dtype: the
 * latency's (NAS_DT_I8 / NAS_DT_BF16), or NAS_DT_I32 with NAS_DT_I8 latency --
 * the cost stays the exact sum_m WA[p,m] * L[m,n] for any int32 traffic (the
 * engine keeps an int8 plane for the MFMA and adds the few entries outside
 * [-128, 127] exactly in the contraction's epilogue); NAS_DT_F32 with
 * NAS_DT_F32 latency. */
int nas_upload_traffic_dense(nas_ctx *ctx, const void *WA, int32_t dtype, int32_t P, int32_t n);

/* Same from a sparse pod-communication graph: for pod p the peers are
 * peer_node[row_ptr[p] .. row_ptr[p+1]) (node of an already-bound peer, or
 * -1 for an unbound peer, which is skipped) with weights weight[...]:
 * int8 (NAS_DT_I8) or int32 (NAS_DT_I32) with int8 latency -- summed exactly
 * (no saturation; an aggregate outside int32 is NAS_ERR_UNSUPPORTED) -- or
 * bf16 bits (NAS_DT_BF16), summed in fp32 on the device and rounded once,
 * or fp32 (NAS_DT_F32), summed in fp64 on the host and rounded once. */
int nas_upload_traffic_csr(nas_ctx *ctx, const int32_t *row_ptr, const int32_t *peer_node,
                           const void *weight, int32_t dtype, int32_t P, int32_t n,
                           int64_t nnz);

/* Resource-fit filter over all pod x node pairs against the working capacity.
 * mask_out (optional) receives ceil(n/64) * P uint64 words, node-chunk major:
 * bit j of mask_out[c * P + p] == pod p fits node 64c + j. */
int nas_filter(nas_ctx *ctx, uint64_t *mask_out);

/* Place all uploaded pods: fit, cost = WA x L on MFMA with the top-k fused
 * in the epilogue, then greedy commit in pod order with capacity update.
 * node_out[P]: chosen node or NAS_EMPTY.  cost_out[P] (optional): the
 * chosen node's cost as float.  int_score_out[P] (optional): the chosen
 * node's exact integer cost (NAS_DT_I8; 0 for bf16 or NAS_EMPTY). */
int nas_place(nas_ctx *ctx, int32_t *node_out, float *cost_out, int64_t *int_score_out);

/* Scoring pass only (fit + cost/top-k + merge, no commit) against the
 * working capacity; its lists are then read with nas_get_candidates. */
int nas_score(nas_ctx *ctx);

/* Candidate lists of the last scoring pass (nas_score, or nas_place after
 * its rescore rounds): cand_node[P*K] sorted by (cost, node), -1 past
 * count; count[P] = number of leading entries that are exactly the pod's
 * best fitting nodes in order (at least min(4, #fitting nodes); entries past
 * count are not returned); cand_cost_i[P*K] exact int cost (NAS_DT_I8),
 * cand_cost_f[P*K] cost as float; complete[P] = 1 iff the list holds every
 * node that fit when it was scored.  Any output may be NULL. */
int nas_get_candidates(nas_ctx *ctx, int32_t *cand_node, int64_t *cand_cost_i,
                       float *cand_cost_f, int32_t *count, int32_t *complete);

/* ---- multi-tenant batches (BASELINE config C5) ----------------------------
 * n_clusters independent clusters of the same shape (nodes, pods, dtype)
 * placed by one call: every extended-mode array passed to the upload calls,
 * nas_get_capacity, nas_place and nas_get_candidates then holds the
 * clusters back to back (cluster b's L at L + b*n*n, its pods at b*P, ...).
 * Call before the extended uploads; not combinable with node shards, CSR
 * traffic, nas_filter or the host-driven steps.  Clusters are independent:
 * each one's placements equal a single-cluster nas_place on its inputs. */
int nas_set_batch(nas_ctx *ctx, int32_t n_clusters);

/* ---- multi-GPU: node axis sharded over the GPUs of one node ---------------
 * Rank r of `world` owns node columns [r*n/world, (r+1)*n/world) of L; pods,
 * WA and capacities are replicated.  Per-pod candidate lists are exchanged
 * with an RCCL all-gather over xGMI and merged; the commit is replicated, so
 * every rank returns the same placements.  world = 1 builds a real
 * communicator too (the exchange then runs as a one-rank all-gather: the
 * whole RCCL path on a single GPU). */
int nas_comm_unique_id(uint8_t id_out[128]);
int nas_comm_init(nas_ctx *ctx, const uint8_t id[128], int32_t rank, int32_t world);

/* In-process transport instead of RCCL: `world` contexts of ONE process (on
 * any devices, each driven by its own host thread) form a node-sharded
 * placement whose exchanges are device-to-device pulls behind host barriers.
 * Every call of nas_place / nas_score / nas_score_range / nas_score_reference
 * then runs exactly the RCCL path's kernels, merges and commit with the
 * all-gather replaced -- so G ranks' distinct candidate lists meet the
 * cross-rank merge on one GPU (tests), or one host process drives the GPUs
 * of a node without RCCL.  All ranks must make the same calls; a rank that
 * does not arrive within NAS_OPT_COMM_TIMEOUT_MS breaks the group
 * (NAS_ERR_COMM, contexts poisoned).  The group must outlive nas_comm_init_local;
 * contexts keep it alive after nas_local_group_destroy. */
typedef struct nas_local_group nas_local_group;
int nas_local_group_create(int32_t world, nas_local_group **out);
void nas_local_group_destroy(nas_local_group *group);
int nas_comm_init_local(nas_ctx *ctx, nas_local_group *group, int32_t rank);

/* Node shard without a communicator: this context keeps and scores only node
 * columns [rank*n/world, (rank+1)*n/world) (call before the extended
 * uploads).  For hosts that exchange candidate lists themselves (nas_score +
 * nas_get_candidate_keys, then merge: keep the 8 smallest keys, bound =
 * min(bounds, kept[7])); nas_place needs nas_comm_init instead. */
int nas_set_shard(nas_ctx *ctx, int32_t rank, int32_t world);

/* Raw candidate lists of the last scoring pass: keys[P*8] (orderable cost
 * << 32 | global node index, ascending; ~0 = empty) and bounds[P] (every
 * fitting key <= bound is in the list; ~0 = nothing was dropped). */
int nas_get_candidate_keys(nas_ctx *ctx, uint64_t *keys, uint64_t *bounds);

/* ---- host-driven steps of nas_place -------------------------------------
 * For hosts that run the placement loop themselves -- e.g. node shards
 * (nas_set_shard) whose candidate lists travel over the host's own
 * transport: score a pod range on this context's node columns, read the raw
 * lists, write back the lists merged across shards, and commit:
 *
 *   nas_score_range(0, P) -> get keys -> [exchange + merge] -> set keys
 *   stop = 0; while (stop < P) {
 *     nas_commit(stop, ..., &stop);          // replicated on every shard
 *     if (stop < P) { nas_score_range(stop, min(P, stop + 1024)); get/merge/set }
 *   }
 *
 * Merge rule for lists of several shards: keep the 8 smallest keys, bound =
 * min(all bounds, kept[7]).  Every shard runs the same commit on the same
 * merged lists, so all of them return the same placements. */

/* Scoring pass (fit against the WORKING capacity, cost/top-k, merge over
 * this context's node tiles) for pods [p_lo, p_hi). */
int nas_score_range(nas_ctx *ctx, int32_t p_lo, int32_t p_hi);

/* Raw candidate lists of pods [p_lo, p_lo + n): keys[n*8], bounds[n]
 * (encoding of nas_get_candidate_keys). */
int nas_get_candidate_keys_range(nas_ctx *ctx, int32_t p_lo, int32_t n, uint64_t *keys,
                                 uint64_t *bounds);
int nas_set_candidate_keys(nas_ctx *ctx, int32_t p_lo, int32_t n, const uint64_t *keys,
                           const uint64_t *bounds);

/* Greedy commit of pods [p_begin, P) in order on the current lists and the
 * working capacity.  Stops at the first pod none of whose usable candidates
 * fits while its list is incomplete (score it again first): *stop_out = that
 * pod, or P when every pod was placed.  node_out / cost_out / int_score_out
 * (length P; cost_out and int_score_out may be NULL) receive entries
 * [p_begin, *stop_out) only. */
int nas_commit(nas_ctx *ctx, int32_t p_begin, int32_t *node_out, float *cost_out,
               int64_t *int_score_out, int32_t *stop_out);

/* ---- synthetic inputs generated in HBM (benchmarks; seeded, deterministic) */
/* Reference-mode snapshots per SURVEY.md §8(d) C1/C3. */
int nas_synth_snapshots(nas_ctx *ctx, uint64_t seed, int32_t n_nodes, int32_t n_snapshots);
/* Nodes [node_lo, node_lo + n_local) of the snapshots nas_synth_snapshots
 * generates with the same seed and sizes (a node shard of them). */
int nas_synth_snapshots_shard(nas_ctx *ctx, uint64_t seed, int32_t n_nodes, int32_t node_lo,
                              int32_t n_local, int32_t n_snapshots);
/* Read back snapshot s (to check sampled pods against a CPU oracle). */
int nas_read_snapshot(nas_ctx *ctx, int32_t s, double *cpu, double *mem, int64_t *rx,
                      int64_t *tx, double *bw, int64_t *disk);
/* Extended-mode cluster: racks of 32 nodes in zones of 16 racks; latency by
 * distance class; each pod has `peers` bound peers in one rack, traffic
 * concentrated there; capacity and requests per SURVEY.md §8(d) C2/C3. */
int nas_synth_cluster(nas_ctx *ctx, uint64_t seed, int32_t n_nodes, int32_t P, int32_t dtype,
                      int32_t peers);
/* A batch of n_clusters synthetic clusters; cluster b is the cluster
 * nas_synth_cluster(seed + b, ...) generates (sets the batch). */
int nas_synth_batch(nas_ctx *ctx, uint64_t seed, int32_t n_clusters, int32_t n_nodes, int32_t P,
                    int32_t dtype, int32_t peers);
/* Read back rows of the device-resident inputs (for sampled oracle checks):
 * WA rows [p0, p0+np) -- int32 [np][n] exact traffic for int8 scoring, bf16
 * bits [np][n] otherwise --, the full L, capacity and requests (cluster 0 of a
 * batch). */
int nas_read_inputs(nas_ctx *ctx, int32_t p0, int32_t np, void *WA_rows, void *L,
                    int32_t *cap_cpu, int32_t *cap_mem, int32_t *cap_pods, int32_t *req_cpu,
                    int32_t *req_mem, int32_t *req_pods);

#ifdef __cplusplus
}
#endif
#endif /* NAS_H_ */
