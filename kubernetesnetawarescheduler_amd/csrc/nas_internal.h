// nas_internal.h -- context, device buffers and kernel launch interfaces of
// the MI355X placement engine (gfx950 only).  See DESIGN.md for the data
// layout in HBM and the roofline of each kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nas.h"

struct ncclComm;

namespace nas {

constexpr int KC = NAS_K_CANDIDATES;  // candidates per pod

// Cost contraction tile (see k_cost.hip): BM nodes x BN pods, 128-byte K stage.
constexpr int COST_BM = 256;
constexpr int COST_BN = 256;
// rows allocated past the last traffic row: the wide cost tile (384 pods over
// launches of 256 k pods, ceil(256 k / 384) tiles) reads up to 256 rows past a
// launch's end (k = 2 mod 3), whose results it discards
constexpr int WA_PAD_ROWS = 256;
constexpr int COST_BKB = 128;  // bytes of K per stage (128 int8 or 64 bf16)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    template <typename T>
    T *as() const { return static_cast<T *>(p); }
};

// per-cluster commit control words in ctx->status: halt (pod to rescore or
// -1), device-side rescores, commit rounds, spare
constexpr int STATUS_INTS = 4;

// packed candidate key: orderable 32-bit cost in the high word, node index
// in the low word; ascending key == ascending (cost, node).
constexpr uint64_t KEY_INVALID = ~0ull;

// Exact int32 traffic on the int8 MFMA path: WA = plane + E, where the plane
// (the MFMA operand) holds every entry clamped to [-128, 127] and E the few
// entries outside it as per-pod lists (row r of the pod array: entries
// [ptr[r], ptr[r+1]) of (node m, excess e = WA - clamp(WA))).  The cost
// kernel's epilogue adds e * L[m][n] for the tile's nodes from Lr, a
// row-major copy of this rank's latency columns (Lr[m][i] = L[m][Nloc0 + i],
// row stride Mp).  row_pod maps a gathered view's rows to pods (nullptr:
// row = pod); rows >= *row_count of a view are never read.
// The cost kernel's fused fit (k_cost.hip; every launch over a main pod range,
// i.e. not a rescore window): the capacity the scoring reads (live `cap`, or
// `cap_snap` beside the L2 commit) and the requests, read by the cost
// workgroups themselves instead of a k_fit mask (batches: cluster cb at
// cap + cb*3*N, req + cb*3*Pp)
struct FitSrc {
    const int32_t *cap = nullptr;  // [3][N]
    const int32_t *req = nullptr;  // [3][Pp] (row stride = the launch's Pp)
    int N = 0;                     // row stride of cap
    int n0 = 0;                    // first node of this shard
    int nloc = 0;                  // valid local nodes
};

struct Ovf {
    const int32_t *ptr = nullptr;  // [B * Pp + 1] absolute offsets (nullptr: no entries)
    const int32_t *m = nullptr;
    const int32_t *e = nullptr;
    const signed char *Lr = nullptr;  // [B][N][Mp]
    const int32_t *row_pod = nullptr;
    const int32_t *row_count = nullptr;
    int N = 0;  // rows of one cluster's Lr
};

// In-process transport (nas_comm_init_local): G contexts of one process, each
// driven by its own host thread, exchange candidate lists through device
// memory instead of RCCL.  Kernel argument of k_local_gather: the G ranks'
// send buffers of one exchange.
constexpr int LOCAL_MAX_WORLD = 64;
struct LocalSrcs {
    const void *p[LOCAL_MAX_WORLD];
};
struct LocalGroup;  // nas_api.hip
struct CommInit;    // nas_api.hip: state shared with a nas_comm_init helper thread

}  // namespace nas

struct nas_ctx {
    int device = 0;
    int n_cu = 256;                    // compute units of the device
    hipStream_t stream = nullptr;      // main stream (uploads, scoring, results)
    hipStream_t stream2 = nullptr;     // second scoring stream (chunk tails overlap)
    hipStream_t stream_commit = nullptr;  // commit walks, pipelined behind scoring
    // a node-shard pass's chunk merges and all-gathers, ahead of their commits
    // (so one chunk's exchange runs beside the previous chunk's commit)
    hipStream_t stream_x = nullptr;
    int32_t cu_reserve = 0;               // CUs per XCD kept for stream_commit (set_stream_masks)
    std::string err;
    hipEvent_t ev[12] = {};
    nas_timings timings = {};

    // ---- reference mode
    int32_t snap_n = 0, snap_s = 0;   // nodes (whole cluster), snapshots
    int32_t snap_lo = 0, snap_nl = 0; // node slice held here: [snap_lo, snap_lo + snap_nl)
    bool snap_sharded = false;        // uploaded as a node shard (nas_upload_snapshot_shard)
    int64_t snap_ns = 0;              // padded row stride of the slice (even)
    nas::DevBuf snap[6];              // cpu, mem, bw (f64) ; rx, tx, disk (i64)  [S][ns]
    int32_t n_orders = 0;
    bool orders_per_pod = false;      // nas_upload_pod_orders: set p belongs to pod p
    // gathered slots the previous nas_place of shape (P, N) needed: enqueued
    // speculatively by the next pass of that shape
    int32_t slot_hint = 0, slot_hint_P = -1, slot_hint_N = -1;
    int32_t last_rescore_rounds = 0;  // of the previous nas_place of shape (slot_hint_P, _N)
    // cost-row cache (NAS_OPT_COST_CACHE): [Pp][Mp] orderable keys of the
    // current pass's main cost launches, read by its gathered rescore slots
    nas::DevBuf cost_cache;
    bool cache_active = false;
    // NAS_DT_F32: the operands as six-segment bf16 splits (prepare_split);
    // the fp32 Lt / WA stay for read-back and host-side updates
    nas::DevBuf Lt6, WA6;
    bool split_valid = false;
    int64_t ord_ns = 0;               // row stride of order arrays
    nas::DevBuf order1, pos1;         // [n_orders][ord_ns]
    nas::DevBuf order2, pos2;         // [n_orders][ord_ns + 2]  (n+1 keys)
    nas::DevBuf pod_snap, best, winners;
    nas::DevBuf snap_best, snap_win;  // per-snapshot results
    nas::DevBuf vote_part, vote_gather;
    nas::DevBuf xsend[3];  // per gather slot: a chunk's lists to all-gather, [np][8] keys | [np] bounds  // node-shard partial records [S], [world][S]

    // ---- extended mode
    int32_t N = 0;           // nodes
    int32_t P = 0;           // pending pods
    int32_t dtype = 0;       // element type of L and WA
    int32_t Kp = 0;          // padded contraction length (row bytes / elt)
    int32_t Nloc0 = 0, Nloc = 0;  // node shard [Nloc0, Nloc0+Nloc) owned by this rank
    int32_t Mp = 0;          // padded local node count (multiple of COST_BM)
    int32_t Pp = 0;          // padded pod count (multiple of COST_BN)
    int32_t B = 1;           // independent clusters of equal shape (nas_set_batch)
    int32_t cur_cluster = 0; // target of per-cluster uploads / reads (nas_select_cluster)
    bool have_L = false, have_cap = false, have_pods = false, have_wa = false;
    int32_t L_n = 0, L_dtype = 0, cap_n = 0, req_P = 0, wa_P = 0, wa_n = 0, wa_dtype = 0;
    nas::DevBuf Lt;          // [Mp][Kp] elements: Lt[i][m] = L[m][Nloc0 + i]
    nas::DevBuf WA;          // [Pp][Kp] elements
    nas::DevBuf cap0, cap;   // [3][N] int32 (initial, working)
    nas::DevBuf cap_snap;    // [3][N] published capacity: start minus committed pods (L2 commit)
    nas::DevBuf req;         // [3][Pp] int32
    nas::DevBuf mask;        // [ceil(Mp/64)][Pp] uint64, local nodes
    nas::DevBuf partial;     // [Mp/BM][Pp][KC] uint64 keys per node tile
    nas::DevBuf pbound;      // [Mp/BM][Pp] uint64 exactness bound per node tile
    nas::DevBuf cand_key;    // [Pp][KC] uint64 (global node ids), after merge
    nas::DevBuf cand_bound;  // [Pp] uint64
    nas::DevBuf gather[3];   // per scoring stream: [world][chunk][KC] uint64 (multi-GPU exchange)
    nas::DevBuf gbound[3];   // per scoring stream: [world][chunk] uint64
    nas::DevBuf resc_key, resc_bound;      // rescore slot staging [win][KC] / [win] (multi-GPU)
    nas::DevBuf gather_r, gbound_r;        // rescore slot exchange [world][win][KC] / [world][win]
    nas::DevBuf out_node, out_cost_f, out_cost_i;  // [Pp]
    nas::DevBuf g_words, g_idx;            // gathered rescore: dry-pod ballots, indices + count
    nas::DevBuf g_key, g_bound;  // gathered rescore view's lists (rows read in place, row map g_idx)
    nas::DevBuf g_gk, g_gb;                // gathered rescore exchange [world][R][KC] / [world][R]
    nas::DevBuf status;      // small device scratch for commit control
    nas::DevBuf commit_flag;  // the pass's last commit sequence number (launch_flag_set)
    uint64_t commit_seq = 0;  // host copy: sequence numbers only grow, across passes
    nas::DevBuf host_status; // pinned
    nas::DevBuf ref_stage;   // pinned: nas_score_reference results [P] best | [P][6] winners
    nas::DevBuf scratch;
    // exact int32 traffic (nas::Ovf): entries outside the int8 plane, and Lr
    nas::DevBuf ovf_ptr, ovf_m, ovf_e, Lr;
    int64_t ovf_n = 0;          // entries (0: the plane is the traffic)
    bool lr_valid = false;      // Lr matches the uploaded latency
    int64_t wa_abs_row_max = 0; // max over pods of sum_m |WA[p,m]| (int8 path)
    int32_t L_abs_max = 0;      // max |L| (int8 path)
    bool scored = false;        // a scoring pass filled cand_key
    // zero-traffic pods (k_commit.hip): zrow[B][Pp], valid for the uploaded
    // traffic; L_finite: no Inf / NaN latency (float dtypes; 0 x Inf is not 0)
    nas::DevBuf zrow;
    bool zrow_valid = false;
    bool L_finite = true;
    bool synth_valid = false;   // inputs came from nas_synth_cluster(synth_seed)
    uint64_t synth_seed = 0;
    int32_t synth_profile = 0;  // the profile the synthetic inputs were generated with

    // ---- multi-GPU
    ncclComm *comm = nullptr;    // scoring chunks on `stream` and host-side rescores
    ncclComm *comm2 = nullptr;   // scoring chunks on `stream2`
    ncclComm *comm_c = nullptr;  // rescore slots on `stream_commit`
    // the non-blocking communicator the three above are split from (nas_comm_init
    // polls it under a deadline and can abort it); it issues no collectives
    ncclComm *comm_root = nullptr;
    int32_t rank = 0, world = 1;
    // diagnostic (NAS_REHEARSE_WORLD=G with a one-rank communicator): shard
    // geometry of rank 0 of G, the other G-1 ranks' lists stood in for by
    // copies of this rank's shifted to their node ranges -- times one rank of
    // a G-GPU pass on a single GPU; placements are not meaningful
    int32_t rehearse = 0;
    bool virtual_shard = false;  // nas_set_shard: shard geometry, no exchange
    // in-process transport instead of RCCL (nas_comm_init_local): the group,
    // per channel (0 = scoring stream, 1 = scoring stream 2, 2 = commit
    // stream) the exchange count and two events per parity {send ready, copies
    // done}, and the peer devices this context already reads from
    std::shared_ptr<nas::LocalGroup> local;
    uint32_t lg_round[3] = {0, 0, 0};
    hipEvent_t lg_ev[3][2][2] = {};
    uint64_t lg_peers = 0;
    // nas_comm_init helper threads still inside RCCL after an abandoned init
    // (joined by the next nas_comm_init once finished, or by nas_destroy)
    std::vector<std::thread> comm_helpers;
    std::vector<std::shared_ptr<nas::CommInit>> comm_helper_state;
    // options (nas_set_option)
    bool opt_stage_timings = true;
    int64_t opt_comm_timeout_ms = 120000;
    int32_t opt_rehearse_world = 0;
    int64_t opt_inject_stall_ms = 0;
    int64_t opt_commit_wait_ms = 0;         // 0: automatic (NAS_OPT_COMMIT_WAIT_MS)
    int64_t opt_inject_commit_stall_ms = 0;
    int32_t opt_synth_profile = 0;          // NAS_OPT_SYNTH_PROFILE
    int32_t opt_commit_cus = 0;             // NAS_OPT_COMMIT_CUS (world 1)
    int32_t opt_cost_cache = 2;             // NAS_OPT_COST_CACHE: 0 off, 1 on, 2 auto
    int32_t opt_herd_plan = 2;              // NAS_OPT_HERD_PLAN: 0 off, 1 on, 2 auto
    int32_t herd_P = -1, herd_N = -1;       // auto: the shape whose passes run the herd plan
    bool poisoned = false;       // a collective missed its deadline: communicators aborted
    // timing events, created once and reused by every call (hipEventCreate
    // per mark cost a small placement more than its kernels)
    std::vector<hipEvent_t> ev_pool;
    hipEvent_t sync_ev = nullptr;  // sync_stream's event (created on first use)
    size_t ev_used = 0;
};

namespace nas {

// hipFuncSetAttribute(max dynamic LDS) once per kernel and device (the
// attribute is per device; contexts on several devices may share a process)
inline hipError_t set_lds_once(const void *fn, int bytes, std::atomic<unsigned long long> &done) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

int fail(nas_ctx *ctx, int code, const std::string &msg);
int hip_fail(nas_ctx *ctx, hipError_t e, const char *what);
int ensure(nas_ctx *ctx, DevBuf &b, size_t bytes);

// kernel launchers (k_*.hip); all enqueue on `stream` and return hipError_t
hipError_t launch_vote(hipStream_t st, const nas_ctx *c, int n_snapshots_used);
// per-pod order sets (nas_upload_pod_orders): pod p scores snapshot
// pod_snap[p] (device array) with order set p -> best[p], win[p][6]
hipError_t launch_vote_pods(hipStream_t st, const nas_ctx *c, const int32_t *pod_snap, int P,
                            int32_t *best, int32_t *win);
// node-shard form: partial records of the context's slice -> part[S]
hipError_t launch_vote_partial(hipStream_t st, const nas_ctx *c, int S, nas_vote_partial *part);
// merge parts[n_parts][S] -> best[S], win[S][6] with the context's orders
hipError_t launch_vote_merge(hipStream_t st, const nas_ctx *c, const nas_vote_partial *parts,
                             int n_parts, int S, int32_t *best, int32_t *win);
hipError_t launch_vote_gather(hipStream_t st, const int32_t *pod_snap, int P,
                              const int32_t *snap_best, const int32_t *snap_win, int32_t *best,
                              int32_t *win);

// A rescore slot's pod window, decided on the device: the kernels read the
// window start from *start (the commit's halt word; < 0 = nothing to do) and
// cover pods [start, min(start + win, hi)).  Grids are sized for `win`.
// Batched launches (batch > 1 independent clusters of equal shape, laid out
// back to back; the cluster index is a grid dimension) read cluster b's
// start at start[b * STATUS_INTS].
struct Dyn {
    const int32_t *start;
    int win;
    int hi;
    const int32_t *hi_ptr = nullptr;  // when set, hi is read on the device (per cluster)
};
constexpr int MERGE_SRC_WINDOW = 1;  // k_merge source lists indexed from the window start
constexpr int MERGE_DST_WINDOW = 2;  // k_merge destination indexed from the window start

// rowmap (gathered rescore view, batch 1): view row q is pod rowmap[q] -- its
// requests (k_fit, main array with row stride req_stride) and traffic row
// (k_cost_topk, main WA) are read in place, no gathered copy
hipError_t launch_fit(hipStream_t st, const int32_t *cap, int N, int n0, int nloc, int Mp,
                      const int32_t *req, int P, int Pp, int p0, int np, uint64_t *mask,
                      const Dyn *dyn = nullptr, int batch = 1, const int32_t *rowmap = nullptr,
                      int req_stride = 0);

// pods per tile of the wide cost kernel for this (compute) dtype when it is
// built in (384), else COST_BN
int cost_tile_pods(int dtype);
hipError_t launch_cost_topk(hipStream_t st, int dtype, const void *Lt, const void *WA, int Mp,
                            int Kp, int Pp, int p0, int np, const uint64_t *mask,
                            uint64_t *partial, uint64_t *pbound, int node_base,
                            const Dyn *dyn = nullptr, int batch = 1, const Ovf *ovf = nullptr,
                            const int32_t *rowmap = nullptr, bool wide = false,
                            const FitSrc *fit = nullptr, uint32_t *cache = nullptr);
// cache (main pod ranges only): every (pod, local node) cost of the launch as
// its orderable 32-bit key into cache[cluster][Pp][Mp] (the cost-row cache,
// rescored from by launch_rescore_cached)
hipError_t launch_merge(hipStream_t st, const uint64_t *keys, const uint64_t *bounds, int n_lists,
                        int64_t stride, int64_t bstride, int src_p0, int p0, int np,
                        uint64_t *cand_key, uint64_t *cand_bound, int dst_p0 = 0,
                        const Dyn *dyn = nullptr, int dyn_flags = 0, int batch = 1,
                        int64_t dst_cluster_pods = 0, const int32_t *dst_idx = nullptr,
                        int32_t *init_status = nullptr);
// the commit keeps the working capacity in LDS (and publishes only final
// values, at the end of each launch) for clusters of up to this many nodes
bool commit_in_lds(int N);
hipError_t launch_commit(hipStream_t st, const uint64_t *cand_key, const uint64_t *cand_bound,
                         const int32_t *req, int Pp, int p_begin, int p_end, int32_t *cap, int N,
                         int32_t *out_node, int32_t *out_cost_i, int32_t *halt, int batch = 1,
                         int32_t *pub = nullptr, const uint8_t *zrow = nullptr,
                         int32_t *stage_node = nullptr, int32_t *stage_cost = nullptr,
                         int32_t *stage_status = nullptr);
// stage_status (batch 1): after the walk the commit copies the status words
// status[0 .. COMMIT_STATUS_WORDS) there (pinned host memory)
constexpr int COMMIT_STATUS_WORDS = STATUS_INTS + 3;
// zrow[r] = 1 iff traffic row r (row_bytes bytes of WA) is all zero bytes and
// has no overflow entries (ovf_ptr may be null): the pod's every cost is 0
hipError_t launch_zero_rows(hipStream_t st, const void *WA, int64_t rows, int64_t row_bytes,
                            const int32_t *ovf_ptr, uint8_t *zrow);

// gathered rescore (k_rescore.hip)
int stale_words(int P);
// p0 < 0: the scan starts at the commit's halt word *p0_dev (nothing to do if
// it is < 0); ctl receives {window start (0, or -1 when no pod is dry),
// count, running total of rescored pods}
hipError_t launch_stale_scan(hipStream_t st, const uint64_t *key, const uint64_t *bound,
                             const int32_t *req, int Pp, const int32_t *cap, int N, int p0, int P,
                             uint64_t *words, int R, int32_t *idx, int32_t *ctl,
                             const int32_t *p0_dev = nullptr);
// one workgroup: the flagged pods among [*p0_dev, min(P, *p0_dev + W)), the
// first R of them, same ctl protocol (the herd plan's in-loop slots)
hipError_t launch_stale_window(hipStream_t st, const uint64_t *key, const uint64_t *bound,
                               const int32_t *req, int Pp, const int32_t *cap, int N, int P, int W,
                               int R, int32_t *idx, int32_t *ctl, const int32_t *p0_dev);

// rescore from the cost-row cache (cache[Pp][stride], this rank's nloc local
// nodes from global node n0): view row q < ctl[1] (nothing if ctl[0] < 0) is
// pod idx[q]; its 8-list + bound against the capacity now go to view row q
// (to_view) or to the pod's own slot p of key_out / bound_out
hipError_t launch_rescore_cached(hipStream_t st, const uint32_t *cache, int stride, int nloc,
                                 int n0, const int32_t *cap, int N, const int32_t *req, int Pp,
                                 const int32_t *idx, const int32_t *ctl, int R, uint64_t *key_out,
                                 uint64_t *bound_out, bool to_view);

// start of a nas_place pass: status[0] = -1 (halt), status[1 .. 2*STATUS_INTS)
// = 0; cap_snap[0, n) = cap[0, n) when cap_snap is non-null
// the commit order across the commit stream and the tail chunk's stream
// (k_misc.hip): flag_set stores v into *flag behind the stream's work so far,
// flag_wait holds the stream until *flag >= v, for at most budget_ms; on
// timeout it writes FLAG_TIMEOUT_HALT into *halt (an impossible halt word:
// halts are pod indices), which the pass reports as its own error
constexpr int32_t FLAG_TIMEOUT_HALT = 0x7ffffff0;
hipError_t launch_flag_set(hipStream_t st, uint64_t *flag, uint64_t v);
hipError_t launch_flag_wait(hipStream_t st, const uint64_t *flag, uint64_t v, int32_t *halt,
                            int64_t budget_ms);
// dst[0, n) = src[0, n) on st (16-byte moves when both are 16-byte aligned)
hipError_t launch_copy_i32(hipStream_t st, int32_t *dst, const int32_t *src, int64_t n);
hipError_t launch_pass_init(hipStream_t st, int32_t *status, const int32_t *cap, int32_t *cap_snap,
                            int n);
// rehearsal: rank slots 1..G-1 of an all-gathered buffer [G][n] of keys
// (or bounds) = slot 0 with node indices shifted to rank r's first node
// (r * N / G); ~0 stays
hipError_t launch_rehearse_replicate(hipStream_t st, uint64_t *buf, size_t n, int G, int N);
// in-process all-gather (nas_comm_init_local): dst[r * bytes ..] = srcs.p[r][0 .. bytes)
// for r < G (bytes a multiple of 8), on the receiving rank's stream
hipError_t launch_local_gather(hipStream_t st, const LocalSrcs &srcs, int G, void *dst,
                               size_t bytes);
hipError_t launch_transpose_L(hipStream_t st, const void *L_dev, int dtype, int N, int n0,
                              int nloc, int Mp, int Kp, void *Lt);
// bf16 CSR traffic -> dense WA rows (fp32 sums, rounded once)
hipError_t launch_csr_aggregate_bf16(hipStream_t st, const int32_t *row_ptr, const int32_t *peer,
                                     const uint16_t *w, int P, int N, int Kp, uint16_t *WA);
// fp32 rows WA[p][m] = v for host-aggregated (pod, node, value) triples
// fp32 operand -> six bf16 K-segments (pattern 0: latency h h m h l m,
// 1: traffic h m h l h m), rows of 6 * Kp elements (k_misc.hip k_split6)
hipError_t launch_split6(hipStream_t st, const float *src, uint16_t *dst, int64_t rows, int Kp,
                         int pattern);
hipError_t launch_scatter_f32(hipStream_t st, const int32_t *pod, const int32_t *node,
                              const float *val, int64_t n, int Kp, float *WA);
// int8 plane entries WA[p][m] = v for host-aggregated (pod, node, value) triples
hipError_t launch_plane_scatter(hipStream_t st, const int32_t *pod, const int32_t *node,
                                const signed char *val, int64_t n, int Kp, signed char *WA);
// Lr[m][i] = Lt[i][m] for m < N, i < Mp (one cluster)
hipError_t launch_make_lr(hipStream_t st, const signed char *Lt, int N, int Mp, int Kp,
                          signed char *Lr);
// *out = max(*out, max_r sum_k |WA[r][k]| + sum of |plane + e| - |plane| over r's overflow
// entries) for rows [0, rows): the exact sum_m |WA[p,m]| (out zeroed by the caller)
hipError_t launch_row_abs_max(hipStream_t st, const signed char *WA, int64_t rows, int Kp,
                              const int32_t *ovf_ptr, const int32_t *ovf_m, const int32_t *ovf_e,
                              unsigned long long *out);
// *out = max(*out, max |Lt|) (out zeroed by the caller)
hipError_t launch_abs_max_i8(hipStream_t st, const signed char *a, int64_t n, unsigned *out);
// a device-side delay of `ms` milliseconds on st (NAS_OPT_INJECT_STALL_MS)
hipError_t launch_stall(hipStream_t st, int64_t ms);

// nodes [lo, lo + nl) of an n-node synthetic snapshot set, row stride ns
hipError_t launch_synth_snapshots(hipStream_t st, uint64_t seed, int n, int lo, int nl,
                                  int64_t ns, int S, double *cpu, double *mem, double *bw,
                                  int64_t *rx, int64_t *tx, int64_t *disk);
hipError_t launch_synth_cluster(hipStream_t st, uint64_t seed, int N, int P, int dtype, int peers,
                                int n0, int nloc, int Mp, int Kp, int Pp, void *Lt, void *WA,
                                int32_t *cap, int32_t *req, void *L_full /* optional N*N */,
                                int profile /* NAS_OPT_SYNTH_PROFILE */);
// int8 synthetic traffic is exact: pass 0 writes the plane and ovf_cnt[p] (the
// entries of pod p outside [-128, 127]); pass 1 (after the host's prefix sum
// into ovf_ptr) writes the entries.  Peer aggregates are recomputed from the
// seed in both passes, so nothing else is kept between them.
hipError_t launch_synth_overflow(hipStream_t st, uint64_t seed, int N, int P, int peers, int Kp,
                                 int pass, const signed char *WA, int32_t *ovf_cnt,
                                 const int32_t *ovf_ptr, int32_t *ovf_m, int32_t *ovf_e);

}  // namespace nas
