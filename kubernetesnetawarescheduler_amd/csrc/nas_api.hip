// nas_api.hip -- C ABI (include/nas.h) of the MI355X placement engine:
// context, uploads into the HBM layouts of DESIGN.md, and the orchestration
// of fit -> cost/top-k -> merge -> (RCCL exchange) -> commit with the rescore
// loop.  Every entry re-binds the context's device and synchronises its
// stream before returning (blocking semantics of the Go call it replaces).
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <cstdlib>
#include <mutex>
#include <new>
#include <numeric>
#include <thread>
#include <vector>

#include "nas_internal.h"

using nas::DevBuf;
using nas::KC;

// roctx range around every C-ABI entry (rocprofv3 --marker-trace shows the
// host call that issued each kernel); a no-op call without a profiler
namespace {
struct RoctxRange {
    explicit RoctxRange(const char *name) { roctxRangePush(name); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange &) = delete;
    RoctxRange &operator=(const RoctxRange &) = delete;
};
}  // namespace
#define NAS_RANGE(name) const RoctxRange nas_range_(name)

namespace nas {

int fail(nas_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int hip_fail(nas_ctx *ctx, hipError_t e, const char *what) {
    return fail(ctx, NAS_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(nas_ctx *ctx, DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.p && b.bytes >= bytes) return NAS_OK;
    if (b.p) {
        (void)hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        b.p = nullptr;
        return fail(ctx, NAS_ERR_NOMEM,
                    "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    }
    b.bytes = bytes;
    return NAS_OK;
}

}  // namespace nas

#define HIPCK(expr)                                                  \
    do {                                                             \
        hipError_t e_ = (expr);                                      \
        if (e_ != hipSuccess) return nas::hip_fail(ctx, e_, #expr);  \
    } while (0)
#define OK(expr)                   \
    do {                           \
        int r_ = (expr);           \
        if (r_ != NAS_OK) return r_; \
    } while (0)

namespace {

constexpr int RESCORE_PODS = 1024;  // pods per device-side rescore slot (multiple of COST_BN)
// dry pods rescored per gathered slot (gathered_slot).  1024, not 4096: a
// bf16 C3 halt (the last chunk's lists, scored against capacity two chunks
// stale, run dry in a herd) flags > 4096 pods with STALE_MIN_FIT 2, but the
// first 1024 of them always let the walk finish -- the slot's cost launch
// 690 -> 235 us, the halting pass's slots 0.9 -> 0.37 ms (traced); 256 / 512
// need more slots (profiles/r04_ab_gather_pods.txt)
// (round 6: 6 tiles = 1,536 pods for C3 -- still one wave of cost workgroups
// over 40 node tiles -- took 65 instead of 89 slots through the full-range
// herd but 31.6 instead of 29.4 ms, same box: profiles/r06b_ab_slots.txt)
constexpr int GATHER_PODS = 1024;
// a pass with the cost-row cache rescores from cached rows (k_rescore_cached:
// no cost launch), so its slots take more pods
constexpr int GATHER_PODS_CACHED = 2048;
// NAS_OPT_COST_CACHE auto: the previous pass's rescore rounds that turn the
// cache on, and its largest size (C4 at world 1 would need 100 GB)
constexpr int CACHE_MIN_ROUNDS = 4;
constexpr size_t CACHE_MAX_BYTES = (size_t)16 << 30;
// NAS_OPT_HERD_PLAN auto: rescore rounds of one pass that make its shape a herd
constexpr int HERD_MIN_ROUNDS = 8;
// gathered slots behind each chunk's commit in the herd plan
constexpr int HERD_SLOTS = 1;
// ... of at most this many pods (they run on the CUs a chunk's wave leaves
// free, C3: 16, where a 2,048-pod rescore takes ~190 us; 512-pod slots
// measured no faster and less stable: profiles/r06e_ab_herd.txt)
constexpr int HERD_SLOT_PODS = 2048;
constexpr int GATHER_SLOTS_PER_SYNC = 4;  // gathered slots enqueued per host check of the halt word
constexpr int MAX_SPEC_SLOTS = 8;         // speculative slots at most (nas_place, slot_hint)
// ... except the second check: a walk still halted after a full batch is
// usually nearly done (C2: 5 slots), and an idle slot's ~8 launches cost about
// what one more host round trip does, so the second batch is one slot (C2
// median 1.17 / 1.07 / 1.04 ms with a second batch of 4 / 2 / 1, same
// placements).  With the cost-row cache (a herd; an idle slot is 3 launches)
// 8 slots per check from the fourth on
int gather_batch(int check, bool cached) {
    return check == 2 ? 1 : (cached && check > 3) ? 8 : GATHER_SLOTS_PER_SYNC;
}
int plan_n_mt(const nas_ctx *ctx);
// (a one-slot FIRST batch for walks halting near their end helped a 12-pod
// rescore, 0.39 -> 0.26 ms, but cost bench C1's 3-slot case two extra round
// trips, 0.39 -> 0.52 ms: with a round trip ~2 idle slots, 4 then 1 is the
// robust order)
// pinned staging of nas_place results in host_status: behind the status words
// of every cluster of a batch (B * STATUS_INTS ints; nas_set_batch allows up to
// 65535 clusters), page-aligned
size_t host_out_offset(int B) {
    const size_t status_bytes = (size_t)std::max(B, 1) * (nas::STATUS_INTS + 4) * 4;
    return std::max<size_t>(4096, (status_bytes + 4095) & ~(size_t)4095);
}
// Rescore slots run only for a walk known to have halted (after the
// pipeline): an idle gathered slot still costs ~0.1 ms of launches (C3,
// measured), more than the host round trip a stop costs once the pipeline is
// done -- the results fetch brings the halt word back with the placements --
// and scoring against the live capacity makes stops rare.

int bind(nas_ctx *ctx) {
    if (!ctx) return NAS_ERR_ARG;
    ctx->err.clear();
    if (ctx->poisoned)
        return nas::fail(ctx, NAS_ERR_COMM,
                         "context poisoned: a collective missed its deadline and the "
                         "communicators were aborted (destroy the context)");
    HIPCK(hipSetDevice(ctx->device));
    return NAS_OK;
}

size_t esz(int dtype) { return dtype == NAS_DT_I8 ? 1 : dtype == NAS_DT_F32 ? 4 : 2; }

// contraction length padded to whole 128-byte K-steps of the cost kernel
int64_t kpad(int n, int dtype) { return nas::round_up(n, 128 / (int)esz(dtype)); }

bool valid_dtype(int dtype) {
    return dtype == NAS_DT_I8 || dtype == NAS_DT_BF16 || dtype == NAS_DT_F32;
}

// event pool for per-stage device timing on the context stream
struct Timer {
    nas_ctx *ctx;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> spans;
    // events come from the context's pool (every call synchronises before it
    // returns, so the previous call's events are complete when reused)
    explicit Timer(nas_ctx *c) : ctx(c) { ctx->ev_used = 0; }
    ~Timer() { ctx->ev_used = 0; }
    hipEvent_t ev() {
        if (ctx->ev_used < ctx->ev_pool.size()) return ctx->ev_pool[ctx->ev_used++];
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        ctx->ev_pool.push_back(e);
        ctx->ev_used = ctx->ev_pool.size();
        return e;
    }
    hipEvent_t mark(hipStream_t st = nullptr) {
        hipEvent_t e = ev();
        if (e) (void)hipEventRecord(e, st ? st : ctx->stream);
        return e;
    }
    // a timing-only mark: none when stage timings are off
    // (NAS_OPT_STAGE_TIMINGS = 0), so the pass records only the events it
    // synchronises on
    hipEvent_t fine(hipStream_t st = nullptr) {
        return ctx->opt_stage_timings ? mark(st) : nullptr;
    }
    void span(int which, hipEvent_t a, hipEvent_t b) { spans.push_back({which, {a, b}}); }
    float total(int which) {
        float s = 0;
        for (auto &x : spans) {
            if (x.first != which || !x.second.first || !x.second.second) continue;
            float ms = 0;
            if (hipEventElapsedTime(&ms, x.second.first, x.second.second) == hipSuccess) s += ms;
        }
        return s;
    }
};
enum { T_FIT, T_COST, T_MERGE, T_COMMIT, T_VOTE, T_TOTAL };

int validate_perm(const int32_t *o, int n, std::vector<int32_t> &pos) {
    pos.assign(n, -1);
    for (int i = 0; i < n; ++i) {
        if (o[i] < 0 || o[i] >= n || pos[o[i]] != -1) return -1;
        pos[o[i]] = i;
    }
    return 0;
}

int upload_orders(nas_ctx *ctx, const int32_t *order1, const int32_t *order2, int32_t n_orders,
                  bool per_pod = false) {
    const int n = ctx->snap_n;
    if (n <= 0) return nas::fail(ctx, NAS_ERR_STATE, "upload a snapshot before its orders");
    if (!order1 || !order2 || n_orders <= 0) return nas::fail(ctx, NAS_ERR_ARG, "orders");
    const int64_t ns = nas::round_up(n, 2), ns2 = ns + 2;
    std::vector<int32_t> o1((size_t)n_orders * ns, 0), p1((size_t)n_orders * ns, 0);
    std::vector<int32_t> o2((size_t)n_orders * ns2, 0), p2((size_t)n_orders * ns2, 0);
    std::vector<int32_t> pos;
    for (int o = 0; o < n_orders; ++o) {
        const int32_t *a = order1 + (size_t)o * n;
        if (validate_perm(a, n, pos))
            return nas::fail(ctx, NAS_ERR_ARG, "order1 set " + std::to_string(o) + " is not a permutation");
        std::copy(a, a + n, o1.begin() + (size_t)o * ns);
        std::copy(pos.begin(), pos.end(), p1.begin() + (size_t)o * ns);
        const int32_t *b = order2 + (size_t)o * (n + 1);
        if (validate_perm(b, n + 1, pos))
            return nas::fail(ctx, NAS_ERR_ARG, "order2 set " + std::to_string(o) + " is not a permutation");
        std::copy(b, b + n + 1, o2.begin() + (size_t)o * ns2);
        std::copy(pos.begin(), pos.end(), p2.begin() + (size_t)o * ns2);
    }
    OK(nas::ensure(ctx, ctx->order1, o1.size() * 4));
    OK(nas::ensure(ctx, ctx->pos1, p1.size() * 4));
    OK(nas::ensure(ctx, ctx->order2, o2.size() * 4));
    OK(nas::ensure(ctx, ctx->pos2, p2.size() * 4));
    HIPCK(hipMemcpyAsync(ctx->order1.p, o1.data(), o1.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipMemcpyAsync(ctx->pos1.p, p1.data(), p1.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipMemcpyAsync(ctx->order2.p, o2.data(), o2.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipMemcpyAsync(ctx->pos2.p, p2.data(), p2.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));  // host vectors die here
    ctx->n_orders = n_orders;
    ctx->orders_per_pod = per_pod;
    ctx->ord_ns = ns;
    return NAS_OK;
}

// shard geometry of the extended mode for n nodes / dtype
void set_geometry(nas_ctx *ctx, int n, int dtype) {
    ctx->N = n;
    ctx->dtype = dtype;
    ctx->Kp = (int32_t)kpad(n, dtype);
    const int64_t a = (int64_t)ctx->rank * n / ctx->world;
    const int64_t b = (int64_t)(ctx->rank + 1) * n / ctx->world;
    ctx->Nloc0 = (int32_t)a;
    ctx->Nloc = (int32_t)(b - a);
    ctx->Mp = (int32_t)nas::round_up(std::max<int64_t>(ctx->Nloc, 1), nas::COST_BM);
}

// ---- exact int32 traffic on the int8 path (nas::Ovf, nas_internal.h)

// overflow lists of every pod row: ptr[B * Pp + 1] absolute offsets, entries
// (node, excess); none -> ovf_n = 0 and the plane is the traffic
int upload_ovf(nas_ctx *ctx, const std::vector<int32_t> &ptr, const std::vector<int32_t> &m,
               const std::vector<int32_t> &e) {
    ctx->ovf_n = (int64_t)m.size();
    if (m.empty()) return NAS_OK;
    OK(nas::ensure(ctx, ctx->ovf_ptr, ptr.size() * 4));
    OK(nas::ensure(ctx, ctx->ovf_m, m.size() * 4));
    OK(nas::ensure(ctx, ctx->ovf_e, e.size() * 4));
    HIPCK(hipMemcpyAsync(ctx->ovf_ptr.p, ptr.data(), ptr.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipMemcpyAsync(ctx->ovf_m.p, m.data(), m.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipMemcpyAsync(ctx->ovf_e.p, e.data(), e.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));  // host vectors die with the caller
    return NAS_OK;
}

// after the plane and the lists are on the device: the largest sum_m |WA[p,m]|
// over pods, for the int32 range check of check_extended
int finish_traffic_i8(nas_ctx *ctx) {
    OK(nas::ensure(ctx, ctx->scratch, 64));
    auto *mx = ctx->scratch.as<unsigned long long>();
    HIPCK(hipMemsetAsync(mx, 0, 8, ctx->stream));
    const bool o = ctx->ovf_n > 0;
    HIPCK(nas::launch_row_abs_max(ctx->stream, ctx->WA.as<signed char>(), (int64_t)ctx->B * ctx->Pp,
                                  ctx->Kp, o ? ctx->ovf_ptr.as<int32_t>() : nullptr,
                                  o ? ctx->ovf_m.as<int32_t>() : nullptr,
                                  o ? ctx->ovf_e.as<int32_t>() : nullptr, mx));
    unsigned long long h = 0;
    HIPCK(hipMemcpyAsync(&h, mx, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    ctx->wa_abs_row_max = (int64_t)h;
    return NAS_OK;
}

// the epilogue's view of the lists (no entries -> ptr null, the kernel skips it)
nas::Ovf make_ovf(const nas_ctx *ctx, const int32_t *row_pod = nullptr,
                  const int32_t *row_count = nullptr) {
    nas::Ovf o;
    if (ctx->dtype != NAS_DT_I8 || ctx->ovf_n == 0) return o;
    o.ptr = ctx->ovf_ptr.as<int32_t>();
    o.m = ctx->ovf_m.as<int32_t>();
    o.e = ctx->ovf_e.as<int32_t>();
    o.Lr = ctx->Lr.as<signed char>();
    o.row_pod = row_pod;
    o.row_count = row_count;
    o.N = ctx->N;
    return o;
}

// Lr (row-major latency columns for the epilogue's correction), built from Lt
// on the main stream when lists exist and the latency changed
int prepare_ovf(nas_ctx *ctx) {
    if (ctx->dtype != NAS_DT_I8 || ctx->ovf_n == 0 || ctx->lr_valid) return NAS_OK;
    const size_t per = (size_t)ctx->N * ctx->Mp;
    OK(nas::ensure(ctx, ctx->Lr, per * ctx->B));
    for (int b = 0; b < ctx->B; ++b)
        HIPCK(nas::launch_make_lr(ctx->stream, ctx->Lt.as<signed char>() + (size_t)b * ctx->Mp * ctx->Kp,
                                  ctx->N, ctx->Mp, ctx->Kp, ctx->Lr.as<signed char>() + b * per));
    ctx->lr_valid = true;
    return NAS_OK;
}

// zero-traffic pods (k_commit.hip's scan past an exhausted list), once per
// traffic upload, on the main stream like the other per-upload preparations
int prepare_zrow(nas_ctx *ctx) {
    if (ctx->zrow_valid) return NAS_OK;
    const int64_t rows = (int64_t)ctx->B * ctx->Pp;
    OK(nas::ensure(ctx, ctx->zrow, (size_t)rows));
    HIPCK(nas::launch_zero_rows(ctx->stream, ctx->WA.p, rows, (int64_t)ctx->Kp * esz(ctx->dtype),
                                ctx->ovf_n ? ctx->ovf_ptr.as<int32_t>() : nullptr,
                                ctx->zrow.as<uint8_t>()));
    ctx->zrow_valid = true;
    return NAS_OK;
}

// the commit's zero-traffic flags, or nullptr when 0 x L may not be 0
// (a float latency matrix holding Inf / NaN)
const uint8_t *zrow_ptr(const nas_ctx *ctx) {
    if (!ctx->zrow_valid || (ctx->dtype != NAS_DT_I8 && !ctx->L_finite)) return nullptr;
    return ctx->zrow.as<uint8_t>();
}

// NAS_DT_F32 scores on the bf16 MFMA: both operands split into six K-segments
// of bf16 planes (k_misc.hip k_split6), once per upload; every cost launch
// then runs the bf16 kernel over K' = 6 Kp (launch_cost below)
int prepare_split(nas_ctx *ctx) {
    if (ctx->dtype != NAS_DT_F32 || ctx->split_valid) return NAS_OK;
    const int64_t lrows = (int64_t)ctx->B * ctx->Mp, wrows = (int64_t)ctx->B * ctx->Pp;
    OK(nas::ensure(ctx, ctx->Lt6, (size_t)lrows * 6 * ctx->Kp * 2));
    OK(nas::ensure(ctx, ctx->WA6, (size_t)(wrows + nas::WA_PAD_ROWS) * 6 * ctx->Kp * 2));
    HIPCK(nas::launch_split6(ctx->stream, ctx->Lt.as<float>(), ctx->Lt6.as<uint16_t>(), lrows,
                             ctx->Kp, 0));
    HIPCK(nas::launch_split6(ctx->stream, ctx->WA.as<float>(), ctx->WA6.as<uint16_t>(), wrows,
                             ctx->Kp, 1));
    ctx->split_valid = true;
    return NAS_OK;
}

// one cost/top-k launch over the main traffic rows (or a row-mapped view)
// The wide cost tile (256 nodes x 384 pods, 12 waves) for the main scoring
// pass of one whole cluster with many pods (full launch 3.5% (int8) / 6%
// (bf16) faster than 256 x 256: profiles/r02_s4_ab_wide*.txt), for batches of
// clusters (C5: launch frac 0.42 -> 0.45 although a 5,000-pod cluster is
// 13.02 wide tiles, profiles/r04_ab_narrow_fit_wide.txt) and for node shards,
// there together with CU-masked streams (below; the wide tile alone lost on
// shards in round 2: longer workgroups, coarser tails).  Small clusters,
// rescore windows and row-mapped views keep 256 x 256.
constexpr int WIDE_MIN_PODS = 32768;
// On a node shard (world > 1) the scoring streams leave RESERVE_SHARD_CUS
// CUs per XCD to the commit stream (set_stream_masks), so the merge /
// exchange / commit chain runs beside the wide cost tile instead of waiting
// for one of its workgroups to drain (profiles/r04_ab_reserve.txt)
constexpr int RESERVE_SHARD_CUS = 2;  // per XCD; 3 from 4 ranks, 4 from 8 (shard_reserve)
bool wide_ok(const nas_ctx *ctx) {
    const bool shard = ctx->world > 1 || ctx->rehearse > 1;
    if (ctx->B > 1) return !shard;
    return ctx->Pp >= WIDE_MIN_PODS || shard;
}
int tile_pods(const nas_ctx *ctx) {
    return wide_ok(ctx) ? nas::cost_tile_pods(ctx->dtype == NAS_DT_F32 ? NAS_DT_BF16 : ctx->dtype)
                        : nas::COST_BN;
}

// A launch over a main pod range (no rescore window, no row map) decides the
// fit itself from `fit` (k_cost.hip: fused fit), so no k_fit launch sits
// between two cost launches of a scoring stream; windows keep the k_fit mask.
hipError_t launch_cost(nas_ctx *ctx, hipStream_t st, int Pp, int p0, int np, const uint64_t *mask,
                       const nas::Dyn *dyn, int batch, const nas::Ovf *ov,
                       const int32_t *rowmap = nullptr, const nas::FitSrc *fit = nullptr,
                       bool narrow = false, uint32_t *cache = nullptr) {
    const bool wide = !narrow && wide_ok(ctx);
    if (ctx->dtype == NAS_DT_F32)
        return nas::launch_cost_topk(st, NAS_DT_BF16, ctx->Lt6.p, ctx->WA6.p, ctx->Mp, 6 * ctx->Kp,
                                     Pp, p0, np, mask, ctx->partial.as<uint64_t>(),
                                     ctx->pbound.as<uint64_t>(), ctx->Nloc0, dyn, batch, nullptr,
                                     rowmap, wide, fit, cache);
    return nas::launch_cost_topk(st, ctx->dtype, ctx->Lt.p, ctx->WA.p, ctx->Mp, ctx->Kp, Pp, p0, np,
                                 mask, ctx->partial.as<uint64_t>(), ctx->pbound.as<uint64_t>(),
                                 ctx->Nloc0, dyn, batch, ov, rowmap, wide, fit, cache);
}

// exact traffic row (n values, each within int32) -> the int8 plane row and
// the row's overflow entries (node, excess)
void split_row(const int64_t *v, int n, signed char *plane, std::vector<int32_t> &m,
               std::vector<int32_t> &e) {
    for (int j = 0; j < n; ++j) {
        const int64_t x = v[j];
        const int64_t c = x < -128 ? -128 : x > 127 ? 127 : x;
        plane[j] = (signed char)c;
        if (x != c) {
            m.push_back(j);
            e.push_back((int32_t)(x - c));
        }
    }
}

// the call issued collectives other ranks must join (waits get deadlines)
bool has_coll(const nas_ctx *ctx) { return ctx->comm != nullptr || ctx->local != nullptr; }
int set_stream_masks(nas_ctx *ctx, int reserve);  // (multi-GPU section)

int check_extended(nas_ctx *ctx) {
    if (!ctx->have_L || !ctx->have_cap || !ctx->have_pods || !ctx->have_wa)
        return nas::fail(ctx, NAS_ERR_STATE,
                         "nas_place needs latency, capacity, pods and traffic uploaded");
    if (ctx->L_n != ctx->cap_n || ctx->L_n != ctx->wa_n)
        return nas::fail(ctx, NAS_ERR_ARG, "node counts of latency / capacity / traffic differ");
    if (ctx->req_P != ctx->wa_P)
        return nas::fail(ctx, NAS_ERR_ARG, "pod counts of requests / traffic differ");
    if (ctx->L_dtype != ctx->wa_dtype)
        return nas::fail(ctx, NAS_ERR_ARG, "dtypes of latency / traffic differ");
    if (ctx->N != ctx->L_n || ctx->P != ctx->req_P || ctx->dtype != ctx->L_dtype)
        return nas::fail(ctx, NAS_ERR_STATE, "re-upload latency and traffic after resizing");
    if (ctx->world > 1 && !has_coll(ctx) && !ctx->virtual_shard)
        return nas::fail(ctx, NAS_ERR_STATE, "node shard without a communicator");
    // int8 path: exact int32 costs need sum_m |WA[p,m]| * |L[m,n]| <= INT32_MAX
    if (ctx->dtype == NAS_DT_I8 && ctx->wa_abs_row_max * (int64_t)ctx->L_abs_max > 0x7fffffffLL)
        return nas::fail(ctx, NAS_ERR_UNSUPPORTED,
                         "int8 path: a pod's sum_m |WA[p,m]| * max|L| = " +
                             std::to_string(ctx->wa_abs_row_max) + " * " +
                             std::to_string(ctx->L_abs_max) + " exceeds int32");
    return NAS_OK;
}

void abort_comms(nas_ctx *ctx);

// The communicators are NON-blocking (nas_comm_init): a collective may return
// ncclInProgress while RCCL finishes enqueueing it (e.g. a lazy connection
// set-up); poll the communicator until it is enqueued, under the same
// NAS_OPT_COMM_TIMEOUT_MS deadline as the waits (abort + poison on expiry).
int nccl_enqueued(nas_ctx *ctx, ncclComm *cm, ncclResult_t r, const char *what) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    while (r == ncclInProgress) {
        ncclResult_t a = ncclInProgress;
        const ncclResult_t q = ncclCommGetAsyncError(reinterpret_cast<ncclComm_t>(cm), &a);
        r = q != ncclSuccess ? q : a;
        if (r != ncclInProgress) break;
        if (ctx->opt_comm_timeout_ms > 0 &&
            clk::now() - t0 > std::chrono::milliseconds(ctx->opt_comm_timeout_ms)) {
            abort_comms(ctx);
            return nas::fail(ctx, NAS_ERR_COMM,
                             std::string(what) + " was not enqueued within " +
                                 std::to_string(ctx->opt_comm_timeout_ms) +
                                 " ms (NAS_OPT_COMM_TIMEOUT_MS): communicators aborted, "
                                 "context poisoned");
        }
        // spin (yield) for the first ms: a sleep costs ~60-80 us of timer
        // slack per poll, on the pass's critical path when the enqueue of a
        // chunk's all-gather is what the commit stream waits for
        if (clk::now() - t0 < std::chrono::milliseconds(1)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (r != ncclSuccess)
        return nas::fail(ctx, NAS_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
    return NAS_OK;
}

// ---- collectives: RCCL (nas_comm_init) or the in-process transport
// (nas_comm_init_local).  A channel is the stream family that issues them --
// each keeps its own issue order on every rank: CH_SCORE (ctx->stream and
// scoring stream 1), CH_SCORE2 (scoring stream 2), CH_COMMIT (the commit
// stream and the pass's chunk merges).
enum { CH_SCORE = 0, CH_SCORE2 = 1, CH_COMMIT = 2 };

ncclComm *chan_comm(const nas_ctx *ctx, int ch) {
    return ch == CH_SCORE2 ? ctx->comm2 : ch == CH_COMMIT ? ctx->comm_c : ctx->comm;
}

// a communicator exchanges even at world 1 (nas_comm_init with world 1
// builds one: the whole RCCL path on a single GPU, all-gather = copy)
bool exchanging(const nas_ctx *ctx) { return has_coll(ctx) && !ctx->virtual_shard; }

}  // namespace

// The in-process group: one rendezvous per channel.  An exchange is two
// host-side barriers.  (1) Every rank records "send ready" on its stream and
// posts {send buffers, event}; after the barrier each rank makes its stream
// wait for every peer's event and PULLS all ranks' buffers into its receive
// buffer with one k_local_gather launch per segment.  (2) Every rank records
// "copies done" and posts it; after the barrier each stream waits for every
// peer's copies, so no rank overwrites a send buffer a peer still reads (the
// completion guarantee an RCCL all-gather gives its caller).  Every stream
// wait is enqueued after the event it waits on was recorded (the barriers),
// so streams sharing a hardware queue cannot deadlock.  Events alternate by
// exchange parity: a rank re-records a parity only after every peer passed the
// next exchange's first barrier, i.e. finished waiting on it.  A barrier that
// misses NAS_OPT_COMM_TIMEOUT_MS breaks the group: every rank's pending and
// later exchanges fail with NAS_ERR_COMM.
struct nas::LocalGroup {
    struct Seg {
        const void *send = nullptr;
        size_t bytes = 0;
    };
    struct Post {
        Seg seg[2];
        int nseg = 0;
        hipEvent_t ev = nullptr;
        int device = 0;
    };
    struct Chan {
        uint64_t gen = 0;
        int arrived = 0;
        std::vector<Post> send, done;
    };
    explicit LocalGroup(int w) : world(w), joined(w, false) {
        for (Chan &c : ch) {
            c.send.resize(w);
            c.done.resize(w);
        }
    }
    const int world;
    std::mutex mu;
    std::condition_variable cv;
    bool broken = false;
    std::vector<bool> joined;
    Chan ch[3];

    // under lk; false: timed out or broken (the group is then broken)
    bool barrier(Chan &c, std::unique_lock<std::mutex> &lk, int64_t timeout_ms) {
        if (broken) return false;
        const uint64_t gen = c.gen;
        if (++c.arrived == world) {
            c.arrived = 0;
            ++c.gen;
            cv.notify_all();
            return true;
        }
        auto passed = [&] { return c.gen != gen || broken; };
        if (timeout_ms > 0) {
            if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), passed)) broken = true;
        } else {
            cv.wait(lk, passed);
        }
        if (c.gen != gen) return true;
        broken = true;
        cv.notify_all();
        return false;
    }
    void break_group() {
        std::lock_guard<std::mutex> g(mu);
        broken = true;
        cv.notify_all();
    }
};

struct nas_local_group {
    std::shared_ptr<nas::LocalGroup> g;
};

namespace {

struct GatherSeg {
    const void *send;
    void *recv;
    size_t bytes;  // per rank; recv holds world * bytes, rank-major
};

void abort_comms(nas_ctx *ctx);

int local_fail(nas_ctx *ctx, const std::string &what) {
    abort_comms(ctx);
    return nas::fail(ctx, NAS_ERR_COMM,
                     what + " (in-process group): a rank did not join within " +
                         std::to_string(ctx->opt_comm_timeout_ms) +
                         " ms (NAS_OPT_COMM_TIMEOUT_MS) or the group is broken; context poisoned");
}

int local_allgather(nas_ctx *ctx, int ch, hipStream_t st, const GatherSeg *segs, int nseg,
                    const char *what) {
    nas::LocalGroup &g = *ctx->local;
    const int G = g.world, me = ctx->rank;
    const int par = (int)(ctx->lg_round[ch]++ & 1);
    hipEvent_t ready = ctx->lg_ev[ch][par][0], copied = ctx->lg_ev[ch][par][1];
    HIPCK(hipEventRecord(ready, st));
    std::vector<nas::LocalGroup::Post> peers;
    nas::LocalGroup::Chan &c = g.ch[ch];
    {
        std::unique_lock<std::mutex> lk(g.mu);
        nas::LocalGroup::Post &p = c.send[me];
        p.nseg = nseg;
        for (int s = 0; s < nseg; ++s) p.seg[s] = {segs[s].send, segs[s].bytes};
        p.ev = ready;
        p.device = ctx->device;
        if (!g.barrier(c, lk, ctx->opt_comm_timeout_ms)) {
            lk.unlock();
            return local_fail(ctx, what);
        }
        peers = c.send;
    }
    for (int j = 0; j < G; ++j) {
        bool same = peers[j].nseg == nseg;
        for (int s = 0; same && s < nseg; ++s) same = peers[j].seg[s].bytes == segs[s].bytes;
        if (!same) {
            g.break_group();
            return local_fail(ctx, std::string(what) + ": ranks issued different exchanges");
        }
        if (j == me) continue;
        HIPCK(hipStreamWaitEvent(st, peers[j].ev, 0));
        const int pd = peers[j].device;
        if (pd != ctx->device && !(ctx->lg_peers >> (pd & 63) & 1)) {
            const hipError_t e = hipDeviceEnablePeerAccess(pd, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                return nas::hip_fail(ctx, e, "hipDeviceEnablePeerAccess");
            (void)hipGetLastError();
            ctx->lg_peers |= 1ull << (pd & 63);
        }
    }
    for (int s = 0; s < nseg; ++s) {
        nas::LocalSrcs src{};
        for (int j = 0; j < G; ++j) src.p[j] = peers[j].seg[s].send;
        HIPCK(nas::launch_local_gather(st, src, G, segs[s].recv, segs[s].bytes));
    }
    HIPCK(hipEventRecord(copied, st));
    {
        std::unique_lock<std::mutex> lk(g.mu);
        c.done[me].ev = copied;
        if (!g.barrier(c, lk, ctx->opt_comm_timeout_ms)) {
            lk.unlock();
            return local_fail(ctx, what);
        }
        peers = c.done;
    }
    for (int j = 0; j < G; ++j)
        if (j != me) HIPCK(hipStreamWaitEvent(st, peers[j].ev, 0));
    return NAS_OK;
}

// all-gather of nseg (<= 2) segments on channel ch, stream st: each rank's
// segs[s].send (bytes each, a multiple of 8) into segs[s].recv [world][bytes]
int allgather(nas_ctx *ctx, int ch, hipStream_t st, const GatherSeg *segs, int nseg,
              const char *what) {
    if (ctx->local) return local_allgather(ctx, ch, st, segs, nseg, what);
    ncclComm *cm = chan_comm(ctx, ch);
    auto comm = reinterpret_cast<ncclComm_t>(cm);
    ncclResult_t r = nseg > 1 ? ncclGroupStart() : ncclSuccess;
    for (int s = 0; s < nseg && r == ncclSuccess; ++s)
        r = ncclAllGather(segs[s].send, segs[s].recv, segs[s].bytes / 8, ncclUint64, comm, st);
    if (nseg > 1) {
        const ncclResult_t r2 = ncclGroupEnd();
        if (r == ncclSuccess) r = r2;
    }
    return nccl_enqueued(ctx, cm, r, what);
}

// all-gather each rank's per-pod lists (keys [np][KC] + bounds [np]) into
// gk [world][np][KC] / gb [world][np] on `st` over channel ch
int exchange(nas_ctx *ctx, int ch, hipStream_t st, const uint64_t *keys, const uint64_t *bounds,
             size_t np, uint64_t *gk, uint64_t *gb) {
    const GatherSeg segs[2] = {{keys, gk, np * KC * 8}, {bounds, gb, np * 8}};
    OK(allgather(ctx, ch, st, segs, 2, "ncclAllGather"));
    if (ctx->rehearse > 1) {
        HIPCK(nas::launch_rehearse_replicate(st, gk, np * KC, ctx->rehearse, ctx->N));
        HIPCK(nas::launch_rehearse_replicate(st, gb, np, ctx->rehearse, ctx->N));
    }
    return NAS_OK;
}

// The pod arrays a scoring pass reads and writes: the context's own, or the
// gathered scratch view of a rescore (k_rescore.hip) with its own row stride.
struct PodView {
    const void *WA;
    const int32_t *req;
    int Pp;  // row stride of req / mask / partial lists
    uint64_t *key, *bound;
};

PodView main_view(nas_ctx *ctx) {
    return {ctx->WA.p, ctx->req.as<int32_t>(), ctx->Pp, ctx->cand_key.as<uint64_t>(),
            ctx->cand_bound.as<uint64_t>()};
}

// merge of pods [p_lo, p_hi)'s node-tile lists (-> exchange over `cm` and
// merge across ranks), on stream st behind their cost launch; gbuf picks the
// gathered-list scratch (one per stream that exchanges)
int merge_range(nas_ctx *ctx, Timer &tm, int p_lo, int p_hi, hipStream_t st, int ch,
                int gbuf, const PodView &v, int32_t *init_status = nullptr) {
    const int pr0 = p_lo / nas::COST_BN * nas::COST_BN;
    const int pr1 = (int)nas::round_up(p_hi, nas::COST_BN);
    const int np = pr1 - pr0;
    hipEvent_t e2 = tm.fine(st);
    const int n_lists = ctx->Mp / nas::COST_BM;
    if (!exchanging(ctx)) {
        HIPCK(nas::launch_merge(st, ctx->partial.as<uint64_t>(), ctx->pbound.as<uint64_t>(),
                                n_lists, (int64_t)v.Pp * KC, v.Pp, 0, p_lo, p_hi - p_lo, v.key,
                                v.bound, 0, nullptr, 0, 1, 0, nullptr, init_status));
    } else {
        if (init_status) return nas::fail(ctx, NAS_ERR_STATE, "status init rides a local merge only");
        // this rank's lists of pods [pr0, pr1) go straight into one send
        // buffer ([np][8] keys, then [np] bounds), so one all-gather moves
        // them; the cross-rank merge reads the rank-major result in place
        const size_t seg = (size_t)np * (KC + 1);
        OK(nas::ensure(ctx, ctx->xsend[gbuf], seg * 8));
        auto *xs = ctx->xsend[gbuf].as<uint64_t>();
        auto *gx = ctx->gather[gbuf].as<uint64_t>();
        HIPCK(nas::launch_merge(st, ctx->partial.as<uint64_t>(), ctx->pbound.as<uint64_t>(),
                                n_lists, (int64_t)v.Pp * KC, v.Pp, 0, p_lo, p_hi - p_lo, xs,
                                xs + (size_t)np * KC, pr0));
        const GatherSeg g1{xs, gx, seg * 8};
        OK(allgather(ctx, ch, st, &g1, 1, "ncclAllGather"));
        if (ctx->rehearse > 1)
            HIPCK(nas::launch_rehearse_replicate(st, gx, seg, ctx->rehearse, ctx->N));
        HIPCK(nas::launch_merge(st, gx, gx + (size_t)np * KC, ctx->world, (int64_t)seg,
                                (int64_t)seg, pr0, p_lo, p_hi - p_lo, v.key, v.bound));
    }
    tm.span(T_MERGE, e2, tm.fine(st));
    return NAS_OK;
}

// scoring for pods [p_lo, p_hi) on stream st against capacity `cap`:
// fit -> cost/top-k, then (merge = true) merge_range on the same stream over
// the stream's communicator
int score_range(nas_ctx *ctx, Timer &tm, int p_lo, int p_hi, hipStream_t st = nullptr,
                const int32_t *cap = nullptr, const PodView *view = nullptr, bool merge = true) {
    if (!st) st = ctx->stream;
    if (!cap) cap = ctx->cap.as<int32_t>();
    const PodView v = view ? *view : main_view(ctx);
    const int sidx = st == ctx->stream2 ? 1 : 0;
    const int pr0 = p_lo / nas::COST_BN * nas::COST_BN;
    const int pr1 = (int)nas::round_up(p_hi, nas::COST_BN);
    const int np = pr1 - pr0;
    auto *mask = ctx->mask.as<uint64_t>();
    // the cost launch decides the fit itself (fused fit): no k_fit before it.
    // Node shards fuse too since they run the wide tile on CU-masked streams
    // (round 4): the commit stream's merge / exchange / commit kernels have
    // CUs of their own, so the k_fit launch between two cost launches is no
    // longer needed as a gap for them (with the 256 x 256 tile and unmasked
    // streams each of them had waited ~100 us for a cost workgroup to drain:
    // profiles/r03_g8_timeline_before.txt, r03_ab_fuse_shard.txt)
    const bool fuse = ctx->world == 1 || wide_ok(ctx);
    const nas::FitSrc fit{cap, v.req, ctx->N, ctx->Nloc0, ctx->Nloc};
    hipEvent_t e0 = tm.fine(st);
    if (!fuse)
        HIPCK(nas::launch_fit(st, cap, ctx->N, ctx->Nloc0, ctx->Nloc, ctx->Mp, v.req, p_hi, v.Pp,
                              p_lo, p_hi - p_lo, mask));
    hipEvent_t e1 = fuse ? e0 : tm.fine(st);
    const nas::Ovf ov = make_ovf(ctx);
    // (a pass with the cost-row cache: the main launches store every cost too)
    uint32_t *cache = ctx->cache_active && !view ? ctx->cost_cache.as<uint32_t>() : nullptr;
    HIPCK(launch_cost(ctx, st, v.Pp, pr0, np, mask, nullptr, 1, &ov, nullptr, fuse ? &fit : nullptr,
                      false, cache));
    hipEvent_t e2 = tm.fine(st);
    tm.span(T_FIT, e0, e1);
    tm.span(T_COST, e1, e2);
    ctx->timings.cost_launches += 1;
    if (merge) OK(merge_range(ctx, tm, p_lo, p_hi, st, sidx ? CH_SCORE2 : CH_SCORE, sidx, v));
    return NAS_OK;
}

// Gathered rescore slot, all on the device (k_rescore.hip): if the commit walk
// has halted (halt word >= 0), every pending pod in [halt, hi) whose list is
// dry against the capacity now -- up to R of them (GATHER_PODS), in pod order, the
// halted pod first -- is copied into a scratch view, scored there by the
// ordinary fit / cost / merge kernels (+ the exchange across ranks), its list
// written back, and the walk resumed from the halt.  Nothing halted: every
// kernel exits at once (the exchange still runs, so all ranks issue the same
// collectives).  Slots need no host round trip, so a crowded cluster's many
// stops cost launches, not synchronisations.
int gathered_slot(nas_ctx *ctx, Timer &tm, hipStream_t st, int ch, int32_t *pub, int hi,
                  int r_max = 0) {
    const int R = std::min({ctx->cache_active ? GATHER_PODS_CACHED : GATHER_PODS, ctx->Pp,
                            r_max > 0 ? r_max : ctx->Pp});
    OK(nas::ensure(ctx, ctx->g_words, (size_t)nas::stale_words(ctx->Pp) * 8));
    OK(nas::ensure(ctx, ctx->g_idx, (size_t)R * 4));
    OK(nas::ensure(ctx, ctx->g_key, (size_t)R * KC * 8));
    OK(nas::ensure(ctx, ctx->g_bound, (size_t)R * 8));
    int32_t *halt = ctx->status.as<int32_t>();
    int32_t *ctl = halt + nas::STATUS_INTS;  // {view start, count, rescored total}
    int32_t *idx = ctx->g_idx.as<int32_t>();
    auto *gk = ctx->g_key.as<uint64_t>();
    auto *gb = ctx->g_bound.as<uint64_t>();
    hipEvent_t e0 = tm.fine(st);
    // (a bounded slot -- the herd plan's, beside a cost wave -- scans a window
    // of 2R pods from the halt in one workgroup: no release fences)
    if (r_max > 0)
        HIPCK(nas::launch_stale_window(st, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                                       ctx->req.as<int32_t>(), ctx->Pp, ctx->cap.as<int32_t>(),
                                       ctx->N, hi, 2 * R, R, idx, ctl, halt));
    else
        HIPCK(nas::launch_stale_scan(st, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                                     ctx->req.as<int32_t>(), ctx->Pp, ctx->cap.as<int32_t>(), ctx->N,
                                     -1, hi, ctx->g_words.as<uint64_t>(), R, idx, ctl, halt));
    const bool xch = exchanging(ctx);
    auto *ck = ctx->cand_key.as<uint64_t>();
    auto *cbnd = ctx->cand_bound.as<uint64_t>();
    if (ctx->cache_active) {
        // the pods' costs are in the cost-row cache: each view row's list from
        // its cached row against the capacity now (k_rescore_cached), straight
        // into the pod's own slot -- or into the view rows for the exchange
        hipEvent_t e1 = tm.fine(st);
        HIPCK(nas::launch_rescore_cached(st, ctx->cost_cache.as<uint32_t>(), ctx->Mp, ctx->Nloc,
                                         ctx->Nloc0, ctx->cap.as<int32_t>(), ctx->N,
                                         ctx->req.as<int32_t>(), ctx->Pp, idx, ctl, R,
                                         xch ? gk : ck, xch ? gb : cbnd, xch));
        hipEvent_t e3 = tm.fine(st);
        nas::Dyn dyn{ctl, R, 0, ctl + 1};
        if (xch) {
            OK(nas::ensure(ctx, ctx->g_gk, (size_t)ctx->world * R * KC * 8));
            OK(nas::ensure(ctx, ctx->g_gb, (size_t)ctx->world * R * 8));
            auto *xk = ctx->g_gk.as<uint64_t>();
            auto *xb = ctx->g_gb.as<uint64_t>();
            OK(exchange(ctx, ch, st, gk, gb, (size_t)R, xk, xb));
            HIPCK(nas::launch_merge(st, xk, xb, ctx->world, (int64_t)R * KC, R, 0, 0, 0, ck, cbnd, 0,
                                    &dyn, 0, 1, 0, idx));
        }
        hipEvent_t e4 = tm.fine(st);
        HIPCK(nas::launch_commit(st, ck, cbnd, ctx->req.as<int32_t>(), ctx->Pp, -1, hi,
                                 ctx->cap.as<int32_t>(), ctx->N, ctx->out_node.as<int32_t>(),
                                 ctx->out_cost_i.as<int32_t>(), halt, 1, pub, zrow_ptr(ctx)));
        tm.span(T_COST, e1, e3);
        tm.span(T_MERGE, e3, e4);
        tm.span(T_COMMIT, e0, e1);
        tm.span(T_COMMIT, e4, tm.fine(st));
        return NAS_OK;
    }
    nas::Dyn dyn{ctl, R, 0, ctl + 1};
    auto *mask = ctx->mask.as<uint64_t>();
    hipEvent_t e1 = tm.fine(st);
    HIPCK(nas::launch_fit(st, ctx->cap.as<int32_t>(), ctx->N, ctx->Nloc0, ctx->Nloc, ctx->Mp,
                          ctx->req.as<int32_t>(), R, R, 0, R, mask, &dyn, 1, idx, ctx->Pp));
    hipEvent_t e2 = tm.fine(st);
    const nas::Ovf ov = make_ovf(ctx, idx, ctl + 1);  // view row r is pod idx[r]
    HIPCK(launch_cost(ctx, st, R, 0, 0, mask, &dyn, 1, &ov, idx));
    hipEvent_t e3 = tm.fine(st);
    const int n_lists = ctx->Mp / nas::COST_BM;
    // the last merge writes the fresh lists straight into the pods' own list
    // slots (idx); with an exchange, the local merge first fills the view
    HIPCK(nas::launch_merge(st, ctx->partial.as<uint64_t>(), ctx->pbound.as<uint64_t>(), n_lists,
                            (int64_t)R * KC, R, 0, 0, 0, xch ? gk : ck, xch ? gb : cbnd, 0, &dyn,
                            0, 1, 0, xch ? nullptr : idx));
    if (xch) {
        OK(nas::ensure(ctx, ctx->g_gk, (size_t)ctx->world * R * KC * 8));
        OK(nas::ensure(ctx, ctx->g_gb, (size_t)ctx->world * R * 8));
        auto *xk = ctx->g_gk.as<uint64_t>();
        auto *xb = ctx->g_gb.as<uint64_t>();
        OK(exchange(ctx, ch, st, gk, gb, (size_t)R, xk, xb));
        HIPCK(nas::launch_merge(st, xk, xb, ctx->world, (int64_t)R * KC, R, 0, 0, 0, ck, cbnd, 0,
                                &dyn, 0, 1, 0, idx));
    }
    hipEvent_t e4 = tm.fine(st);
    HIPCK(nas::launch_commit(st, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                             ctx->req.as<int32_t>(), ctx->Pp, -1, hi, ctx->cap.as<int32_t>(),
                             ctx->N, ctx->out_node.as<int32_t>(), ctx->out_cost_i.as<int32_t>(),
                             halt, 1, pub, zrow_ptr(ctx)));
    tm.span(T_FIT, e1, e2);
    tm.span(T_COST, e2, e3);
    tm.span(T_MERGE, e3, e4);
    tm.span(T_COMMIT, e0, e1);
    tm.span(T_COMMIT, e4, tm.fine(st));
    return NAS_OK;
}

float decode_cost(uint32_t raw, int dtype);
void unpack_range(int32_t *__restrict__ node_out, float *__restrict__ cost_out,
                  int64_t *__restrict__ int_score_out, const int32_t *__restrict__ from,
                  const int32_t *__restrict__ raw_in, int lo, int hi, int dtype, int &unsched);

int no_batch(nas_ctx *ctx, const char *what) {
    if (ctx->B > 1)
        return nas::fail(ctx, NAS_ERR_UNSUPPORTED, std::string(what) + " with a cluster batch");
    return NAS_OK;
}

// A rescore slot on the commit stream, enqueued behind a chunk's commit: if
// the walk halted at pod s (halt word), rescore pods [s, min(s + RESCORE_PODS,
// hi)) against the working capacity and resume the walk from s to hi; if it
// did not halt, every kernel exits at once (the exchange still runs, so all
// ranks issue the same collectives).  Every pod of [s, hi) belongs to chunks
// whose scoring the commit stream has already waited for: no other stream
// touches their masks, partial lists or candidate lists.
int rescore_slot(nas_ctx *ctx, hipStream_t sc, int hi, int32_t *pub = nullptr) {
    int32_t *halt = ctx->status.as<int32_t>();
    const nas::Dyn dyn{halt, RESCORE_PODS, hi};
    const int B = ctx->B;  // batched: every cluster with a stop gets its own window
    auto *mask = ctx->mask.as<uint64_t>();
    HIPCK(nas::launch_fit(sc, ctx->cap.as<int32_t>(), ctx->N, ctx->Nloc0, ctx->Nloc, ctx->Mp,
                          ctx->req.as<int32_t>(), ctx->P, ctx->Pp, 0, RESCORE_PODS, mask, &dyn, B));
    const nas::Ovf ov = make_ovf(ctx);
    HIPCK(launch_cost(ctx, sc, ctx->Pp, 0, 0, mask, &dyn, B, &ov));
    const int n_lists = ctx->Mp / nas::COST_BM;
    if (!exchanging(ctx)) {
        HIPCK(nas::launch_merge(sc, ctx->partial.as<uint64_t>(), ctx->pbound.as<uint64_t>(),
                                n_lists, (int64_t)ctx->Pp * KC, ctx->Pp, 0, 0, 0,
                                ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(), 0,
                                &dyn, 0, B, ctx->Pp));
    } else {
        auto *rk = ctx->resc_key.as<uint64_t>();
        auto *rb = ctx->resc_bound.as<uint64_t>();
        auto *gk = ctx->gather_r.as<uint64_t>();
        auto *gb = ctx->gbound_r.as<uint64_t>();
        HIPCK(nas::launch_merge(sc, ctx->partial.as<uint64_t>(), ctx->pbound.as<uint64_t>(),
                                n_lists, (int64_t)ctx->Pp * KC, ctx->Pp, 0, 0, 0, rk, rb, 0, &dyn,
                                nas::MERGE_DST_WINDOW));
        OK(exchange(ctx, CH_COMMIT, sc, rk, rb, RESCORE_PODS, gk, gb));
        HIPCK(nas::launch_merge(sc, gk, gb, ctx->world, (int64_t)RESCORE_PODS * KC, RESCORE_PODS,
                                0, 0, 0, ctx->cand_key.as<uint64_t>(),
                                ctx->cand_bound.as<uint64_t>(), 0, &dyn, nas::MERGE_SRC_WINDOW));
    }
    HIPCK(nas::launch_commit(sc, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                             ctx->req.as<int32_t>(), ctx->Pp, -1, hi, ctx->cap.as<int32_t>(),
                             ctx->N, ctx->out_node.as<int32_t>(), ctx->out_cost_i.as<int32_t>(),
                             halt, B, pub, zrow_ptr(ctx)));
    return NAS_OK;
}

// Scoring pass over every cluster of a batch: one cost/top-k launch (with
// the fused fit) and one merge launch, against the working capacity (cluster
// = a grid dimension).
int score_batch(nas_ctx *ctx, Timer &tm) {
    hipStream_t st = ctx->stream;
    const int B = ctx->B, P = ctx->P, Pp = ctx->Pp, N = ctx->N;
    auto *mask = ctx->mask.as<uint64_t>();
    hipEvent_t e0 = tm.mark(st);
    hipEvent_t e1 = e0;
    const nas::Ovf ov = make_ovf(ctx);
    const nas::FitSrc fit{ctx->cap.as<int32_t>(), ctx->req.as<int32_t>(), N, 0, N};
    // whole wide tiles (384 pods) over the pods a multiple of 768 (a launch
    // covers 256-pod units) reaches, 256 x 256 tiles over the rest: C5's 5,000
    // pods (Pp 5,120) are 12 wide + 2 narrow tiles per cluster instead of 14
    // wide ones, the last of them 8 pods of 384
    const int W = tile_pods(ctx) != nas::COST_BN ? Pp / 768 * 768 : 0;
    if (W > 0) HIPCK(launch_cost(ctx, st, Pp, 0, W, mask, nullptr, B, &ov, nullptr, &fit));
    if (W < Pp) HIPCK(launch_cost(ctx, st, Pp, W, Pp - W, mask, nullptr, B, &ov, nullptr, &fit, true));
    hipEvent_t e2 = tm.mark(st);
    const int n_lists = ctx->Mp / nas::COST_BM;
    HIPCK(nas::launch_merge(st, ctx->partial.as<uint64_t>(), ctx->pbound.as<uint64_t>(), n_lists,
                            (int64_t)Pp * KC, Pp, 0, 0, P, ctx->cand_key.as<uint64_t>(),
                            ctx->cand_bound.as<uint64_t>(), 0, nullptr, 0, B, Pp));
    tm.span(T_FIT, e0, e1);
    tm.span(T_COST, e1, e2);
    tm.span(T_MERGE, e2, tm.mark(st));
    ctx->timings.cost_launches += 1;
    return NAS_OK;
}

// Batched placement (B > 1 independent clusters): one fit / cost / merge
// launch covers every cluster (cluster = a grid dimension), one commit
// workgroup per cluster walks them in parallel, and batched rescore slots
// serve every cluster's stop at once until none is left.
int place_batch(nas_ctx *ctx, Timer &tm, int32_t *node_out, float *cost_out,
                int64_t *int_score_out) {
    hipStream_t st = ctx->stream;
    const int B = ctx->B, P = ctx->P, Pp = ctx->Pp, N = ctx->N;
    int32_t *halt = ctx->status.as<int32_t>();
    int32_t *hs = ctx->host_status.as<int32_t>();
    hipEvent_t t0 = tm.mark(st);
    for (int b = 0; b < B; ++b) {
        hs[b * nas::STATUS_INTS] = -1;
        for (int j = 1; j < nas::STATUS_INTS; ++j) hs[b * nas::STATUS_INTS + j] = 0;
    }
    HIPCK(hipMemcpyAsync(halt, hs, (size_t)B * nas::STATUS_INTS * 4, hipMemcpyHostToDevice, st));
    OK(score_batch(ctx, tm));
    hipEvent_t e3 = tm.mark(st);
    // every cluster's placements (and raw scores) go to the pinned stage from
    // the commit kernel itself, before the status words: when no cluster
    // stopped, the one status round trip brings the results with it
    int32_t *stage = reinterpret_cast<int32_t *>(ctx->host_status.as<char>() + host_out_offset(ctx->B));
    const size_t BP = (size_t)B * P;
    const bool want_raw = cost_out || int_score_out;
    HIPCK(nas::launch_commit(st, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                             ctx->req.as<int32_t>(), Pp, 0, P, ctx->cap.as<int32_t>(), N,
                             ctx->out_node.as<int32_t>(), ctx->out_cost_i.as<int32_t>(), halt, B,
                             nullptr, zrow_ptr(ctx), stage, want_raw ? stage + BP : nullptr));
    tm.span(T_COMMIT, e3, tm.mark(st));
    auto fetch = [&]() -> int {
        HIPCK(hipMemcpy2DAsync(stage, (size_t)P * 4, ctx->out_node.p, (size_t)Pp * 4,
                               (size_t)P * 4, B, hipMemcpyDeviceToHost, st));
        if (want_raw)
            HIPCK(hipMemcpy2DAsync(stage + BP, (size_t)P * 4, ctx->out_cost_i.p, (size_t)Pp * 4,
                                   (size_t)P * 4, B, hipMemcpyDeviceToHost, st));
        return NAS_OK;
    };
    hipEvent_t t1 = tm.mark(st);
    int slots = 0;
    while (true) {
        HIPCK(hipMemcpyAsync(hs, halt, (size_t)B * nas::STATUS_INTS * 4, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        bool any = false;
        for (int b = 0; b < B; ++b) {
            const int h = hs[b * nas::STATUS_INTS];
            if (h >= P) return nas::fail(ctx, NAS_ERR_HIP, "commit halt word corrupt");
            any |= h >= 0;
        }
        if (!any) break;
        if (++slots > P + 1) return nas::fail(ctx, NAS_ERR_HIP, "commit made no progress");
        hipEvent_t c0 = tm.mark(st);
        OK(rescore_slot(ctx, st, P));
        tm.span(T_COMMIT, c0, tm.mark(st));
        ctx->timings.cost_launches += 1;
    }
    if (slots > 0) {  // the walk moved on after the speculative copies
        OK(fetch());
        t1 = tm.mark(st);
        HIPCK(hipStreamSynchronize(st));
    }
    tm.span(T_TOTAL, t0, t1);
    int unsched = 0, dev_rounds = 0, rounds = 0;
    for (int b = 0; b < B; ++b) {
        dev_rounds += hs[b * nas::STATUS_INTS + 1];
        rounds += hs[b * nas::STATUS_INTS + 2];
    }
    unpack_range(node_out, cost_out, int_score_out, stage, stage + BP, 0, (int)BP, ctx->dtype, unsched);
    ctx->timings.fit_ms = tm.total(T_FIT);
    ctx->timings.cost_ms = tm.total(T_COST);
    ctx->timings.merge_ms = tm.total(T_MERGE);
    ctx->timings.commit_ms = tm.total(T_COMMIT);
    ctx->timings.total_ms = tm.total(T_TOTAL);
    ctx->timings.rescore_rounds = dev_rounds;
    ctx->timings.unschedulable = unsched;
    ctx->timings.commit_rounds = rounds;
    ctx->scored = true;
    return NAS_OK;
}

// Abort every communicator of a context whose collective missed its deadline:
// the stuck collective kernels return, later calls fail fast (bind).
void abort_comms(nas_ctx *ctx) {
    for (ncclComm **c : {&ctx->comm, &ctx->comm2, &ctx->comm_c, &ctx->comm_root}) {
        if (*c) (void)ncclCommAbort(reinterpret_cast<ncclComm_t>(*c));
        *c = nullptr;
    }
    // in-process group: every peer's pending and later exchanges fail too
    if (ctx->local) ctx->local->break_group();
    ctx->poisoned = true;
}

// Wait for an event.  Without a communicator: hipEventSynchronize.  With one
// (the call issued collectives that other ranks must join), poll under the
// NAS_OPT_COMM_TIMEOUT_MS deadline -- a rank whose peers never arrive would
// otherwise block in the collective forever -- and on expiry abort the
// communicators and poison the context.  (Polling measured equal to the
// blocking wait on the G = 8 rehearsal: 1.38-1.41 ms per pass either way.)
// The host waits by polling the event (WAIT_SPIN_MS, then a blocking wait):
// past its active-wait window the runtime's own wait sleeps on an interrupt,
// and the wake-up lands on the pass's critical path at its last event (the
// host unpacks each chunk as it lands, so only the last wait is exposed)
// (each host thread that waits spins on its core for up to WAIT_SPIN_MS:
// an in-process group of G ranks, one thread each, keeps G cores busy
// during a pass -- INTEGRATION.md, threading)
constexpr int WAIT_SPIN_MS = 20;
int wait_event(nas_ctx *ctx, hipEvent_t e) {
    if (!has_coll(ctx) || ctx->opt_comm_timeout_ms <= 0) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        while (clk::now() - t0 < std::chrono::milliseconds(WAIT_SPIN_MS)) {
            const hipError_t r = hipEventQuery(e);
            if (r == hipSuccess) return NAS_OK;
            if (r != hipErrorNotReady) return nas::hip_fail(ctx, r, "hipEventQuery");
            __builtin_ia32_pause();
        }
        HIPCK(hipEventSynchronize(e));
        return NAS_OK;
    }
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto limit = std::chrono::milliseconds(ctx->opt_comm_timeout_ms);
    for (;;) {
        const hipError_t r = hipEventQuery(e);
        if (r == hipSuccess) return NAS_OK;
        if (r != hipErrorNotReady) return nas::hip_fail(ctx, r, "hipEventQuery");
        const auto waited = clk::now() - t0;
        if (waited > limit) {
            abort_comms(ctx);
            return nas::fail(ctx, NAS_ERR_COMM,
                             "collective did not complete within " +
                                 std::to_string(ctx->opt_comm_timeout_ms) +
                                 " ms (NAS_OPT_COMM_TIMEOUT_MS): communicators aborted, "
                                 "context poisoned");
        }
        if (waited < std::chrono::milliseconds(2)) __builtin_ia32_pause();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// stream synchronisation through wait_event (the spin, and the deadline of
// calls that may have issued collectives), on the context's own event
// (created once, destroyed by nas_destroy)
int sync_stream(nas_ctx *ctx, hipStream_t st) {
    if (!ctx->sync_ev) HIPCK(hipEventCreateWithFlags(&ctx->sync_ev, hipEventDisableTiming));
    const hipError_t r = hipEventRecord(ctx->sync_ev, st);
    return r == hipSuccess ? wait_event(ctx, ctx->sync_ev) : nas::hip_fail(ctx, r, "hipEventRecord");
}

// NAS_OPT_INJECT_STALL_MS (tests): delay the stream a call waits on, once,
// behind the call's collectives (so the abort it provokes finds them done)
void inject_stall(nas_ctx *ctx, hipStream_t st) {
    if (ctx->opt_inject_stall_ms > 0) {
        (void)nas::launch_stall(st, ctx->opt_inject_stall_ms);
        ctx->opt_inject_stall_ms = 0;
    }
}

// pods per pipelined scoring chunk starting at pod lo: at least 32 pod
// tiles, and enough tiles that one chunk's cost launch has ~512 workgroups on
// this rank's node tiles (node shards have few node tiles).  The first chunk
// is 32 tiles, so the commit stream starts early, and the last is at most
// about 32, so the commit left after the scoring ends (the serial tail, which
// matters most on a node shard's short scoring) is short.
constexpr int CHUNK_WORKGROUPS = 512;  // cost workgroups per big chunk (measured best)
// a node shard's chunks after the first, on shards of up to
// SHARD_CHUNKS_MAX_MT node tiles (C3 from G = 4 on)
constexpr int SHARD_CHUNKS = 6;
constexpr int SHARD_CHUNKS_MAX_MT = 10;
// 256-pod units per chunk on the wide tile: 32 tiles of 384 (1,280 workgroups
// at 40 node tiles, as the 256-pod form's 32-unit chunks); 24 / 33 units
// measured 0.5-2% slower (profiles/r02_s4_ab_chunk.txt)
constexpr int CHUNK_TILES_WIDE = 48;
// node tiles per rank for chunk planning: the LARGEST shard's, the same on
// every rank (rank shards differ by up to one node, so their own Mp can
// differ by a tile, e.g. 2,049 nodes over 8 ranks: 256 vs 257 nodes); every
// rank must plan the same chunks, or their per-chunk all-gathers mismatch
int plan_n_mt(const nas_ctx *ctx) {
    const int64_t widest = ((int64_t)ctx->N + ctx->world - 1) / ctx->world;
    return (int)(nas::round_up(std::max<int64_t>(widest, 1), nas::COST_BM) / nas::COST_BM);
}

int chunk_pods(const nas_ctx *ctx, int c, int lo) {
    const int wgs = CHUNK_WORKGROUPS;
    const int n_mt = plan_n_mt(ctx);
    const int big = std::max(32, (wgs + n_mt - 1) / n_mt);
    // 32-tile chunks (whole waves of workgroups at 8+ node tiles) with a
    // short last one; when the workgroup target sets the size (a node shard
    // with few node tiles), equal chunks: on rank 0 of a G = 8 rehearsal
    // 1.45 ms vs 1.56 ms per C3 pass, while at G = 1 the 32-tile form is
    // 2.5% ahead (8.15 vs 8.37 ms)
    const int mode = big > 32 ? 2 : 0;
    const int left = (ctx->P - lo + nas::COST_BN - 1) / nas::COST_BN;  // pod tiles left
    int tiles = c == 0 ? 32 : big;
    // (one cluster, G = 1) the wide tile's chunks: the first chunk of the
    // second scoring stream is half as long, so the two streams' chunk
    // boundaries stay half a chunk apart -- a stream's next chunk waits for
    // its previous one to complete, and while that drains its last round the
    // other stream still has undispatched workgroups to fill the CUs (with
    // equal chunks both streams drained together: ~20 us of idle CUs per
    // chunk pair in the C3 pass timeline)
    if (tile_pods(ctx) != nas::COST_BN && ctx->world == 1)
        tiles = c == 1 ? CHUNK_TILES_WIDE / 2 : CHUNK_TILES_WIDE;
    // a pass whose pods fit one big chunk (C2: 40 pod tiles on 4 node tiles)
    // is one chunk: pipelining its short tail would save less than the
    // cross-stream hops and launches it adds (device time 0.96 -> 0.92 ms, C2)
    if (c == 0 && left <= big) tiles = left;
    if (mode == 0) {
        // a big last chunk is split in two so that the last is 32 tiles (unless
        // the first part would be a sliver of under 16)
        if (c > 0 && left > 32 && left <= big && left - 32 >= 16) tiles = left - 32;
    } else if (mode == 2 && c > 0) {
        // the rest in equal chunks: SHARD_CHUNKS of them (counting from
        // chunk 1; fewer when a chunk would drop below 32 units) on shards of
        // up to SHARD_CHUNKS_MAX_MT node tiles, else of at most `big` tiles
        // (~512 workgroups).  Six measured best on the C3 rehearsal: G = 8
        // 1.213 vs 1.227 ms, G = 4 2.105 vs 2.174 ms, but G = 3 (14 node
        // tiles, 560-workgroup chunks) 2.850 vs 2.812 ms; three to seven
        // swept (profiles/r05ab_ab_shard_chunks.txt).  (A short last chunk of
        // 16 / 32 tiles, to shorten the commit left after the scoring,
        // measured 7-13% slower at G = 8 and 2-3% at G = 4: one more chunk
        // costs more cross-stream hops than its shorter commit saves)
        //  the six-way split is capped at 2 x `big` tiles per chunk
        // (~1,024 workgroups), so a much larger P keeps chunks -- and the
        // serial merge / exchange / commit of the tail chunk after the
        // scoring -- bounded instead of growing linearly with P; C3's plans
        // are unchanged (G = 4: 60-tile chunks under a 104-tile cap, G = 8:
        // 60 under 206)
        const int n = n_mt <= SHARD_CHUNKS_MAX_MT
                          ? std::max({1, std::min(SHARD_CHUNKS - c + 1, left / 32),
                                      (left + 2 * big - 1) / (2 * big)})
                          : (left + big - 1) / big;
        tiles = (left + n - 1) / n;
    }  // (decreasing chunk sizes n, n-1, ..., 1 measured 7-10% slower at G = 4 / 8)
    // whole cost tiles per chunk: the wide tile (384 pods) needs multiples of
    // 3 units, or a chunk's last tile would score pods of the next chunk
    const int unit = tile_pods(ctx) / std::gcd(tile_pods(ctx), nas::COST_BN);
    tiles = std::min(left, (tiles + unit - 1) / unit * unit);
    return tiles * nas::COST_BN;
}

// The pass's scoring chunks [lo, hi) in pod order; chunk c runs on scoring
// stream c & 1.  On the wide tile (one cluster, G = 1) the two streams'
// totals are balanced at the end: the remainder after the 48-unit chunks is
// split over one last chunk per stream, sized so that both streams carry the
// same number of units and finish together (with the last chunks alternating
// as before, the stream that drew the first full chunk carried ~37 more wide
// tiles of 261 at C3, and ran alone -- one partial wave of idle CUs per
// chunk -- for the last ~1.4 ms of the scoring: profiles/r03_pass_timeline_c3_*.txt,
// r03_ab_balance_ksweep.txt)
// Node shards keep equal chunks (chunk_pods mode 2): the balanced plan put
// two chunk chains in the pass's tail and measured 4-8% slower at G = 8 and
// 1% at G = 4 (profiles/r03_ab_chunk_plan_shard.txt).  Putting the half-length
// chunk first (chunks then finish in pod order) measured the same or 0.5%
// slower, and so did moving units from a stream's short last chunk to its
// previous one (r03_ab_chunk_order.txt).
std::vector<std::pair<int, int>> plan_chunks(const nas_ctx *ctx, bool herd = false) {
    std::vector<std::pair<int, int>> chunks;
    const int P = ctx->P;
    const bool wide = tile_pods(ctx) != nas::COST_BN && ctx->world == 1;
    if (herd) {
        // the herd plan's chunks (nas_place): ONE wave of cost workgroups
        // each -- as many pod tiles as the CUs hold beside this rank's node
        // tiles (C3: 6 wide tiles = 2,304 pods over 40 node tiles = 240
        // workgroups), so the commit stream keeps the CUs left over -- and at
        // most ~1.25 pods per node (a chunk's own pods compete for the nodes
        // its fit saw free; tools/herd_model.py: 0 slots at 3,072 pods per
        // chunk, 5 at 6,144, 18 at 12,288 for 36,864 pods over 10k nodes)
        const int tp = tile_pods(ctx);
        int tiles = std::min(ctx->n_cu / std::max(plan_n_mt(ctx), 1),
                             std::max(1, (int)((5LL * ctx->N / 4) / tp)));
        if (tp != nas::COST_BN) tiles = std::max(2, tiles / 2 * 2);  // whole 256-pod units
        tiles = std::max(tiles, 1);
        const int step = tiles * tp;
        for (int lo = 0; lo < P; lo += step) chunks.push_back({lo, std::min(P, lo + step)});
        return chunks;
    }
    if (!wide) {
        for (int c = 0, lo = 0; lo < P; ++c) {
            const int hi = std::min(P, lo + chunk_pods(ctx, c, lo));
            chunks.push_back({lo, hi});
            lo = hi;
        }
        return chunks;
    }
    const int unit = tile_pods(ctx) / std::gcd(tile_pods(ctx), nas::COST_BN);  // wide: 3 (256-pod units)
    const int total = (P + nas::COST_BN - 1) / nas::COST_BN;                   // 256-pod units
    std::vector<int> sizes;
    int load[2] = {0, 0}, left = total;
    auto take = [&](int u) {
        u = std::min(left, (u + unit - 1) / unit * unit);
        sizes.push_back(u);
        load[(sizes.size() - 1) & 1] += u;
        left -= u;
    };
    // 48-unit chunks, the second stream's first one half as long
    const int big = CHUNK_TILES_WIDE;
    if (left <= big) {
        take(left);
    } else {
        take(big);
        take(big / 2);
        while (left > 0) {
            // can the rest end as one chunk on the next stream s and one on
            // the other, both at most `big`, with equal stream totals?
            const int s = sizes.size() & 1;
            const int x = std::max(0, (left + load[s ^ 1] - load[s]) / 2) / unit * unit;
            if (x >= unit && x <= big && left - x <= big) {
                take(x);
                if (left > 0) take(left);
                break;
            }
            if (x < unit && left <= big) {  // stream s is ahead: one last chunk
                take(left);
                break;
            }
            take(big);
        }
    }
    for (int lo = 0, i = 0; i < (int)sizes.size(); ++i) {
        const int hi = std::min(P, lo + sizes[i] * nas::COST_BN);
        chunks.push_back({lo, hi});
        lo = hi;
    }
    return chunks;
}

int alloc_extended(nas_ctx *ctx) {
    const size_t chunks = ctx->Mp / 64, B = ctx->B;
    OK(nas::ensure(ctx, ctx->mask, B * chunks * ctx->Pp * 8));
    OK(nas::ensure(ctx, ctx->partial, B * (ctx->Mp / nas::COST_BM) * ctx->Pp * KC * 8));
    OK(nas::ensure(ctx, ctx->pbound, B * (ctx->Mp / nas::COST_BM) * ctx->Pp * 8));
    OK(nas::ensure(ctx, ctx->cand_key, B * ctx->Pp * KC * 8));
    OK(nas::ensure(ctx, ctx->cand_bound, B * ctx->Pp * 8));
    OK(nas::ensure(ctx, ctx->out_node, B * ctx->Pp * 4));
    OK(nas::ensure(ctx, ctx->out_cost_i, B * ctx->Pp * 4));
    OK(nas::ensure(ctx, ctx->status, std::max<size_t>(256, B * nas::STATUS_INTS * 4)));
    OK(nas::ensure(ctx, ctx->cap_snap, (size_t)3 * ctx->N * 4));
    if (!ctx->commit_flag.p) {
        OK(nas::ensure(ctx, ctx->commit_flag, 8));
        HIPCK(hipMemset(ctx->commit_flag.p, 0, 8));
        ctx->commit_seq = 0;
    }
    if (exchanging(ctx)) {
        for (int i = 0; i < 3; ++i) {
            OK(nas::ensure(ctx, ctx->gather[i], (size_t)ctx->world * ctx->Pp * (KC + 1) * 8));
            OK(nas::ensure(ctx, ctx->gbound[i], (size_t)ctx->world * ctx->Pp * 8));
        }
        OK(nas::ensure(ctx, ctx->resc_key, (size_t)RESCORE_PODS * KC * 8));
        OK(nas::ensure(ctx, ctx->resc_bound, (size_t)RESCORE_PODS * 8));
        OK(nas::ensure(ctx, ctx->gather_r, (size_t)ctx->world * RESCORE_PODS * KC * 8));
        OK(nas::ensure(ctx, ctx->gbound_r, (size_t)ctx->world * RESCORE_PODS * 8));
    }
    // pinned: the status words, then (from host_out_offset(B)) a staging area
    // for the placements and scores so their copies back are DMA, not staged,
    // and a second one for nas_place's speculative full copy (below)
    const size_t hs_bytes = host_out_offset((int)B) + 4 * B * (size_t)ctx->Pp * 4;
    if (ctx->host_status.bytes < hs_bytes) {
        if (ctx->host_status.p) (void)hipHostFree(ctx->host_status.p);
        ctx->host_status.p = nullptr;
        ctx->host_status.bytes = 0;
        HIPCK(hipHostMalloc(&ctx->host_status.p, hs_bytes, hipHostMallocDefault));
        ctx->host_status.bytes = hs_bytes;
    }
    return NAS_OK;
}

void unpack_range(int32_t *__restrict__ node_out, float *__restrict__ cost_out,
                  int64_t *__restrict__ int_score_out, const int32_t *__restrict__ from,
                  const int32_t *__restrict__ raw_in, int lo, int hi, int dtype, int &unsched) {
    const uint32_t *__restrict__ raw = reinterpret_cast<const uint32_t *>(raw_in);
    int none = 0;
    if (dtype == NAS_DT_I8 && cost_out && int_score_out) {
        // the common case in one pass over the stage (host-memory bound:
        // 24 B per pod; 0.24 vs 0.49 ms per 100k pods for the per-pod loop
        // with the dtype test and a possibly aliased counter inside)
        for (int i = lo; i < hi; ++i) {
            const int32_t n = from[i];
            const int32_t v = (int32_t)(raw[i] ^ 0x80000000u);
            const bool z = n < 0;
            node_out[i] = n;
            none += z;
            cost_out[i] = z ? 0.f : (float)v;
            int_score_out[i] = z ? 0 : (int64_t)v;
        }
        unsched += none;
        return;
    }
    std::memcpy(node_out + lo, from + lo, (size_t)(hi - lo) * 4);
    for (int i = lo; i < hi; ++i) none += from[i] < 0;
    unsched += none;
    if (cost_out)
        for (int i = lo; i < hi; ++i) cost_out[i] = from[i] < 0 ? 0.f : decode_cost(raw[i], dtype);
    if (int_score_out) {
        if (dtype == NAS_DT_I8) {
            for (int i = lo; i < hi; ++i)
                int_score_out[i] = from[i] < 0 ? 0 : (int64_t)(int32_t)(raw[i] ^ 0x80000000u);
        } else {
            std::memset(int_score_out + lo, 0, (size_t)(hi - lo) * 8);
        }
    }
}

float decode_cost(uint32_t raw, int dtype) {
    if (dtype == NAS_DT_I8) return (float)(int32_t)(raw ^ 0x80000000u);
    const uint32_t u = (raw & 0x80000000u) ? (raw & 0x7fffffffu) : ~raw;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

void destroy_comms(nas_ctx *ctx) {
    // non-blocking communicators: finalize (flush, in RCCL's async job), poll
    // it to completion, then destroy; a finalize that fails or does not
    // finish within 10 s -- one deadline for all three, so peers that already
    // exited cost 10 s, not 30 -- is aborted instead (local, no peer
    // handshake); a poisoned context (a collective missed its deadline)
    // aborts at once
    const auto limit = std::chrono::steady_clock::now() + std::chrono::seconds(10);
    for (ncclComm **c : {&ctx->comm, &ctx->comm2, &ctx->comm_c}) {
        if (!*c) continue;
        auto comm = reinterpret_cast<ncclComm_t>(*c);
        ncclResult_t r = ctx->poisoned ? ncclInvalidUsage : ncclCommFinalize(comm);
        while (r == ncclInProgress && std::chrono::steady_clock::now() < limit) {
            ncclResult_t a = ncclInProgress;
            const ncclResult_t q = ncclCommGetAsyncError(comm, &a);
            r = q != ncclSuccess ? q : a;
            if (r == ncclInProgress) std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        if (r == ncclSuccess) (void)ncclCommDestroy(comm);
        else (void)ncclCommAbort(comm);
        *c = nullptr;
    }
    // the non-blocking root issued no collectives and owns nothing the
    // children use (no splitShare): aborting it needs no peer
    if (ctx->comm_root) (void)ncclCommAbort(reinterpret_cast<ncclComm_t>(ctx->comm_root));
    ctx->comm_root = nullptr;
    // in-process group: give the rank back (callers synchronised the streams
    // that waited on the events)
    if (ctx->local) {
        {
            std::lock_guard<std::mutex> g(ctx->local->mu);
            ctx->local->joined[ctx->rank] = false;
        }
        ctx->local.reset();
        for (auto &c : ctx->lg_ev)
            for (auto &p : c)
                for (hipEvent_t &e : p) {
                    if (e) (void)hipEventDestroy(e);
                    e = nullptr;
                }
    }
}

}  // namespace

// state of one nas_comm_init, shared with its helper thread (see there)
struct nas::CommInit {
    enum { ROOT = 3 };  // handle index: 0..2 the children, 3 the root
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    unsigned claimed = 0;  // bit i: handle i is the main thread's to abort (or already aborted)
    ncclComm_t root = nullptr;                         // written by RCCL from the helper
    ncclComm_t kids[3] = {nullptr, nullptr, nullptr};  // likewise
    ncclResult_t r = ncclSuccess;
    std::string what;
};

namespace {
// join the parked helpers of earlier abandoned inits that have finished;
// with detach_ms >= 0 (nas_destroy) poll up to that long for the others,
// then DETACH those still inside RCCL: a helper owns only the shared
// CommInit record and its own stream, event and buffers (it captures no
// context pointer), so it may outlive the context, and a helper that never
// returns from RCCL must not hang the context's teardown
void reap_comm_helpers(nas_ctx *ctx, int detach_ms = -1) {
    using clk = std::chrono::steady_clock;
    const auto until = clk::now() + std::chrono::milliseconds(std::max(detach_ms, 0));
    for (;;) {
        for (size_t i = 0; i < ctx->comm_helpers.size();) {
            bool done;
            {
                std::lock_guard<std::mutex> g(ctx->comm_helper_state[i]->mu);
                done = ctx->comm_helper_state[i]->done;
            }
            if (!done) {
                ++i;
                continue;
            }
            ctx->comm_helpers[i].join();
            ctx->comm_helpers.erase(ctx->comm_helpers.begin() + i);
            ctx->comm_helper_state.erase(ctx->comm_helper_state.begin() + i);
        }
        if (detach_ms < 0 || ctx->comm_helpers.empty()) return;
        if (clk::now() >= until) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    for (std::thread &t : ctx->comm_helpers) t.detach();
    ctx->comm_helpers.clear();
    ctx->comm_helper_state.clear();
}
// Process-wide pool of CU-masked streams.  A masked
// stream is a hardware queue of its own with the CU mask programmed into it
// (hipExtStreamCreateWithCUMask); contexts that reserve CUs for their commit
// stream (node shards, set_stream_masks) BORROW their masked streams from this
// pool and give them back idle when they drop the reservation or are
// destroyed, so a process that creates and destroys contexts keeps a bounded
// set of masked queues -- as many as its most concurrent contexts used -- and
// the runtime's create / destroy path for them runs once per (device, mask)
// slot, not once per context (tools/stream_churn_probe.hip measures what
// churning them costs).  Idle pooled streams live until the process exits
// (drain_masked_pool).
struct MaskedPool {
    struct Slot {
        int dev;
        std::vector<uint32_t> mask;
        hipStream_t s;
    };
    std::mutex mu;
    std::vector<Slot> idle;
    int64_t created = 0, lent = 0;
};
MaskedPool &masked_pool() {
    static MaskedPool *p = new MaskedPool;  // (intentionally leaked: outlives static teardown)
    return *p;
}
// at exit the idle pooled streams are destroyed while the runtime is still up
// (the handler is registered after the runtime initialised, so it runs before
// the runtime's own teardown): left to that teardown, a process under
// rocprofv3 with masked queues alive crashed in __cxa_finalize after the
// profiler had finalised (the G = 8 rehearsal trace, gpurun_out/r06k)
void drain_masked_pool() {
    MaskedPool &mp = masked_pool();
    std::lock_guard<std::mutex> g(mp.mu);
    for (const MaskedPool::Slot &sl : mp.idle) {
        (void)hipSetDevice(sl.dev);
        (void)hipStreamDestroy(sl.s);
    }
    mp.idle.clear();
}
std::atomic<int64_t> g_live_contexts{0};

hipError_t masked_acquire(int dev, const std::vector<uint32_t> &mask, hipStream_t *out) {
    MaskedPool &mp = masked_pool();
    {
        std::lock_guard<std::mutex> g(mp.mu);
        for (size_t i = 0; i < mp.idle.size(); ++i)
            if (mp.idle[i].dev == dev && mp.idle[i].mask == mask) {
                *out = mp.idle[i].s;
                mp.idle.erase(mp.idle.begin() + i);
                ++mp.lent;
                return hipSuccess;
            }
    }
    const hipError_t e = hipExtStreamCreateWithCUMask(out, (uint32_t)mask.size(), mask.data());
    if (e != hipSuccess) return e;
    static std::once_flag at_exit;
    std::call_once(at_exit, [] { std::atexit(drain_masked_pool); });
    std::lock_guard<std::mutex> g(masked_pool().mu);
    ++mp.created;
    ++mp.lent;
    return hipSuccess;
}
// s must be idle (synchronised by the caller)
void masked_release(int dev, const std::vector<uint32_t> &mask, hipStream_t s) {
    MaskedPool &mp = masked_pool();
    std::lock_guard<std::mutex> g(mp.mu);
    mp.idle.push_back({dev, mask, s});
    --mp.lent;
}
// the scoring-stream and commit-stream masks of a reservation of `reserve`
// CUs per XCD (bit i = CU i / 8 of XCD i % 8, tools/cumask_probe.hip)
void reserve_masks(int ncu, int reserve, std::vector<uint32_t> &ms, std::vector<uint32_t> &mc) {
    const int words = (ncu + 31) / 32;
    ms.assign(words, 0);
    mc.assign(words, 0);
    for (int b = 0; b < ncu; ++b) (b < 8 * reserve ? mc : ms)[b / 32] |= 1u << (b % 32);
}
// give a context's streams back: masked ones to the pool, plain ones destroyed
// (all idle); stream_x is cleared
void drop_streams(nas_ctx *ctx) {
    if (ctx->cu_reserve > 0) {
        int ncu = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device);
        std::vector<uint32_t> ms, mc;
        reserve_masks(ncu, ctx->cu_reserve, ms, mc);
        masked_release(ctx->device, ms, ctx->stream);
        masked_release(ctx->device, ms, ctx->stream2);
        masked_release(ctx->device, mc, ctx->stream_commit);
        if (ctx->stream_x) masked_release(ctx->device, mc, ctx->stream_x);
    } else {
        for (hipStream_t s : {ctx->stream, ctx->stream2, ctx->stream_commit, ctx->stream_x})
            if (s) (void)hipStreamDestroy(s);
    }
    ctx->stream = ctx->stream2 = ctx->stream_commit = ctx->stream_x = nullptr;
}
}  // namespace

extern "C" {

int nas_version(void) { return NAS_ABI_VERSION; }

int nas_create(nas_ctx **out, const nas_config *cfg) {
    NAS_RANGE("nas_create");
    if (!out) return NAS_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) return NAS_ERR_HIP;
    const int dev = cfg ? cfg->device : 0;
    if (dev < 0 || dev >= ndev) return NAS_ERR_ARG;
    nas_ctx *ctx = new (std::nothrow) nas_ctx();
    if (!ctx) return NAS_ERR_NOMEM;
    ctx->device = dev;
    if (hipDeviceGetAttribute(&ctx->n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ctx->n_cu <= 0)
        ctx->n_cu = 256;
    // the commit stream runs at the highest priority: its one-workgroup walks
    // and rescore slots take the next CU a scoring workgroup frees instead of
    // queueing behind a whole scoring launch
    int prio_lo = 0, prio_hi = 0;
    if (hipSetDevice(dev) != hipSuccess ||
        hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stream_commit, hipStreamNonBlocking, prio_hi) != hipSuccess) {
        delete ctx;
        return NAS_ERR_HIP;
    }
    *out = ctx;
    g_live_contexts.fetch_add(1);
    return NAS_OK;
}

int nas_debug_counters(int64_t *out, int32_t n) {
    if (!out || n < 0) return NAS_ERR_ARG;
    MaskedPool &mp = masked_pool();
    int64_t v[NAS_DBG_COUNT];
    {
        std::lock_guard<std::mutex> g(mp.mu);
        v[NAS_DBG_MASKED_STREAMS_CREATED] = mp.created;
        v[NAS_DBG_MASKED_STREAMS_LENT] = mp.lent;
        v[NAS_DBG_MASKED_STREAMS_IDLE] = (int64_t)mp.idle.size();
    }
    v[NAS_DBG_LIVE_CONTEXTS] = g_live_contexts.load();
    for (int i = 0; i < n && i < NAS_DBG_COUNT; ++i) out[i] = v[i];
    return NAS_OK;
}

void nas_destroy(nas_ctx *ctx) {
    NAS_RANGE("nas_destroy");
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    // a poisoned context's communicators go first: a collective left stuck on
    // a stream (a peer died) returns only once its communicator is aborted,
    // and the synchronisations below would otherwise wait for it forever
    if (ctx->poisoned) destroy_comms(ctx);
    for (hipStream_t st : {ctx->stream, ctx->stream2, ctx->stream_commit, ctx->stream_x})
        if (st) (void)hipStreamSynchronize(st);
    DevBuf *bufs[] = {&ctx->snap[0], &ctx->snap[1], &ctx->snap[2], &ctx->snap[3], &ctx->snap[4],
                      &ctx->snap[5], &ctx->order1, &ctx->pos1, &ctx->order2, &ctx->pos2,
                      &ctx->pod_snap, &ctx->best, &ctx->winners, &ctx->snap_best, &ctx->snap_win,
                      &ctx->Lt, &ctx->WA, &ctx->cap0, &ctx->cap, &ctx->cap_snap, &ctx->req, &ctx->mask,
                      &ctx->partial, &ctx->pbound, &ctx->cand_key, &ctx->cand_bound,
                      &ctx->gather[0], &ctx->gbound[0], &ctx->gather[1], &ctx->gbound[1],
                      &ctx->gather[2], &ctx->gbound[2], &ctx->xsend[2],
                      &ctx->resc_key, &ctx->resc_bound, &ctx->gather_r, &ctx->gbound_r,
                      &ctx->out_node, &ctx->out_cost_f, &ctx->out_cost_i,
                      &ctx->g_words, &ctx->g_idx, &ctx->g_key,
                      &ctx->g_bound, &ctx->g_gk, &ctx->g_gb, &ctx->status, &ctx->scratch,
                      &ctx->vote_part, &ctx->vote_gather, &ctx->xsend[0], &ctx->xsend[1],
                      &ctx->ovf_ptr, &ctx->ovf_m, &ctx->ovf_e, &ctx->Lr, &ctx->Lt6, &ctx->WA6,
                      &ctx->commit_flag, &ctx->zrow, &ctx->cost_cache};
    for (DevBuf *b : bufs)
        if (b->p) (void)hipFree(b->p);
    if (ctx->host_status.p) (void)hipHostFree(ctx->host_status.p);
    if (ctx->ref_stage.p) (void)hipHostFree(ctx->ref_stage.p);
    destroy_comms(ctx);
    reap_comm_helpers(ctx, 2000);
    for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
    if (ctx->sync_ev) (void)hipEventDestroy(ctx->sync_ev);
    drop_streams(ctx);  // (synchronised above; masked ones back to the pool)
    g_live_contexts.fetch_sub(1);
    delete ctx;
}

const char *nas_last_error(nas_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int nas_get_timings(nas_ctx *ctx, nas_timings *out) {
    if (!ctx || !out) return NAS_ERR_ARG;
    *out = ctx->timings;
    return NAS_OK;
}

int nas_set_option(nas_ctx *ctx, int32_t key, int64_t value) {
    if (!ctx) return NAS_ERR_ARG;
    ctx->err.clear();
    switch (key) {
    case NAS_OPT_STAGE_TIMINGS:
        if (value != 0 && value != 1) break;
        ctx->opt_stage_timings = value != 0;
        return NAS_OK;
    case NAS_OPT_COMM_TIMEOUT_MS:
        if (value < 0) break;
        ctx->opt_comm_timeout_ms = value;
        return NAS_OK;
    case NAS_OPT_REHEARSE_WORLD:
        if (value < 0 || value > 64) break;
        if (has_coll(ctx)) return nas::fail(ctx, NAS_ERR_STATE, "set NAS_OPT_REHEARSE_WORLD before nas_comm_init");
        ctx->opt_rehearse_world = (int32_t)value;
        return NAS_OK;
    case NAS_OPT_INJECT_STALL_MS:
        if (value < 0 || value > 60000) break;
        ctx->opt_inject_stall_ms = value;
        return NAS_OK;
    case NAS_OPT_COMMIT_WAIT_MS:
        if (value < 0 || value > 3600000) break;
        ctx->opt_commit_wait_ms = value;
        return NAS_OK;
    case NAS_OPT_HERD_PLAN:
        if (value < 0 || value > 2) break;
        ctx->opt_herd_plan = (int32_t)value;
        return NAS_OK;
    case NAS_OPT_COST_CACHE:
        if (value < 0 || value > 2) break;
        ctx->opt_cost_cache = (int32_t)value;
        return NAS_OK;
    case NAS_OPT_COMMIT_CUS:
        if (value < 0 || value > 4) break;
        ctx->opt_commit_cus = (int32_t)value;
        return NAS_OK;
    case NAS_OPT_SYNTH_PROFILE:
        if (value < 0 || value > 1) break;
        ctx->opt_synth_profile = (int32_t)value;
        return NAS_OK;
    case NAS_OPT_INJECT_COMMIT_STALL_MS:
        if (value < 0 || value > 60000) break;
        ctx->opt_inject_commit_stall_ms = value;
        return NAS_OK;
    default:
        return nas::fail(ctx, NAS_ERR_ARG, "nas_set_option: unknown key " + std::to_string(key));
    }
    return nas::fail(ctx, NAS_ERR_ARG, "nas_set_option: value out of range for key " + std::to_string(key));
}

// ---------------------------------------------------------------- reference
namespace {
// Snapshot slice [lo, lo + nl) of an n-node cluster, n_snapshots rows.
int upload_snapshot_slice(nas_ctx *ctx, const double *cpu, const double *mem, const int64_t *rx,
                          const int64_t *tx, const double *bw, const int64_t *disk, int32_t n,
                          int32_t lo, int32_t nl, int32_t n_snapshots, bool sharded) {
    if (!cpu || !mem || !rx || !tx || !bw || !disk || n <= 0 || nl <= 0 || n_snapshots <= 0)
        return nas::fail(ctx, NAS_ERR_ARG, "snapshot upload: null array or empty size");
    if (lo < 0 || (int64_t)lo + nl > n)
        return nas::fail(ctx, NAS_ERR_ARG, "snapshot upload: node slice outside [0, n_nodes)");
    const int64_t ns = nas::round_up(nl, 2);
    const void *src[6] = {cpu, mem, bw, rx, tx, disk};
    for (int f = 0; f < 6; ++f) {
        OK(nas::ensure(ctx, ctx->snap[f], (size_t)ns * n_snapshots * 8));
        HIPCK(hipMemcpy2DAsync(ctx->snap[f].p, ns * 8, src[f], (size_t)nl * 8, (size_t)nl * 8,
                               n_snapshots, hipMemcpyHostToDevice, ctx->stream));
    }
    if (ctx->snap_n != n) ctx->n_orders = 0;  // orders no longer match
    ctx->snap_n = n;
    ctx->snap_lo = lo;
    ctx->snap_nl = nl;
    ctx->snap_sharded = sharded;
    ctx->snap_s = n_snapshots;
    ctx->snap_ns = ns;
    HIPCK(hipStreamSynchronize(ctx->stream));
    return NAS_OK;
}

// nas_score_reference's argument checks and order upload, shared by the
// node-shard entries.  Per-snapshot sets must cover the `need` snapshots the
// call votes on; per-pod sets (nas_upload_pod_orders) are checked by the caller.
int prepare_orders(nas_ctx *ctx, const int32_t *order1, const int32_t *order2, int need,
                   bool pods_ok = false) {
    if (ctx->snap_s <= 0) return nas::fail(ctx, NAS_ERR_STATE, "no snapshot uploaded");
    if ((order1 == nullptr) != (order2 == nullptr))
        return nas::fail(ctx, NAS_ERR_ARG, "order1 and order2 must both be given or both NULL");
    if (order1) OK(upload_orders(ctx, order1, order2, 1));
    if (ctx->n_orders <= 0) return nas::fail(ctx, NAS_ERR_STATE, "no orders uploaded");
    if (ctx->orders_per_pod) {
        if (!pods_ok)
            return nas::fail(ctx, NAS_ERR_STATE,
                             "per-pod order sets serve nas_score_reference on an unsharded snapshot only");
        return NAS_OK;
    }
    if (ctx->n_orders != 1 && ctx->n_orders < need)
        return nas::fail(ctx, NAS_ERR_STATE, "orders: need 1 set or one per snapshot voted on");
    return NAS_OK;
}
}  // namespace

int nas_upload_snapshot(nas_ctx *ctx, const double *cpu, const double *mem, const int64_t *rx,
                        const int64_t *tx, const double *bw, const int64_t *disk, int32_t n_nodes,
                        int32_t n_snapshots) {
    NAS_RANGE("nas_upload_snapshot");
    OK(bind(ctx));
    return upload_snapshot_slice(ctx, cpu, mem, rx, tx, bw, disk, n_nodes, 0, n_nodes, n_snapshots,
                                 false);
}

int nas_upload_snapshot_shard(nas_ctx *ctx, const double *cpu, const double *mem,
                              const int64_t *rx, const int64_t *tx, const double *bw,
                              const int64_t *disk, int32_t n_nodes, int32_t node_lo,
                              int32_t n_local, int32_t n_snapshots) {
    NAS_RANGE("nas_upload_snapshot_shard");
    OK(bind(ctx));
    return upload_snapshot_slice(ctx, cpu, mem, rx, tx, bw, disk, n_nodes, node_lo, n_local,
                                 n_snapshots, true);
}

int nas_vote_partials(nas_ctx *ctx, const int32_t *order1, const int32_t *order2, int32_t S,
                      nas_vote_partial *out) {
    NAS_RANGE("nas_vote_partials");
    OK(bind(ctx));
    OK(prepare_orders(ctx, order1, order2, S));
    if (S < 0 || S > ctx->snap_s || (S > 0 && !out))
        return nas::fail(ctx, NAS_ERR_ARG, "nas_vote_partials: S / out");
    if (S == 0) return NAS_OK;
    OK(nas::ensure(ctx, ctx->vote_part, (size_t)S * sizeof(nas_vote_partial)));
    Timer tm(ctx);
    std::memset(&ctx->timings, 0, sizeof(ctx->timings));
    hipEvent_t a = tm.mark();
    HIPCK(nas::launch_vote_partial(ctx->stream, ctx, S, ctx->vote_part.as<nas_vote_partial>()));
    hipEvent_t b = tm.mark();
    HIPCK(hipMemcpyAsync(out, ctx->vote_part.p, (size_t)S * sizeof(nas_vote_partial),
                         hipMemcpyDeviceToHost, ctx->stream));
    hipEvent_t c = tm.mark();
    HIPCK(hipStreamSynchronize(ctx->stream));
    tm.span(T_VOTE, a, b);
    tm.span(T_TOTAL, a, c);
    ctx->timings.vote_ms = tm.total(T_VOTE);
    ctx->timings.total_ms = tm.total(T_TOTAL);
    return NAS_OK;
}

int nas_vote_merge(nas_ctx *ctx, const nas_vote_partial *parts, int32_t n_parts, int32_t S,
                   int32_t *best_out, int32_t *winners_out) {
    NAS_RANGE("nas_vote_merge");
    OK(bind(ctx));
    OK(prepare_orders(ctx, nullptr, nullptr, 1));
    if (n_parts < 1 || S < 0 || (S > 0 && (!parts || !best_out)))
        return nas::fail(ctx, NAS_ERR_ARG, "nas_vote_merge: parts / n_parts / S / best_out");
    if (ctx->n_orders != 1 && S > ctx->n_orders)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_vote_merge: S exceeds the per-snapshot order sets");
    for (int64_t i = 0; i < (int64_t)n_parts * S; ++i)
        for (int f = 0; f < 6; ++f) {
            const int32_t q = parts[i].m[f].pos1;
            if (q != NAS_VOTE_NOPOS && (q < 0 || q >= ctx->snap_n))
                return nas::fail(ctx, NAS_ERR_ARG, "nas_vote_merge: pos1 outside [0, n_nodes)");
        }
    if (S == 0) return NAS_OK;
    const size_t pb = (size_t)n_parts * S * sizeof(nas_vote_partial);
    OK(nas::ensure(ctx, ctx->vote_gather, pb));
    OK(nas::ensure(ctx, ctx->snap_best, (size_t)S * 4));
    OK(nas::ensure(ctx, ctx->snap_win, (size_t)S * 24));
    Timer tm(ctx);
    std::memset(&ctx->timings, 0, sizeof(ctx->timings));
    hipEvent_t a = tm.mark();
    HIPCK(hipMemcpyAsync(ctx->vote_gather.p, parts, pb, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(nas::launch_vote_merge(ctx->stream, ctx, ctx->vote_gather.as<nas_vote_partial>(), n_parts,
                                 S, ctx->snap_best.as<int32_t>(), ctx->snap_win.as<int32_t>()));
    HIPCK(hipMemcpyAsync(best_out, ctx->snap_best.p, (size_t)S * 4, hipMemcpyDeviceToHost,
                         ctx->stream));
    if (winners_out)
        HIPCK(hipMemcpyAsync(winners_out, ctx->snap_win.p, (size_t)S * 24, hipMemcpyDeviceToHost,
                             ctx->stream));
    hipEvent_t b = tm.mark();
    HIPCK(hipStreamSynchronize(ctx->stream));
    tm.span(T_TOTAL, a, b);
    ctx->timings.total_ms = tm.total(T_TOTAL);
    return NAS_OK;
}

int nas_upload_orders(nas_ctx *ctx, const int32_t *order1, const int32_t *order2,
                      int32_t n_orders) {
    NAS_RANGE("nas_upload_orders");
    OK(bind(ctx));
    return upload_orders(ctx, order1, order2, n_orders);
}

int nas_upload_pod_orders(nas_ctx *ctx, const int32_t *order1, const int32_t *order2,
                          int32_t n_pods) {
    NAS_RANGE("nas_upload_pod_orders");
    OK(bind(ctx));
    return upload_orders(ctx, order1, order2, n_pods, true);
}

int nas_score_reference(nas_ctx *ctx, const int32_t *order1, const int32_t *order2,
                        const int32_t *pod_snapshot, int32_t P, int32_t *best_out,
                        int32_t *winners_out) {
    NAS_RANGE("nas_score_reference");
    OK(bind(ctx));
    if (ctx->snap_s <= 0) return nas::fail(ctx, NAS_ERR_STATE, "no snapshot uploaded");
    if (P < 0 || (P > 0 && !best_out)) return nas::fail(ctx, NAS_ERR_ARG, "P / best_out");
    const bool per_pod = ctx->orders_per_pod && !order1;
    OK(prepare_orders(ctx, order1, order2, pod_snapshot ? ctx->snap_s : P, !ctx->snap_sharded));
    if (per_pod && ctx->n_orders != P)
        return nas::fail(ctx, NAS_ERR_ARG, "per-pod order sets: P must equal the uploaded set count (" +
                                               std::to_string(ctx->n_orders) + ")");
    if (ctx->snap_sharded && !exchanging(ctx))
        return nas::fail(ctx, NAS_ERR_STATE,
                         "node-sharded snapshot: nas_score_reference needs nas_comm_init "
                         "(or use nas_vote_partials + nas_vote_merge)");
    if (!pod_snapshot && P > ctx->snap_s)
        return nas::fail(ctx, NAS_ERR_ARG, "pod_snapshot NULL needs P <= n_snapshots");
    if (pod_snapshot)
        for (int p = 0; p < P; ++p)
            if (pod_snapshot[p] < 0 || pod_snapshot[p] >= ctx->snap_s)
                return nas::fail(ctx, NAS_ERR_ARG, "pod_snapshot index out of range");
    if (P == 0) return NAS_OK;
    const int S = ctx->snap_s;
    OK(nas::ensure(ctx, ctx->snap_best, (size_t)S * 4));
    OK(nas::ensure(ctx, ctx->snap_win, (size_t)S * 6 * 4));
    Timer tm(ctx);
    std::memset(&ctx->timings, 0, sizeof(ctx->timings));
    hipEvent_t a = tm.mark(), b = nullptr;
    const int Sused = pod_snapshot ? S : P;
    const int32_t *best_d = ctx->snap_best.as<int32_t>();
    const int32_t *win_d = ctx->snap_win.as<int32_t>();
    if (per_pod) {
        // one block per pod: its snapshot, its own order set; no per-pod
        // snapshot copies and no gather
        OK(nas::ensure(ctx, ctx->best, (size_t)P * 4));
        OK(nas::ensure(ctx, ctx->winners, (size_t)P * 24));
        const int32_t *ps = nullptr;
        if (pod_snapshot) {
            OK(nas::ensure(ctx, ctx->pod_snap, (size_t)P * 4));
            HIPCK(hipMemcpyAsync(ctx->pod_snap.p, pod_snapshot, (size_t)P * 4, hipMemcpyHostToDevice,
                                 ctx->stream));
            ps = ctx->pod_snap.as<int32_t>();
        }
        HIPCK(nas::launch_vote_pods(ctx->stream, ctx, ps, P, ctx->best.as<int32_t>(),
                                    ctx->winners.as<int32_t>()));
        b = tm.mark();
        best_d = ctx->best.as<int32_t>();
        win_d = ctx->winners.as<int32_t>();
    } else if (ctx->snap_sharded) {
        // node shards: partial records of this rank's slice, all-gathered
        // over RCCL, merged in rank order (every rank gets the full result)
        const size_t rb = (size_t)Sused * sizeof(nas_vote_partial);
        const int ranks = ctx->rehearse > 1 ? 1 : ctx->world;  // the communicator's size
        OK(nas::ensure(ctx, ctx->vote_part, rb));
        OK(nas::ensure(ctx, ctx->vote_gather, rb * ranks));
        HIPCK(nas::launch_vote_partial(ctx->stream, ctx, Sused, ctx->vote_part.as<nas_vote_partial>()));
        b = tm.mark();  // vote_ms: the slice's HBM pass alone
        const GatherSeg g1{ctx->vote_part.p, ctx->vote_gather.p, rb};
        OK(allgather(ctx, CH_SCORE, ctx->stream, &g1, 1, "vote all-gather"));
        HIPCK(nas::launch_vote_merge(ctx->stream, ctx, ctx->vote_gather.as<nas_vote_partial>(),
                                     ranks, Sused, ctx->snap_best.as<int32_t>(),
                                     ctx->snap_win.as<int32_t>()));
    } else {
        HIPCK(nas::launch_vote(ctx->stream, ctx, Sused));
        b = tm.mark();
    }
    if (pod_snapshot && !per_pod) {
        OK(nas::ensure(ctx, ctx->pod_snap, (size_t)P * 4));
        OK(nas::ensure(ctx, ctx->best, (size_t)P * 4));
        OK(nas::ensure(ctx, ctx->winners, (size_t)P * 24));
        HIPCK(hipMemcpyAsync(ctx->pod_snap.p, pod_snapshot, (size_t)P * 4, hipMemcpyHostToDevice,
                             ctx->stream));
        HIPCK(nas::launch_vote_gather(ctx->stream, ctx->pod_snap.as<int32_t>(), P, best_d, win_d,
                                      ctx->best.as<int32_t>(), ctx->winners.as<int32_t>()));
        best_d = ctx->best.as<int32_t>();
        win_d = ctx->winners.as<int32_t>();
    }
    // results come back through a pinned staging buffer (a copy into the
    // caller's pageable memory is a blocking staged copy each: C1, 100 pods,
    // spent most of its per-call time in the two of them)
    const size_t stage_bytes = (size_t)P * 28;
    if (ctx->ref_stage.bytes < stage_bytes) {
        if (ctx->ref_stage.p) (void)hipHostFree(ctx->ref_stage.p);
        ctx->ref_stage.p = nullptr;
        ctx->ref_stage.bytes = 0;
        HIPCK(hipHostMalloc(&ctx->ref_stage.p, stage_bytes, hipHostMallocDefault));
        ctx->ref_stage.bytes = stage_bytes;
    }
    int32_t *stage = ctx->ref_stage.as<int32_t>();
    HIPCK(hipMemcpyAsync(stage, best_d, (size_t)P * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (winners_out)
        HIPCK(hipMemcpyAsync(stage + P, win_d, (size_t)P * 24, hipMemcpyDeviceToHost, ctx->stream));
    if (ctx->snap_sharded && has_coll(ctx)) inject_stall(ctx, ctx->stream);
    hipEvent_t c = tm.mark();
    if (ctx->snap_sharded) OK(sync_stream(ctx, ctx->stream));
    else HIPCK(hipStreamSynchronize(ctx->stream));
    std::memcpy(best_out, stage, (size_t)P * 4);
    if (winners_out) std::memcpy(winners_out, stage + P, (size_t)P * 24);
    tm.span(T_VOTE, a, b);
    tm.span(T_TOTAL, a, c);
    ctx->timings.vote_ms = tm.total(T_VOTE);
    ctx->timings.total_ms = tm.total(T_TOTAL);
    return NAS_OK;
}

// ----------------------------------------------------------------- extended
int nas_upload_latency(nas_ctx *ctx, const void *L, int32_t dtype, int32_t n) {
    NAS_RANGE("nas_upload_latency");
    OK(bind(ctx));
    if (!L || n <= 0 || !valid_dtype(dtype))
        return nas::fail(ctx, NAS_ERR_ARG, "nas_upload_latency: L / n / dtype");
    set_geometry(ctx, n, dtype);
    if (dtype == NAS_DT_I8) {  // max |L| over the whole matrix (the same on every rank)
        const auto *l = static_cast<const signed char *>(L);
        int mx = 0;
        for (size_t i = 0, e = (size_t)ctx->B * n * n; i < e; ++i) mx = std::max(mx, std::abs((int)l[i]));
        ctx->L_abs_max = mx;
    }
    // float latency: a zero-traffic pod's costs are exactly 0 only if no entry
    // is Inf / NaN (the whole matrix: every rank decides the same)
    ctx->L_finite = true;
    if (dtype == NAS_DT_F32) {
        const auto *l = static_cast<const uint32_t *>(L);
        for (size_t i = 0, e = (size_t)ctx->B * n * n; i < e && ctx->L_finite; ++i)
            ctx->L_finite = (l[i] & 0x7f800000u) != 0x7f800000u;
    } else if (dtype == NAS_DT_BF16) {
        const auto *l = static_cast<const uint16_t *>(L);
        for (size_t i = 0, e = (size_t)ctx->B * n * n; i < e && ctx->L_finite; ++i)
            ctx->L_finite = (l[i] & 0x7f80u) != 0x7f80u;
    }
    if (ctx->have_wa && (ctx->wa_n != n || ctx->wa_dtype != dtype)) ctx->have_wa = false;
    const size_t e = esz(dtype);
    const size_t lt_b = (size_t)ctx->Mp * ctx->Kp * e;  // one cluster's Lt
    OK(nas::ensure(ctx, ctx->Lt, lt_b * ctx->B));
    DevBuf tmp;
    OK(nas::ensure(ctx, tmp, (size_t)n * n * e));
    hipError_t he = hipSuccess;
    for (int b = 0; b < ctx->B && he == hipSuccess; ++b) {
        he = hipMemcpyAsync(tmp.p, static_cast<const char *>(L) + (size_t)b * n * n * e,
                            (size_t)n * n * e, hipMemcpyHostToDevice, ctx->stream);
        if (he == hipSuccess)
            he = nas::launch_transpose_L(ctx->stream, tmp.p, dtype, n, ctx->Nloc0, ctx->Nloc,
                                         ctx->Mp, ctx->Kp, ctx->Lt.as<char>() + b * lt_b);
    }
    if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
    (void)hipFree(tmp.p);
    if (he != hipSuccess) return nas::hip_fail(ctx, he, "upload latency");
    ctx->have_L = true;
    ctx->L_n = n;
    ctx->L_dtype = dtype;
    ctx->synth_valid = false;
    ctx->lr_valid = false;
    ctx->split_valid = false;
    ctx->zrow_valid = false;
    ctx->scored = false;
    return NAS_OK;
}

int nas_upload_capacity(nas_ctx *ctx, const int32_t *cpu_milli, const int32_t *mem_kib,
                        const int32_t *pods, int32_t n) {
    NAS_RANGE("nas_upload_capacity");
    OK(bind(ctx));
    if (!cpu_milli || !mem_kib || !pods || n <= 0)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_upload_capacity");
    if (!ctx->have_L && !ctx->have_wa) set_geometry(ctx, n, ctx->dtype ? ctx->dtype : NAS_DT_I8);
    const size_t B = ctx->B;
    OK(nas::ensure(ctx, ctx->cap0, B * 3 * n * 4));
    OK(nas::ensure(ctx, ctx->cap, B * 3 * n * 4));
    const int32_t *src[3] = {cpu_milli, mem_kib, pods};
    for (size_t b = 0; b < B; ++b)
        for (int r = 0; r < 3; ++r)
            HIPCK(hipMemcpyAsync(ctx->cap0.as<int32_t>() + (b * 3 + r) * n, src[r] + b * n,
                                 (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipMemcpyAsync(ctx->cap.p, ctx->cap0.p, B * 3 * n * 4, hipMemcpyDeviceToDevice,
                         ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    ctx->have_cap = true;
    ctx->cap_n = n;
    return NAS_OK;
}

int nas_reset_capacity(nas_ctx *ctx) {
    NAS_RANGE("nas_reset_capacity");
    OK(bind(ctx));
    if (!ctx->have_cap) return nas::fail(ctx, NAS_ERR_STATE, "no capacity uploaded");
    // stream-ordered, no host wait: every later entry point's device work runs
    // on ctx->stream or behind an event recorded on it (nas_place's other
    // streams start behind `ready`), and every host read of the capacity syncs
    // ctx->stream -- the round trip here cost each reset-then-place cycle a
    // launch + wait (~30-50 us; C2's whole pass is ~450 us)
    // (a copy kernel: hipMemcpyAsync's device-to-device path cost the host
    // 15-36 us per reset, k_misc.hip k_copy_i32)
    HIPCK(nas::launch_copy_i32(ctx->stream, ctx->cap.as<int32_t>(), ctx->cap0.as<int32_t>(),
                               (int64_t)ctx->B * 3 * ctx->cap_n));
    return NAS_OK;
}

int nas_get_capacity(nas_ctx *ctx, int32_t *cpu_milli, int32_t *mem_kib, int32_t *pods,
                     int32_t n) {
    NAS_RANGE("nas_get_capacity");
    OK(bind(ctx));
    if (!ctx->have_cap) return nas::fail(ctx, NAS_ERR_STATE, "no capacity uploaded");
    if (n != ctx->cap_n || !cpu_milli || !mem_kib || !pods)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_get_capacity");
    int32_t *dst[3] = {cpu_milli, mem_kib, pods};
    for (size_t b = 0; b < (size_t)ctx->B; ++b)
        for (int r = 0; r < 3; ++r)
            HIPCK(hipMemcpyAsync(dst[r] + b * n, ctx->cap.as<int32_t>() + (b * 3 + r) * n,
                                 (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    return NAS_OK;
}

int nas_upload_pods(nas_ctx *ctx, const int32_t *rc, const int32_t *rm, const int32_t *rp,
                    int32_t P) {
    NAS_RANGE("nas_upload_pods");
    OK(bind(ctx));
    if (!rc || !rm || !rp || P <= 0) return nas::fail(ctx, NAS_ERR_ARG, "nas_upload_pods");
    const size_t B = ctx->B;
    for (size_t p = 0; p < B * P; ++p)
        if (rc[p] < 0 || rm[p] < 0 || rp[p] < 0)
            return nas::fail(ctx, NAS_ERR_ARG, "negative resource request");
    const int Pp = (int)nas::round_up(P, nas::COST_BN);
    std::vector<int32_t> h(B * 3 * Pp, 0);  // [B][3][Pp]
    for (size_t b = 0; b < B; ++b) {
        const size_t o = b * 3 * Pp, q = b * P;
        std::copy(rc + q, rc + q + P, h.begin() + o);
        std::copy(rm + q, rm + q + P, h.begin() + o + Pp);
        std::copy(rp + q, rp + q + P, h.begin() + o + 2 * (size_t)Pp);
    }
    OK(nas::ensure(ctx, ctx->req, h.size() * 4));
    HIPCK(hipMemcpyAsync(ctx->req.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    if (!ctx->have_wa) {
        ctx->P = P;
        ctx->Pp = Pp;
    }
    if (P != ctx->req_P) ctx->scored = false;  // lists of another pod set
    ctx->req_P = P;
    ctx->have_pods = true;
    return NAS_OK;
}

// dtype here is the COMPUTE dtype (NAS_DT_I8 for int8 / int32 traffic)
static int traffic_common(nas_ctx *ctx, int32_t dtype, int32_t P, int32_t n) {
    if (P <= 0 || n <= 0 || !valid_dtype(dtype))
        return nas::fail(ctx, NAS_ERR_ARG, "traffic: P / n / dtype");
    if (!ctx->have_L || ctx->L_n != n || ctx->L_dtype != dtype) {
        set_geometry(ctx, n, dtype);
        ctx->have_L = false;  // its layout no longer matches: re-upload latency
    }
    ctx->P = P;
    ctx->Pp = (int32_t)nas::round_up(P, nas::COST_BN);
    const size_t wa_bytes = (size_t)ctx->B * ctx->Pp * ctx->Kp * esz(dtype);
    OK(nas::ensure(ctx, ctx->WA, wa_bytes + (size_t)nas::WA_PAD_ROWS * ctx->Kp * esz(dtype)));
    HIPCK(hipMemsetAsync(ctx->WA.p, 0, wa_bytes, ctx->stream));
    ctx->wa_P = P;
    ctx->wa_n = n;
    ctx->wa_dtype = dtype;
    ctx->ovf_n = 0;
    ctx->wa_abs_row_max = 0;
    ctx->split_valid = false;
    ctx->zrow_valid = false;
    ctx->scored = false;  // the lists (and their buffers' sizes) belong to the old inputs
    ctx->have_wa = false;
    return NAS_OK;
}

int nas_upload_traffic_dense(nas_ctx *ctx, const void *WA, int32_t dtype, int32_t P, int32_t n) {
    NAS_RANGE("nas_upload_traffic_dense");
    OK(bind(ctx));
    if (!WA) return nas::fail(ctx, NAS_ERR_ARG, "WA null");
    if (dtype == NAS_DT_I32) {
        // exact int32 traffic: the int8 plane (clamped) + overflow lists,
        // split on the host in row blocks
        OK(traffic_common(ctx, NAS_DT_I8, P, n));
        const auto *src = static_cast<const int32_t *>(WA);
        const int B = ctx->B, Pp = ctx->Pp, Kp = ctx->Kp;
        std::vector<int32_t> ptr((size_t)B * Pp + 1, 0), om, oe;
        const int rows_blk = std::max(1, (int)std::min<int64_t>(P, (64 << 20) / std::max(1, n)));
        std::vector<signed char> plane((size_t)rows_blk * n);
        std::vector<int64_t> row(n);
        for (int b = 0; b < B; ++b)
            for (int p0 = 0; p0 < P; p0 += rows_blk) {
                const int nr = std::min(rows_blk, P - p0);
                for (int i = 0; i < nr; ++i) {
                    const int32_t *r = src + ((size_t)b * P + p0 + i) * n;
                    for (int j = 0; j < n; ++j) row[j] = r[j];
                    split_row(row.data(), n, plane.data() + (size_t)i * n, om, oe);
                    ptr[(size_t)b * Pp + p0 + i + 1] = (int32_t)om.size();
                }
                HIPCK(hipMemcpy2DAsync(ctx->WA.as<char>() + ((size_t)b * Pp + p0) * Kp, (size_t)Kp,
                                       plane.data(), (size_t)n, (size_t)n, nr,
                                       hipMemcpyHostToDevice, ctx->stream));
                HIPCK(hipStreamSynchronize(ctx->stream));  // plane is reused
            }
        // padding rows carry the running offset
        for (size_t r = 1; r < ptr.size(); ++r) ptr[r] = std::max(ptr[r], ptr[r - 1]);
        if (om.size() > 0x7fffffffu) return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "too many overflow entries");
        OK(upload_ovf(ctx, ptr, om, oe));
        OK(finish_traffic_i8(ctx));
        ctx->have_wa = true;
        ctx->synth_valid = false;
        return NAS_OK;
    }
    OK(traffic_common(ctx, dtype, P, n));
    const size_t e = esz(dtype);
    for (size_t b = 0; b < (size_t)ctx->B; ++b)
        HIPCK(hipMemcpy2DAsync(ctx->WA.as<char>() + b * ctx->Pp * ctx->Kp * e, (size_t)ctx->Kp * e,
                               static_cast<const char *>(WA) + b * P * n * e, (size_t)n * e,
                               (size_t)n * e, P, hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    if (dtype == NAS_DT_I8) OK(finish_traffic_i8(ctx));
    ctx->have_wa = true;
    ctx->synth_valid = false;
    return NAS_OK;
}

int nas_upload_traffic_csr(nas_ctx *ctx, const int32_t *row_ptr, const int32_t *peer_node,
                           const void *weight, int32_t dtype, int32_t P, int32_t n, int64_t nnz) {
    NAS_RANGE("nas_upload_traffic_csr");
    OK(bind(ctx));
    if (!row_ptr || nnz < 0 || (nnz > 0 && (!peer_node || !weight)))
        return nas::fail(ctx, NAS_ERR_ARG, "csr arrays");
    if (dtype != NAS_DT_I8 && dtype != NAS_DT_I32 && dtype != NAS_DT_BF16 && dtype != NAS_DT_F32)
        return nas::fail(ctx, NAS_ERR_ARG, "csr weight dtype");
    if (ctx->B > 1) return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "CSR traffic with a cluster batch");
    if (P <= 0 || row_ptr[0] != 0 || row_ptr[P] != nnz)
        return nas::fail(ctx, NAS_ERR_ARG, "row_ptr bounds");
    for (int p = 0; p < P; ++p)
        if (row_ptr[p + 1] < row_ptr[p]) return nas::fail(ctx, NAS_ERR_ARG, "row_ptr not monotone");
    if (dtype == NAS_DT_F32) {
        // fp32 traffic: per-node sums in fp64 on the host, rounded to fp32
        // once, scattered into the dense rows on the device
        OK(traffic_common(ctx, NAS_DT_F32, P, n));
        std::vector<int32_t> tp, tn;
        std::vector<float> tv;
        std::vector<std::pair<int32_t, double>> agg;
        const auto *wf = static_cast<const float *>(weight);
        for (int p = 0; p < P; ++p) {
            agg.clear();
            for (int64_t x = row_ptr[p]; x < row_ptr[p + 1]; ++x)
                if (peer_node[x] >= 0 && peer_node[x] < n) agg.push_back({peer_node[x], (double)wf[x]});
            std::sort(agg.begin(), agg.end(),
                      [](const auto &a, const auto &b) { return a.first < b.first; });
            for (size_t i = 0; i < agg.size();) {
                const int32_t m = agg[i].first;
                double v = 0;
                for (; i < agg.size() && agg[i].first == m; ++i) v += agg[i].second;
                tp.push_back(p);
                tn.push_back(m);
                tv.push_back((float)v);
            }
        }
        DevBuf dp, dn, dv;
        int rc = nas::ensure(ctx, dp, tp.size() * 4 + 4);
        if (rc == NAS_OK) rc = nas::ensure(ctx, dn, tn.size() * 4 + 4);
        if (rc == NAS_OK) rc = nas::ensure(ctx, dv, tv.size() * 4 + 4);
        hipError_t he = hipSuccess;
        if (rc == NAS_OK && !tp.empty()) {
            he = hipMemcpyAsync(dp.p, tp.data(), tp.size() * 4, hipMemcpyHostToDevice, ctx->stream);
            if (he == hipSuccess)
                he = hipMemcpyAsync(dn.p, tn.data(), tn.size() * 4, hipMemcpyHostToDevice, ctx->stream);
            if (he == hipSuccess)
                he = hipMemcpyAsync(dv.p, tv.data(), tv.size() * 4, hipMemcpyHostToDevice, ctx->stream);
            if (he == hipSuccess)
                he = nas::launch_scatter_f32(ctx->stream, dp.as<int32_t>(), dn.as<int32_t>(),
                                             dv.as<float>(), (int64_t)tp.size(), ctx->Kp,
                                             ctx->WA.as<float>());
        }
        (void)hipStreamSynchronize(ctx->stream);
        for (DevBuf *b : {&dp, &dn, &dv})
            if (b->p) (void)hipFree(b->p);
        if (rc != NAS_OK) return rc;
        if (he != hipSuccess) return nas::hip_fail(ctx, he, "csr f32 scatter");
        ctx->have_wa = true;
        ctx->synth_valid = false;
        return NAS_OK;
    }
    if (dtype != NAS_DT_BF16) {
        // exact integer aggregation on the host (int64 sums, then int32 range):
        // the plane entries are scattered on the device, the rest is overflow
        OK(traffic_common(ctx, NAS_DT_I8, P, n));
        std::vector<int32_t> ptr((size_t)ctx->Pp + 1, 0), om, oe, tp, tn;
        std::vector<signed char> tv;
        std::vector<std::pair<int32_t, int64_t>> agg;
        for (int p = 0; p < P; ++p) {
            agg.clear();
            for (int64_t x = row_ptr[p]; x < row_ptr[p + 1]; ++x) {
                const int32_t m = peer_node[x];
                if (m < 0 || m >= n) continue;  // unbound peer (or off-cluster): skipped
                const int64_t w = dtype == NAS_DT_I8 ? (int64_t) static_cast<const int8_t *>(weight)[x]
                                                     : (int64_t) static_cast<const int32_t *>(weight)[x];
                agg.push_back({m, w});
            }
            std::sort(agg.begin(), agg.end(),
                      [](const auto &a, const auto &b) { return a.first < b.first; });
            for (size_t i = 0; i < agg.size();) {
                const int32_t m = agg[i].first;
                int64_t v = 0;
                for (; i < agg.size() && agg[i].first == m; ++i) v += agg[i].second;
                if (v < INT32_MIN || v > INT32_MAX)
                    return nas::fail(ctx, NAS_ERR_UNSUPPORTED,
                                     "traffic of pod " + std::to_string(p) + " to node " +
                                         std::to_string(m) + " exceeds int32");
                if (v == 0) continue;
                const int64_t c = v < -128 ? -128 : v > 127 ? 127 : v;
                tp.push_back(p);
                tn.push_back(m);
                tv.push_back((signed char)c);
                if (v != c) {
                    om.push_back(m);
                    oe.push_back((int32_t)(v - c));
                }
            }
            ptr[p + 1] = (int32_t)om.size();
        }
        for (size_t r = (size_t)P + 1; r < ptr.size(); ++r) ptr[r] = ptr[r - 1];
        DevBuf dp, dn, dv;
        int rc = nas::ensure(ctx, dp, tp.size() * 4 + 4);
        if (rc == NAS_OK) rc = nas::ensure(ctx, dn, tn.size() * 4 + 4);
        if (rc == NAS_OK) rc = nas::ensure(ctx, dv, tv.size() + 4);
        hipError_t he = hipSuccess;
        if (rc == NAS_OK && !tp.empty()) {
            he = hipMemcpyAsync(dp.p, tp.data(), tp.size() * 4, hipMemcpyHostToDevice, ctx->stream);
            if (he == hipSuccess)
                he = hipMemcpyAsync(dn.p, tn.data(), tn.size() * 4, hipMemcpyHostToDevice, ctx->stream);
            if (he == hipSuccess)
                he = hipMemcpyAsync(dv.p, tv.data(), tv.size(), hipMemcpyHostToDevice, ctx->stream);
            if (he == hipSuccess)
                he = nas::launch_plane_scatter(ctx->stream, dp.as<int32_t>(), dn.as<int32_t>(),
                                               dv.as<signed char>(), (int64_t)tp.size(), ctx->Kp,
                                               ctx->WA.as<signed char>());
        }
        (void)hipStreamSynchronize(ctx->stream);
        for (DevBuf *b : {&dp, &dn, &dv})
            if (b->p) (void)hipFree(b->p);
        if (rc != NAS_OK) return rc;
        if (he != hipSuccess) return nas::hip_fail(ctx, he, "csr plane scatter");
        OK(upload_ovf(ctx, ptr, om, oe));
        OK(finish_traffic_i8(ctx));
        ctx->have_wa = true;
        ctx->synth_valid = false;
        return NAS_OK;
    }
    OK(traffic_common(ctx, dtype, P, n));
    DevBuf rp, pn, w;
    int rc = nas::ensure(ctx, rp, (size_t)(P + 1) * 4);
    if (rc == NAS_OK) rc = nas::ensure(ctx, pn, (size_t)nnz * 4);
    if (rc == NAS_OK) rc = nas::ensure(ctx, w, (size_t)nnz * 2);
    hipError_t he = hipSuccess;
    if (rc == NAS_OK) {
        he = hipMemcpyAsync(rp.p, row_ptr, (size_t)(P + 1) * 4, hipMemcpyHostToDevice, ctx->stream);
        if (he == hipSuccess && nnz)
            he = hipMemcpyAsync(pn.p, peer_node, (size_t)nnz * 4, hipMemcpyHostToDevice, ctx->stream);
        if (he == hipSuccess && nnz)
            he = hipMemcpyAsync(w.p, weight, (size_t)nnz * 2, hipMemcpyHostToDevice, ctx->stream);
        if (he == hipSuccess)
            he = nas::launch_csr_aggregate_bf16(ctx->stream, rp.as<int32_t>(), pn.as<int32_t>(),
                                                w.as<uint16_t>(), P, n, ctx->Kp,
                                                ctx->WA.as<uint16_t>());
        if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
    }
    (void)hipStreamSynchronize(ctx->stream);
    for (DevBuf *b : {&rp, &pn, &w})
        if (b->p) (void)hipFree(b->p);
    if (rc != NAS_OK) return rc;
    if (he != hipSuccess) return nas::hip_fail(ctx, he, "csr aggregate");
    ctx->have_wa = true;
    ctx->synth_valid = false;
    return NAS_OK;
}

int nas_filter(nas_ctx *ctx, uint64_t *mask_out) {
    NAS_RANGE("nas_filter");
    OK(bind(ctx));
    OK(no_batch(ctx, "nas_filter"));
    if (!ctx->have_cap || !ctx->have_pods || ctx->N <= 0)
        return nas::fail(ctx, NAS_ERR_STATE, "nas_filter needs capacity and pods");
    if (ctx->cap_n != ctx->N || ctx->req_P != ctx->P)
        return nas::fail(ctx, NAS_ERR_STATE, "nas_filter: capacity/pods do not match the geometry");
    OK(alloc_extended(ctx));
    Timer tm(ctx);
    hipEvent_t a = tm.mark();
    HIPCK(nas::launch_fit(ctx->stream, ctx->cap.as<int32_t>(), ctx->N, ctx->Nloc0, ctx->Nloc,
                          ctx->Mp, ctx->req.as<int32_t>(), ctx->P, ctx->Pp, 0, ctx->P,
                          ctx->mask.as<uint64_t>()));
    hipEvent_t b = tm.mark();
    if (mask_out) {
        const int chunks = (ctx->Nloc + 63) / 64;
        HIPCK(hipMemcpy2DAsync(mask_out, (size_t)ctx->P * 8, ctx->mask.p, (size_t)ctx->Pp * 8,
                               (size_t)ctx->P * 8, chunks, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCK(hipStreamSynchronize(ctx->stream));
    tm.span(T_FIT, a, b);
    ctx->timings.fit_ms = tm.total(T_FIT);
    return NAS_OK;
}

int nas_score(nas_ctx *ctx) {
    NAS_RANGE("nas_score");
    OK(bind(ctx));
    OK(check_extended(ctx));
    OK(alloc_extended(ctx));
    OK(prepare_ovf(ctx));
    OK(prepare_split(ctx));
    OK(prepare_zrow(ctx));
    std::memset(&ctx->timings, 0, sizeof(ctx->timings));
    Timer tm(ctx);
    if (ctx->B > 1) OK(score_batch(ctx, tm));
    else OK(score_range(ctx, tm, 0, ctx->P));
    if (has_coll(ctx)) inject_stall(ctx, ctx->stream);
    OK(sync_stream(ctx, ctx->stream));
    ctx->timings.fit_ms = tm.total(T_FIT);
    ctx->timings.cost_ms = tm.total(T_COST);
    ctx->timings.merge_ms = tm.total(T_MERGE);
    ctx->scored = true;
    return NAS_OK;
}

namespace {
// The exchange stream of node-shard passes (nas_place), made on first use --
// a world-1 context never has it: one more stream than the hardware queues a
// process gets (4 on the pool's boxes) made a C3 world-1 pass 0.7% slower
// (profiles/r05ae_ab_exchange_stream.txt) -- with the commit stream's CU mask
// when the context reserves CUs for it, else at the commit stream's priority
int exchange_stream(nas_ctx *ctx, hipStream_t *out) {
    if (!ctx->stream_x) {
        hipError_t e = hipSuccess;
        if (ctx->cu_reserve > 0) {
            int ncu = 0;
            HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
            std::vector<uint32_t> ms, mc;
            reserve_masks(ncu, ctx->cu_reserve, ms, mc);
            e = masked_acquire(ctx->device, mc, &ctx->stream_x);
        } else {
            int lo = 0, hi = 0;
            e = hipDeviceGetStreamPriorityRange(&lo, &hi);
            if (e == hipSuccess) e = hipStreamCreateWithPriority(&ctx->stream_x, hipStreamNonBlocking, hi);
        }
        if (e != hipSuccess) {
            ctx->stream_x = nullptr;
            return nas::hip_fail(ctx, e, "exchange stream");
        }
    }
    *out = ctx->stream_x;
    return NAS_OK;
}
}  // namespace

int nas_place(nas_ctx *ctx, int32_t *node_out, float *cost_out, int64_t *int_score_out) {
    NAS_RANGE("nas_place");
    OK(bind(ctx));
    OK(check_extended(ctx));
    if (ctx->virtual_shard)
        return nas::fail(ctx, NAS_ERR_STATE,
                         "nas_place on a shard needs nas_comm_init (nas_set_shard scores only)");
    if (!node_out) return nas::fail(ctx, NAS_ERR_ARG, "node_out null");
    // world 1: the commit stream's own CUs (NAS_OPT_COMMIT_CUS), so chunk
    // merges and commits run as chunks land instead of queueing behind the
    // wide cost workgroups (node shards set theirs in nas_comm_init)
    if (ctx->world == 1 && !has_coll(ctx) && ctx->cu_reserve != ctx->opt_commit_cus)
        OK(set_stream_masks(ctx, ctx->opt_commit_cus));
    OK(alloc_extended(ctx));
    OK(prepare_ovf(ctx));
    OK(prepare_split(ctx));
    OK(prepare_zrow(ctx));
    std::memset(&ctx->timings, 0, sizeof(ctx->timings));
    Timer tm(ctx);
    if (ctx->B > 1) return place_batch(ctx, tm, node_out, cost_out, int_score_out);
    hipStream_t st = ctx->stream, sc = ctx->stream_commit;
    const int P = ctx->P, N = ctx->N;
    int32_t *halt = ctx->status.as<int32_t>();
    // The cost-row cache (NAS_OPT_COST_CACHE, k_rescore_cached): in auto mode
    // when the previous pass of this shape needed CACHE_MIN_ROUNDS rescore
    // rounds or more (a herd: consecutive passes over similar clusters stop
    // alike, as the speculative slots below assume too).  It costs the main
    // cost launches a 4-byte store per (pod, node) and saves every gathered
    // slot its fit / cost / merge launches.  Same placements either way.
    struct CacheOff {
        nas_ctx *c;
        ~CacheOff() { c->cache_active = false; }
    } cache_off{ctx};
    ctx->cache_active = false;
    // (the herd plan below, auto: sticky for a shape once one of its passes
    // needed HERD_MIN_ROUNDS rescore rounds; it turns the cache on too)
    const bool herd_shape = !has_coll(ctx) &&
                            (ctx->opt_herd_plan == 1 ||
                             (ctx->opt_herd_plan == 2 && ctx->herd_P == P && ctx->herd_N == N));
    if (ctx->opt_cost_cache != 0) {
        const bool herd = ctx->slot_hint_P == P && ctx->slot_hint_N == N &&
                          ctx->last_rescore_rounds >= CACHE_MIN_ROUNDS;
        const size_t bytes = (size_t)ctx->Pp * ctx->Mp * 4;
        if ((ctx->opt_cost_cache == 1 || herd || herd_shape) && bytes <= CACHE_MAX_BYTES)
            ctx->cache_active = nas::ensure(ctx, ctx->cost_cache, bytes) == NAS_OK;
        if (!ctx->cache_active) ctx->err.clear();  // (no memory: the slots recompute)
    }
    const bool herd = herd_shape;
    hipEvent_t t0 = tm.mark(st);
    // Each chunk is filtered against the working capacity as the commit
    // stream has left it so far: every value read is >= the capacity at the
    // chunk's pods' own (later) turn, so every node that will fit them is
    // scored (the lists stay exact) and the lists are far fresher than a
    // snapshot at entry -- fewer pods exhaust them.  The LDS commit publishes
    // final values only; the L2 commit's speculative reservations could dip
    // below them, so it also maintains a published copy (cap_snap, start
    // minus committed pods) that scoring reads instead.
    const bool live_cap = nas::commit_in_lds(N);
    const int32_t *score_cap = live_cap ? ctx->cap.as<int32_t>() : ctx->cap_snap.as<int32_t>();
    int32_t *pub = live_cap ? nullptr : ctx->cap_snap.as<int32_t>();
    // one launch: halt = -1, rescores / rounds / slot control = 0 (and the
    // published capacity for the L2 commit) -- three memsets and a copy cost
    // ~60 us of serial enqueue before the first chunk
    auto pass_init = [&](hipStream_t s) -> int {
        HIPCK(nas::launch_pass_init(s, halt, live_cap ? nullptr : ctx->cap.as<int32_t>(),
                                    live_cap ? nullptr : ctx->cap_snap.as<int32_t>(), 3 * N));
        return NAS_OK;
    };
    int32_t *hs = ctx->host_status.as<int32_t>();
    int32_t *stage = reinterpret_cast<int32_t *>(ctx->host_status.as<char>() + host_out_offset(ctx->B));
    // the speculative slots' full copy lands in its own area: the host may
    // still be unpacking chunks from `stage` while that copy runs
    int32_t *stage_spec = stage + 2 * (size_t)ctx->Pp;
    const bool want_raw = cost_out || int_score_out;
    struct Landed { int lo, hi; hipEvent_t ev; };
    std::vector<Landed> landed;
    // chunk bounds; every scoring launch is enqueued before any commit-stream
    // work, so the host's enqueue time of merges / commits / copies never
    // delays the next chunk's cost launch
    const std::vector<std::pair<int, int>> chunks = plan_chunks(ctx, herd);
    // a one-chunk pass without a communicator has nothing to pipeline: its
    // merge / commit / copies stay on the scoring stream, which saves the
    // cross-stream event hops (~15-20 us each) that dominate a small pass
    // (C1 extended 0.41 -> 0.385 ms per nas_place)
    const bool one_stream = chunks.size() == 1 && !has_coll(ctx);
    if (one_stream) sc = st;
    // With the LDS commit nothing the scoring kernels read comes from the
    // pass init (capacity is read live), so the first chunk's fit and cost are
    // the first launches of the pass and the init goes to the commit stream
    // behind the scoring enqueues (C3: the first cost launch started ~45 us
    // after the init, host enqueue time).  The L2 commit's scoring reads the
    // published copy the init makes: init first, on st.  Either way the other
    // streams start behind st's work so far -- the inputs prepared on st
    // above (overflow lists, latency rows, fp32 splits) are read by every
    // chunk's cost launch.
    if (!live_cap) OK(pass_init(st));
    // the two scoring streams (on a node shard CU-masked by set_stream_masks:
    // they leave 2-3 CUs per XCD to the commit stream, profiles/r04_ab_reserve.txt;
    // round 3's masks that reserved 8-16 CUs beside the narrow tile measured
    // 25-35% slower, r03_ab_reserve_cus.txt)
    const int spec = (!herd && !has_coll(ctx) && ctx->slot_hint_P == P && ctx->slot_hint_N == N)
                         ? ctx->slot_hint : 0;
    // (the herd plan's slots run inside its chunk loop, behind each commit;
    // pods they place after their chunk's rows were staged are unpacked again
    // at the end, like the speculative slots' -- `late_slots`)
    const bool late_slots = spec > 0 || herd;
    // (an injected stall, NAS_OPT_INJECT_STALL_MS, sits on st behind the
    // pass: the host must wait on st then)
    // (the pass's last commit writes the status words to the pinned host area)
    const bool status_in_commit = !late_slots && ctx->opt_inject_stall_ms == 0;
    // its bound: with collectives the communicator deadline -- the
    // commit stream's last commit may wait on an all-gather whose peer died --
    // so the pass fails as a communicator failure (below), never with a
    // shorter fixed budget that makes the tail "complete" while RCCL is stuck
    const int64_t commit_wait_ms =
        ctx->opt_commit_wait_ms > 0 ? ctx->opt_commit_wait_ms
        : has_coll(ctx)             ? (ctx->opt_comm_timeout_ms > 0 ? ctx->opt_comm_timeout_ms : 600000)
                                    : 2000;
    if (herd) {
        // The herd plan: chunks of one wave of cost workgroups, scored and
        // merged back to back on one stream; each chunk's commit and
        // HERD_SLOTS gathered slots run on the commit stream, on the CUs that
        // wave leaves free, while the next chunk's workgroups run their main loop
        // -- so the next chunk's fused fit, read after that loop, sees this
        // chunk's commits (lag ~1) instead of a capacity two or more chunks
        // stale.  In a global herd (configs.C3_fullrange: every pod ranks the
        // same nodes first) the pipelined plan's stale lists run dry for most
        // pods: ~90 gathered slots per C3 pass.  The slots here rescore from
        // the cost-row cache only (their recomputing form would share the
        // scoring buffers with the next chunk's launch); without it a halt
        // waits for the host loop.
        if (live_cap) OK(pass_init(st));
        HIPCK(hipStreamWaitEvent(sc, tm.mark(st), 0));
        for (size_t c = 0; c < chunks.size(); ++c) {
            const int lo = chunks[c].first, hi = chunks[c].second;
            const bool last = c + 1 == chunks.size();
            // (the merge on the scoring stream, behind its cost launch, with
            // the whole GPU: ~10 us; on the commit stream's leftover CUs it
            // took ~60 us, and the commit stream fell behind the scoring)
            OK(score_range(ctx, tm, lo, hi, st, score_cap, nullptr, false));
            OK(merge_range(ctx, tm, lo, hi, st, CH_SCORE, 0, main_view(ctx)));
            HIPCK(hipStreamWaitEvent(sc, tm.mark(st), 0));
            hipEvent_t c0 = tm.fine(sc);
            HIPCK(nas::launch_commit(sc, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                                     ctx->req.as<int32_t>(), ctx->Pp, lo, hi, ctx->cap.as<int32_t>(),
                                     N, ctx->out_node.as<int32_t>(), ctx->out_cost_i.as<int32_t>(),
                                     halt, 1, pub, zrow_ptr(ctx), stage, want_raw ? stage + P : nullptr,
                                     last && status_in_commit ? hs : nullptr));
            tm.span(T_COMMIT, c0, tm.fine(sc));
            // a walk halted in this chunk resumes here, before the chunk after
            // next is scored (a halt they leave is resumed by a later chunk's
            // slots or the host loop below); idle slots are three launches
            // that exit at once
            if (ctx->cache_active)
                for (int r = 0; r < HERD_SLOTS; ++r)
                    OK(gathered_slot(ctx, tm, sc, CH_SCORE, pub, hi, HERD_SLOT_PODS));
            landed.push_back({lo, hi, tm.mark(sc)});
        }
        HIPCK(hipStreamWaitEvent(st, tm.mark(sc), 0));
    } else {
        const hipStream_t ss2[2] = {st, ctx->stream2};
        if (!one_stream) {
            hipEvent_t ready = tm.mark(st);
            for (hipStream_t s : {ss2[0], ss2[1], sc})
                if (s != st) HIPCK(hipStreamWaitEvent(s, ready, 0));
        }
        std::vector<hipEvent_t> scored(chunks.size());
        // fit + cost only on the two scoring streams (a chunk's tail blocks overlap
        // the next chunk; a third scoring stream measured 5% slower at G = 1 and
        // 6-25% at G = 8); the commit stream merges (and exchanges, over its own
        // communicator) each chunk right before committing it, so no cost launch
        // ever waits behind a merge or an all-gather
        for (size_t c = 0; c < chunks.size(); ++c) {
            hipStream_t ss = ss2[c & 1];
            OK(score_range(ctx, tm, chunks[c].first, chunks[c].second, ss, score_cap, nullptr, false));
            // (one stream: nothing waits on it -- every event record or wait is a
            // packet the queue processes between two kernels)
            scored[c] = one_stream ? nullptr : tm.mark(ss);
        }
        // (one stream: the chunk's merge starts the status words itself)
        const bool init_in_merge = one_stream && live_cap;
        if (live_cap && !init_in_merge) OK(pass_init(sc));
        // speculative slots: as many as the previous pass of this shape needed
        // (consecutive passes over similar clusters stop alike), enqueued before
        // the first status round trip; a slot whose walk is not halted exits at
        // once.  Not with a communicator: every rank must issue the same slots.
        // A node-shard pass's chunks merge and exchange on their own stream (sx,
        // the commit stream's communicator and CUs) and the commit stream only
        // commits, each commit waiting for its chunk's merged lists: with every
        // chunk's merge -> all-gather -> merge -> commit chain on the commit
        // stream the chains of the last two chunks ran back to back after the
        // scoring (~108 us each at G = 8 with six shard chunks); now one chunk's
        // exchange overlaps the previous chunk's commit.  The tail chunk merges
        // and exchanges on its scoring stream right behind its cost launch (its
        // stream's own communicator and gather buffers, so the collectives of
        // each communicator stay on one stream in one order) and commits there
        // after the commit stream's last commit.
        const bool xs_mode = exchanging(ctx) && !one_stream;
        // the tail chunk's stream waits for the commit stream's last commit: by
        // the device word behind each commit (launch_flag_set / flag_wait) once a
        // commit has run on the commit stream, else by an event (a one-chunk pass
        // with a communicator: only the pass init is on the commit stream)
        auto *cflag = ctx->commit_flag.as<uint64_t>();
        auto after_commits = [&](hipStream_t s) -> int {
            if (chunks.size() > 1)
                HIPCK(nas::launch_flag_wait(s, cflag, ctx->commit_seq, halt, commit_wait_ms));
            else HIPCK(hipStreamWaitEvent(s, tm.mark(sc), 0));
            return NAS_OK;
        };
        hipStream_t sx = nullptr;
        if (xs_mode) OK(exchange_stream(ctx, &sx));
        for (size_t c = 0; c < chunks.size(); ++c) {
            const int lo = chunks[c].first, hi = chunks[c].second;
            // the last chunk is merged and committed on its own scoring stream
            // behind the commit stream's earlier work (long finished by then), so
            // the pass's serial tail after the last cost launch has no
            // cross-stream hop in front of its merge (the communicator is the
            // commit stream's: its collectives stay in one order)
            const bool tail = !one_stream && c + 1 == chunks.size();
            const bool last = c + 1 == chunks.size();
            hipStream_t cs = sc;
            if (xs_mode) {
                if (tail) {
                    cs = ss2[c & 1];
                    OK(merge_range(ctx, tm, lo, hi, cs, (c & 1) ? CH_SCORE2 : CH_SCORE, (int)(c & 1),
                                   main_view(ctx)));
                    OK(after_commits(cs));
                } else {
                    HIPCK(hipStreamWaitEvent(sx, scored[c], 0));
                    OK(merge_range(ctx, tm, lo, hi, sx, CH_COMMIT, 2, main_view(ctx)));
                    HIPCK(hipStreamWaitEvent(sc, tm.mark(sx), 0));
                }
            } else {
                if (tail) {
                    cs = ss2[c & 1];
                    OK(after_commits(cs));
                } else if (!one_stream) {
                    HIPCK(hipStreamWaitEvent(sc, scored[c], 0));
                }
                // (merging the tail chunk locally before this wait, gated before
                // its exchange / commit, measured within noise at G = 1 and 8:
                // profiles/r04_ab_tail.txt)
                OK(merge_range(ctx, tm, lo, hi, cs, CH_COMMIT, 0, main_view(ctx),
                               init_in_merge ? halt : nullptr));
            }
            hipEvent_t c0 = tm.fine(cs);
            // the pass's last commit also writes the status words into the pinned
            // host area when nothing follows it (no speculative slots): the host
            // then waits for that commit alone, with no status copy behind it
            HIPCK(nas::launch_commit(cs, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                                     ctx->req.as<int32_t>(), ctx->Pp, lo, hi, ctx->cap.as<int32_t>(), N,
                                     ctx->out_node.as<int32_t>(), ctx->out_cost_i.as<int32_t>(), halt,
                                     1, pub, zrow_ptr(ctx), stage, want_raw ? stage + P : nullptr,
                                     last && status_in_commit ? hs : nullptr));
            // (releases the tail chunk's commit)
            if (!one_stream && !last) {
                if (c + 2 == chunks.size() && ctx->opt_inject_commit_stall_ms > 0) {
                    (void)nas::launch_stall(cs, ctx->opt_inject_commit_stall_ms);  // (test option)
                    ctx->opt_inject_commit_stall_ms = 0;
                }
                HIPCK(nas::launch_flag_set(cs, cflag, ++ctx->commit_seq));
            }
            tm.span(T_COMMIT, c0, tm.fine(cs));
            // the commit wrote this chunk's results into the pinned stage as it
            // ended, and the host unpacks them while later chunks still run.
            // Stage ordering rule: every stage row the host reads
            // has ONE writer in the pass -- this commit kernel (to_stage), or
            // fetch()'s copies on `st` issued after the host has waited for every
            // landed event -- and the host reads it only after waiting on an
            // event recorded on the writer's stream behind the writer.  No D2H
            // copy into the stage runs on a scoring stream (round 4's TAIL_SDMA
            // variant moved the last chunk's rows to such a copy and returned
            // stale rows: profiles/r05e_stage_order_probe.txt)
            landed.push_back({lo, hi, tm.mark(cs)});
        }
        // st must follow everything: the last chunk's stream followed the commit
        // stream, which followed every earlier chunk's scoring (and, with xs_mode,
        // every earlier chunk's exchange); so st waits only when the last chunk
        // ran on another stream
        if (!one_stream && ss2[(chunks.size() - 1) & 1] != st)
            HIPCK(hipStreamWaitEvent(st, tm.mark(ss2[(chunks.size() - 1) & 1]), 0));
        // (the tail followed the commit stream by the device word, not a stream
        // wait: st follows the commit stream itself)
        if (!one_stream && chunks.size() > 1) HIPCK(hipStreamWaitEvent(st, tm.mark(sc), 0));
    }
    if (has_coll(ctx)) inject_stall(ctx, st);  // behind every collective of the pass
    for (int r = 0; r < spec; ++r) OK(gathered_slot(ctx, tm, st, CH_SCORE, nullptr, P));
    if (late_slots) {
        // behind the slots, all placements again: when they finished the walk,
        // the status round trip below brings the final results with it
        HIPCK(hipMemcpyAsync(stage_spec, ctx->out_node.p, (size_t)P * 4, hipMemcpyDeviceToHost,
                             st));
        if (want_raw)
            HIPCK(hipMemcpyAsync(stage_spec + P, ctx->out_cost_i.p, (size_t)P * 4,
                                 hipMemcpyDeviceToHost, st));
    }
    hipEvent_t t1 = nullptr;
    // status words in one copy: halt[0..2] = halt word, slot resumes, commit
    // rounds; halt[STATUS_INTS + 2] (slot control) = pods rescored
    constexpr int NSTAT = nas::COMMIT_STATUS_WORDS, RESCORED = nas::STATUS_INTS + 2;
    auto fetch = [&]() -> int {
        HIPCK(hipMemcpyAsync(hs, halt, NSTAT * 4, hipMemcpyDeviceToHost, st));
        HIPCK(hipMemcpyAsync(stage, ctx->out_node.p, (size_t)P * 4, hipMemcpyDeviceToHost, st));
        if (want_raw)
            HIPCK(hipMemcpyAsync(stage + P, ctx->out_cost_i.p, (size_t)P * 4, hipMemcpyDeviceToHost,
                                 st));
        t1 = tm.mark(st);
        return wait_event(ctx, t1);
    };
    int unsched = 0;
    // decode pods [lo, hi) from a staging area (placements, then raw keys)
    // (the last chunks land together at the end of the pass, so their unpack
    // is on the pass's critical path: one tight loop per output with the
    // dtype hoisted and no aliasing, so each vectorises)
    auto unpack = [&](int lo, int hi, const int32_t *from) {
        unpack_range(node_out, cost_out, int_score_out, from, from + P, lo, hi, ctx->dtype, unsched);
    };
    // the walk's status comes back in one round trip on `st`; meanwhile the
    // host unpacks each chunk as its copy lands.  Values copied behind a commit
    // are final unless the walk halted there -- then (rare) more slots run and
    // everything is fetched and unpacked again.
    if (status_in_commit) {
        t1 = landed.back().ev;  // the last commit wrote hs itself
    } else {
        HIPCK(hipMemcpyAsync(hs, halt, NSTAT * 4, hipMemcpyDeviceToHost, st));
        t1 = tm.mark(st);
    }
    for (const Landed &l : landed) {
        OK(wait_event(ctx, l.ev));
        unpack(l.lo, l.hi, stage);
    }
    OK(wait_event(ctx, t1));  // t1 follows the status words (copy, or the last commit)
    int checks = 0;
    if (late_slots && hs[0] < 0 && hs[1] > 0) {
        // speculative slots finished a walk that had halted: the per-chunk
        // copies behind the commits predate them; the full copy behind the
        // slots (same round trip, its own staging area) holds the final
        // placements -- from the first halt on (status word 3, the first
        // resume's pod): the pods before it were final in their chunks' copies
        const int h0 = std::min(std::max(hs[3], 0), P);
        unsched = 0;
        for (int i = 0; i < h0; ++i) unsched += node_out[i] < 0;
        unpack(h0, P, stage_spec);
    }
    // the first halt the host sees: every pod before it was final in its
    // chunk's copy, unpacked as it landed (the slots resume the walk there),
    // so only [h0, P) is unpacked again -- a bf16 C3 halt sits in the last
    // chunk, and re-unpacking all 100k pods cost ~0.25 ms of host time
    int h0 = -1;
    if (hs[0] == nas::FLAG_TIMEOUT_HALT) {
        // the tail commit's wait for the commit stream ran out (k_flag_wait):
        // with collectives a peer is gone or stuck -- abort, as a missed
        // deadline does (the stuck collective kernels return, so the streams
        // drain and nas_destroy cannot block on them)
        const std::string why = "the last commit's wait for the commit stream exceeded " +
                                std::to_string(commit_wait_ms) + " ms";
        if (has_coll(ctx)) {
            abort_comms(ctx);
            return nas::fail(ctx, NAS_ERR_COMM,
                             why + " (NAS_OPT_COMM_TIMEOUT_MS): communicators aborted, context poisoned");
        }
        return nas::fail(ctx, NAS_ERR_HIP, why + " (NAS_OPT_COMMIT_WAIT_MS)");
    }
    while (hs[0] >= 0) {
        // still halted after the pipeline: more gathered slots, checked in batches
        if (hs[0] >= P) return nas::fail(ctx, NAS_ERR_HIP, "commit halt word corrupt");
        if (++checks > P + 1) return nas::fail(ctx, NAS_ERR_HIP, "commit made no progress");
        // (with speculative slots the walk may have resumed and halted again:
        // its first halt is status word 3)
        if (h0 < 0) h0 = late_slots ? (hs[1] > 0 ? std::min(std::max(hs[3], 0), hs[0]) : hs[0]) : hs[0];
        for (int r = 0, n = gather_batch(checks, ctx->cache_active); r < n; ++r)
            OK(gathered_slot(ctx, tm, st, CH_SCORE, nullptr, P));
        OK(fetch());
        if (hs[0] < 0) {
            unsched = 0;
            for (int i = 0; i < h0; ++i) unsched += node_out[i] < 0;
            unpack(h0, P, stage);
        }
    }
    tm.span(T_TOTAL, t0, t1);
    ctx->timings.fit_ms = tm.total(T_FIT);
    ctx->timings.cost_ms = tm.total(T_COST);
    ctx->timings.merge_ms = tm.total(T_MERGE);
    ctx->timings.commit_ms = tm.total(T_COMMIT);
    ctx->timings.total_ms = tm.total(T_TOTAL);
    ctx->timings.rescore_rounds = hs[1];
    ctx->timings.rescored_pods = hs[RESCORED];
    ctx->timings.unschedulable = unsched;
    ctx->timings.commit_rounds = hs[2];
    ctx->slot_hint = std::min(hs[1], MAX_SPEC_SLOTS);
    ctx->last_rescore_rounds = hs[1];
    if (hs[1] >= HERD_MIN_ROUNDS) {
        ctx->herd_P = P;
        ctx->herd_N = N;
    }
    ctx->slot_hint_P = P;
    ctx->slot_hint_N = N;
    ctx->scored = true;
    return NAS_OK;
}

int nas_get_candidates(nas_ctx *ctx, int32_t *cand_node, int64_t *cand_cost_i, float *cand_cost_f,
                       int32_t *count, int32_t *complete) {
    NAS_RANGE("nas_get_candidates");
    OK(bind(ctx));
    if (!ctx->scored) return nas::fail(ctx, NAS_ERR_STATE, "no scoring pass yet");
    const int64_t P = (int64_t)ctx->B * ctx->P;  // a batch: B clusters back to back
    std::vector<uint64_t> keys((size_t)P * KC), bounds(P);
    HIPCK(hipMemcpy2DAsync(keys.data(), (size_t)ctx->P * KC * 8, ctx->cand_key.p,
                           (size_t)ctx->Pp * KC * 8, (size_t)ctx->P * KC * 8, ctx->B,
                           hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipMemcpy2DAsync(bounds.data(), (size_t)ctx->P * 8, ctx->cand_bound.p, (size_t)ctx->Pp * 8,
                           (size_t)ctx->P * 8, ctx->B, hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    for (int64_t p = 0; p < P; ++p) {
        int c = 0;
        for (int j = 0; j < KC; ++j) {
            const uint64_t k = keys[(size_t)p * KC + j];
            const bool ok = k != nas::KEY_INVALID && k <= bounds[p];  // exact prefix only
            c += ok;
            if (cand_node) cand_node[(size_t)p * KC + j] = ok ? (int32_t)(uint32_t)k : -1;
            const uint32_t raw = (uint32_t)(k >> 32);
            if (cand_cost_i)
                cand_cost_i[(size_t)p * KC + j] =
                    (ok && ctx->dtype == NAS_DT_I8) ? (int64_t)(int32_t)(raw ^ 0x80000000u) : 0;
            if (cand_cost_f) cand_cost_f[(size_t)p * KC + j] = ok ? decode_cost(raw, ctx->dtype) : 0.f;
        }
        if (count) count[p] = c;
        if (complete) complete[p] = bounds[p] == nas::KEY_INVALID;
    }
    return NAS_OK;
}

// ------------------------------------------------------- host-driven steps
int nas_score_range(nas_ctx *ctx, int32_t p_lo, int32_t p_hi) {
    NAS_RANGE("nas_score_range");
    OK(bind(ctx));
    OK(no_batch(ctx, "nas_score_range"));
    OK(check_extended(ctx));
    if (p_lo < 0 || p_hi > ctx->P || p_lo >= p_hi)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_score_range: pod range");
    OK(alloc_extended(ctx));
    OK(prepare_ovf(ctx));
    OK(prepare_split(ctx));
    OK(prepare_zrow(ctx));
    std::memset(&ctx->timings, 0, sizeof(ctx->timings));
    Timer tm(ctx);
    OK(score_range(ctx, tm, p_lo, p_hi));
    if (has_coll(ctx)) inject_stall(ctx, ctx->stream);
    OK(sync_stream(ctx, ctx->stream));
    ctx->timings.fit_ms = tm.total(T_FIT);
    ctx->timings.cost_ms = tm.total(T_COST);
    ctx->timings.merge_ms = tm.total(T_MERGE);
    ctx->scored = true;
    return NAS_OK;
}

static int keys_range_ok(nas_ctx *ctx, int32_t p_lo, int32_t n, const void *keys,
                         const void *bounds) {
    if (!ctx->scored) return nas::fail(ctx, NAS_ERR_STATE, "no scoring pass yet");
    if (p_lo < 0 || n < 0 || p_lo + n > ctx->P || (n > 0 && (!keys || !bounds)))
        return nas::fail(ctx, NAS_ERR_ARG, "candidate key range");
    return NAS_OK;
}

int nas_get_candidate_keys_range(nas_ctx *ctx, int32_t p_lo, int32_t n, uint64_t *keys,
                                 uint64_t *bounds) {
    NAS_RANGE("nas_get_candidate_keys_range");
    OK(bind(ctx));
    OK(no_batch(ctx, "candidate key ranges"));
    OK(keys_range_ok(ctx, p_lo, n, keys, bounds));
    if (n == 0) return NAS_OK;
    HIPCK(hipMemcpyAsync(keys, ctx->cand_key.as<uint64_t>() + (size_t)p_lo * KC, (size_t)n * KC * 8,
                         hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipMemcpyAsync(bounds, ctx->cand_bound.as<uint64_t>() + p_lo, (size_t)n * 8,
                         hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    return NAS_OK;
}

int nas_set_candidate_keys(nas_ctx *ctx, int32_t p_lo, int32_t n, const uint64_t *keys,
                           const uint64_t *bounds) {
    NAS_RANGE("nas_set_candidate_keys");
    OK(bind(ctx));
    OK(no_batch(ctx, "candidate key ranges"));
    OK(check_extended(ctx));
    OK(alloc_extended(ctx));  // lists sized for the current pods
    if (p_lo < 0 || n < 0 || p_lo + n > ctx->P || (n > 0 && (!keys || !bounds)))
        return nas::fail(ctx, NAS_ERR_ARG, "candidate key range");
    // the commit relies on sorted lists with in-range node ids
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        const uint64_t *k = keys + i * KC;
        for (int j = 0; j < KC; ++j) {
            if (j && k[j] < k[j - 1])
                return nas::fail(ctx, NAS_ERR_ARG, "candidate keys not ascending");
            if (k[j] != nas::KEY_INVALID && (int64_t)(uint32_t)k[j] >= ctx->N)
                return nas::fail(ctx, NAS_ERR_ARG, "candidate key names a node out of range");
        }
    }
    if (n == 0) return NAS_OK;
    HIPCK(hipMemcpyAsync(ctx->cand_key.as<uint64_t>() + (size_t)p_lo * KC, keys, (size_t)n * KC * 8,
                         hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipMemcpyAsync(ctx->cand_bound.as<uint64_t>() + p_lo, bounds, (size_t)n * 8,
                         hipMemcpyHostToDevice, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    ctx->scored = true;
    return NAS_OK;
}

int nas_commit(nas_ctx *ctx, int32_t p_begin, int32_t *node_out, float *cost_out,
               int64_t *int_score_out, int32_t *stop_out) {
    NAS_RANGE("nas_commit");
    OK(bind(ctx));
    OK(no_batch(ctx, "nas_commit"));
    OK(check_extended(ctx));
    if (!ctx->scored) return nas::fail(ctx, NAS_ERR_STATE, "nas_commit needs candidate lists");
    if (!node_out || !stop_out || p_begin < 0 || p_begin > ctx->P)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_commit arguments");
    OK(alloc_extended(ctx));  // (scored implies they match; cheap when they do)
    OK(prepare_zrow(ctx));
    const int P = ctx->P;
    *stop_out = P;
    if (p_begin == P) return NAS_OK;
    std::memset(&ctx->timings, 0, sizeof(ctx->timings));
    Timer tm(ctx);
    hipStream_t st = ctx->stream;
    int32_t *halt = ctx->status.as<int32_t>();
    HIPCK(hipMemsetAsync(halt, 0xff, 4, st));
    HIPCK(hipMemsetAsync(halt + 1, 0, 8, st));
    hipEvent_t c0 = tm.mark(st);
    HIPCK(nas::launch_commit(st, ctx->cand_key.as<uint64_t>(), ctx->cand_bound.as<uint64_t>(),
                             ctx->req.as<int32_t>(), ctx->Pp, p_begin, P, ctx->cap.as<int32_t>(),
                             ctx->N, ctx->out_node.as<int32_t>(), ctx->out_cost_i.as<int32_t>(),
                             halt, 1, nullptr, zrow_ptr(ctx)));
    tm.span(T_COMMIT, c0, tm.mark(st));
    int32_t *hs = ctx->host_status.as<int32_t>();
    HIPCK(hipMemcpyAsync(hs, halt, 12, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    const int stop = hs[0] >= 0 ? hs[0] : P;
    if (stop < p_begin || stop > P) return nas::fail(ctx, NAS_ERR_HIP, "commit halt word corrupt");
    const int n = stop - p_begin;
    std::vector<uint32_t> raw(n);
    if (n) {
        HIPCK(hipMemcpyAsync(node_out + p_begin, ctx->out_node.as<int32_t>() + p_begin,
                             (size_t)n * 4, hipMemcpyDeviceToHost, st));
        HIPCK(hipMemcpyAsync(raw.data(), ctx->out_cost_i.as<int32_t>() + p_begin, (size_t)n * 4,
                             hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
    }
    for (int i = 0; i < n; ++i) {
        const bool none = node_out[p_begin + i] < 0;
        if (cost_out) cost_out[p_begin + i] = none ? 0.f : decode_cost(raw[i], ctx->dtype);
        if (int_score_out)
            int_score_out[p_begin + i] = (none || ctx->dtype != NAS_DT_I8)
                                             ? 0 : (int64_t)(int32_t)(raw[i] ^ 0x80000000u);
    }
    *stop_out = stop;
    ctx->timings.commit_ms = tm.total(T_COMMIT);
    ctx->timings.commit_rounds = hs[2];
    return NAS_OK;
}

// ---------------------------------------------------------------- multi-GPU
namespace {
// CUs per XCD kept for the commit and exchange streams on a node shard of
// `world` ranks: same-box A/B (profiles/r04_ab_reserve.txt), rank-0
// rehearsal ms per pass at reserve 0 (narrow tile) / 2 / 3 / 4: G = 2
// 4.13-4.21 / 3.92-3.97 / 3.96-4.00 / 3.99-4.03, G = 4 2.27-2.29 / 2.19-2.20
// / 2.20-2.22 / 2.16-2.20, G = 8 1.28-1.32 / 1.27-1.28 / 1.24-1.26 /
// 1.24-1.29.  With six shard chunks and the exchange stream (round 5) the
// chains want one CU more: G = 8 4 vs 3 1.186 vs 1.196 ms, G = 4 3 vs 2
// 2.107 vs 2.117 ms (profiles/r05an_ab_reserve.txt)
int shard_reserve(int world) {
    if (world <= 1) return 0;
    return world >= 8 ? RESERVE_SHARD_CUS + 2 : world >= 4 ? RESERVE_SHARD_CUS + 1 : RESERVE_SHARD_CUS;
}
// Recreate the context's three streams: reserve > 0 keeps `reserve` CUs of
// every XCD for the commit stream alone and the rest for the two scoring
// streams (hipExtStreamCreateWithCUMask: mask bit i is CU i / 8 of XCD i % 8,
// tools/cumask_probe.hip; an XCD whose bits are all clear would run on ALL its
// CUs, so every mask keeps CUs on every XCD); reserve 0 restores plain
// streams.  Only between calls (nothing in flight).  The masked streams are
// BLOCKING streams at the default priority (the CU-mask constructor takes no
// flags): they serialise with the legacy NULL stream, which nothing of the
// engine uses (every call works on its own streams and waits on its own
// events), and the commit stream needs no priority there because it has CUs
// of its own.
int set_stream_masks(nas_ctx *ctx, int reserve) {
    if (reserve == ctx->cu_reserve) return NAS_OK;
    int ncu = 0;
    HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    if (reserve > 0 && (ncu % 8 || ncu / 8 <= 2 * reserve)) reserve = 0;  // not an 8-XCD part
    if (reserve == ctx->cu_reserve) return NAS_OK;
    for (hipStream_t s : {ctx->stream, ctx->stream2, ctx->stream_commit, ctx->stream_x})
        if (s) HIPCK(hipStreamSynchronize(s));
    hipStream_t ns[3] = {nullptr, nullptr, nullptr};
    hipError_t e = hipSuccess;
    std::vector<uint32_t> ms, mc;
    if (reserve > 0) {
        reserve_masks(ncu, reserve, ms, mc);
        for (int i = 0; i < 3 && e == hipSuccess; ++i)
            e = masked_acquire(ctx->device, i == 2 ? mc : ms, &ns[i]);
    } else {
        int lo = 0, hi = 0;
        e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&ns[0], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&ns[1], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&ns[2], hipStreamNonBlocking, hi);
    }
    if (e != hipSuccess) {
        for (int i = 0; i < 3; ++i)
            if (ns[i]) {
                if (reserve > 0) masked_release(ctx->device, i == 2 ? mc : ms, ns[i]);
                else (void)hipStreamDestroy(ns[i]);
            }
        return nas::hip_fail(ctx, e, "set_stream_masks");
    }
    // the old streams go back (masked ones to the pool); the exchange stream
    // is made again on first use, on the commit stream's CUs
    drop_streams(ctx);
    ctx->stream = ns[0];
    ctx->stream2 = ns[1];
    ctx->stream_commit = ns[2];
    ctx->cu_reserve = reserve;
    return NAS_OK;
}
}  // namespace



int nas_comm_unique_id(uint8_t id_out[128]) {
    NAS_RANGE("nas_comm_unique_id");
    if (!id_out) return NAS_ERR_ARG;
    ncclUniqueId id;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    if (ncclGetUniqueId(&id) != ncclSuccess) return NAS_ERR_COMM;
    std::memcpy(id_out, &id, 128);
    return NAS_OK;
}

int nas_comm_init(nas_ctx *ctx, const uint8_t id[128], int32_t rank, int32_t world) {
    NAS_RANGE("nas_comm_init");
    OK(bind(ctx));
    if (!id || world < 1 || rank < 0 || rank >= world)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_comm_init: rank/world");
    if (ctx->have_L || ctx->have_wa || ctx->have_cap)
        return nas::fail(ctx, NAS_ERR_STATE, "nas_comm_init must precede the extended uploads");
    if (ctx->B > 1 && world > 1)
        return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "node shards of a cluster batch");
    destroy_comms(ctx);
    // the previous communicators are gone: until this call succeeds the
    // context is a single rank (a context left at world > 1 without
    // communicators would fail every sharded call with a null communicator),
    // on plain streams (no CUs kept for a commit stream of a shard)
    ctx->rank = 0;
    ctx->world = 1;
    ctx->rehearse = 0;
    ctx->virtual_shard = false;
    OK(set_stream_masks(ctx, 0));
    int32_t eff_world = world, rehearse = 0;
    if (ctx->opt_rehearse_world > 1 && world == 1) {
        // diagnostic (NAS_OPT_REHEARSE_WORLD): one rank of a G-GPU pass
        rehearse = ctx->opt_rehearse_world;
        eff_world = rehearse;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    // ncclCommInitRank waits in RCCL's bootstrap until every rank has joined,
    // in the calling thread (RCCL 2.27, blocking or not), so a rank whose
    // peers never arrive would block forever.  The communicators are built
    // on a helper thread, all NON-blocking (config.blocking = 0): a root,
    // whose handle RCCL publishes as soon as it exists, and three children
    // initialised from ids rank 0 broadcasts over the root (no ncclCommSplit:
    // RCCL 2.26 fails a split of a non-blocking root with an internal error)
    // (one per stream that issues collectives: scoring stream 1,
    // scoring stream 2, commit stream -- each keeps its own issue order on
    // every rank), each warmed up by one small all-gather so its connections
    // exist before the first pass (the pass's collectives then enqueue at
    // once; nccl_enqueued polls the rare ncclInProgress).  This thread waits
    // under NAS_OPT_COMM_TIMEOUT_MS; on expiry it CLAIMS every published
    // handle under the state's mutex and aborts it, which ends the helper's
    // bootstrap wait (measured: the helper returns ~2.5 s after the abort).
    // Handle ownership: the helper touches a handle only under the mutex and
    // only while it is unclaimed (except inside the init call that creates
    // it), so no RCCL call of the helper races the main thread's abort; a
    // handle that appears after the claim is aborted by the helper itself.
    // A helper still inside RCCL 30 s after the aborts is parked in the
    // context: joined by the next nas_comm_init once done, or by nas_destroy,
    // which waits up to 2 s for it and then detaches it (it holds no
    // reference to the context).  Every communicator is non-blocking
    // (config.blocking = 0, root and children), so the RCCL calls `guarded`
    // makes under the mutex (broadcast, warm-up all-gathers, async-error
    // polls) return at once (ncclInProgress at worst) and never hold the
    // mutex against the main thread's claim-and-abort.
    reap_comm_helpers(ctx);
    auto st = std::make_shared<nas::CommInit>();
    const int dev = ctx->device;
    using CI = nas::CommInit;
    std::thread helper([st, dev, uid, rank, world]() mutable {
        auto load = [](ncclComm_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); };
        auto slot = [&](int i) -> ncclComm_t * { return i == CI::ROOT ? &st->root : &st->kids[i]; };
        // run f(handle i) under the mutex unless the init was abandoned or
        // the main thread claimed the handle
        auto guarded = [&](int i, auto &&f) -> ncclResult_t {
            std::lock_guard<std::mutex> g(st->mu);
            if (st->abandoned || (st->claimed >> i & 1u)) return ncclInvalidUsage;
            return f(load(slot(i)));
        };
        // poll handle i until its pending work is done
        auto settle = [&](int i) -> ncclResult_t {
            for (;;) {
                ncclResult_t a = ncclInProgress;
                const ncclResult_t q = guarded(i, [&](ncclComm_t c) { return ncclCommGetAsyncError(c, &a); });
                if (q != ncclSuccess) return q;
                if (a != ncclInProgress) return a;
                std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
        };
        // an init call returned: if the call was abandoned meanwhile, the
        // handle it published after the main thread's claim is ours to abort
        auto after_init = [&](int i, ncclResult_t r) -> ncclResult_t {
            std::lock_guard<std::mutex> g(st->mu);
            if (!st->abandoned) return r;
            ncclComm_t c = load(slot(i));
            if (c && !(st->claimed >> i & 1u)) {
                st->claimed |= 1u << i;
                (void)ncclCommAbort(c);
            }
            return ncclInvalidUsage;
        };
        auto abandoned = [&] {
            std::lock_guard<std::mutex> g(st->mu);
            return st->abandoned;
        };
        ncclResult_t r = hipSetDevice(dev) == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
        std::string what = "hipSetDevice";
        if (r == ncclSuccess) {
            what = "ncclCommInitRankConfig";
            ncclConfig_t rc = NCCL_CONFIG_INITIALIZER;
            rc.blocking = 0;
            r = after_init(CI::ROOT, ncclCommInitRankConfig(&st->root, world, uid, rank, &rc));
            if (r == ncclInProgress && load(&st->root)) r = settle(CI::ROOT);
            if (r == ncclSuccess && !load(&st->root)) r = ncclInternalError;
        }
        hipStream_t s = nullptr;
        void *buf = nullptr;
        hipEvent_t ev = nullptr;
        // device scratch: 3 child ids (broadcast) and the warm-up all-gathers
        const size_t scratch = 3 * sizeof(ncclUniqueId) + 8 * ((size_t)world + 1);
        if (r == ncclSuccess &&
            (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
             hipMalloc(&buf, scratch) != hipSuccess ||
             hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess))
            r = ncclUnhandledCudaError;
        // wait for everything enqueued on s (polled, so an abandoned init ends)
        auto drain = [&]() -> ncclResult_t {
            if (hipEventRecord(ev, s) != hipSuccess) return ncclUnhandledCudaError;
            for (;;) {
                const hipError_t q = hipEventQuery(ev);
                if (q == hipSuccess) return ncclSuccess;
                if (q != hipErrorNotReady) return ncclUnhandledCudaError;
                if (abandoned()) return ncclInvalidUsage;
                std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
        };
        bool inflight = false;  // collectives enqueued on s and not yet drained
        // the three children: rank 0 draws their ids and broadcasts them over
        // the root, every rank then initialises them as ordinary non-blocking
        // communicators (ncclCommSplit of a non-blocking root returns
        // ncclInternalError on torch's RCCL 2.26.6: see the round-3 GPU test log)
        ncclUniqueId *kid_ids = nullptr;  // pinned: the copies never block the thread
        const size_t ids_bytes = 3 * sizeof(ncclUniqueId);
        if (r == ncclSuccess && hipHostMalloc(reinterpret_cast<void **>(&kid_ids), ids_bytes,
                                              hipHostMallocDefault) != hipSuccess)
            r = ncclUnhandledCudaError;
        if (r == ncclSuccess) {
            what = "child ids";
            std::memset(kid_ids, 0, ids_bytes);
            if (rank == 0)
                for (int i = 0; i < 3 && r == ncclSuccess; ++i) r = ncclGetUniqueId(&kid_ids[i]);
            if (r == ncclSuccess &&
                hipMemcpyAsync(buf, kid_ids, ids_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
                r = ncclUnhandledCudaError;
            if (r == ncclSuccess) {
                r = guarded(CI::ROOT, [&](ncclComm_t root) {
                    return ncclBroadcast(buf, buf, ids_bytes, ncclUint8, 0, root, s);
                });
                if (r == ncclInProgress) r = settle(CI::ROOT);
                inflight = r == ncclSuccess;
            }
            if (r == ncclSuccess &&
                hipMemcpyAsync(kid_ids, buf, ids_bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
                r = ncclUnhandledCudaError;
            if (r == ncclSuccess) r = drain();
            if (r == ncclSuccess) inflight = false;
        }
        for (int i = 0; i < 3 && r == ncclSuccess; ++i) {
            what = "ncclCommInitRankConfig (child)";
            ncclConfig_t kc = NCCL_CONFIG_INITIALIZER;
            kc.blocking = 0;
            r = after_init(i, ncclCommInitRankConfig(&st->kids[i], world, kid_ids[i], rank, &kc));
            if (r == ncclInProgress && load(&st->kids[i])) r = settle(i);
            if (r == ncclSuccess && !load(&st->kids[i])) r = ncclInternalError;
        }
        if (r == ncclSuccess) {
            // warm-up: one 8-byte all-gather per child (connections set up now,
            // inside the deadline, not in the first pass)
            what = "warm-up all-gather";
            char *w = static_cast<char *>(buf) + ids_bytes;
            for (int i = 0; i < 3 && r == ncclSuccess; ++i) {
                r = guarded(i, [&](ncclComm_t k) { return ncclAllGather(w, w + 8, 1, ncclUint64, k, s); });
                if (r == ncclInProgress) r = settle(i);
                inflight = inflight || r == ncclSuccess;
            }
            if (r == ncclSuccess) r = drain();
            if (r == ncclSuccess) inflight = false;
        }
        bool drained = !inflight;
        if (!drained && ev) {
            // abandoned with collectives in flight: the aborts end them;
            // give them a bounded while, then leak the scratch
            (void)hipEventRecord(ev, s);
            for (int i = 0; i < 50000 && hipEventQuery(ev) == hipErrorNotReady; ++i)
                std::this_thread::sleep_for(std::chrono::microseconds(200));
            drained = hipEventQuery(ev) == hipSuccess;
        }
        if (drained) {
            if (ev) (void)hipEventDestroy(ev);
            if (buf) (void)hipFree(buf);
            if (kid_ids) (void)hipHostFree(kid_ids);
            if (s) (void)hipStreamDestroy(s);
        }
        std::lock_guard<std::mutex> g(st->mu);
        if (r == ncclSuccess && st->abandoned) r = ncclInvalidUsage;
        if (r != ncclSuccess) {
            // abort (local, no peer handshake) every handle the main thread
            // did not claim; the claimed ones are its to abort
            for (int i = 0; i < 4; ++i) {
                ncclComm_t c = load(slot(i));
                if (c && !(st->claimed >> i & 1u)) (void)ncclCommAbort(c);
                st->claimed |= 1u << i;
            }
            for (ncclComm_t &k : st->kids) k = nullptr;
            st->root = nullptr;
        }
        st->r = r;
        st->what = what;
        st->done = true;
        st->cv.notify_all();
    });
    std::unique_lock<std::mutex> lk(st->mu);
    bool expired = false;
    if (ctx->opt_comm_timeout_ms > 0) {
        const auto limit = std::chrono::milliseconds(ctx->opt_comm_timeout_ms);
        expired = !st->cv.wait_for(lk, limit, [&] { return st->done; });
        if (expired) {
            // the root's handle appears ~1 s into the init: wait for it (or for
            // the helper to finish) a bounded while, then claim and abort what
            // exists -- claimed under the mutex, aborted outside it (the
            // helper may need the mutex to leave the RCCL call the abort ends)
            st->abandoned = true;
            const auto grace = std::chrono::steady_clock::now() + std::chrono::seconds(30);
            while (!st->done && !__atomic_load_n(&st->root, __ATOMIC_ACQUIRE) &&
                   std::chrono::steady_clock::now() < grace)
                st->cv.wait_for(lk, std::chrono::milliseconds(20));
            if (!st->done) {
                std::vector<ncclComm_t> mine;
                for (int i = 0; i < 4; ++i) {
                    ncclComm_t c = __atomic_load_n(i == CI::ROOT ? &st->root : &st->kids[i], __ATOMIC_ACQUIRE);
                    if (c && !(st->claimed >> i & 1u)) {
                        st->claimed |= 1u << i;
                        mine.push_back(c);
                    }
                }
                lk.unlock();
                for (ncclComm_t h : mine) (void)ncclCommAbort(h);  // ends the helper's waits
                lk.lock();
            }
            st->cv.wait_until(lk, grace, [&] { return st->done; });
        }
    } else {
        st->cv.wait(lk, [&] { return st->done; });
    }
    const bool finished = st->done;
    lk.unlock();
    if (finished) {
        helper.join();
    } else {
        // (the aborts did not release it within 30 s) parked, joined later
        ctx->comm_helpers.push_back(std::move(helper));
        ctx->comm_helper_state.push_back(st);
    }
    if (expired)
        return nas::fail(ctx, NAS_ERR_COMM,
                         "nas_comm_init: the communicators did not complete within " +
                             std::to_string(ctx->opt_comm_timeout_ms) +
                             " ms (NAS_OPT_COMM_TIMEOUT_MS): a rank did not join; "
                             "communicators aborted" +
                             (finished ? "" : " (the helper thread is still inside RCCL: parked in the "
                                              "context, joined later or detached by nas_destroy)"));
    if (st->r != ncclSuccess)
        return nas::fail(ctx, NAS_ERR_COMM, st->what + ": " + ncclGetErrorString(st->r));
    ctx->rank = rank;
    ctx->world = eff_world;
    ctx->rehearse = rehearse;
    ctx->virtual_shard = false;
    ctx->comm_root = reinterpret_cast<ncclComm *>(st->root);
    ctx->comm = reinterpret_cast<ncclComm *>(st->kids[0]);
    ctx->comm2 = reinterpret_cast<ncclComm *>(st->kids[1]);
    ctx->comm_c = reinterpret_cast<ncclComm *>(st->kids[2]);
    return set_stream_masks(ctx, shard_reserve(eff_world));
}

int nas_local_group_create(int32_t world, nas_local_group **out) {
    NAS_RANGE("nas_local_group_create");
    if (!out) return NAS_ERR_ARG;
    *out = nullptr;
    if (world < 1 || world > nas::LOCAL_MAX_WORLD) return NAS_ERR_ARG;
    auto *g = new (std::nothrow) nas_local_group();
    if (!g) return NAS_ERR_NOMEM;
    g->g = std::make_shared<nas::LocalGroup>(world);
    *out = g;
    return NAS_OK;
}

void nas_local_group_destroy(nas_local_group *g) {
    NAS_RANGE("nas_local_group_destroy");
    delete g;
}

int nas_comm_init_local(nas_ctx *ctx, nas_local_group *group, int32_t rank) {
    NAS_RANGE("nas_comm_init_local");
    OK(bind(ctx));
    if (!group || !group->g) return nas::fail(ctx, NAS_ERR_ARG, "nas_comm_init_local: group");
    const int world = group->g->world;
    if (rank < 0 || rank >= world) return nas::fail(ctx, NAS_ERR_ARG, "nas_comm_init_local: rank");
    if (ctx->have_L || ctx->have_wa || ctx->have_cap)
        return nas::fail(ctx, NAS_ERR_STATE, "nas_comm_init_local must precede the extended uploads");
    if (ctx->B > 1 && world > 1)
        return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "node shards of a cluster batch");
    destroy_comms(ctx);
    ctx->rank = 0;
    ctx->world = 1;
    ctx->rehearse = 0;
    ctx->virtual_shard = false;
    OK(set_stream_masks(ctx, 0));  // (as nas_comm_init: a failed join leaves plain streams)
    {
        std::lock_guard<std::mutex> g(group->g->mu);
        if (group->g->broken) return nas::fail(ctx, NAS_ERR_COMM, "nas_comm_init_local: group is broken");
        if (group->g->joined[rank])
            return nas::fail(ctx, NAS_ERR_STATE, "nas_comm_init_local: rank already joined");
        group->g->joined[rank] = true;
    }
    ctx->local = group->g;
    for (auto &c : ctx->lg_ev)
        for (auto &p : c)
            for (hipEvent_t &e : p)
                if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                    destroy_comms(ctx);
                    return nas::fail(ctx, NAS_ERR_HIP, "nas_comm_init_local: hipEventCreate");
                }
    for (uint32_t &r : ctx->lg_round) r = 0;
    ctx->lg_peers = 0;
    ctx->rank = rank;
    ctx->world = world;
    return set_stream_masks(ctx, shard_reserve(world));
}

int nas_set_shard(nas_ctx *ctx, int32_t rank, int32_t world) {
    NAS_RANGE("nas_set_shard");
    OK(bind(ctx));
    if (world < 1 || rank < 0 || rank >= world)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_set_shard: rank/world");
    if (has_coll(ctx)) return nas::fail(ctx, NAS_ERR_STATE, "context already has a communicator");
    if (ctx->have_L || ctx->have_wa || ctx->have_cap)
        return nas::fail(ctx, NAS_ERR_STATE, "nas_set_shard must precede the extended uploads");
    if (ctx->B > 1 && world > 1)
        return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "node shards of a cluster batch");
    ctx->rank = rank;
    ctx->world = world;
    ctx->virtual_shard = world > 1;
    return NAS_OK;
}

int nas_get_candidate_keys(nas_ctx *ctx, uint64_t *keys, uint64_t *bounds) {
    NAS_RANGE("nas_get_candidate_keys");
    OK(bind(ctx));
    OK(no_batch(ctx, "nas_get_candidate_keys"));
    if (!ctx->scored) return nas::fail(ctx, NAS_ERR_STATE, "no scoring pass yet");
    if (keys)
        HIPCK(hipMemcpyAsync(keys, ctx->cand_key.p, (size_t)ctx->P * KC * 8, hipMemcpyDeviceToHost,
                             ctx->stream));
    if (bounds)
        HIPCK(hipMemcpyAsync(bounds, ctx->cand_bound.p, (size_t)ctx->P * 8, hipMemcpyDeviceToHost,
                             ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    return NAS_OK;
}

// ---------------------------------------------------------------- synthetic
namespace {
int synth_snapshot_slice(nas_ctx *ctx, uint64_t seed, int32_t n, int32_t lo, int32_t nl,
                         int32_t n_snapshots, bool sharded) {
    if (n <= 0 || nl <= 0 || n_snapshots <= 0 || lo < 0 || (int64_t)lo + nl > n)
        return nas::fail(ctx, NAS_ERR_ARG, "synth sizes / node slice");
    const int64_t ns = nas::round_up(nl, 2);
    for (int f = 0; f < 6; ++f) OK(nas::ensure(ctx, ctx->snap[f], (size_t)ns * n_snapshots * 8));
    HIPCK(nas::launch_synth_snapshots(ctx->stream, seed, n, lo, nl, ns, n_snapshots,
                                      ctx->snap[0].as<double>(), ctx->snap[1].as<double>(),
                                      ctx->snap[2].as<double>(), ctx->snap[3].as<int64_t>(),
                                      ctx->snap[4].as<int64_t>(), ctx->snap[5].as<int64_t>()));
    HIPCK(hipStreamSynchronize(ctx->stream));
    if (ctx->snap_n != n) ctx->n_orders = 0;
    ctx->snap_n = n;
    ctx->snap_lo = lo;
    ctx->snap_nl = nl;
    ctx->snap_sharded = sharded;
    ctx->snap_s = n_snapshots;
    ctx->snap_ns = ns;
    return NAS_OK;
}
}  // namespace

int nas_synth_snapshots(nas_ctx *ctx, uint64_t seed, int32_t n_nodes, int32_t n_snapshots) {
    NAS_RANGE("nas_synth_snapshots");
    OK(bind(ctx));
    return synth_snapshot_slice(ctx, seed, n_nodes, 0, n_nodes, n_snapshots, false);
}

int nas_synth_snapshots_shard(nas_ctx *ctx, uint64_t seed, int32_t n_nodes, int32_t node_lo,
                              int32_t n_local, int32_t n_snapshots) {
    NAS_RANGE("nas_synth_snapshots_shard");
    OK(bind(ctx));
    return synth_snapshot_slice(ctx, seed, n_nodes, node_lo, n_local, n_snapshots, true);
}

int nas_read_snapshot(nas_ctx *ctx, int32_t s, double *cpu, double *mem, int64_t *rx, int64_t *tx,
                      double *bw, int64_t *disk) {
    NAS_RANGE("nas_read_snapshot");
    OK(bind(ctx));
    if (s < 0 || s >= ctx->snap_s) return nas::fail(ctx, NAS_ERR_ARG, "snapshot index");
    void *dst[6] = {cpu, mem, bw, rx, tx, disk};
    for (int f = 0; f < 6; ++f) {
        if (!dst[f]) continue;
        HIPCK(hipMemcpyAsync(dst[f], ctx->snap[f].as<char>() + (size_t)s * ctx->snap_ns * 8,
                             (size_t)ctx->snap_nl * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCK(hipStreamSynchronize(ctx->stream));
    return NAS_OK;
}

int nas_set_batch(nas_ctx *ctx, int32_t n_clusters) {
    NAS_RANGE("nas_set_batch");
    OK(bind(ctx));
    if (n_clusters < 1 || n_clusters > 65535)
        return nas::fail(ctx, NAS_ERR_ARG, "nas_set_batch: n_clusters");
    if (ctx->have_L || ctx->have_wa || ctx->have_cap || ctx->have_pods)
        return nas::fail(ctx, NAS_ERR_STATE, "nas_set_batch must precede the extended uploads");
    if (ctx->world > 1 && n_clusters > 1)
        return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "node shards of a cluster batch");
    ctx->B = n_clusters;
    return NAS_OK;
}

static int synth(nas_ctx *ctx, uint64_t seed, int32_t B, int32_t n_nodes, int32_t P,
                 int32_t dtype, int32_t peers) {
    if (n_nodes <= 0 || P <= 0 || peers < 1 || peers > 16 || B < 1 || !valid_dtype(dtype))
        return nas::fail(ctx, NAS_ERR_ARG, "nas_synth_cluster arguments");
    if (B > 1 && ctx->world > 1)
        return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "node shards of a cluster batch");
    // (profile 1 has no bound peers: traffic within the int8 plane, no overflow)
    const int profile = ctx->opt_synth_profile;
    const int ovf_peers = profile == 1 ? 0 : peers;
    ctx->B = B;
    set_geometry(ctx, n_nodes, dtype);
    ctx->P = P;
    ctx->Pp = (int32_t)nas::round_up(P, nas::COST_BN);
    const size_t e = esz(dtype);
    const size_t lt_b = (size_t)ctx->Mp * ctx->Kp * e, wa_b = (size_t)ctx->Pp * ctx->Kp * e;
    OK(nas::ensure(ctx, ctx->Lt, lt_b * B));
    OK(nas::ensure(ctx, ctx->WA, wa_b * B + (size_t)nas::WA_PAD_ROWS * ctx->Kp * e));
    OK(nas::ensure(ctx, ctx->cap0, (size_t)B * 3 * n_nodes * 4));
    OK(nas::ensure(ctx, ctx->cap, (size_t)B * 3 * n_nodes * 4));
    OK(nas::ensure(ctx, ctx->req, (size_t)B * 3 * ctx->Pp * 4));
    for (int b = 0; b < B; ++b)  // cluster b is the single cluster of seed + b
        HIPCK(nas::launch_synth_cluster(ctx->stream, seed + b, n_nodes, P, dtype, peers,
                                        ctx->Nloc0, ctx->Nloc, ctx->Mp, ctx->Kp, ctx->Pp,
                                        ctx->Lt.as<char>() + b * lt_b, ctx->WA.as<char>() + b * wa_b,
                                        ctx->cap0.as<int32_t>() + (size_t)b * 3 * n_nodes,
                                        ctx->req.as<int32_t>() + (size_t)b * 3 * ctx->Pp, nullptr,
                                        profile));
    HIPCK(hipMemcpyAsync(ctx->cap.p, ctx->cap0.p, (size_t)B * 3 * n_nodes * 4,
                         hipMemcpyDeviceToDevice, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    ctx->ovf_n = 0;
    ctx->lr_valid = false;
    ctx->split_valid = false;
    ctx->zrow_valid = false;
    ctx->L_finite = true;  // the synthetic latency classes are finite
    ctx->scored = false;
    if (dtype == NAS_DT_I8) {
        // exact traffic: peer aggregates beyond the int8 plane go to the
        // overflow lists (counts, host prefix sum, entries)
        const size_t rows = (size_t)B * ctx->Pp;
        DevBuf cnt;
        OK(nas::ensure(ctx, cnt, rows * 4));
        hipError_t he = hipMemsetAsync(cnt.p, 0, rows * 4, ctx->stream);
        for (int b = 0; b < B && he == hipSuccess; ++b)
            he = nas::launch_synth_overflow(ctx->stream, seed + b, n_nodes, P, ovf_peers, ctx->Kp, 0,
                                            nullptr, cnt.as<int32_t>() + (size_t)b * ctx->Pp,
                                            nullptr, nullptr, nullptr);
        std::vector<int32_t> c(rows), ptr(rows + 1, 0);
        if (he == hipSuccess)
            he = hipMemcpyAsync(c.data(), cnt.p, rows * 4, hipMemcpyDeviceToHost, ctx->stream);
        if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
        (void)hipFree(cnt.p);
        if (he != hipSuccess) return nas::hip_fail(ctx, he, "synth overflow counts");
        int64_t tot = 0;
        for (size_t r = 0; r < rows; ++r) {
            tot += c[r];
            if (tot > 0x7fffffff) return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "too many overflow entries");
            ptr[r + 1] = (int32_t)tot;
        }
        if (tot > 0) {
            OK(nas::ensure(ctx, ctx->ovf_ptr, ptr.size() * 4));
            OK(nas::ensure(ctx, ctx->ovf_m, (size_t)tot * 4));
            OK(nas::ensure(ctx, ctx->ovf_e, (size_t)tot * 4));
            HIPCK(hipMemcpyAsync(ctx->ovf_ptr.p, ptr.data(), ptr.size() * 4, hipMemcpyHostToDevice,
                                 ctx->stream));
            for (int b = 0; b < B; ++b)
                HIPCK(nas::launch_synth_overflow(ctx->stream, seed + b, n_nodes, P, ovf_peers, ctx->Kp, 1,
                                                 nullptr, nullptr,
                                                 ctx->ovf_ptr.as<int32_t>() + (size_t)b * ctx->Pp,
                                                 ctx->ovf_m.as<int32_t>(), ctx->ovf_e.as<int32_t>()));
            HIPCK(hipStreamSynchronize(ctx->stream));
            ctx->ovf_n = tot;
        }
        ctx->L_abs_max = 127;  // bound of the synthetic latency (<= 104; profile 1 <= 127), every rank
        ctx->B = B;
        OK(finish_traffic_i8(ctx));
    }
    ctx->have_L = ctx->have_cap = ctx->have_pods = ctx->have_wa = true;
    ctx->L_n = ctx->cap_n = ctx->wa_n = n_nodes;
    ctx->req_P = ctx->wa_P = P;
    ctx->L_dtype = ctx->wa_dtype = dtype;
    ctx->synth_valid = true;
    ctx->synth_seed = seed;
    ctx->synth_profile = profile;
    return NAS_OK;
}

int nas_synth_cluster(nas_ctx *ctx, uint64_t seed, int32_t n_nodes, int32_t P, int32_t dtype,
                      int32_t peers) {
    NAS_RANGE("nas_synth_cluster");
    OK(bind(ctx));
    return synth(ctx, seed, 1, n_nodes, P, dtype, peers);
}

int nas_synth_batch(nas_ctx *ctx, uint64_t seed, int32_t n_clusters, int32_t n_nodes, int32_t P,
                    int32_t dtype, int32_t peers) {
    NAS_RANGE("nas_synth_batch");
    OK(bind(ctx));
    return synth(ctx, seed, n_clusters, n_nodes, P, dtype, peers);
}

int nas_read_inputs(nas_ctx *ctx, int32_t p0, int32_t np, void *WA_rows, void *L, int32_t *cap_cpu,
                    int32_t *cap_mem, int32_t *cap_pods, int32_t *req_cpu, int32_t *req_mem,
                    int32_t *req_pods) {
    NAS_RANGE("nas_read_inputs");
    OK(bind(ctx));
    OK(check_extended(ctx));
    const int N = ctx->N;
    const size_t e = esz(ctx->dtype);
    if (WA_rows) {
        if (p0 < 0 || np < 0 || p0 + np > ctx->P) return nas::fail(ctx, NAS_ERR_ARG, "pod rows");
        if (np && ctx->dtype != NAS_DT_I8) {
            HIPCK(hipMemcpy2DAsync(WA_rows, (size_t)N * e, ctx->WA.as<char>() + (size_t)p0 * ctx->Kp * e,
                                   (size_t)ctx->Kp * e, (size_t)N * e, np, hipMemcpyDeviceToHost,
                                   ctx->stream));
        } else if (np) {
            // int8 scoring: the exact int32 traffic = plane + overflow entries
            std::vector<signed char> pl((size_t)np * N);
            HIPCK(hipMemcpy2DAsync(pl.data(), (size_t)N, ctx->WA.as<char>() + (size_t)p0 * ctx->Kp,
                                   (size_t)ctx->Kp, (size_t)N, np, hipMemcpyDeviceToHost, ctx->stream));
            std::vector<int32_t> ptr(np + 1, 0), om, oe;
            if (ctx->ovf_n) {
                HIPCK(hipMemcpyAsync(ptr.data(), ctx->ovf_ptr.as<int32_t>() + p0, (size_t)(np + 1) * 4,
                                     hipMemcpyDeviceToHost, ctx->stream));
                HIPCK(hipStreamSynchronize(ctx->stream));
                const size_t ne = (size_t)(ptr[np] - ptr[0]);
                om.resize(ne);
                oe.resize(ne);
                if (ne) {
                    HIPCK(hipMemcpyAsync(om.data(), ctx->ovf_m.as<int32_t>() + ptr[0], ne * 4,
                                         hipMemcpyDeviceToHost, ctx->stream));
                    HIPCK(hipMemcpyAsync(oe.data(), ctx->ovf_e.as<int32_t>() + ptr[0], ne * 4,
                                         hipMemcpyDeviceToHost, ctx->stream));
                }
            }
            HIPCK(hipStreamSynchronize(ctx->stream));
            auto *out = static_cast<int32_t *>(WA_rows);
            for (size_t i = 0; i < pl.size(); ++i) out[i] = pl[i];
            if (ctx->ovf_n)
                for (int r = 0; r < np; ++r)
                    for (int j = ptr[r]; j < ptr[r + 1]; ++j)
                        out[(size_t)r * N + om[j - ptr[0]]] += oe[j - ptr[0]];
        }
    }
    if (L) {
        if (ctx->synth_valid) {
            DevBuf tmp;
            OK(nas::ensure(ctx, tmp, (size_t)N * N * e));
            hipError_t he = nas::launch_synth_cluster(ctx->stream, ctx->synth_seed, N, ctx->P,
                                                      ctx->dtype, 1, 0, 0, 0, 0, 0, nullptr,
                                                      nullptr, nullptr, nullptr, tmp.p,
                                                      ctx->synth_profile);
            if (he == hipSuccess)
                he = hipMemcpyAsync(L, tmp.p, (size_t)N * N * e, hipMemcpyDeviceToHost, ctx->stream);
            if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
            (void)hipFree(tmp.p);
            if (he != hipSuccess) return nas::hip_fail(ctx, he, "read L");
        } else if (ctx->world == 1) {
            std::vector<char> lt((size_t)N * ctx->Kp * e);
            HIPCK(hipMemcpyAsync(lt.data(), ctx->Lt.p, lt.size(), hipMemcpyDeviceToHost, ctx->stream));
            HIPCK(hipStreamSynchronize(ctx->stream));
            char *out = static_cast<char *>(L);
            for (int i = 0; i < N; ++i)
                for (int m = 0; m < N; ++m)
                    std::memcpy(out + ((size_t)m * N + i) * e, lt.data() + ((size_t)i * ctx->Kp + m) * e, e);
        } else {
            return nas::fail(ctx, NAS_ERR_UNSUPPORTED, "full L is not resident on a sharded rank");
        }
    }
    int32_t *cdst[3] = {cap_cpu, cap_mem, cap_pods};
    for (int r = 0; r < 3; ++r)
        if (cdst[r])
            HIPCK(hipMemcpyAsync(cdst[r], ctx->cap0.as<int32_t>() + (size_t)r * N, (size_t)N * 4,
                                 hipMemcpyDeviceToHost, ctx->stream));
    int32_t *rdst[3] = {req_cpu, req_mem, req_pods};
    for (int r = 0; r < 3; ++r)
        if (rdst[r])
            HIPCK(hipMemcpyAsync(rdst[r], ctx->req.as<int32_t>() + (size_t)r * ctx->Pp,
                                 (size_t)ctx->P * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    return NAS_OK;
}

}  // extern "C"
