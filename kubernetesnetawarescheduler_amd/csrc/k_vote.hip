// k_vote.hip -- reference-mode vote scorer on gfx950.
//
// Restates scheduler/scheduler.go:248-394 (prioritize + findBestNode) as an
// associative reduction:
//   * each of the six metric loops of :334-359 is a strict, first-occurrence
//     arg-extremum in iteration order (order1) -> a lexicographic reduction
//     of (value, pos1[node]) keys, valid only if the value beats the sentinel
//     of :258-265 (strict IEEE compare, so NaN never wins, as in Go);
//   * bestNetSentNode (:347-354, the bandwidth winner is written into it) is
//     whichever of {argmin tx, argmax bw} sits later in order1;
//   * votes +3/+2/+1/+1/+3("none")/+1 (:360-365), then findBestNode (:384-394)
//     = the key with the max score, first in order2 (maxP = 0, strict >).
//
// One workgroup (4 wave64) per snapshot; each lane streams node pairs with
// 16-byte loads from the SoA snapshot (48 B/node, HBM-bound), reduces in
// registers, then wave shuffles and an LDS step across the 4 waves.
#include "nas_internal.h"

namespace nas {
namespace {

constexpr int VOTE_THREADS = 256;
constexpr int NOPOS = 0x7fffffff;

constexpr double SENT_CPU = 99999999999.0;  // scheduler.go:260
constexpr double SENT_MEM = 99999999999.0;  // :261
constexpr long long SENT_RX = 99999999999LL;  // :262
constexpr long long SENT_TX = 99999999999LL;  // :263
constexpr long long SENT_DISK = 999;          // :264
constexpr double SENT_BW = 0.0;               // field omitted at :258-265

struct MinF {  // (value, pos) lexicographic min, pos NOPOS = none
    double v; int p;
    __device__ void init() { v = 0.0; p = NOPOS; }
    __device__ void add(double x, int q) {
        if (p == NOPOS || x < v || (!(v < x) && q < p)) { v = x; p = q; }
    }
};
struct MaxF {
    double v; int p;
    __device__ void init() { v = 0.0; p = NOPOS; }
    __device__ void add(double x, int q) {
        if (p == NOPOS || x > v || (!(v > x) && q < p)) { v = x; p = q; }
    }
};
struct MinI {
    long long v; int p;
    __device__ void init() { v = 0; p = NOPOS; }
    __device__ void add(long long x, int q) {
        if (p == NOPOS || x < v || (x == v && q < p)) { v = x; p = q; }
    }
};

struct VoteAcc {
    MinF cpu, mem;
    MaxF bw;
    MinI rx, tx, disk;
    __device__ void init() { cpu.init(); mem.init(); bw.init(); rx.init(); tx.init(); disk.init(); }
    __device__ void merge(const VoteAcc &b) {
        if (b.cpu.p != NOPOS) cpu.add(b.cpu.v, b.cpu.p);
        if (b.mem.p != NOPOS) mem.add(b.mem.v, b.mem.p);
        if (b.bw.p != NOPOS) bw.add(b.bw.v, b.bw.p);
        if (b.rx.p != NOPOS) rx.add(b.rx.v, b.rx.p);
        if (b.tx.p != NOPOS) tx.add(b.tx.v, b.tx.p);
        if (b.disk.p != NOPOS) disk.add(b.disk.v, b.disk.p);
    }
    // one node: the six guarded comparisons of scheduler.go:335-355
    __device__ void node(double c, double m, double b, long long r, long long t, long long d, int q) {
        if (c < SENT_CPU) cpu.add(c, q);
        if (m < SENT_MEM) mem.add(m, q);
        if (r < SENT_RX) rx.add(r, q);
        if (t < SENT_TX) tx.add(t, q);
        if (b > SENT_BW) bw.add(b, q);
        if (d < SENT_DISK && d != 0) disk.add(d, q);
    }
};

template <typename T>
__device__ __forceinline__ void shfl_merge(T &a, int off);

template <>
__device__ __forceinline__ void shfl_merge<MinF>(MinF &a, int off) {
    double x = __shfl_xor(a.v, off);
    int q = __shfl_xor(a.p, off);
    if (q != NOPOS) a.add(x, q);
}
template <>
__device__ __forceinline__ void shfl_merge<MaxF>(MaxF &a, int off) {
    double x = __shfl_xor(a.v, off);
    int q = __shfl_xor(a.p, off);
    if (q != NOPOS) a.add(x, q);
}
template <>
__device__ __forceinline__ void shfl_merge<MinI>(MinI &a, int off) {
    long long x = __shfl_xor(a.v, off);
    int q = __shfl_xor(a.p, off);
    if (q != NOPOS) a.add(x, q);
}

// One snapshot's six extrema over this block's node slice: lanes stream node
// pairs (16-byte SoA loads), reduce in registers, then wave shuffles and one
// LDS step across the 4 waves.  The result is valid in thread 0.  Local node
// i is node lo + i of the cluster; pos1 is indexed by cluster node.
template <bool SLICE>
__device__ __forceinline__ VoteAcc reduce_snapshot(
    const double *__restrict__ cpu, const double *__restrict__ mem, const double *__restrict__ bw,
    const long long *__restrict__ rx, const long long *__restrict__ tx,
    const long long *__restrict__ disk, size_t base, int lo, int nl, const int *__restrict__ p1) {
    const int tid = threadIdx.x;
    VoteAcc acc;
    acc.init();
    for (int i = 2 * tid; i < nl; i += 2 * VOTE_THREADS) {
        const double2 c = *reinterpret_cast<const double2 *>(cpu + base + i);
        const double2 m = *reinterpret_cast<const double2 *>(mem + base + i);
        const double2 b = *reinterpret_cast<const double2 *>(bw + base + i);
        const longlong2 r = *reinterpret_cast<const longlong2 *>(rx + base + i);
        const longlong2 t = *reinterpret_cast<const longlong2 *>(tx + base + i);
        const longlong2 d = *reinterpret_cast<const longlong2 *>(disk + base + i);
        int2 q;
        if constexpr (SLICE) {  // lo may be odd: two 4-byte loads (pos1 is L2-resident)
            q.x = p1[lo + i];
            q.y = i + 1 < nl ? p1[lo + i + 1] : 0;
        } else {
            q = *reinterpret_cast<const int2 *>(p1 + i);
        }
        acc.node(c.x, m.x, b.x, r.x, t.x, d.x, q.x);
        if (i + 1 < nl) acc.node(c.y, m.y, b.y, r.y, t.y, d.y, q.y);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        shfl_merge(acc.cpu, off);
        shfl_merge(acc.mem, off);
        shfl_merge(acc.bw, off);
        shfl_merge(acc.rx, off);
        shfl_merge(acc.tx, off);
        shfl_merge(acc.disk, off);
    }
    __shared__ VoteAcc red[VOTE_THREADS / 64];
    const int wave = tid >> 6;
    if ((tid & 63) == 0) red[wave] = acc;
    __syncthreads();
    VoteAcc a = red[0];
    if (tid == 0) {
        for (int w = 1; w < VOTE_THREADS / 64; ++w) a.merge(red[w]);
    }
    return a;
}

// From the six merged extrema to the decision: net-sent (:347-354), votes
// (:360-365) and findBestNode over order2 (:384-394).  n = cluster nodes
// (key n == "none").
__device__ void vote_decide(const VoteAcc &a, int n, const int *__restrict__ o1,
                            const int *__restrict__ p2, int *__restrict__ best_out,
                            int *__restrict__ win_out) {
    // net-sent: the later (in order1) of the tx and bw winners (:347-354)
    int ps = a.tx.p;
    if (a.bw.p != NOPOS && (ps == NOPOS || a.bw.p > ps)) ps = a.bw.p;
    auto node_at = [&](int p) { return p == NOPOS ? n : o1[p]; };  // key n == "none"
    int key[6];
    key[NAS_W_CPU] = node_at(a.cpu.p);
    key[NAS_W_MEM] = node_at(a.mem.p);
    key[NAS_W_NETSENT] = node_at(ps);
    key[NAS_W_NETREC] = node_at(a.rx.p);
    key[NAS_W_BANDWIDTH] = n;  // bestNetBandwith is never assigned (:271, :364)
    key[NAS_W_DISK] = node_at(a.disk.p);
    const int weight[6] = {3, 2, 1, 1, 3, 1};  // :360-365
    int best = NAS_EMPTY, best_score = 0, best_pos = NOPOS;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        int sc = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) sc += key[j] == key[i] ? weight[j] : 0;
        const int q = p2[key[i]];
        // findBestNode: first key in order2 holding the max score, max > 0
        if (sc > best_score || (sc == best_score && q < best_pos)) {
            best_score = sc;
            best_pos = q;
            best = key[i] == n ? NAS_NONE : key[i];
        }
    }
    *best_out = best;
    if (win_out) {
#pragma unroll
        for (int i = 0; i < 6; ++i) win_out[i] = key[i] == n ? NAS_NONE : key[i];
    }
}

__global__ void __launch_bounds__(VOTE_THREADS)
k_vote(const double *__restrict__ cpu, const double *__restrict__ mem,
       const double *__restrict__ bw, const long long *__restrict__ rx,
       const long long *__restrict__ tx, const long long *__restrict__ disk, int n, long long ns,
       const int *__restrict__ order1, const int *__restrict__ pos1,
       const int *__restrict__ pos2, long long ord_ns, int n_orders,
       int *__restrict__ best_out, int *__restrict__ win_out, const int *__restrict__ pod_snap) {
    // block b: one snapshot (pod_snap null), or one pod scoring snapshot
    // pod_snap[b] with its own order set b (nas_upload_pod_orders)
    const int b = blockIdx.x;
    const int s = pod_snap ? pod_snap[b] : b;
    const int o = n_orders == 1 ? 0 : b;
    const VoteAcc a = reduce_snapshot<false>(cpu, mem, bw, rx, tx, disk, (size_t)s * ns, 0, n,
                                             pos1 + (size_t)o * ord_ns);
    if (threadIdx.x != 0) return;
    vote_decide(a, n, order1 + (size_t)o * ord_ns, pos2 + (size_t)o * (ord_ns + 2), best_out + b,
                win_out ? win_out + (size_t)b * 6 : nullptr);
}

// Node-shard partial: the six extrema of nodes [lo, lo + nl) -> part[s]
// (include/nas.h nas_vote_partial: value bits, pos1).
__global__ void __launch_bounds__(VOTE_THREADS)
k_vote_partial(const double *__restrict__ cpu, const double *__restrict__ mem,
               const double *__restrict__ bw, const long long *__restrict__ rx,
               const long long *__restrict__ tx, const long long *__restrict__ disk, int lo,
               int nl, long long ns, const int *__restrict__ pos1, long long ord_ns,
               int n_orders, long long *__restrict__ part) {
    const int s = blockIdx.x;
    const int o = n_orders == 1 ? 0 : s;
    const VoteAcc a = reduce_snapshot<true>(cpu, mem, bw, rx, tx, disk, (size_t)s * ns, lo, nl,
                                            pos1 + (size_t)o * ord_ns);
    if (threadIdx.x != 0) return;
    long long *r = part + (size_t)s * 12;
    const long long v[6] = {__double_as_longlong(a.cpu.v), __double_as_longlong(a.mem.v),
                            __double_as_longlong(a.bw.v), a.rx.v, a.tx.v, a.disk.v};
    const int p[6] = {a.cpu.p, a.mem.p, a.bw.p, a.rx.p, a.tx.p, a.disk.p};
#pragma unroll
    for (int f = 0; f < 6; ++f) {
        r[2 * f] = p[f] == NOPOS ? 0 : v[f];
        r[2 * f + 1] = (long long)(unsigned)p[f];  // pos1 in the low word, reserved = 0
    }
}

// Merge n_parts slices' records per snapshot (one lane per snapshot; the
// (value, pos1) order is total, so the merge order does not matter), then
// decide as k_vote does.
__global__ void __launch_bounds__(256)
k_vote_merge(const long long *__restrict__ parts, int n_parts, int S, int n,
             const int *__restrict__ order1, const int *__restrict__ pos2, long long ord_ns,
             int n_orders, int *__restrict__ best_out, int *__restrict__ win_out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    VoteAcc a;
    a.init();
    for (int k = 0; k < n_parts; ++k) {
        const long long *r = parts + ((size_t)k * S + s) * 12;
        const int p[6] = {(int)r[1], (int)r[3], (int)r[5], (int)r[7], (int)r[9], (int)r[11]};
        if (p[0] != NOPOS) a.cpu.add(__longlong_as_double(r[0]), p[0]);
        if (p[1] != NOPOS) a.mem.add(__longlong_as_double(r[2]), p[1]);
        if (p[2] != NOPOS) a.bw.add(__longlong_as_double(r[4]), p[2]);
        if (p[3] != NOPOS) a.rx.add(r[6], p[3]);
        if (p[4] != NOPOS) a.tx.add(r[8], p[4]);
        if (p[5] != NOPOS) a.disk.add(r[10], p[5]);
    }
    const int o = n_orders == 1 ? 0 : s;
    vote_decide(a, n, order1 + (size_t)o * ord_ns, pos2 + (size_t)o * (ord_ns + 2), best_out + s,
                win_out ? win_out + (size_t)s * 6 : nullptr);
}

__global__ void k_vote_gather(const int *__restrict__ pod_snap, int P, const int *__restrict__ sb,
                              const int *__restrict__ sw, int *__restrict__ best,
                              int *__restrict__ win) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int s = pod_snap[p];
    best[p] = sb[s];
    if (win) {
#pragma unroll
        for (int i = 0; i < 6; ++i) win[(size_t)p * 6 + i] = sw[(size_t)s * 6 + i];
    }
}

}  // namespace

hipError_t launch_vote(hipStream_t st, const nas_ctx *c, int S) {
    if (S <= 0) return hipSuccess;
    k_vote<<<S, VOTE_THREADS, 0, st>>>(
        c->snap[0].as<double>(), c->snap[1].as<double>(), c->snap[2].as<double>(),
        c->snap[3].as<long long>(), c->snap[4].as<long long>(), c->snap[5].as<long long>(),
        c->snap_n, c->snap_ns, c->order1.as<int>(), c->pos1.as<int>(), c->pos2.as<int>(),
        c->ord_ns, c->n_orders, c->snap_best.as<int>(), c->snap_win.as<int>(), nullptr);
    return hipGetLastError();
}

hipError_t launch_vote_pods(hipStream_t st, const nas_ctx *c, const int32_t *pod_snap, int P,
                            int32_t *best, int32_t *win) {
    if (P <= 0) return hipSuccess;
    k_vote<<<P, VOTE_THREADS, 0, st>>>(
        c->snap[0].as<double>(), c->snap[1].as<double>(), c->snap[2].as<double>(),
        c->snap[3].as<long long>(), c->snap[4].as<long long>(), c->snap[5].as<long long>(),
        c->snap_n, c->snap_ns, c->order1.as<int>(), c->pos1.as<int>(), c->pos2.as<int>(),
        c->ord_ns, c->n_orders, best, win, pod_snap);
    return hipGetLastError();
}

hipError_t launch_vote_partial(hipStream_t st, const nas_ctx *c, int S, nas_vote_partial *part) {
    if (S <= 0) return hipSuccess;
    k_vote_partial<<<S, VOTE_THREADS, 0, st>>>(
        c->snap[0].as<double>(), c->snap[1].as<double>(), c->snap[2].as<double>(),
        c->snap[3].as<long long>(), c->snap[4].as<long long>(), c->snap[5].as<long long>(),
        c->snap_lo, c->snap_nl, c->snap_ns, c->pos1.as<int>(), c->ord_ns, c->n_orders,
        reinterpret_cast<long long *>(part));
    return hipGetLastError();
}

hipError_t launch_vote_merge(hipStream_t st, const nas_ctx *c, const nas_vote_partial *parts,
                             int n_parts, int S, int32_t *best, int32_t *win) {
    if (S <= 0) return hipSuccess;
    k_vote_merge<<<(S + 255) / 256, 256, 0, st>>>(
        reinterpret_cast<const long long *>(parts), n_parts, S, c->snap_n, c->order1.as<int>(),
        c->pos2.as<int>(), c->ord_ns, c->n_orders, best, win);
    return hipGetLastError();
}

hipError_t launch_vote_gather(hipStream_t st, const int32_t *pod_snap, int P,
                              const int32_t *snap_best, const int32_t *snap_win, int32_t *best,
                              int32_t *win) {
    if (P <= 0) return hipSuccess;
    k_vote_gather<<<(P + 255) / 256, 256, 0, st>>>(pod_snap, P, snap_best, snap_win, best, win);
    return hipGetLastError();
}

}  // namespace nas
