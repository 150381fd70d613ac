// k_rescore.hip -- gathered rescoring after a commit stop.
//
// When the commit halts at pod s (its usable candidates all taken), the pods
// after it whose lists are ALSO dry against the current capacity are the ones
// that would halt it next.  Rescoring a contiguous window [s, s + W) only
// refreshes the few of them inside the window: in a crowded cluster (a rack
// filled up) the dry pods are spread thinly over the whole pod order and the
// walk stops again and again.  Instead:
//   1. k_stale: one thread per pending pod p >= s flags it when its list is
//      incomplete (bound != KEY_INVALID) and no usable candidate fits the
//      current capacity; flags are wave ballots, one 64-bit word per 64 pods.
//   2. the last k_stale block to finish prefix-sums the word popcounts and
//      writes the first R flagged pods in pod order (s is always among them:
//      it halted for exactly this reason).
//   3. the ordinary fit / cost / merge kernels (and the RCCL exchange) score
//      them as a "view" of R rows whose row q is pod idx[q]: the kernels read
//      the pod's requests and traffic row in place through that row map.
//   4. k_merge's store puts the fresh lists back into the pods' list slots.
// Lists computed against the capacity now stay valid for every later turn of
// these pods (capacity only shrinks), so the walk resumes from s unchanged.
#include "klist.h"

#include <algorithm>

namespace nas {
namespace {

constexpr int STALE_THREADS = 256;
// a pod is flagged when fewer than this many of its usable candidates still
// fit: the dry ones (0) and those a few commits away from running dry, whose
// lists a herd of neighbours is about to drain.  4 (was 2): the full-range
// herd's rescore rounds 27-56 -> 3-5 per pass and its pass 10.9 -> 9.7 ms
// median on one box; 3, 6 and 8 within noise of 4, the pipelined passes
// unchanged (profiles/r06w_ab_stale_min_fit.txt)
constexpr int STALE_MIN_FIT = 4;

// One launch: every block flags its pods (ballot words), and the LAST block
// to finish (ticket counter ctl[3], zeroed at the start of every pass and
// reset by that block) prefix-sums the words' popcounts and writes the first R
// flagged pods in pod order -- the stale scan and the compaction without a
// second launch on the slot's critical path.  Publication: each block's
// words are stored, drained (vmcnt(0)), released at agent scope by thread 0,
// then the ticket is drawn; the last block acquires before reading
// (cdna_hip_programming.md, the split-K counter recipe).
// pod p's list is dry: incomplete (bound != KEY_INVALID) and fewer than
// STALE_MIN_FIT of its usable candidates fit the capacity now
__device__ __forceinline__ bool stale_pod(const u64 *__restrict__ key, const u64 *__restrict__ bound,
                                          const int *__restrict__ req, int Pp,
                                          const int *__restrict__ cap, int N, int p) {
    const u64 b = bound[p];
    if (b == KEY_INVALID) return false;
    u64 k[KC];
    load8(key + (size_t)p * KC, k);
    const int r0 = req[p], r1 = req[Pp + p], r2 = req[2 * Pp + p];
    int fits = 0;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        if (k[j] == KEY_INVALID || k[j] > b) break;
        const int n = (int)(unsigned)k[j];
        fits += (r0 <= cap[n] && r1 <= cap[N + n] && r2 <= cap[2 * N + n]) ? 1 : 0;
        if (fits >= STALE_MIN_FIT) break;
    }
    return fits < STALE_MIN_FIT;
}

__global__ void __launch_bounds__(STALE_THREADS)
k_stale(const u64 *__restrict__ key, const u64 *__restrict__ bound, const int *__restrict__ req,
        int Pp, const int *__restrict__ cap, int N, int p0, int P, u64 *__restrict__ words,
        int n_words, int R, int *__restrict__ idx, int *__restrict__ ctl,
        const int *__restrict__ p0_dev) {
    __shared__ int part[STALE_THREADS];
    __shared__ int last;
    const int tid = threadIdx.x;
    // device-side slot: pods from the halt word on; nothing halted -> an
    // empty view, published by block 0 alone
    const int first = p0_dev ? *p0_dev : p0;
    // blocks wholly below the first pod take no part (no words, no ticket):
    // the launch covers [p0, P) but the halt is usually far into it (the
    // herd plan's slots scan from the pass's start behind every chunk)
    const int b_first = first < 0 ? 0 : (first - p0) / STALE_THREADS;
    if (first < 0 || b_first >= (int)gridDim.x) {  // (or a halt word past the scan)
        if (blockIdx.x == 0 && tid == 0) {
            ctl[0] = -1;
            ctl[1] = 0;
        }
        return;
    }
    {
        const int t = blockIdx.x * STALE_THREADS + tid;
        const int p = p0 + t;
        if ((int)blockIdx.x < b_first) return;
        const int participants = (int)gridDim.x - b_first;
        const bool dry = p < P && p >= first && stale_pod(key, bound, req, Pp, cap, N, p);
        const u64 m = __ballot(dry);
        if ((tid & 63) == 0) words[t >> 6] = m;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int ticket = __hip_atomic_fetch_add(ctl + 3, 1, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            last = ticket == participants - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        if (!last) return;
    }
    // ---- compaction by the last block (words of the participating blocks)
    const int wbase = b_first * (STALE_THREADS / 64), nw = n_words - wbase;
    const int per = (nw + STALE_THREADS - 1) / STALE_THREADS;
    const int w0 = wbase + min(nw, tid * per), w1 = min(n_words, w0 + per);
    int c = 0;
    for (int w = w0; w < w1; ++w) c += __popcll(words[w]);
    part[tid] = c;
    __syncthreads();
    for (int d = 1; d < STALE_THREADS; d <<= 1) {  // inclusive Hillis-Steele scan
        const int v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int off = part[tid] - c;
    if (tid == STALE_THREADS - 1) {
        const int n = min(part[tid], R);
        ctl[0] = n > 0 ? 0 : -1;  // the view's window start, read like a halt word
        ctl[1] = n;
        ctl[2] += n;              // running total, reported in nas_timings
        ctl[3] = 0;               // the ticket counter, for the next slot
    }
    for (int w = w0; w < w1 && off < R; ++w) {
        u64 mm = words[w];
        while (mm && off < R) {
            const int bit = __ffsll((long long)mm) - 1;
            idx[off++] = p0 + w * 64 + bit;
            mm &= mm - 1;
        }
    }
}

// The herd plan's in-loop slots (nas_place): one workgroup scans the W pods
// from the halt word on and compacts the flagged ones itself -- no per-block
// agent-scope release and ticket.  Beside a wave of cost workgroups that
// store their cost rows (dirty L2 lines), k_stale's per-block release fences
// (an L2 write-back each) ran 125-165 us per slot against 11 us on an idle
// GPU (profiles/r06e_herd_timeline.txt); in a herd nearly every pod after the
// halt is flagged, so W = 2R pods fill the view.
constexpr int SW_THREADS = 1024;
__global__ void __launch_bounds__(SW_THREADS)
k_stale_window(const u64 *__restrict__ key, const u64 *__restrict__ bound,
               const int *__restrict__ req, int Pp, const int *__restrict__ cap, int N, int P,
               int W, int R, int *__restrict__ idx, int *__restrict__ ctl,
               const int *__restrict__ p0_dev) {
    __shared__ int wc[SW_THREADS / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int first = *p0_dev;
    if (first < 0 || first >= P) {  // nothing halted (or past the scan): an empty view
        if (tid == 0) {
            ctl[0] = -1;
            ctl[1] = 0;
        }
        return;
    }
    const int end = min(P, first + W);
    int off = 0;  // flagged pods so far (block-uniform)
    for (int b = first; b < end && off < R; b += SW_THREADS) {
        const int p = b + tid;
        const bool dry = p < end && stale_pod(key, bound, req, Pp, cap, N, p);
        const u64 m = __ballot(dry);
        if (lane == 0) wc[w] = __popcll(m);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int v = 0; v < SW_THREADS / 64; ++v) {
            before += v < w ? wc[v] : 0;
            total += wc[v];
        }
        const int pos = off + before + __popcll(m & ((1ull << lane) - 1));
        if (dry && pos < R) idx[pos] = p;
        off += total;
        __syncthreads();  // (wc is rewritten next round)
    }
    if (tid == 0) {
        const int n = min(off, R);
        ctl[0] = n > 0 ? 0 : -1;
        ctl[1] = n;
        ctl[2] += n;
    }
}

// Cost-row cache rescoring (round 6).  In a global herd -- every pod ranks
// the same nodes first (configs.C3_fullrange: uniform random latency, so a
// node's column sum dominates every pod's cost) -- most pods' lists, scored
// against capacity a few thousand pods stale, run dry at their turn, and the
// walk rescored ~90% of C3's pods through gathered slots whose cost launch
// recomputes the whole contraction (a workgroup's full-K loop, ~150 us per
// slot).  When the pass keeps the cost-row cache (the main cost launches
// store every (pod, node) key, k_cost.hip), a slot's pods are rescored from
// their cached rows instead: one wave per view row reads the pod's Mp keys
// (coalesced), tests each node's fit against the capacity now (exactly
// k_fit's rule), keeps a per-lane top-4 in ascending node order (klist.h
// Top4) and merges the 64 lanes' lists by xor shuffles into the pod's 8-list
// with its exactness bound -- the list the fit + cost + merge kernels would
// have produced, for a read of 4 B per (pod, node) instead of 2 K MACs.
// Output: the view rows (to_view: [R][8] keys, [R] bounds, for the node-shard
// exchange) or straight into the pods' own list slots (row q -> pod idx[q]).
constexpr int RC_THREADS = 256;  // one workgroup (4 waves) per view row
constexpr int RC_UNROLL = 8;     // nodes per thread in flight (cost + 3 capacities each)
__global__ void __launch_bounds__(RC_THREADS)
k_rescore_cached(const unsigned *__restrict__ cc, int stride, int nloc, int n0,
                 const int *__restrict__ cap, int N, const int *__restrict__ req, int Pp,
                 const int *__restrict__ idx, const int *__restrict__ ctl,
                 u64 *__restrict__ key_out, u64 *__restrict__ bound_out, int to_view) {
    __shared__ u64 xl[RC_THREADS / 64][KC + 1];
    const int q = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (ctl[0] < 0 || q >= ctl[1]) return;  // (block-uniform) nothing halted / past the view
    const int p = idx[q];
    const int r0 = req[p], r1 = req[Pp + p], r2 = req[2 * Pp + p];
    const unsigned *row = cc + (size_t)p * stride;
    const int *c0 = cap + n0, *c1 = cap + N + n0, *c2 = cap + 2 * N + n0;
    // thread t visits nodes t, t + 256, ... (ascending: Top4's tie rule);
    // RC_UNROLL of them per round trip -- the walk is latency-bound otherwise
    // (one wave per row with 4 in flight ran 146 us per 2,048-row slot)
    Top4 t;
    t.init();
    int i = tid;
    for (; i + (RC_UNROLL - 1) * RC_THREADS < nloc; i += RC_UNROLL * RC_THREADS) {
        unsigned x[RC_UNROLL];
        int a[RC_UNROLL], b[RC_UNROLL], c[RC_UNROLL];
#pragma unroll
        for (int u = 0; u < RC_UNROLL; ++u) {
            const int j = i + RC_THREADS * u;
            x[u] = row[j];
            a[u] = c0[j];
            b[u] = c1[j];
            c[u] = c2[j];
        }
#pragma unroll
        for (int u = 0; u < RC_UNROLL; ++u)
            t.insert((r0 <= a[u] && r1 <= b[u] && r2 <= c[u]) ? x[u] : 0xffffffffu,
                     (unsigned)(n0 + i + RC_THREADS * u));
    }
    for (; i < nloc; i += RC_THREADS) {
        const unsigned x = row[i];
        const bool f = r0 <= c0[i] && r1 <= c1[i] && r2 <= c2[i];
        t.insert(f ? x : 0xffffffffu, (unsigned)(n0 + i));
    }
    // the wave's 64 lists -> one 8-list + bound (xor shuffles), then the
    // four waves' lists through LDS
    u64 k4[4], o4[4], kl[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) k4[j] = t.c[j] == 0xffffffffu ? KEY_INVALID : t.key(j);
#pragma unroll
    for (int j = 0; j < 4; ++j) o4[j] = shfl_xor64(k4[j], 1);
    merge44(k4, o4, kl);
    u64 bl = umin64(k4[3], o4[3]);
#pragma unroll
    for (int m = 2; m < 64; m <<= 1) {
        u64 o8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o8[j] = shfl_xor64(kl[j], m);
        bl = umin64(bl, shfl_xor64(bl, m));
        merge88(kl, o8);
    }
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < KC; ++j) xl[w][j] = kl[j];
        xl[w][KC] = bl;
    }
    __syncthreads();
    if (tid != 0) return;
#pragma unroll
    for (int v = 1; v < RC_THREADS / 64; ++v) {
        u64 o8[8];
#pragma unroll
        for (int j = 0; j < KC; ++j) o8[j] = xl[v][j];
        bl = umin64(bl, xl[v][KC]);
        merge88(kl, o8);
    }
    bl = umin64(bl, kl[7]);
    const size_t r = to_view ? (size_t)q : (size_t)p;
    store8(key_out + r * KC, kl);
    bound_out[r] = bl;
}

}  // namespace

hipError_t launch_rescore_cached(hipStream_t st, const uint32_t *cache, int stride, int nloc,
                                 int n0, const int32_t *cap, int N, const int32_t *req, int Pp,
                                 const int32_t *idx, const int32_t *ctl, int R, uint64_t *key_out,
                                 uint64_t *bound_out, bool to_view) {
    if (R <= 0) return hipSuccess;
    k_rescore_cached<<<R, RC_THREADS, 0, st>>>(
        reinterpret_cast<const unsigned *>(cache), stride, nloc, n0, cap, N, req, Pp, idx, ctl,
        reinterpret_cast<u64 *>(key_out), reinterpret_cast<u64 *>(bound_out), to_view ? 1 : 0);
    return hipGetLastError();
}

int stale_words(int P) { return (P + STALE_THREADS - 1) / STALE_THREADS * (STALE_THREADS / 64); }

hipError_t launch_stale_scan(hipStream_t st, const uint64_t *key, const uint64_t *bound,
                             const int32_t *req, int Pp, const int32_t *cap, int N, int p0, int P,
                             uint64_t *words, int R, int32_t *idx, int32_t *ctl,
                             const int32_t *p0_dev) {
    if (p0 < 0) p0 = 0;  // device-side start: scan every pod, k_stale skips those before it
    const int n = P - p0;
    if (n <= 0) return hipErrorInvalidValue;
    const int blocks = (n + STALE_THREADS - 1) / STALE_THREADS;
    auto *w = reinterpret_cast<u64 *>(words);
    k_stale<<<blocks, STALE_THREADS, 0, st>>>(reinterpret_cast<const u64 *>(key),
                                              reinterpret_cast<const u64 *>(bound), req, Pp, cap, N,
                                              p0, P, w, blocks * (STALE_THREADS / 64), R, idx, ctl,
                                              p0_dev);
    return hipGetLastError();
}


hipError_t launch_stale_window(hipStream_t st, const uint64_t *key, const uint64_t *bound,
                               const int32_t *req, int Pp, const int32_t *cap, int N, int P, int W,
                               int R, int32_t *idx, int32_t *ctl, const int32_t *p0_dev) {
    if (!p0_dev || W <= 0 || R <= 0) return hipErrorInvalidValue;
    k_stale_window<<<1, SW_THREADS, 0, st>>>(reinterpret_cast<const u64 *>(key),
                                            reinterpret_cast<const u64 *>(bound), req, Pp, cap, N,
                                            P, W, R, idx, ctl, p0_dev);
    return hipGetLastError();
}


}  // namespace nas
