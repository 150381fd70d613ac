// k_commit.hip -- conflict-resolving greedy commit with capacity update.
//
// Sequential semantics (the extended-mode oracle, oracle/oracle.c or_place):
// pods in order take the (cost, node)-smallest node that still fits the
// remaining capacity, which is then decremented.  Each pod arrives with a
// candidate list (klist.h): keys <= its bound are exactly the best nodes that
// fit some EARLIER capacity state.  Capacity only shrinks, so the pod's
// sequential choice is its first usable candidate that fits now -- every
// better node is either ahead of it in the list and does not fit, or never
// fit.  If no usable candidate fits: a complete list (bound = KEY_INVALID)
// means no node fits (NAS_EMPTY); otherwise the pod needs a rescore against
// the current capacity (host loop in nas_api.hip).
//
// Parallel form: one wave64 takes 64 consecutive pods (a chunk).  Every
// not-yet-committed lane picks its first fitting usable candidate against the
// current capacity.  Lanes whose picks are pairwise distinct are independent
// of one another, so the prefix of lanes before the first repeated pick
// (detected with an LDS atomicMin bucket table; a hash collision only
// shortens the prefix) is committed at once -- exactly what the sequential
// walk does -- and the remaining lanes of the same chunk pick again against
// the updated capacity.  Chunks stay aligned, so the next ones are prefetched
// RING chunks ahead into a statically indexed register ring, hiding the
// global-load latency behind the walk.
// The working capacity lives in LDS (3 x N int32) when it fits, else in L2;
// the whole workgroup copies it in and out, one wave runs the walk.
#include "klist.h"

namespace nas {
namespace {

constexpr int THREADS = 256;  // 4 waves copy the capacity in and out; wave 0 walks
constexpr int HBUCKETS = 4096;
constexpr int FREE_SLOT = 0x7fffffff;
constexpr int LDS_CAP_MAX_NODES = (160 * 1024 - HBUCKETS * 4 - 64) / 12;

template <bool LDS_CAP>
__global__ void __launch_bounds__(THREADS)
k_commit(const u64 *__restrict__ cand_key, const u64 *__restrict__ cand_bound,
         const int *__restrict__ req, int Pp, int p_begin, int p_end, int *__restrict__ cap_g,
         int N, int *__restrict__ out_node, unsigned *__restrict__ out_cost,
         int *__restrict__ halt) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    int *table = smem;
    int *capl = smem + HBUCKETS;
    const int tid = threadIdx.x;
    // an earlier commit launch on this stream stopped at a pod that needs a
    // rescore: every later pod must wait for it (sequential semantics)
    if (__hip_atomic_load(halt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 0) return;
    for (int i = tid; i < HBUCKETS; i += THREADS) table[i] = FREE_SLOT;
    if (LDS_CAP)
        for (int i = tid; i < 3 * N; i += THREADS) capl[i] = cap_g[i];
    int *cap = LDS_CAP ? capl : cap_g;
    __syncthreads();

    if (tid < 64) {
        const int lane = tid;
        auto ld = [&](int idx) -> int {
            if (LDS_CAP) return cap[idx];
            return __hip_atomic_load(cap + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        struct Chunk {
            u64 k[KC];
            u64 bound;
            int r0, r1, r2;
        };
        // branch-free (a branchy fill kept Chunk fields in scratch): lanes
        // past p_end read a clamped, in-bounds pod and mark it inactive
        auto load = [&](int base, Chunk &c) {
            const int i = base + lane;
            const bool ok = i < p_end;
            const int ii = min(i, Pp - 1);
            load8(cand_key + (size_t)ii * KC, c.k);
            const u64 b = cand_bound[ii];
            const int r0 = req[ii], r1 = req[Pp + ii], r2 = req[2 * Pp + ii];
#pragma unroll
            for (int j = 0; j < KC; ++j) c.k[j] = ok ? c.k[j] : KEY_INVALID;
            c.bound = ok ? b : KEY_INVALID;
            c.r0 = ok ? r0 : 0;
            c.r1 = ok ? r1 : 0;
            c.r2 = ok ? r2 : 0;
        };
        // walk one chunk to completion; returns the pod that needs a rescore,
        // or -1 when every lane of the chunk is committed
        auto walk = [&](const Chunk &cur, int base) -> int {
            bool done = base + lane >= p_end;
            while (true) {
                bool fit[KC];
#pragma unroll
                for (int j = 0; j < KC; ++j) {
                    const bool usable = cur.k[j] != KEY_INVALID && cur.k[j] <= cur.bound;
                    const int n = usable ? (int)(unsigned)cur.k[j] : 0;
                    const int a = ld(n), b = ld(N + n), c = ld(2 * N + n);
                    fit[j] = usable && cur.r0 <= a && cur.r1 <= b && cur.r2 <= c;
                }
                int choice = -1;
                unsigned ccost = 0;
#pragma unroll
                for (int j = KC - 1; j >= 0; --j) {
                    if (fit[j]) {
                        choice = (int)(unsigned)cur.k[j];
                        ccost = (unsigned)(cur.k[j] >> 32);
                    }
                }
                if (done) choice = -1;
                const bool rescore = !done && choice < 0 && cur.bound != KEY_INVALID;
                // repeated picks: the lowest lane per bucket wins (one wave:
                // LDS operations complete in issue order, no barrier needed)
                const int h = choice & (HBUCKETS - 1);
                if (choice >= 0) atomicMin(&table[h], lane);
                const bool dup = choice >= 0 && table[h] != lane;
                if (choice >= 0) table[h] = FREE_SLOT;
                const u64 bad = __ballot(rescore || dup);
                const int f = bad ? __ffsll((long long)bad) - 1 : 64;
                if (!done && lane < f) {
                    const int i = base + lane;
                    if (choice >= 0) {
                        // picks of lanes < f are pairwise distinct: plain updates
                        if (LDS_CAP) {
                            cap[choice] -= cur.r0; cap[N + choice] -= cur.r1;
                            cap[2 * N + choice] -= cur.r2;
                        } else {
                            atomicSub(cap + choice, cur.r0); atomicSub(cap + N + choice, cur.r1);
                            atomicSub(cap + 2 * N + choice, cur.r2);
                        }
                    }
                    out_node[i] = choice >= 0 ? choice : NAS_EMPTY;
                    out_cost[i] = ccost;
                    done = true;
                }
                if (f < 64 && ((__ballot(rescore) >> f) & 1ull)) return base + f;
                if (__ballot(!done) == 0) return -1;
            }
        };

        constexpr int RING = 6;
        Chunk ring[RING];
#pragma unroll
        for (int s = 0; s < RING; ++s) load(p_begin + 64 * s, ring[s]);
        int stop = p_end;
        int base = p_begin;
        while (base < p_end && stop == p_end) {
#pragma unroll
            for (int s = 0; s < RING; ++s) {  // static slot index: the ring stays in VGPRs
                if (base < p_end && stop == p_end) {
                    const int r = walk(ring[s], base);
                    if (r >= 0) {
                        stop = r;
                    } else {
                        load(base + 64 * RING, ring[s]);
                        base += 64;
                    }
                }
            }
        }
        if (lane == 0 && stop < p_end) *halt = stop;
    }
    __syncthreads();
    if (LDS_CAP)
        for (int i = tid; i < 3 * N; i += THREADS) cap_g[i] = capl[i];
}

}  // namespace

hipError_t launch_commit(hipStream_t st, const uint64_t *cand_key, const uint64_t *cand_bound,
                         const int32_t *req, int Pp, int p_begin, int p_end, int32_t *cap, int N,
                         int32_t *out_node, int32_t *out_cost, int32_t *halt) {
    const auto *ck = reinterpret_cast<const u64 *>(cand_key);
    const auto *cb = reinterpret_cast<const u64 *>(cand_bound);
    auto *oc = reinterpret_cast<unsigned *>(out_cost);
    if (N <= LDS_CAP_MAX_NODES) {
        const size_t lds = (HBUCKETS + 3 * (size_t)N) * 4;
        static bool attr = false;
        if (!attr) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_commit<true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               160 * 1024);
            if (e != hipSuccess) return e;
            attr = true;
        }
        k_commit<true><<<1, THREADS, lds, st>>>(ck, cb, req, Pp, p_begin, p_end, cap, N, out_node,
                                                oc, halt);
    } else {
        k_commit<false><<<1, THREADS, HBUCKETS * 4, st>>>(ck, cb, req, Pp, p_begin, p_end, cap, N,
                                                          out_node, oc, halt);
    }
    return hipGetLastError();
}

}  // namespace nas
