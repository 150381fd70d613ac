// k_commit.hip -- conflict-resolving greedy commit with capacity update.
//
// Sequential semantics (the extended-mode oracle, oracle/oracle.c or_place):
// pods in order take the (cost, node)-smallest node that still fits the
// remaining capacity, which is then decremented.  Given per-pod candidate
// lists (the top-4 among nodes that fit some EARLIER capacity state), a pod's
// sequential choice is its first candidate that fits now: capacity only
// shrinks, so every better node either is in the list ahead of it and does
// not fit, or never fit.  If all 4 fail and the list was full, the pod needs
// a rescore against the current capacity (host loop in nas_api.cpp).
//
// Parallel form: one wave64 takes 64 consecutive pods.  Each lane picks its
// first fitting candidate against the capacity at the start of the chunk.
// Lanes whose picks are pairwise distinct are independent of one another, so
// the prefix of lanes before the first repeated pick (detected with an LDS
// atomicMin bucket table; a hash collision only shortens the prefix) is
// committed at once -- exactly what the sequential walk would do -- and the
// next chunk starts at the first repeated (or rescore-needing) lane.
// The working capacity lives in LDS (3 x N int32) when it fits, else in L2.
#include "nas_internal.h"

namespace nas {
namespace {

constexpr int HBUCKETS = 4096;
constexpr int FREE_SLOT = 0x7fffffff;
constexpr int LDS_CAP_MAX_NODES = (160 * 1024 - HBUCKETS * 4 - 64) / 12;

template <bool LDS_CAP>
__global__ void __launch_bounds__(64)
k_commit(const unsigned long long *__restrict__ cand_key, const int *__restrict__ req, int Pp,
         int p_begin, int p_end, int *__restrict__ cap_g, int N, int *__restrict__ out_node,
         unsigned *__restrict__ out_cost, int *__restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    int *table = smem;
    int *capl = smem + HBUCKETS;
    const int lane = threadIdx.x;
    for (int i = lane; i < HBUCKETS; i += 64) table[i] = FREE_SLOT;
    if (LDS_CAP)
        for (int i = lane; i < 3 * N; i += 64) capl[i] = cap_g[i];
    int *cap = LDS_CAP ? capl : cap_g;
    __syncthreads();

    auto ld = [&](int idx) -> int {
        if (LDS_CAP) return cap[idx];
        return __hip_atomic_load(cap + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };

    // candidates + requests of 64 consecutive pods, one pod per lane;
    // two chunks are prefetched ahead (the common advance is a full 64)
    struct Chunk {
        unsigned long long k[KC];
        int r0, r1, r2;
    };
    auto load = [&](int base, Chunk &c) {
        const int i = base + lane;
        if (i < p_end) {
            const ulonglong2 *s = reinterpret_cast<const ulonglong2 *>(cand_key + (size_t)i * KC);
            const ulonglong2 x = s[0], y = s[1];
            c.k[0] = x.x; c.k[1] = x.y; c.k[2] = y.x; c.k[3] = y.y;
            c.r0 = req[i]; c.r1 = req[Pp + i]; c.r2 = req[2 * Pp + i];
        } else {
#pragma unroll
            for (int j = 0; j < KC; ++j) c.k[j] = KEY_INVALID;
            c.r0 = c.r1 = c.r2 = 0;
        }
    };

    int stop = p_end;
    int p = p_begin;
    Chunk cur, nx1, nx2;
    load(p, cur);
    load(p + 64, nx1);
    load(p + 128, nx2);
    while (p < p_end) {
        const int i = p + lane;
        const bool active = i < p_end;
        int choice = -1, nvalid = 0;
        unsigned ccost = 0;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
            if (cur.k[j] != KEY_INVALID) {
                ++nvalid;
                if (choice < 0) {
                    const int n = (int)(unsigned)cur.k[j];
                    if (cur.r0 <= ld(n) && cur.r1 <= ld(N + n) && cur.r2 <= ld(2 * N + n)) {
                        choice = n;
                        ccost = (unsigned)(cur.k[j] >> 32);
                    }
                }
            }
        }
        const bool rescore = active && choice < 0 && nvalid == KC;
        // repeated picks inside the chunk: the lowest lane per bucket wins
        // (one wave: LDS operations complete in issue order, no barrier)
        const int h = choice & (HBUCKETS - 1);
        if (choice >= 0) atomicMin(&table[h], lane);
        const bool dup = choice >= 0 && table[h] != lane;
        if (choice >= 0) table[h] = FREE_SLOT;
        const unsigned long long bad = __ballot(rescore || dup);
        const int f = bad ? __ffsll((long long)bad) - 1 : 64;
        if (active && lane < f) {
            if (choice >= 0) {
                // picks of lanes < f are pairwise distinct: plain updates
                if (LDS_CAP) {
                    cap[choice] -= cur.r0; cap[N + choice] -= cur.r1; cap[2 * N + choice] -= cur.r2;
                } else {
                    atomicSub(cap + choice, cur.r0); atomicSub(cap + N + choice, cur.r1);
                    atomicSub(cap + 2 * N + choice, cur.r2);
                }
            }
            out_node[i] = choice >= 0 ? choice : NAS_EMPTY;
            out_cost[i] = ccost;
        }
        if (f < 64 && ((__ballot(rescore) >> f) & 1ull)) {
            stop = p + f;
            break;
        }
        p += f;
        if (f == 64) {
            cur = nx1;
            nx1 = nx2;
            load(p + 128, nx2);
        } else {
            load(p, cur);
            load(p + 64, nx1);
            load(p + 128, nx2);
        }
    }
    __syncthreads();
    if (LDS_CAP)
        for (int i = lane; i < 3 * N; i += 64) cap_g[i] = capl[i];
    if (lane == 0) status[0] = stop;
}

}  // namespace

hipError_t launch_commit(hipStream_t st, const uint64_t *cand_key, const int32_t *cand_cnt,
                         const int32_t *req, int Pp, int p_begin, int p_end, int32_t *cap, int N,
                         int32_t *out_node, int32_t *out_cost, int32_t *status) {
    (void)cand_cnt;
    const auto *ck = reinterpret_cast<const unsigned long long *>(cand_key);
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
        k_commit<true><<<1, 64, lds, st>>>(ck, req, Pp, p_begin, p_end, cap, N, out_node,
                                           reinterpret_cast<unsigned *>(out_cost), status);
    } else {
        k_commit<false><<<1, 64, HBUCKETS * 4, st>>>(ck, req, Pp, p_begin, p_end, cap, N, out_node,
                                                     reinterpret_cast<unsigned *>(out_cost), status);
    }
    return hipGetLastError();
}

}  // namespace nas
