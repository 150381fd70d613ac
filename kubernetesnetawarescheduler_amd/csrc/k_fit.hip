// k_fit.hip -- batched resource-fit filter over all pod x node pairs.
//
// The reference's filter stage is findNodesThatFit (scheduler/scheduler.go:239-246),
// which lists the nodes and filters nothing; the north star's filter is the
// Kubernetes NodeResourcesFit rule: pod p fits node n iff
// req[r][p] <= free[r][n] for r in {cpu millicores, memory KiB, pod slots}.
//
// Layout: lane-per-NODE.  Each wave owns one 64-node chunk c (lane j = node
// 64c + j, its three free capacities in VGPRs, read once, plus the chunk's
// minima and maxima, wave-uniform) and walks its pods 64 at a time, lane i
// holding pod i's requests:
//   * three v_cmp against the chunk minima decide, for all 64 pods at once,
//     the pods that fit EVERY valid node of the chunk (word = valid-node
//     mask), three against the maxima the pods that fit NONE (word = 0);
//   * each remaining pod is broadcast (v_readlane) and compared against the
//     64 lanes' capacities: three ballots ANDed are its word, written
//     into its lane;
// and the 64 words leave in one coalesced 8-byte-per-lane store:
//   mask[c * Pp + p]  bit j  <=>  pod p fits local node 64c + j.
// Requests are small against node capacity until nodes fill up, so most
// (pod, chunk) pairs cost 1/64 of a compare; the kernel runs near the rate of
// its mask write (P*N/8 bytes, HBM) -- see DESIGN.md.
#include "nas_internal.h"

namespace nas {
namespace {

constexpr int FIT_THREADS = 256;  // 4 waves = 4 node chunks per block
constexpr int FIT_WAVES = FIT_THREADS / 64;
constexpr int FIT_GROUPS_MAX = 8;  // 64-pod groups per block (at most 512 pods)
constexpr int FIT_PF = 2;          // groups of requests in flight ahead of the one decided

// G = 64-pod groups per wave (compile time: the group loop is unrolled and the
// request ring stays in registers).  Measured at the C3 shape (10k nodes x 100k
// pods, tools/mb_fit.hip): 29.0 us for the round-2 kernel (runtime group loop,
// one group prefetched), 25.5 us unrolled with the uniform bounds in SGPRs,
// 24.5 us with non-temporal mask stores (the mask is written once).
template <int G>
__global__ void __launch_bounds__(FIT_THREADS)
k_fit(const int *cap, int N, int n0, int nloc, int n_chunks,
      const int *__restrict__ req, int Pp, int p0, int p_end, unsigned long long *__restrict__ mask,
      const int *__restrict__ dyn_start, int dyn_win, const int *__restrict__ dyn_hi_ptr,
      const int *__restrict__ rowmap, int rs) {
    // rowmap (gathered rescore view): row q's requests are pod rowmap[q]'s,
    // in the main request array (row stride rs); the mask keeps view rows
    if (dyn_start) {  // window [*dyn_start, +dyn_win) read from device memory (rescore slots)
        const int s = dyn_start[blockIdx.z * STATUS_INTS];
        if (s < 0) return;
        p0 = s;
        if (dyn_hi_ptr) p_end = dyn_hi_ptr[blockIdx.z * STATUS_INTS];
        p_end = min(p_end, s + dyn_win);
    }
    const int pb0 = p0 + (int)blockIdx.x * 64 * G;
    if (pb0 >= p_end) return;  // whole block (no barriers below)
    const int cb = blockIdx.z;  // cluster of a batched launch
    cap += (size_t)cb * 3 * N;
    req += (size_t)cb * 3 * rs;
    mask += (size_t)cb * n_chunks * Pp;
    const int lane = threadIdx.x & 63;
    const int c = (int)blockIdx.y * FIT_WAVES + (int)(threadIdx.x >> 6);
    if (c >= n_chunks) return;
    const int nl = c * 64 + lane;
    const int pend = min(p_end, pb0 + 64 * G);
    // lane i holds pod pb + i's requests (one coalesced load per resource),
    // FIT_PF groups ahead of the one being decided; rows past the range are
    // clamped to its last row (loaded, never stored)
    auto row = [&](int r) { const int q = min(r, p_end - 1); return rowmap ? rowmap[q] : q; };
    constexpr int RING = FIT_PF + 1 < G ? FIT_PF + 1 : G;
    int ra[RING], rb[RING], rd[RING];
#pragma unroll
    for (int g = 0; g < RING; ++g) {
        const int q = row(pb0 + 64 * g + lane);
        ra[g] = req[q];
        rb[g] = req[rs + q];
        rd[g] = req[2 * (size_t)rs + q];
    }
    // relaxed atomic loads: nas_place filters against the working capacity
    // while the commit stream publishes into it; padding nodes never fit
    int fc = -1, fm = -1, fp = -1;
    if (nl < nloc) {
        int *cp = const_cast<int *>(cap) + n0 + nl;
        fc = __hip_atomic_load(cp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fm = __hip_atomic_load(cp + N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fp = __hip_atomic_load(cp + 2 * (size_t)N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the chunk's valid nodes, its smallest and largest capacities (padding
    // lanes excluded: they fit nothing), wave-uniform (SGPRs)
    const bool real = nl < nloc;
    const unsigned long long valid = __builtin_amdgcn_ballot_w64(real);
    int mc = real ? fc : 0x7fffffff, mm = real ? fm : 0x7fffffff, mp = real ? fp : 0x7fffffff;
    int xc = real ? fc : (int)0x80000000, xm = real ? fm : (int)0x80000000;
    int xp = real ? fp : (int)0x80000000;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        mc = min(mc, __shfl_xor(mc, o));
        mm = min(mm, __shfl_xor(mm, o));
        mp = min(mp, __shfl_xor(mp, o));
        xc = max(xc, __shfl_xor(xc, o));
        xm = max(xm, __shfl_xor(xm, o));
        xp = max(xp, __shfl_xor(xp, o));
    }
    mc = __builtin_amdgcn_readfirstlane(mc);
    mm = __builtin_amdgcn_readfirstlane(mm);
    mp = __builtin_amdgcn_readfirstlane(mp);
    xc = __builtin_amdgcn_readfirstlane(xc);
    xm = __builtin_amdgcn_readfirstlane(xm);
    xp = __builtin_amdgcn_readfirstlane(xp);
    const unsigned vlo = (unsigned)valid, vhi = (unsigned)(valid >> 32);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int pb = pb0 + 64 * g;
        if (pb >= pend) break;
        const int sl = g % RING;
        const int a0 = ra[sl], b0 = rb[sl], d0 = rd[sl];
        if (g + RING < G) {  // refill the slot just consumed
            const int q = row(pb + 64 * RING + lane);
            ra[sl] = req[q];
            rb[sl] = req[rs + q];
            rd[sl] = req[2 * (size_t)rs + q];
        }
        const bool in = pb + lane < pend;
        // 64 pods at once against the chunk's extremes: fits every valid node
        // (requests <= the minima) or none (some request > its maximum)
        const unsigned long long all = __builtin_amdgcn_ballot_w64(in && a0 <= mc && b0 <= mm && d0 <= mp);
        const unsigned long long none = __builtin_amdgcn_ballot_w64(in && (a0 > xc || b0 > xm || d0 > xp));
        unsigned long long rest = __builtin_amdgcn_ballot_w64(in) & ~all & ~none;
        unsigned lo = ((all >> lane) & 1) ? vlo : 0u, hi = ((all >> lane) & 1) ? vhi : 0u;
        // the others one by one: the pod's (broadcast) requests against the
        // lanes' capacities, three ballots ANDed, written into its lane
        while (rest) {
            const int i = (int)__builtin_ctzll(rest);
            rest &= rest - 1;
            const int a = __builtin_amdgcn_readlane(a0, i), b = __builtin_amdgcn_readlane(b0, i);
            const int d = __builtin_amdgcn_readlane(d0, i);
            const unsigned long long m = __builtin_amdgcn_ballot_w64(a <= fc) &
                                         __builtin_amdgcn_ballot_w64(b <= fm) &
                                         __builtin_amdgcn_ballot_w64(d <= fp);
            if (lane == i) {
                lo = (unsigned)m;
                hi = (unsigned)(m >> 32);
            }
        }
        if (in)
            __builtin_nontemporal_store(((unsigned long long)hi << 32) | lo,
                                        mask + (size_t)c * Pp + pb + lane);
    }
}

// Two pods per lane (pods pb + 2i and pb + 2i + 1 of a 128-pod group): the
// requests arrive as one 8-byte load per resource and the two fit words leave
// as ONE 16-byte store per lane -- half the memory instructions of k_fit per
// pod for the same bytes.  Same decisions as k_fit (the chunk's extremes
// first, then the remaining pods one by one); main pod ranges only (no row
// map: a gathered view's rows are not adjacent).
template <int G>
__global__ void __launch_bounds__(FIT_THREADS)
k_fit2(const int *cap, int N, int n0, int nloc, int n_chunks,
       const int *__restrict__ req, int Pp, int p0, int p_end, unsigned long long *__restrict__ mask,
       const int *__restrict__ dyn_start, int dyn_win, const int *__restrict__ dyn_hi_ptr) {
    if (dyn_start) {
        const int s = dyn_start[blockIdx.z * STATUS_INTS];
        if (s < 0) return;
        p0 = s & ~1;  // pairs start on an even pod (the store is 16-byte aligned)
        if (dyn_hi_ptr) p_end = dyn_hi_ptr[blockIdx.z * STATUS_INTS];
        p_end = min(p_end, s + dyn_win);
    }
    const int pb0 = p0 + (int)blockIdx.x * 128 * G;
    if (pb0 >= p_end) return;
    const int cb = blockIdx.z;
    cap += (size_t)cb * 3 * N;
    req += (size_t)cb * 3 * Pp;
    mask += (size_t)cb * n_chunks * Pp;
    const int lane = threadIdx.x & 63;
    const int c = (int)blockIdx.y * FIT_WAVES + (int)(threadIdx.x >> 6);
    if (c >= n_chunks) return;
    const int nl = c * 64 + lane;
    const int pend = min(p_end, pb0 + 128 * G);
    int fc = -1, fm = -1, fp = -1;
    if (nl < nloc) {
        int *cp = const_cast<int *>(cap) + n0 + nl;
        fc = __hip_atomic_load(cp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fm = __hip_atomic_load(cp + N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fp = __hip_atomic_load(cp + 2 * (size_t)N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool real = nl < nloc;
    const unsigned long long valid = __builtin_amdgcn_ballot_w64(real);
    int mc = real ? fc : 0x7fffffff, mm = real ? fm : 0x7fffffff, mp = real ? fp : 0x7fffffff;
    int xc = real ? fc : (int)0x80000000, xm = real ? fm : (int)0x80000000;
    int xp = real ? fp : (int)0x80000000;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        mc = min(mc, __shfl_xor(mc, o));
        mm = min(mm, __shfl_xor(mm, o));
        mp = min(mp, __shfl_xor(mp, o));
        xc = max(xc, __shfl_xor(xc, o));
        xm = max(xm, __shfl_xor(xm, o));
        xp = max(xp, __shfl_xor(xp, o));
    }
    mc = __builtin_amdgcn_readfirstlane(mc);
    mm = __builtin_amdgcn_readfirstlane(mm);
    mp = __builtin_amdgcn_readfirstlane(mp);
    xc = __builtin_amdgcn_readfirstlane(xc);
    xm = __builtin_amdgcn_readfirstlane(xm);
    xp = __builtin_amdgcn_readfirstlane(xp);
    // requests of the lane's two pods (8-byte loads; rows past the range read
    // the last even pair, loaded, never stored)
    auto load2 = [&](int pb, int2 &a, int2 &b, int2 &d) {
        const int q = min(pb + 2 * lane, (p_end - 1) & ~1);
        a = *reinterpret_cast<const int2 *>(req + q);
        b = *reinterpret_cast<const int2 *>(req + Pp + q);
        d = *reinterpret_cast<const int2 *>(req + 2 * (size_t)Pp + q);
    };
    int2 ra, rb, rd;
    load2(pb0, ra, rb, rd);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int pb = pb0 + 128 * g;
        if (pb >= pend) break;
        const int2 a0 = ra, b0 = rb, d0 = rd;
        if (g + 1 < G) load2(pb + 128, ra, rb, rd);  // next group in flight
        const bool in0 = pb + 2 * lane < pend, in1 = pb + 2 * lane + 1 < pend;
        unsigned long long w0 = 0, w1 = 0;
        // half h: the lanes' pod pb + 2 * lane + h
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int a = h ? a0.y : a0.x, b = h ? b0.y : b0.x, d = h ? d0.y : d0.x;
            const bool in = h ? in1 : in0;
            const unsigned long long all = __builtin_amdgcn_ballot_w64(in && a <= mc && b <= mm && d <= mp);
            const unsigned long long none =
                __builtin_amdgcn_ballot_w64(in && (a > xc || b > xm || d > xp));
            unsigned long long rest = __builtin_amdgcn_ballot_w64(in) & ~all & ~none;
            unsigned long long word = ((all >> lane) & 1) ? valid : 0ull;
            while (rest) {
                const int i = (int)__builtin_ctzll(rest);
                rest &= rest - 1;
                const int ba = __builtin_amdgcn_readlane(a, i), bb = __builtin_amdgcn_readlane(b, i);
                const int bd = __builtin_amdgcn_readlane(d, i);
                const unsigned long long m = __builtin_amdgcn_ballot_w64(ba <= fc) &
                                             __builtin_amdgcn_ballot_w64(bb <= fm) &
                                             __builtin_amdgcn_ballot_w64(bd <= fp);
                if (lane == i) word = m;
            }
            if (h) w1 = word;
            else w0 = word;
        }
        unsigned long long *dst = mask + (size_t)c * Pp + pb + 2 * lane;
        // plain stores: 24.7-24.9 vs 25.1-25.8 us for non-temporal ones at the
        // C3 shape (profiles/r04_ab_fold.txt, fitpl)
        if (in1) {
            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u64x2 *>(dst) = u64x2{w0, w1};
        } else if (in0) {
            *dst = w0;
        }
    }
}

}  // namespace

hipError_t launch_fit(hipStream_t st, const int32_t *cap, int N, int n0, int nloc, int Mp,
                      const int32_t *req, int P, int Pp, int p0, int np, uint64_t *mask,
                      const Dyn *dyn, int batch, const int32_t *rowmap, int req_stride) {
    (void)P;
    if (rowmap && batch != 1) return hipErrorInvalidValue;
    if (np <= 0) return hipSuccess;
    const int n_chunks = Mp / 64;
    if (!rowmap && p0 % 2 == 0) {  // two pods per lane (k_fit2)
        // pods per block: up to 512 (4 groups of 128), fewer on small launches
        const int yb2 = (n_chunks + FIT_WAVES - 1) / FIT_WAVES;
        const long long groups2 = ((long long)np + 127) / 128 * yb2;
        const int k2 = (int)std::max(1LL, std::min<long long>(4, groups2 / 2048));
        const int G2 = k2 >= 4 ? 4 : k2 >= 2 ? 2 : 1;
        dim3 grid2((np + 128 * G2 - 1) / (128 * G2) + (dyn ? 1 : 0), yb2, batch);
        auto *m2 = reinterpret_cast<unsigned long long *>(mask);
        const int pe2 = dyn ? dyn->hi : p0 + np;
        const int *ds2 = dyn ? dyn->start : nullptr, *dh2 = dyn ? dyn->hi_ptr : nullptr;
        const int dw2 = dyn ? dyn->win : 0;
#define NAS_FIT2(GV) \
    k_fit2<GV><<<grid2, FIT_THREADS, 0, st>>>(cap, N, n0, nloc, n_chunks, req, Pp, p0, pe2, m2, ds2, dw2, dh2)
        switch (G2) {
        case 4: NAS_FIT2(4); break;
        case 2: NAS_FIT2(2); break;
        default: NAS_FIT2(1); break;
        }
#undef NAS_FIT2
        return hipGetLastError();
    }
    // pods per block: up to 512, fewer when the launch is small, so a rescore
    // slot's few thousand pods still spread over ~2k blocks (each wave's pod
    // groups run back to back: latency, not work, sets a small launch's time)
    const int yb = (n_chunks + FIT_WAVES - 1) / FIT_WAVES;
    const long long groups = ((long long)np + 63) / 64 * yb;
    const int k = (int)std::max(1LL, std::min<long long>(FIT_GROUPS_MAX, groups / 2048));
    const int G = k >= 8 ? 8 : k >= 4 ? 4 : k >= 2 ? 2 : 1;  // instantiated group counts
    dim3 grid((np + 64 * G - 1) / (64 * G), yb, batch);
    auto *m = reinterpret_cast<unsigned long long *>(mask);
    const int pe = dyn ? dyn->hi : p0 + np;
    const int *ds = dyn ? dyn->start : nullptr, *dh = dyn ? dyn->hi_ptr : nullptr;
    const int dw = dyn ? dyn->win : 0, rs = rowmap ? req_stride : Pp;
#define NAS_FIT(GV) \
    k_fit<GV><<<grid, FIT_THREADS, 0, st>>>(cap, N, n0, nloc, n_chunks, req, Pp, p0, pe, m, ds, dw, dh, rowmap, rs)
    switch (G) {
    case 8: NAS_FIT(8); break;
    case 4: NAS_FIT(4); break;
    case 2: NAS_FIT(2); break;
    default: NAS_FIT(1); break;
    }
#undef NAS_FIT
    return hipGetLastError();
}

}  // namespace nas
