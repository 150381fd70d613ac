// k_fit.hip -- batched resource-fit filter over all pod x node pairs.
//
// The reference's filter stage is findNodesThatFit (scheduler/scheduler.go:239-246),
// which lists the nodes and filters nothing; the north star's filter is the
// Kubernetes NodeResourcesFit rule: pod p fits node n iff
// req[r][p] <= free[r][n] for r in {cpu millicores, memory KiB, pod slots}.
//
// Layout: lane-per-NODE.  Each wave owns one 64-node chunk c (lane j = node
// 64c + j, its three free capacities in VGPRs, read once) and walks pods:
// a pod's requests are wave-uniform (wide scalar loads of 64 pods at a
// time), three v_cmp against
// the lanes' capacities and their AND are the pod's 64-bit fit word for the
// chunk directly -- the ballot -- which v_writelane drops into lane i of the
// group's result, so 64 pods end in one coalesced 8-byte-per-lane store:
//   mask[c * Pp + p]  bit j  <=>  pod p fits local node 64c + j.
// ~8 instructions per (pod, 64 nodes) instead of ~6 per (pod, node) in a
// lane-per-pod form.  Most pods fit every node of a chunk outright (requests
// are small against node capacity until nodes fill up): a pod whose three
// requests are <= the chunk's smallest capacities (wave-uniform, reduced
// once) is settled by three SCALAR compares into a 64-pod "fits everything"
// mask, and one v_cndmask per group writes the chunk's valid-node mask for
// all of them; only the other pods take the ballot path.  The kernel then
// runs near the rate of its mask write (P*N/8 bytes, HBM) -- see DESIGN.md.
#include "nas_internal.h"

namespace nas {
namespace {

// 16 ints at 4-byte alignment: one s_load_dwordx16 from a uniform address
typedef int v16i_a4 __attribute__((ext_vector_type(16), aligned(4)));

constexpr int FIT_THREADS = 256;  // 4 waves = 4 node chunks per block
constexpr int FIT_WAVES = FIT_THREADS / 64;
constexpr int FIT_GROUPS_MAX = 8;  // 64-pod groups per block (at most 512 pods)

__global__ void __launch_bounds__(FIT_THREADS)
k_fit(const int *cap, int N, int n0, int nloc, int n_chunks,
      const int *__restrict__ req, int Pp, int p0, int p_end, unsigned long long *__restrict__ mask,
      const int *__restrict__ dyn_start, int dyn_win, const int *__restrict__ dyn_hi_ptr,
      int block_pods) {
    if (dyn_start) {  // window [*dyn_start, +dyn_win) read from device memory (rescore slots)
        const int s = dyn_start[blockIdx.z * STATUS_INTS];
        if (s < 0) return;
        p0 = s;
        if (dyn_hi_ptr) p_end = dyn_hi_ptr[blockIdx.z * STATUS_INTS];
        p_end = min(p_end, s + dyn_win);
    }
    const int pb0 = p0 + (int)blockIdx.x * block_pods;
    if (pb0 >= p_end) return;  // whole block (no barriers below)
    const int cb = blockIdx.z;  // cluster of a batched launch
    cap += (size_t)cb * 3 * N;
    req += (size_t)cb * 3 * Pp;
    mask += (size_t)cb * n_chunks * Pp;
    const int lane = threadIdx.x & 63;
    const int c = (int)blockIdx.y * FIT_WAVES + (int)(threadIdx.x >> 6);
    if (c >= n_chunks) return;
    const int nl = c * 64 + lane;
    // relaxed atomic loads: nas_place filters against the working capacity
    // while the commit stream publishes into it; padding nodes never fit
    int fc = -1, fm = -1, fp = -1;
    if (nl < nloc) {
        int *cp = const_cast<int *>(cap) + n0 + nl;
        fc = __hip_atomic_load(cp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fm = __hip_atomic_load(cp + N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fp = __hip_atomic_load(cp + 2 * (size_t)N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the chunk's valid nodes and its smallest capacities (padding lanes
    // excluded: they fit nothing), wave-uniform
    const unsigned long long valid = __builtin_amdgcn_ballot_w64(nl < nloc);
    int mc = nl < nloc ? fc : 0x7fffffff, mm = nl < nloc ? fm : 0x7fffffff;
    int mp = nl < nloc ? fp : 0x7fffffff;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        mc = min(mc, __shfl_xor(mc, o));
        mm = min(mm, __shfl_xor(mm, o));
        mp = min(mp, __shfl_xor(mp, o));
    }
    mc = __builtin_amdgcn_readfirstlane(mc);
    mm = __builtin_amdgcn_readfirstlane(mm);
    mp = __builtin_amdgcn_readfirstlane(mp);
    const unsigned vlo = (unsigned)valid, vhi = (unsigned)(valid >> 32);
    const int pend = min(p_end, pb0 + block_pods);
    for (int pb = pb0; pb < pend; pb += 64) {
        unsigned lo = 0, hi = 0;
        unsigned long long all_fit = 0;  // pods of the group that fit every valid node
        // lane i takes pod pb + i's word: three v_cmp of the pod's (uniform)
        // requests against the lanes' capacities straight into SGPR lane
        // masks, ANDed on the scalar unit, v_writelane into lane i
        auto pod = [&](int i, int ra, int rb, int rd) {
            if (ra <= mc && rb <= mm && rd <= mp) {  // uniform: scalar compares only
                all_fit |= 1ull << i;
                return;
            }
            const unsigned long long m = __builtin_amdgcn_ballot_w64(ra <= fc) &
                                         __builtin_amdgcn_ballot_w64(rb <= fm) &
                                         __builtin_amdgcn_ballot_w64(rd <= fp);
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(lo) : "s"((unsigned)m), "i"(i));
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(hi) : "s"((unsigned)(m >> 32)), "i"(i));
        };
        if (pb + 64 <= Pp) {
            // the group's requests through the scalar unit: wide s_loads of
            // 64 consecutive ints per resource, issued together
            const int *qa = req + pb, *qb = req + Pp + pb, *qd = req + 2 * (size_t)Pp + pb;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const v16i_a4 a = *reinterpret_cast<const v16i_a4 *>(qa + 16 * k);
                const v16i_a4 b = *reinterpret_cast<const v16i_a4 *>(qb + 16 * k);
                const v16i_a4 d = *reinterpret_cast<const v16i_a4 *>(qd + 16 * k);
#pragma unroll
                for (int i = 0; i < 16; ++i) pod(16 * k + i, a[i], b[i], d[i]);
            }
        } else {
            // a window running past the padded rows (rescore views): one
            // coalesced load per resource, broadcast with v_readlane
            const int q = min(pb + lane, Pp - 1);
            const int va = req[q], vb = req[Pp + q], vd = req[2 * Pp + q];
#pragma unroll
            for (int i = 0; i < 64; ++i)
                pod(i, __builtin_amdgcn_readlane(va, i), __builtin_amdgcn_readlane(vb, i),
                    __builtin_amdgcn_readlane(vd, i));
        }
        if ((all_fit >> lane) & 1) {
            lo = vlo;
            hi = vhi;
        }
        if (pb + lane < pend) mask[(size_t)c * Pp + pb + lane] = ((unsigned long long)hi << 32) | lo;
    }
}

}  // namespace

hipError_t launch_fit(hipStream_t st, const int32_t *cap, int N, int n0, int nloc, int Mp,
                      const int32_t *req, int P, int Pp, int p0, int np, uint64_t *mask,
                      const Dyn *dyn, int batch) {
    (void)P;
    if (np <= 0) return hipSuccess;
    const int n_chunks = Mp / 64;
    // pods per block: up to 512, fewer when the launch is small, so a rescore
    // slot's few thousand pods still spread over ~2k blocks (each wave's pod
    // groups run back to back: latency, not work, sets a small launch's time)
    const int yb = (n_chunks + FIT_WAVES - 1) / FIT_WAVES;
    const long long groups = ((long long)np + 63) / 64 * yb;
    const int k = (int)std::max(1LL, std::min<long long>(FIT_GROUPS_MAX, groups / 2048));
    const int block_pods = 64 * k;
    dim3 grid((np + block_pods - 1) / block_pods, yb, batch);
    k_fit<<<grid, FIT_THREADS, 0, st>>>(cap, N, n0, nloc, n_chunks, req, Pp, p0,
                                        dyn ? dyn->hi : p0 + np,
                                        reinterpret_cast<unsigned long long *>(mask),
                                        dyn ? dyn->start : nullptr, dyn ? dyn->win : 0,
                                        dyn ? dyn->hi_ptr : nullptr, block_pods);
    return hipGetLastError();
}

}  // namespace nas
