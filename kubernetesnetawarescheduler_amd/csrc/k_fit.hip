// k_fit.hip -- batched resource-fit filter over all pod x node pairs.
//
// The reference's filter stage is findNodesThatFit (scheduler/scheduler.go:239-246),
// which lists the nodes and filters nothing; the north star's filter is the
// Kubernetes NodeResourcesFit rule: pod p fits node n iff
// req[r][p] <= free[r][n] for r in {cpu millicores, memory KiB, pod slots}.
//
// Layout: lane-per-node.  Each wave owns a 64-node chunk and keeps that
// chunk's free capacity in VGPRs (one coalesced SoA read); it then walks the
// pods 64 at a time: one coalesced load of their requests, broadcast to the
// wave with v_readlane, and the three vector compares produce the 64-bit fit
// mask of (pod, chunk) directly in an SGPR pair (a ballot).  64 consecutive pods' masks are collected one per lane and
// written with one coalesced 8-byte-per-lane store:
//   mask[c * Pp + p]  bit j  <=>  pod p fits local node 64c + j.
// HBM-bound on the mask write (P*N/8 bytes) -- see DESIGN.md.
#include "nas_internal.h"

namespace nas {
namespace {

constexpr int FIT_THREADS = 256;       // 4 waves = 4 node chunks per block
constexpr int FIT_PODS_PER_BLOCK = 512;

__global__ void __launch_bounds__(FIT_THREADS)
k_fit(const int *__restrict__ cap, int N, int n0, int nloc, int n_chunks,
      const int *__restrict__ req, int Pp, int p0, int p_end, unsigned long long *__restrict__ mask) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.y * (FIT_THREADS / 64) + (threadIdx.x >> 6);
    if (c >= n_chunks) return;  // wave-uniform
    const int nl = c * 64 + lane;  // local node
    // padding nodes (nl >= nloc) never fit: requests are >= 0
    int fc = -1, fm = -1, fp = -1;
    if (nl < nloc) {
        fc = cap[n0 + nl];
        fm = cap[N + n0 + nl];
        fp = cap[2 * N + n0 + nl];
    }
    const int *rc = req, *rm = req + Pp, *rp = req + 2 * Pp;
    const int pb = p0 + blockIdx.x * FIT_PODS_PER_BLOCK;
    const int pe = min(p_end, pb + FIT_PODS_PER_BLOCK);
    for (int p = pb; p < pe; p += 64) {
        // one coalesced load of 64 pods' requests, broadcast with v_readlane
        const int q = p + lane;
        const int a = q < pe ? rc[q] : 0x7fffffff;
        const int b = q < pe ? rm[q] : 0x7fffffff;
        const int d = q < pe ? rp[q] : 0x7fffffff;
        unsigned long long mine = 0;
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            const int ra = __builtin_amdgcn_readlane(a, i);
            const int rb = __builtin_amdgcn_readlane(b, i);
            const int rd = __builtin_amdgcn_readlane(d, i);
            const unsigned long long m = __ballot(ra <= fc && rb <= fm && rd <= fp);
            mine = lane == i ? m : mine;
        }
        if (q < pe) mask[(size_t)c * Pp + q] = mine;
    }
}

}  // namespace

hipError_t launch_fit(hipStream_t st, const int32_t *cap, int N, int n0, int nloc, int Mp,
                      const int32_t *req, int P, int Pp, int p0, int np, uint64_t *mask) {
    (void)P;
    if (np <= 0) return hipSuccess;
    const int n_chunks = Mp / 64;
    dim3 grid((np + FIT_PODS_PER_BLOCK - 1) / FIT_PODS_PER_BLOCK,
              (n_chunks + FIT_THREADS / 64 - 1) / (FIT_THREADS / 64));
    k_fit<<<grid, FIT_THREADS, 0, st>>>(cap, N, n0, nloc, n_chunks, req, Pp, p0, p0 + np,
                                        reinterpret_cast<unsigned long long *>(mask));
    return hipGetLastError();
}

}  // namespace nas
