// k_fit.hip -- batched resource-fit filter over all pod x node pairs.
//
// The reference's filter stage is findNodesThatFit (scheduler/scheduler.go:239-246),
// which lists the nodes and filters nothing; the north star's filter is the
// Kubernetes NodeResourcesFit rule: pod p fits node n iff
// req[r][p] <= free[r][n] for r in {cpu millicores, memory KiB, pod slots}.
//
// Layout: lane-per-pod.  A block owns 256 consecutive pods (one per lane;
// requests in VGPRs, one coalesced read) and FIT_CHUNKS 64-node chunks, whose
// capacities it stages once in LDS (SoA, padding nodes = -1 so they never
// fit).  Per node, the wave reads the node's three capacities with
// wave-uniform (broadcast) ds_read_b128s, three v_cmp give the fit lane mask
// and one shift-and-add folds it into the lane's 32-bit word (nodes visited
// high to low, so bit j ends up as node j).  Every lane then holds its pod's
// 64-bit word for the chunk and the wave writes them with one coalesced
// 8-byte-per-lane store:
//   mask[c * Pp + p]  bit j  <=>  pod p fits local node 64c + j.
// ~5 VALU per 64 pairs: the kernel runs near the speed of its mask write
// (P*N/8 bytes, HBM) -- see DESIGN.md.
#include "nas_internal.h"

namespace nas {
namespace {

constexpr int FIT_THREADS = 256;  // 4 waves = 256 pods per block
constexpr int FIT_CHUNKS = 8;     // 512 nodes per block

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(FIT_THREADS)
k_fit(const int *cap, int N, int n0, int nloc, int n_chunks,
      const int *__restrict__ req, int Pp, int p0, int p_end, unsigned long long *__restrict__ mask,
      const int *__restrict__ dyn_start, int dyn_win, const int *__restrict__ dyn_hi_ptr) {
    if (dyn_start) {  // window [*dyn_start, +dyn_win) read from device memory (rescore slots)
        const int s = dyn_start[blockIdx.z * STATUS_INTS];
        if (s < 0) return;
        p0 = s;
        if (dyn_hi_ptr) p_end = dyn_hi_ptr[blockIdx.z * STATUS_INTS];
        p_end = min(p_end, s + dyn_win);
        if (p0 + (int)blockIdx.x * FIT_THREADS >= p_end) return;  // whole block
    }
    const int cb = blockIdx.z;  // cluster of a batched launch
    cap += (size_t)cb * 3 * N;
    req += (size_t)cb * 3 * Pp;
    mask += (size_t)cb * n_chunks * Pp;
    __shared__ __attribute__((aligned(16))) int sc[3][FIT_CHUNKS * 64];
    const int tid = threadIdx.x;
    const int c0 = blockIdx.y * FIT_CHUNKS;
    const int c1 = min(n_chunks, c0 + FIT_CHUNKS);
    for (int i = tid; i < FIT_CHUNKS * 64; i += FIT_THREADS) {
        const int nl = c0 * 64 + i;
        const bool real = nl < nloc;
        // relaxed atomic loads: nas_place filters against the working
        // capacity while the commit stream publishes into it
#pragma unroll
        for (int r = 0; r < 3; ++r)
            sc[r][i] = real ? __hip_atomic_load(const_cast<int *>(cap) + (size_t)r * N + n0 + nl, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)
                            : -1;
    }
    const int p = p0 + blockIdx.x * FIT_THREADS + tid;
    const int q = min(p, Pp - 1);
    const int ra = req[q], rb = req[Pp + q], rd = req[2 * Pp + q];
    __syncthreads();
    for (int c = c0; c < c1; ++c) {
        const int *lc = &sc[0][(c - c0) * 64], *lm = &sc[1][(c - c0) * 64];
        const int *lp = &sc[2][(c - c0) * 64];
        unsigned w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            unsigned acc = 0;
#pragma unroll
            for (int j4 = 7; j4 >= 0; --j4) {
                const int o = h * 32 + j4 * 4;
                const v4i fc = *reinterpret_cast<const v4i *>(lc + o);
                const v4i fm = *reinterpret_cast<const v4i *>(lm + o);
                const v4i fp = *reinterpret_cast<const v4i *>(lp + o);
#pragma unroll
                for (int j = 3; j >= 0; --j)
                    acc = acc * 2u + ((ra <= fc[j] && rb <= fm[j] && rd <= fp[j]) ? 1u : 0u);
            }
            w[h] = acc;
        }
        if (p < p_end) mask[(size_t)c * Pp + p] = ((unsigned long long)w[1] << 32) | w[0];
    }
}

}  // namespace

hipError_t launch_fit(hipStream_t st, const int32_t *cap, int N, int n0, int nloc, int Mp,
                      const int32_t *req, int P, int Pp, int p0, int np, uint64_t *mask,
                      const Dyn *dyn, int batch) {
    (void)P;
    if (np <= 0) return hipSuccess;
    const int n_chunks = Mp / 64;
    dim3 grid((np + FIT_THREADS - 1) / FIT_THREADS,
              (n_chunks + FIT_CHUNKS - 1) / FIT_CHUNKS, batch);
    k_fit<<<grid, FIT_THREADS, 0, st>>>(cap, N, n0, nloc, n_chunks, req, Pp, p0,
                                        dyn ? dyn->hi : p0 + np,
                                        reinterpret_cast<unsigned long long *>(mask),
                                        dyn ? dyn->start : nullptr, dyn ? dyn->win : 0,
                                        dyn ? dyn->hi_ptr : nullptr);
    return hipGetLastError();
}

}  // namespace nas
