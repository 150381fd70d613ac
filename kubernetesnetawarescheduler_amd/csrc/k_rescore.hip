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
//   2. k_compact: one workgroup prefix-sums the word popcounts and writes the
//      first R flagged pods in pod order (s is always among them: it halted
//      for exactly this reason).
//   3. k_gather_pods: their traffic rows and requests are copied into a
//      contiguous scratch "view" that the ordinary fit / cost / merge
//      kernels (and the RCCL exchange) score like any pod range.
//   4. k_merge's store puts the fresh lists back into the pods' list slots.
// Lists computed against the capacity now stay valid for every later turn of
// these pods (capacity only shrinks), so the walk resumes from s unchanged.
#include "klist.h"

#include <algorithm>

namespace nas {
namespace {

constexpr int STALE_THREADS = 256;
constexpr int COMPACT_THREADS = 1024;
// a pod is flagged when fewer than this many of its usable candidates still
// fit: the dry ones (0) and those one commit away from running dry, whose
// lists a herd of neighbours is about to drain
#ifndef STALE_MIN_FIT
#define STALE_MIN_FIT 2
#endif

__global__ void __launch_bounds__(STALE_THREADS)
k_stale(const u64 *__restrict__ key, const u64 *__restrict__ bound, const int *__restrict__ req,
        int Pp, const int *__restrict__ cap, int N, int p0, int P, u64 *__restrict__ words,
        const int *__restrict__ p0_dev) {
    const int t = blockIdx.x * STALE_THREADS + threadIdx.x;
    const int p = p0 + t;
    // device-side slot: pods from the halt word on; nothing halted -> k_compact
    // publishes an empty view without reading the words
    const int first = p0_dev ? *p0_dev : p0;
    if (first < 0) return;
    bool dry = false;
    if (p < P && first >= 0 && p >= first) {
        const u64 b = bound[p];
        if (b != KEY_INVALID) {
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
            dry = fits < STALE_MIN_FIT;
        }
    }
    const u64 m = __ballot(dry);
    if ((threadIdx.x & 63) == 0) words[t >> 6] = m;
}

__global__ void __launch_bounds__(COMPACT_THREADS)
k_compact(const u64 *__restrict__ words, int n_words, int p0, int R, int *__restrict__ idx,
          int *__restrict__ ctl, const int *__restrict__ p0_dev) {
    __shared__ int part[COMPACT_THREADS];
    const int tid = threadIdx.x;
    if (p0_dev && *p0_dev < 0) {  // the walk did not halt: empty view
        if (tid == 0) {
            ctl[0] = -1;
            ctl[1] = 0;
        }
        return;
    }
    const int per = (n_words + COMPACT_THREADS - 1) / COMPACT_THREADS;
    const int w0 = min(n_words, tid * per), w1 = min(n_words, w0 + per);
    int c = 0;
    for (int w = w0; w < w1; ++w) c += __popcll(words[w]);
    part[tid] = c;
    __syncthreads();
    // inclusive Hillis-Steele scan over the per-thread counts
    for (int d = 1; d < COMPACT_THREADS; d <<= 1) {
        const int v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int off = part[tid] - c;
    if (tid == COMPACT_THREADS - 1) {
        const int n = min(part[tid], R);
        ctl[0] = n > 0 ? 0 : -1;  // the view's window start, read like a halt word
        ctl[1] = n;
        ctl[2] += n;              // running total, reported in nas_timings
    }
    for (int w = w0; w < w1 && off < R; ++w) {
        u64 m = words[w];
        while (m && off < R) {
            const int b = __ffsll((long long)m) - 1;
            idx[off++] = p0 + w * 64 + b;
            m &= m - 1;
        }
    }
}

// view rows i < count (grid-stride, a workgroup per row): pod idx[i]'s
// traffic row and requests
__global__ void __launch_bounds__(256)
k_gather_pods(const int *__restrict__ idx, const int *__restrict__ count, const uint4 *__restrict__ WA,
              int row_vec, const int *__restrict__ req, int Pp, int Rv, uint4 *__restrict__ WA_v,
              int *__restrict__ req_v) {
    const int n = *count;  // rows past count are scored as garbage and never scattered
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int p = idx[i];
        const uint4 *src = WA + (size_t)p * row_vec;
        uint4 *dst = WA_v + (size_t)i * row_vec;
        for (int v = threadIdx.x; v < row_vec; v += 256) dst[v] = src[v];
        if (threadIdx.x < 3) req_v[threadIdx.x * Rv + i] = req[threadIdx.x * Pp + p];
    }
}


}  // namespace

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
                                              p0, P, w, p0_dev);
    k_compact<<<1, COMPACT_THREADS, 0, st>>>(w, blocks * (STALE_THREADS / 64), p0, R, idx, ctl,
                                             p0_dev);
    return hipGetLastError();
}

hipError_t launch_gather_pods(hipStream_t st, const int32_t *idx, const int32_t *count,
                              const void *WA, size_t row_bytes, const int32_t *req, int Pp, int Rv,
                              void *WA_v, int32_t *req_v) {
    if (row_bytes % 16) return hipErrorInvalidValue;
    k_gather_pods<<<std::min(Rv, 512), 256, 0, st>>>(idx, count, static_cast<const uint4 *>(WA),
                                      (int)(row_bytes / 16), req, Pp, Rv,
                                      static_cast<uint4 *>(WA_v), req_v);
    return hipGetLastError();
}


}  // namespace nas
