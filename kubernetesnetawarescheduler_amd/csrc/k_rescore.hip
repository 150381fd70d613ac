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
// fit: the dry ones (0) and those one commit away from running dry, whose
// lists a herd of neighbours is about to drain
constexpr int STALE_MIN_FIT = 2;

// One launch: every block flags its pods (ballot words), and the LAST block
// to finish (ticket counter ctl[3], zeroed at the start of every pass and
// reset by that block) prefix-sums the words' popcounts and writes the first R
// flagged pods in pod order -- the stale scan and the compaction without a
// second launch on the slot's critical path.  Publication: each block's
// words are stored, drained (vmcnt(0)), released at agent scope by thread 0,
// then the ticket is drawn; the last block acquires before reading
// (cdna_hip_programming.md, the split-K counter recipe).
__global__ void __launch_bounds__(STALE_THREADS)
k_stale(const u64 *__restrict__ key, const u64 *__restrict__ bound, const int *__restrict__ req,
        int Pp, const int *__restrict__ cap, int N, int p0, int P, u64 *__restrict__ words,
        int n_words, int R, int *__restrict__ idx, int *__restrict__ ctl,
        const int *__restrict__ p0_dev) {
    __shared__ int part[STALE_THREADS];
    __shared__ int last;
    const int tid = threadIdx.x;
    const int t = blockIdx.x * STALE_THREADS + tid;
    const int p = p0 + t;
    // device-side slot: pods from the halt word on; nothing halted -> an
    // empty view, published by block 0 alone
    const int first = p0_dev ? *p0_dev : p0;
    if (first < 0) {
        if (blockIdx.x == 0 && tid == 0) {
            ctl[0] = -1;
            ctl[1] = 0;
        }
        return;
    }
    bool dry = false;
    if (p < P && p >= first) {
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
    if ((tid & 63) == 0) words[t >> 6] = m;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int ticket = __hip_atomic_fetch_add(ctl + 3, 1, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        last = ticket == (int)gridDim.x - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last) return;
    // ---- compaction by the last block
    const int per = (n_words + STALE_THREADS - 1) / STALE_THREADS;
    const int w0 = min(n_words, tid * per), w1 = min(n_words, w0 + per);
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
                                              p0, P, w, blocks * (STALE_THREADS / 64), R, idx, ctl,
                                              p0_dev);
    return hipGetLastError();
}


}  // namespace nas
