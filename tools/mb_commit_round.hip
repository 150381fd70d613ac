// mb_commit_round.hip -- microbenchmark of k_commit's round skeleton (DESIGN.md
// §7, round 5): one workgroup over a 120 KB LDS capacity image walks R rounds
// of { per pod: 3 LDS reads (the pick) ; barrier ; per pod: 3 LDS
// fetch-and-subtracts and their undo (the reservation) ; atomicMin of a "bad"
// pod ; barrier ; one LDS read (the lowest bad pod) }, with a window of 1,024
// pods spread over THREADS threads (PPT pods per thread).  It tells how much
// of a ~1.8 us commit round is the skeleton itself, and whether fewer waves
// with more pods each (cheaper barriers, more LDS work per wave) would help;
// the LISTS legs add the next window's 84 B per pod of lists (one or two
// windows ahead).  Measured (profiles/r05ar_mb_commit_round.txt): skeleton
// 0.52 us, +0.76 us with the lists at either distance -- one CU's load
// throughput (~80 KB per round), not their latency.
//   hipcc -O3 --offload-arch=gfx950 tools/mb_commit_round.hip -o tools/mb_commit_round
//   ./tools/mb_commit_round
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(2);                                                            \
        }                                                                            \
    } while (0)

constexpr int N = 10000;  // nodes: 3 x N int32 of capacity in LDS

__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// LISTS: each round also loads the lists (8 keys, a bound and 3 requests per
// pod: 84 B, as k_commit's register prefetch) of the window AHEAD rounds on
// from `lists`, and uses the ones loaded AHEAD - 1 rounds ago at its end (as
// k_commit's window switch, AHEAD = 1; AHEAD = 2 rotates two buffers)
template <int THREADS, int PPT, bool LISTS, int AHEAD = 1>
__global__ void __launch_bounds__(THREADS) k_round(int rounds, int *out, const uint4 *lists, int nwin) {
    extern __shared__ int cap[];
    __shared__ int first_bad;
    const int tid = threadIdx.x;
    for (int i = tid; i < 3 * N; i += THREADS) cap[i] = 1 << 20;
    if (tid == 0) first_bad = 0x7fffffff;
    __syncthreads();
    unsigned s = 0x9E3779B9u * (tid + 1);
    int acc = 0;
    uint4 bA[PPT][5], bB[PPT][5];
    auto issue = [&](int r, uint4(&b)[PPT][5]) {
#pragma unroll
        for (int p = 0; p < PPT; ++p)
#pragma unroll
            for (int q = 0; q < 5; ++q) b[p][q] = lists[((size_t)(r % nwin) * 1024 + p * THREADS + tid) * 5 + q];
    };
    auto use = [&](uint4(&b)[PPT][5]) {
#pragma unroll
        for (int p = 0; p < PPT; ++p)
#pragma unroll
            for (int q = 0; q < 5; ++q) acc += (int)(b[p][q].x ^ b[p][q].w);
    };
    // one round; `ld` receives the lists of round r + AHEAD, `us` holds the
    // ones of round r + 1 (loaded AHEAD - 1 rounds ago) and is used at the end
    auto round = [&](int r, uint4(&ld)[PPT][5], uint4(&us)[PPT][5]) {
        if constexpr (LISTS) issue(r + AHEAD, ld);
        int node[PPT];
        bool fit[PPT];
#pragma unroll
        for (int p = 0; p < PPT; ++p) {
            s = s * 1664525u + 1013904223u;
            node[p] = (int)(s >> 8) % N;
            const int a = cap[node[p]], b = cap[N + node[p]], c = cap[2 * N + node[p]];
            fit[p] = (a > 3) & (b > 3) & (c > 3);
        }
        bar();
        bool bad = false;
#pragma unroll
        for (int p = 0; p < PPT; ++p) {
            if (!fit[p]) continue;
            const int p0 = atomicSub(&cap[node[p]], 1);
            const int p1 = atomicSub(&cap[N + node[p]], 1);
            const int p2 = atomicSub(&cap[2 * N + node[p]], 1);
            bad |= (p0 < 1) | (p1 < 1) | (p2 < 1);
            // keep the image from draining: give the capacity back
            atomicAdd(&cap[node[p]], 1);
            atomicAdd(&cap[N + node[p]], 1);
            atomicAdd(&cap[2 * N + node[p]], 1);
        }
        if (bad) atomicMin(&first_bad, tid);
        bar();
        acc += first_bad;
        if constexpr (LISTS) use(us);
    };
    if constexpr (AHEAD == 1) {
        for (int r = 0; r < rounds; ++r) round(r, bA, bA);
    } else {
        if constexpr (LISTS) issue(1, bB);
        for (int r = 0; r + 1 < rounds; r += 2) {
            round(r, bA, bB);      // loads r + 2 into A, uses r + 1's (B)
            round(r + 1, bB, bA);  // loads r + 3 into B, uses r + 2's (A)
        }
    }
    if (tid == 0) out[0] = acc;
}

template <int THREADS, int PPT, bool LISTS = false, int AHEAD = 1>
void run(int *out, const uint4 *lists, int nwin) {
    const size_t lds = 3 * N * 4;
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_round<THREADS, PPT, LISTS, AHEAD>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int rounds = 2000;
    k_round<THREADS, PPT, LISTS, AHEAD><<<1, THREADS, lds>>>(10, out, lists, nwin);  // warm-up
    CK(hipEventRecord(a));
    k_round<THREADS, PPT, LISTS, AHEAD><<<1, THREADS, lds>>>(rounds, out, lists, nwin);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"threads\": %d, \"pods_per_thread\": %d, \"lists\": %d, \"ahead\": %d, \"us_per_round\": %.3f}\n",
                THREADS, PPT, (int)LISTS, AHEAD, ms * 1e3 / rounds);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    int *out = nullptr;
    CK(hipMalloc(&out, 4));
    // 2,000 windows of lists (172 MB: beyond L2 and most of the Infinity
    // Cache), written by a copy first
    const int nwin = 2000;
    uint4 *lists = nullptr;
    CK(hipMalloc(&lists, (size_t)nwin * 1024 * 5 * 16));
    CK(hipMemset(lists, 1, (size_t)nwin * 1024 * 5 * 16));
    run<1024, 1>(out, lists, nwin);
    run<512, 2>(out, lists, nwin);
    run<256, 4>(out, lists, nwin);
    run<1024, 2>(out, lists, nwin);
    run<1024, 1, true>(out, lists, nwin);
    run<512, 2, true>(out, lists, nwin);
    run<1024, 1, true, 2>(out, lists, nwin);
    run<512, 2, true, 2>(out, lists, nwin);
    CK(hipFree(lists));
    CK(hipDeviceSynchronize());
    CK(hipFree(out));
    return 0;
}
