// mb_cost.hip -- microbenchmark of the cost contraction kernel variants
// (diagnostics only; not part of libnas.so).  Times each variant with HIP
// events over back-to-back launches on random operands, interleaved.
#define NAS_DIAG_VARIANTS
#include "../k_cost.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace nas;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 10000;
    const int P = argc > 2 ? atoi(argv[2]) : 100000;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int Mp = (int)round_up(N, 256), Kp = (int)round_up(N, 128), Pp = (int)round_up(P, 256);
    void *Lt, *WA, *mask, *partial, *pbound;
    CK(hipMalloc(&Lt, (size_t)Mp * Kp));
    CK(hipMalloc(&WA, (size_t)Pp * Kp));
    CK(hipMalloc(&mask, (size_t)(Mp / 64) * Pp * 8));
    CK(hipMalloc(&pbound, (size_t)(Mp / 256) * Pp * 8));
    CK(hipMalloc(&partial, (size_t)(Mp / 256) * Pp * 64 + (size_t)(Mp / 256) * (Pp / 256) * 512 * 4));
    std::vector<signed char> h((size_t)Pp * Kp);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (signed char)((i * 2654435761u >> 13) % 7 - 3);
    CK(hipMemcpy(WA, h.data(), (size_t)Pp * Kp, hipMemcpyHostToDevice));
    CK(hipMemcpy(Lt, h.data(), (size_t)Mp * Kp, hipMemcpyHostToDevice));
    CK(hipMemset(mask, 0xff, (size_t)(Mp / 64) * Pp * 8));
    CK(hipFuncSetAttribute((const void *)&k_cost_topk<NAS_DT_I8, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    CK(hipFuncSetAttribute((const void *)&k_cost_topk<NAS_DT_I8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    CK(hipFuncSetAttribute((const void *)&k_cost_topk<NAS_DT_I8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    const int n_mt = Mp / BM, n_nt = Pp / BN;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double ops = 2.0 * N * (double)N * P;
    for (int r = 0; r < reps; ++r) {
        for (int v = 0; v < 3; ++v) {
            CK(hipEventRecord(a));
#define L(E) k_cost_topk<NAS_DT_I8, E><<<n_mt * n_nt, THREADS, LDS_BYTES>>>( \
                    (const unsigned char *)Lt, (const unsigned char *)WA, Kp, n_mt, n_nt, 0, Pp, \
                    (const u64 *)mask, (u64 *)partial, (u64 *)pbound, 0)
            if (v == 0) L(0); else if (v == 1) L(1); else L(2);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("rep %d %-10s %8.3f ms %8.1f TOPS\n", r, v == 0 ? "top4" : v == 1 ? "no-epi" : "top1", ms, ops / ms / 1e9);
        }
    }
    return 0;
}
