// mb_cost.hip -- microbenchmark of the cost contraction kernel variants
// (diagnostics only; not part of libnas.so).  Times each variant with HIP
// events over back-to-back launches on random operands, interleaved.
#define NAS_DIAG_VARIANTS
#include "k_cost_diag.hip"
#include "k_cost_experiments.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace nas;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 10000;
    const int P = argc > 2 ? atoi(argv[2]) : 100000;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const char *vsel = argc > 4 ? argv[4] : "abcdefgh";  // variants to run (a..)
    const int Mp = (int)round_up(N, 256), Kp = (int)round_up(N, 256), Pp = (int)round_up(P, 768);
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
    // variants: name, kernel
    struct V { const char *name; const void *fn; int lds; int threads = THREADS; };
#define KV(E, S, PP, G) (const void *)&k_cost_topk<NAS_DT_I8, E, S, PP, G>, lds_bytes<PP>()
    const V vars[] = {{"top4/jit", KV(0, 0, 0, 4)},   {"noepi/jit", KV(1, 0, 0, 4)},
                      {"top4/spread", KV(0, 5, 0, 4)}, {"noepi/spread", KV(1, 5, 0, 4)},
                      {"l2hot/spread", KV(3, 5, 0, 4)}, {"top4/pin", KV(0, 1, 0, 4)},
                      {"top4/spr/g8", KV(0, 5, 0, 8)}, {"ldsonly+bar", KV(4, 0, 0, 4)},
                      {"top4/pin/regB", KV(0, 1, 2, 4)}, {"top4/pin/regAB", KV(0, 1, 3, 4)},
                      {"top4/jit/regB", KV(0, 0, 2, 4)}, {"top4/jit/regAB", KV(0, 0, 3, 4)},
                      {"noepi/pin/regB", KV(1, 1, 2, 4)}, {"noepi/pin/regAB", KV(1, 1, 3, 4)},
                      {"top4/phased", KV(0, 0, 4, 4)}, {"noepi/phased", KV(1, 0, 4, 4)},
                      {"top4/phased/g8", KV(0, 0, 4, 8)}, {"top4/phased/g2", KV(0, 0, 4, 2)},
                      {"top4/touch2", KV(0, 0, 5, 4)}, {"top4/touch3", KV(0, 0, 6, 4)},
                      {"top4/touchB2", KV(0, 0, 7, 4)}, {"noepi/touch2", KV(1, 0, 5, 4)},
                      {"top4sel/jit", KV(6, 0, 0, 4)},
#define KV2(E, S, G) (const void *)&k_cost_topk2<NAS_DT_I8, E, S, G>, (S) * TILE_BYTES
                      {"v2/top4/st4", KV2(0, 4, 4)}, {"v2/noepi/st4", KV2(1, 4, 4)},
                      {"v2/l2hot", KV2(3, 4, 4)}, {"v2/ldsonly", KV2(4, 4, 4)},
                      {"v2/top4/st3", KV2(0, 3, 4)}, {"v2/top4/g8", KV2(0, 4, 8)},
                      {"v2/noepi/st3", KV2(1, 3, 4)},
#define KV3(E, S, G) (const void *)&k_cost_topk3<NAS_DT_I8, E, S, G>, (S) * TILE_BYTES
                      {"v3/top4", KV3(0, 4, 4)}, {"v3/noepi", KV3(1, 4, 4)},
                      {"v3/l2hot", KV3(3, 4, 4)}, {"v3/ldsonly", KV3(4, 4, 4)},
                      {"v3/top4/g8", KV3(0, 4, 8)},
                      {"top4/podg2", KV(0, 0, 0, -2)}, {"top4/podg4", KV(0, 0, 0, -4)},
                      {"top4/podg8", KV(0, 0, 0, -8)}, {"top4/g8", KV(0, 0, 0, 8)},
                      {"top4/g2", KV(0, 0, 0, 2)}, {"top4/g16", KV(0, 0, 0, 16)},
#define KV2T(E, S, G) (const void *)&k_cost_topk2<NAS_DT_I8, E, S, G, true>, (S) * TILE_BYTES
#define KV3T(E, S, G) (const void *)&k_cost_topk3<NAS_DT_I8, E, S, G, true>, (S) * TILE_BYTES
                      {"v2T/top4/st4", KV2T(0, 4, 4)}, {"v2T/noepi/st4", KV2T(1, 4, 4)},
                      {"v2T/top4/st3", KV2T(0, 3, 4)}, {"v3T/top4", KV3T(0, 4, 4)},
                      {"v3T/noepi", KV3T(1, 4, 4)},
#define KVW(E, NI) (const void *)&k_cost_wide<NAS_DT_I8, E, false, NI>, 2 * (BM + 128 * NI) * BKB
                      {"wide2/top4", KVW(0, 2)}, {"wide2/noepi", KVW(1, 2)},
                      {"wide3/top4", KVW(0, 3)}, {"wide3/noepi", KVW(1, 3)}};
    const int nv = sizeof(vars) / sizeof(vars[0]);
    for (int v = 0; v < nv; ++v)
        CK(hipFuncSetAttribute(vars[v].fn, hipFuncAttributeMaxDynamicSharedMemorySize, vars[v].lds));
    const int n_mt = Mp / BM, n_nt = Pp / BN;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double ops = 2.0 * N * (double)N * P;
    const unsigned char *lt = (const unsigned char *)Lt, *wa = (const unsigned char *)WA;
    const u64 *mk = (const u64 *)mask;
    u64 *pa = (u64 *)partial, *pb = (u64 *)pbound;
    int zero = 0;
    const int *nodyn = nullptr;
    Ovf noovf{};
    FitSrc nofit{};  // (the mask path; FUSE variants are not benchmarked here)
    for (int r = 0; r < reps; ++r) {
        for (int v = 0; v < nv; ++v) {
            if (!strchr(vsel, v < 26 ? 'a' + v : 'A' + v - 26)) continue;
            // k_cost_topk's trailing row map (none); the experiment kernels
            // take one argument fewer and ignore it
            void *args[] = {&lt, &wa, (void *)&Kp, (void *)&n_mt, (void *)&n_nt, &zero,
                            (void *)&Pp, &mk, &pa, &pb, &zero, &nodyn, &zero, &nodyn, &noovf,
                            &nodyn, &nofit};
            CK(hipEventRecord(a));
            const int thr = strncmp(vars[v].name, "v3", 2) ? THREADS : THREADS3;  // v3 and v3T
            // wide3: 384-pod tiles (Pp rounded to 768 below, so both divide)
            const int nnt = strncmp(vars[v].name, "wide3", 5) ? n_nt : Pp / 384;
            void *argw[] = {&lt, &wa, (void *)&Kp, (void *)&n_mt, (void *)&nnt, &zero,
                            (void *)&Pp, &mk, &pa, &pb, &zero, &nodyn, &zero, &nodyn, &noovf,
                            &nodyn, &nofit};
            CK(hipLaunchKernel(vars[v].fn, dim3(n_mt * nnt), dim3(thr), strncmp(vars[v].name, "wide3", 5) ? args : argw, vars[v].lds, 0));
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("rep %d %-12s %8.3f ms %8.1f TOPS\n", r, vars[v].name, ms, ops / ms / 1e9);
        }
    }
    return 0;
}
