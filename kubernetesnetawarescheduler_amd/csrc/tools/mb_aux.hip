// mb_aux.hip -- lean microbenchmark of the product k_cost_topk (int8,
// pod-group-major tile order) for build-time knobs such as COST_AUX_A/B (the
// LDS-DMA cache policy per operand).  Diagnostics only; not part of libnas.so.
// Build one binary per knob setting (tools/mb_aux.sh) and run them alternately
// on one box: prints "<tag> <variant> <ms>" per launch.
#include "k_cost_diag.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace nas;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

#ifndef MB_TAG
#define MB_TAG "default"
#endif

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 10000;
    const int P = argc > 2 ? atoi(argv[2]) : 100000;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int Mp = (int)round_up(N, 256), Kp = (int)round_up(N, 256), Pp = (int)round_up(P, 256);
    void *Lt, *WA, *mask, *partial, *pbound;
    CK(hipMalloc(&Lt, (size_t)Mp * Kp));
    CK(hipMalloc(&WA, (size_t)Pp * Kp));
    CK(hipMalloc(&mask, (size_t)(Mp / 64) * Pp * 8));
    CK(hipMalloc(&pbound, (size_t)(Mp / 256) * Pp * 8));
    CK(hipMalloc(&partial, (size_t)(Mp / 256) * Pp * 64));
    std::vector<signed char> h((size_t)Pp * Kp);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (signed char)((i * 2654435761u >> 13) % 7 - 3);
    CK(hipMemcpy(WA, h.data(), (size_t)Pp * Kp, hipMemcpyHostToDevice));
    CK(hipMemcpy(Lt, h.data(), (size_t)Mp * Kp, hipMemcpyHostToDevice));
    CK(hipMemset(mask, 0xff, (size_t)(Mp / 64) * Pp * 8));
    // bf16 operands (C3-like: latency 1..105, traffic 0..2, as bf16 values)
    void *Ltb, *WAb;
    CK(hipMalloc(&Ltb, (size_t)Mp * Kp * 2));
    CK(hipMalloc(&WAb, (size_t)Pp * Kp * 2));
    {
        std::vector<unsigned short> hb((size_t)Pp * Kp);
        auto bf = [](float f) { unsigned u; memcpy(&u, &f, 4); return (unsigned short)(u >> 16); };
        for (size_t i = 0; i < hb.size(); ++i) hb[i] = bf((float)((i * 2654435761u >> 13) % 3));
        CK(hipMemcpy(WAb, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
        for (size_t i = 0; i < (size_t)Mp * Kp; ++i) hb[i] = bf((float)(1 + (i * 2246822519u >> 11) % 105));
        CK(hipMemcpy(Ltb, hb.data(), (size_t)Mp * Kp * 2, hipMemcpyHostToDevice));
    }
    struct V { const char *name; const void *fn; int threads; bool b16; };
    const V vars[] = {{"top4", (const void *)&k_cost_topk<NAS_DT_I8, 0, 0, 0, -4, false, 4>, 512, false},
                      {"top4/w4", (const void *)&k_cost_topk<NAS_DT_I8, 0, 0, 0, -4, false, 2>, 256, false},
                      {"noepi/w4", (const void *)&k_cost_topk<NAS_DT_I8, 1, 0, 0, -4, false, 2>, 256, false},
                      {"bf16/top4", (const void *)&k_cost_topk<NAS_DT_BF16, 0, 0, 0, -4, false, 4>, 512, true},
                      {"bf16/top4/w4", (const void *)&k_cost_topk<NAS_DT_BF16, 0, 0, 0, -4, false, 2>, 256, true}};
    for (const V &v : vars)
        CK(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes<0>()));
    const int n_mt = Mp / BM, n_nt = Pp / BN;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned char *lt = (const unsigned char *)Lt, *wa = (const unsigned char *)WA;
    const unsigned char *ltb = (const unsigned char *)Ltb, *wab = (const unsigned char *)WAb;
    const int Kb2 = 2 * Kp;
    const u64 *mk = (const u64 *)mask;
    u64 *pa = (u64 *)partial, *pb = (u64 *)pbound;
    int zero = 0;
    const int *nodyn = nullptr;
    Ovf noovf{};
    FitSrc nofit{};  // (the mask path; FUSE variants are not benchmarked here)
    void *args[] = {&lt, &wa, (void *)&Kp, (void *)&n_mt, (void *)&n_nt, &zero, (void *)&Pp, &mk,
                    &pa, &pb, &zero, &nodyn, &zero, &nodyn, &noovf, &nodyn, &nofit};
    void *argsb[] = {&ltb, &wab, (void *)&Kb2, (void *)&n_mt, (void *)&n_nt, &zero, (void *)&Pp, &mk,
                     &pa, &pb, &zero, &nodyn, &zero, &nodyn, &noovf, &nodyn, &nofit};
    const char *sel = argc > 4 ? argv[4] : nullptr;  // substring filter on variant names
    for (int r = 0; r < reps; ++r)
        for (const V &v : vars) {
            if (sel && !strstr(v.name, sel)) continue;
            CK(hipEventRecord(a));
            CK(hipLaunchKernel(v.fn, dim3(n_mt * n_nt), dim3(v.threads), v.b16 ? argsb : args,
                               lds_bytes<0>(), 0));
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r > 0) printf("%s %s %.3f\n", MB_TAG, v.name, ms);
        }
    return 0;
}
