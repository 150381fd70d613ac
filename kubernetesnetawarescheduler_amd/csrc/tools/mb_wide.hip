// mb_wide.hip -- diagnostic microbenchmark (not part of libnas.so): the
// k_cost_topk main loop (int8 MFMA 32x32x32, LDS-DMA double buffer, source
// swizzle, pod-group-major XCD order) with the pod tile widened from 256 to
// 64 x NWP pods at the same per-wave shape (128 nodes x 64 pods, 4 x 2 MFMA
// tiles): NWP = 4 is the product's 256 x 256 / 8-wave workgroup; NWP = 6 is a
// 256 x 384 / 12-wave workgroup (3 waves per SIMD, 160 KiB of LDS), which
// stages 17% fewer bytes per MAC.  No epilogue: the accumulators are sunk.
// usage: mb_wide [N] [P] [reps]  -> "<variant> <ms> <TOPS>" per launch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
constexpr int BM = 256, BKB = 128;

template <int NI>
__device__ __forceinline__ void rd(const unsigned char *As, const unsigned char *Bs, int kk, int fh,
                                   int fr, int wm, int wn, v4i *ra, v4i *rb) {
    const int c = kk * 2 + fh;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
        const int rw = wm * 128 + mi * 32 + fr;
        ra[mi] = *reinterpret_cast<const v4i *>(As + rw * BKB + ((c ^ ((rw >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
        const int rw = wn * 32 * NI + ni * 32 + fr;
        rb[ni] = *reinterpret_cast<const v4i *>(Bs + rw * BKB + ((c ^ ((rw >> 1) & 7)) << 4));
    }
}

template <int NWP, bool DB, int NI>
__global__ void __launch_bounds__(128 * NWP, 1)
k_wide(const unsigned char *__restrict__ Lt, const unsigned char *__restrict__ WA, int Kb,
       int n_mt, int n_nt) {
    constexpr int NW = 2 * NWP, BN = 32 * NI * NWP;
    constexpr int STAGE = (BM + BN) * BKB, PIECES = (BM + BN) / 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int nwg = n_mt * n_nt, b = blockIdx.x;
    const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    constexpr int PG = 4;
    const int gsize = PG * n_mt, g = v / gsize, r = v % gsize;
    const int first_nt = g * PG, pg = min(n_nt - first_nt, PG);
    const int mt = r / pg, nt = first_nt + r % pg;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w / NWP, wn = w % NWP;
    const unsigned char *Ag = Lt + (size_t)mt * BM * Kb;
    const unsigned char *Bg = WA + (size_t)nt * BN * Kb;
    const int srow_in = lane >> 3, sq = lane & 7;
    // piece j (8 rows x 128 B): rows 0..BM-1 are A, BM.. are B
    auto stage = [&](int buf, int k0) {
        for (int j = w; j < PIECES; j += NW) {
            const int r0 = j * 8, row = r0 + srow_in;
            const bool isA = row < BM;
            const int rr = isA ? row : row - BM;
            const int c = sq ^ ((rr >> 1) & 7);
            const unsigned char *src = (isA ? Ag : Bg) + (size_t)rr * Kb + k0 + c * 16;
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)src,
                                             (void __attribute__((address_space(3))) *)(lds + buf * STAGE + r0 * BKB),
                                             16, 0, 0);
        }
    };
    v16i acc[4][4];  // (only [..NI) used: a dependent bound here loses the host stubs, hipcc 7.2)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = v16i{};
    const int fr = lane & 31, fh = lane >> 5;
    auto compute = [&](int buf) {
        const unsigned char *As = lds + buf * STAGE;
        const unsigned char *Bs = As + BM * BKB;
        auto read = [&](int kk, v4i *ra, v4i *rb) {
            rd<NI>(As, Bs, kk, fh, fr, wm, wn, ra, rb);
        };
        if constexpr (DB) {
            v4i a[2][4], bb[2][NI];
            read(0, a[0], bb[0]);
#pragma unroll
            for (int kk = 0; kk < BKB / 32; ++kk) {
                if (kk + 1 < BKB / 32) read(kk + 1, a[(kk + 1) & 1], bb[(kk + 1) & 1]);
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < NI; ++ni)
                        acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kk & 1][mi], bb[kk & 1][ni],
                                                                            acc[mi][ni], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < BKB / 32; ++kk) {
                v4i a[4], bb[NI];
                read(kk, a, bb);
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < NI; ++ni)
                        acc[mi][ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[mi], bb[ni], acc[mi][ni], 0, 0, 0);
            }
        }
    };
    const int nk = Kb / BKB;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        if (t + 1 < nk) stage(cur ^ 1, (t + 1) * BKB);
        compute(cur);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) asm volatile("" ::"v"(acc[mi][ni]));
}

template <int NWP, bool DB, int NI>
void run(const char *name, const unsigned char *Lt, const unsigned char *WA, int Kp, int Mp, int P,
         int reps) {
    constexpr int BN = 32 * NI * NWP;
    const int Pp = (P + BN - 1) / BN * BN;
    const int n_mt = Mp / BM, n_nt = Pp / BN;
    const int lds = 2 * (BM + BN) * BKB;
    CK(hipFuncSetAttribute((const void *)&k_wide<NWP, DB, NI>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int r = 0; r <= reps; ++r) {
        CK(hipEventRecord(a));
        k_wide<NWP, DB, NI><<<n_mt * n_nt, 128 * NWP, lds>>>(Lt, WA, Kp, n_mt, n_nt);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r > 0) printf("%s %.3f %.1f\n", name, ms, 2.0 * Mp * (double)Pp * Kp / (ms * 1e-3) / 1e12);
    }
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 10000;
    const int P = argc > 2 ? atoi(argv[2]) : 100000;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int Mp = (N + 255) / 256 * 256, Kp = Mp, Pmax = (P + 383) / 384 * 384;
    void *Lt, *WA;
    CK(hipMalloc(&Lt, (size_t)Mp * Kp));
    CK(hipMalloc(&WA, (size_t)Pmax * Kp));
    std::vector<signed char> h((size_t)Pmax * Kp);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (signed char)((i * 2654435761u >> 13) % 7 - 3);
    CK(hipMemcpy(WA, h.data(), (size_t)Pmax * Kp, hipMemcpyHostToDevice));
    CK(hipMemcpy(Lt, h.data(), (size_t)Mp * Kp, hipMemcpyHostToDevice));
    const auto *lt = (const unsigned char *)Lt, *wa = (const unsigned char *)WA;
    for (int i = 0; i < 2; ++i) {
        run<4, true, 2>("w256x256/8w/db", lt, wa, Kp, Mp, P, reps);
        run<6, false, 2>("w256x384/12w/sb", lt, wa, Kp, Mp, P, reps);
        run<6, true, 2>("w256x384/12w/db", lt, wa, Kp, Mp, P, reps);
        run<4, false, 2>("w256x256/8w/sb", lt, wa, Kp, Mp, P, reps);
        run<4, false, 3>("w256x384/8w128x96/sb", lt, wa, Kp, Mp, P, reps);
        run<4, true, 3>("w256x384/8w128x96/db", lt, wa, Kp, Mp, P, reps);
        run<2, false, 4>("w256x256/4w128x128/sb", lt, wa, Kp, Mp, P, reps);
    }
    return 0;
}
