// mb_fit.hip -- microbenchmark of the resource-fit filter (k_fit.hip) at the
// C3 shape (10k nodes x 100k pods): the product kernel against variants with
// more pod groups per wave and a deeper request prefetch ring.  Checks every
// variant's mask against the product kernel's.
//   build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I/opt/rocm/include tools/mb_fit.hip -o tools/mb_fit
//   run:   tools/mb_fit [reps]
#include "../k_fit.hip"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

namespace nas {
namespace {

// G groups of 64 pods per wave, the requests of the next PF groups in flight
template <int G, int PF, int WAVES, bool NT = false>
__global__ void __launch_bounds__(64 * WAVES)
k_fit2(const int *cap, int N, int n0, int nloc, int n_chunks, const int *__restrict__ req, int Pp,
       int p0, int p_end, unsigned long long *__restrict__ mask) {
    const int pb0 = p0 + (int)blockIdx.x * 64 * G;
    if (pb0 >= p_end) return;
    const int lane = threadIdx.x & 63;
    const int c = (int)blockIdx.y * WAVES + (int)(threadIdx.x >> 6);
    if (c >= n_chunks) return;
    const int nl = c * 64 + lane;
    const int pend = min(p_end, pb0 + 64 * G);
    auto row = [&](int r) { return min(r, p_end - 1); };
    int ra[PF + 1], rb[PF + 1], rd[PF + 1];
#pragma unroll
    for (int g = 0; g <= PF; ++g) {
        const int q = row(pb0 + 64 * g + lane);
        ra[g] = req[q];
        rb[g] = req[Pp + q];
        rd[g] = req[2 * (size_t)Pp + q];
    }
    int fc = -1, fm = -1, fp = -1;
    if (nl < nloc) {
        int *cp = const_cast<int *>(cap) + n0 + nl;
        fc = __hip_atomic_load(cp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fm = __hip_atomic_load(cp + N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fp = __hip_atomic_load(cp + 2 * (size_t)N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool real = nl < nloc;
    const unsigned long long valid = __builtin_amdgcn_ballot_w64(real);
    int mc = real ? fc : 0x7fffffff, mm = real ? fm : 0x7fffffff, mp = real ? fp : 0x7fffffff;
    int xc = real ? fc : (int)0x80000000, xm = real ? fm : (int)0x80000000;
    int xp = real ? fp : (int)0x80000000;
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        mc = min(mc, __shfl_xor(mc, o));
        mm = min(mm, __shfl_xor(mm, o));
        mp = min(mp, __shfl_xor(mp, o));
        xc = max(xc, __shfl_xor(xc, o));
        xm = max(xm, __shfl_xor(xm, o));
        xp = max(xp, __shfl_xor(xp, o));
    }
    mc = __builtin_amdgcn_readfirstlane(mc); mm = __builtin_amdgcn_readfirstlane(mm);
    mp = __builtin_amdgcn_readfirstlane(mp); xc = __builtin_amdgcn_readfirstlane(xc);
    xm = __builtin_amdgcn_readfirstlane(xm); xp = __builtin_amdgcn_readfirstlane(xp);
    const unsigned vlo = (unsigned)valid, vhi = (unsigned)(valid >> 32);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int pb = pb0 + 64 * g;
        if (pb >= pend) break;
        const int s = g % (PF + 1);
        const int a0 = ra[s], b0 = rb[s], d0 = rd[s];
        if (g + PF + 1 < G) {  // refill the slot just consumed
            const int q = row(pb + 64 * (PF + 1) + lane);
            ra[s] = req[q];
            rb[s] = req[Pp + q];
            rd[s] = req[2 * (size_t)Pp + q];
        }
        const bool in = pb + lane < pend;
        const unsigned long long all = __builtin_amdgcn_ballot_w64(in && a0 <= mc && b0 <= mm && d0 <= mp);
        const unsigned long long none = __builtin_amdgcn_ballot_w64(in && (a0 > xc || b0 > xm || d0 > xp));
        unsigned long long rest = __builtin_amdgcn_ballot_w64(in) & ~all & ~none;
        unsigned lo = ((all >> lane) & 1) ? vlo : 0u, hi = ((all >> lane) & 1) ? vhi : 0u;
        while (rest) {
            const int i = (int)__builtin_ctzll(rest);
            rest &= rest - 1;
            const int a = __builtin_amdgcn_readlane(a0, i), b = __builtin_amdgcn_readlane(b0, i);
            const int d = __builtin_amdgcn_readlane(d0, i);
            const unsigned long long m = __builtin_amdgcn_ballot_w64(a <= fc) &
                                         __builtin_amdgcn_ballot_w64(b <= fm) &
                                         __builtin_amdgcn_ballot_w64(d <= fp);
            if (lane == i) {
                lo = (unsigned)m;
                hi = (unsigned)(m >> 32);
            }
        }
        if (in) {
            const unsigned long long word = ((unsigned long long)hi << 32) | lo;
            if constexpr (NT) __builtin_nontemporal_store(word, mask + (size_t)c * Pp + pb + lane);
            else mask[(size_t)c * Pp + pb + lane] = word;
        }
    }
}

}  // namespace
}  // namespace nas

using namespace nas;

struct Var {
    const char *name;
    int g, waves;
    const void *fn;
};

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const int N = 10000, P = 100000, Pp = 100096, Mp = 10240, n_chunks = Mp / 64;
    std::vector<int> cap(3 * N), req(3 * (size_t)Pp);
    srand(7);
    for (int n = 0; n < N; ++n) {
        const int big = rand() & 1;
        cap[n] = (big ? 8000 : 4000) - rand() % 600;
        cap[N + n] = (big ? 8 : 4) * 1048576 - rand() % 400000;
        cap[2 * N + n] = 110 - rand() % 12;
    }
    for (int p = 0; p < Pp; ++p) {
        req[p] = 1 + rand() % 540;
        req[Pp + p] = 7464 + rand() % 300000;
        req[2 * (size_t)Pp + p] = 1;
    }
    int *dcap, *dreq;
    unsigned long long *m0, *m1;
    CK(hipMalloc(&dcap, cap.size() * 4));
    CK(hipMalloc(&dreq, req.size() * 4));
    CK(hipMalloc(&m0, (size_t)n_chunks * Pp * 8));
    CK(hipMalloc(&m1, (size_t)n_chunks * Pp * 8));
    CK(hipMemcpy(dcap, cap.data(), cap.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dreq, req.data(), req.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(m0, 0, (size_t)n_chunks * Pp * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const Var vars[] = {
        {"g8pf1w4", 8, 4, (const void *)&k_fit2<8, 1, 4>},
        {"g8pf2w4", 8, 4, (const void *)&k_fit2<8, 2, 4>},
        {"g16pf2w4", 16, 4, (const void *)&k_fit2<16, 2, 4>},
        {"g16pf3w4", 16, 4, (const void *)&k_fit2<16, 3, 4>},
        {"g32pf3w4", 32, 4, (const void *)&k_fit2<32, 3, 4>},
        {"g8pf2w8", 8, 8, (const void *)&k_fit2<8, 2, 8>},
        {"g16pf1w4", 16, 4, (const void *)&k_fit2<16, 1, 4>},
        {"g16pf2w2", 16, 2, (const void *)&k_fit2<16, 2, 2>},
        {"g16pf2w1", 16, 1, (const void *)&k_fit2<16, 2, 1>},
        {"g12pf2w4", 12, 4, (const void *)&k_fit2<12, 2, 4>},
        {"g16pf2w4nt", 16, 4, (const void *)&k_fit2<16, 2, 4, true>},
        {"g8pf2w4nt", 8, 4, (const void *)&k_fit2<8, 2, 4, true>},
    };
    const double bytes = (double)P * n_chunks * 8 + 12.0 * (N + P);
    // the product kernel
    std::vector<float> t(reps);
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        CK(launch_fit(0, dcap, N, 0, N, Mp, dreq, P, Pp, 0, P, (uint64_t *)m0));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&t[r], a, b));
    }
    std::sort(t.begin(), t.end());
    printf("product   median %.2f us  min %.2f us  %.2f TB/s\n", t[reps / 2] * 1e3, t[0] * 1e3,
           bytes / (t[reps / 2] * 1e-3) / 1e12);
    std::vector<unsigned long long> h0((size_t)n_chunks * Pp), h1(h0.size());
    CK(hipMemcpy(h0.data(), m0, h0.size() * 8, hipMemcpyDeviceToHost));
    for (const Var &v : vars) {
        CK(hipMemset(m1, 0xff, (size_t)n_chunks * Pp * 8));
        dim3 grid((P + 64 * v.g - 1) / (64 * v.g), (n_chunks + v.waves - 1) / v.waves);
        int zero = 0, nn = N, nc = n_chunks, pp = Pp, pe = P;
        const int *cp = dcap, *rp = dreq;
        unsigned long long *mp = m1;
        void *args[] = {&cp, &nn, &zero, &nn, &nc, &rp, &pp, &zero, &pe, &mp};
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a));
            CK(hipLaunchKernel(v.fn, grid, dim3(64 * v.waves), args, 0, 0));
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&t[r], a, b));
        }
        std::sort(t.begin(), t.end());
        CK(hipMemcpy(h1.data(), m1, h1.size() * 8, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (int c = 0; c < n_chunks; ++c)
            for (int p = 0; p < P; ++p) bad += h0[(size_t)c * Pp + p] != h1[(size_t)c * Pp + p];
        printf("%-9s median %.2f us  min %.2f us  %.2f TB/s  mismatches %zu\n", v.name,
               t[reps / 2] * 1e3, t[0] * 1e3, bytes / (t[reps / 2] * 1e-3) / 1e12, bad);
    }
    return 0;
}
