// k_cost_pc.hip -- DIAGNOSTIC (included by tools/mb_aux.hip, never built into
// libnas.so): k_cost_topk's main loop with the LDS-DMA staging moved to
// dedicated loader waves.  12 waves per workgroup (3 per SIMD): waves 0-7
// compute the 256 x 256 tile exactly as k_cost_topk (2 x 4 waves of 128 x 64,
// fragments from the swizzled LDS image), waves 8-11 only issue the next
// stage's 64 LDS-DMA pieces (16 each) and wait for them.  One barrier per
// K-step for all 12 waves.  Tests whether the staging stops adding to the
// in-core loop once no MFMA-issuing wave issues DMA.
namespace nas {
namespace {

constexpr int PC_THREADS = 768;

template <int EPI>
__global__ void __launch_bounds__(PC_THREADS, 1)
k_cost_pc(const unsigned char *__restrict__ Lt, const unsigned char *__restrict__ WA, int Kb,
          int n_mt, int n_nt, int p0, int Pp, const u64 *__restrict__ mask,
          u64 *__restrict__ partial, u64 *__restrict__ pbound, int node_base,
          const int *__restrict__ dyn_start, int dyn_hi, const int *__restrict__ dyn_hi_ptr,
          Ovf ov, const int *__restrict__ rowmap) {
    using M = Mma<NAS_DT_I8>;
    using acc_t = typename M::acc_t;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int nwg = n_mt * n_nt;
    const int b = blockIdx.x;
    const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    constexpr int PG = 4;  // pod-group-major, as k_cost_topk's default
    const int gsize = PG * n_mt;
    const int g = v / gsize, r = v % gsize;
    const int first_nt = g * PG;
    const int pg = min(n_nt - first_nt, PG);
    const int mt = r / pg, nt = first_nt + r % pg;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const unsigned char *Ag = Lt + (size_t)mt * BM * Kb;
    const unsigned char *Bg = WA + (size_t)(p0 + nt * BN) * Kb;
    const int nk = Kb / BKB;
    auto abuf = [&](int bf) -> unsigned char * { return lds + bf * STAGE_BYTES; };
    auto bbuf = [&](int bf) -> unsigned char * { return lds + bf * STAGE_BYTES + TILE_BYTES; };

    if (w >= 8) {
        // loader wave lw: pieces p = lw + 4 j (j < 8) of A and of B; piece p
        // fills rows 8p .. 8p+7 (lane l: row 8p + l/8, 16-byte chunk l%8,
        // source-side swizzle chunk ^= (row >> 1) & 7, as k_cost_topk)
        const int lw = w - 8;
        const int srow_in = lane >> 3, sq = lane & 7;
        auto stage = [&](int bf, int k0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int r0 = (lw + 4 * j) * 8, row = r0 + srow_in;
                const int c = sq ^ ((row >> 1) & 7);
                glds16(Ag + (size_t)row * Kb + k0 + c * 16, abuf(bf) + r0 * BKB);
                glds16(Bg + (size_t)row * Kb + k0 + c * 16, bbuf(bf) + r0 * BKB);
            }
        };
        stage(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int t = 0; t < nk; ++t) {
            if (t + 1 < nk) stage((t + 1) & 1, (t + 1) * BKB);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        return;
    }

    const int wm = w >> 2, wn = w & 3;
    const int fr = lane & 31, fh = lane >> 5;
    acc_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = acc_t{};
    auto compute = [&](int bf) {
        const unsigned char *As = abuf(bf);
        const unsigned char *Bs = bbuf(bf);
        v4i a[2][4], bb[2][2];
        auto read = [&](int kk, v4i (&ra)[4], v4i (&rb)[2]) {
            const int c = kk * 2 + fh;
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int rr = wm * 128 + mi * 32 + fr;
                ra[mi] = *reinterpret_cast<const v4i *>(As + rr * BKB + ((c ^ ((rr >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int rr = wn * 64 + ni * 32 + fr;
                rb[ni] = *reinterpret_cast<const v4i *>(Bs + rr * BKB + ((c ^ ((rr >> 1) & 7)) << 4));
            }
        };
        read(0, a[0], bb[0]);
#pragma unroll
        for (int kk = 0; kk < BKB / 32; ++kk) {
            if (kk + 1 < BKB / 32) read(kk + 1, a[(kk + 1) & 1], bb[(kk + 1) & 1]);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
                    acc[mi][ni] = M::mma(a[kk & 1][mi], bb[kk & 1][ni], acc[mi][ni]);
        }
    };
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
        compute(t & 1);
        __syncthreads();
    }
    // checksum of the tile (keeps the accumulators live; EPI 1 = nothing stored)
    int s = 0;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int k = 0; k < 16; ++k) s += acc[mi][ni][k] * (k + 1);
    if (EPI == 0 || s == 0x7fffffff) pbound[(size_t)mt * Pp + p0 + nt * BN + (w * 64 + lane) % BN] = (u64)s;
}

}  // namespace
}  // namespace nas
