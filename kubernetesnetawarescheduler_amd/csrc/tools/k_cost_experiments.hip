// k_cost_experiments.hip -- DIAGNOSTIC ONLY (included by tools/mb_cost.hip,
// never built into libnas.so): two alternative tilings of the cost
// contraction measured against k_cost_topk in round 2 and kept for the
// record ("Measured alternatives").
//   k_cost_topk2  8 waves, each all 256 nodes x 32 pods; Lt via LDS-DMA, WA
//                 rows straight into registers.
//   k_cost_topk3  4 waves (one per SIMD, 256 AGPR accumulators), each all 256
//                 nodes x 64 pods; the K-step hand-scheduled in inline asm
//                 (MFMA pairs interleaved with the next substep's
//                 ds_read_b128), WA rows by inline-asm loads retired by
//                 explicit vmcnt waits.
// Both keep the MFMA pipe ~87% busy on LDS-resident operands (PMC), but lose
// to k_cost_topk once WA is streamed from L2/HBM into registers.
namespace nas {
namespace {

// 16-byte global load the compiler's waitcnt pass does not track (the caller
// retires it with an explicit s_waitcnt vmcnt tied to the destination)
__device__ __forceinline__ v4i gld16(const unsigned char *p) {
    v4i r;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}

// ---------------------------------------------------------------------------
// k_cost_topk2: the same 256-node x 256-pod workgroup tile with the roles of
// the operands split by where they are shared.
//   * Lt (nodes) is shared by every wave: staged once per workgroup into an
//     LDS ring of NST 32-KiB stages by LDS-DMA (4 pieces per wave per K-step,
//     half of k_cost_topk's), DMA'd NST-1 K-steps ahead.
//   * WA (pods) is private: wave w owns pods 32w .. 32w+31 of the tile and
//     streams its rows straight into registers (global_load_dwordx4, 64
//     contiguous bytes per lane per K-step), two K-steps ahead -- no LDS
//     round trip and no LDS-DMA issue cost for the 1-GB operand.
// A K-step's 128 bytes are split by lane half h: half h contracts bytes
// [64h, 64h + 64), 16 per k-substep (the contraction order is free; A's
// fragment reads use the same permutation).  Each wave computes all 256
// nodes x its 32 pods = 8 MFMA tiles: 8 ds_read_b128 + 8 MFMAs per k-substep.
// A lane ends with 128 (node, cost) values of ONE pod, so the top-k needs no
// cross-wave merge: per-lane top-4, one lane^32 exchange, 72 B per pod.
// ---------------------------------------------------------------------------
template <int DT, int EPI = 0, int NST = 4, int GM = COST_GM, bool TB = false>
__global__ void __launch_bounds__(THREADS, 1)
k_cost_topk2(const unsigned char *__restrict__ Lt, const unsigned char *__restrict__ WA, int Kb,
             int n_mt, int n_nt, int p0, int Pp, const u64 *__restrict__ mask,
             u64 *__restrict__ partial, u64 *__restrict__ pbound, int node_base,
             const int *__restrict__ dyn_start, int dyn_hi, const int *__restrict__ dyn_hi_ptr,
             Ovf ov) {
    using M = Mma<DT>;
    using acc_t = typename M::acc_t;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    // ---- XCD-aware tile order (speed only), as k_cost_topk
    const int nwg = n_mt * n_nt;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int gsize = GM * n_nt;
    const int g = v / gsize;
    const int first_mt = g * GM;
    const int gm = min(n_mt - first_mt, GM);
    const int mt = first_mt + (v % gsize) % gm;
    const int nt = (v % gsize) / gm;
    const int cb = blockIdx.y;
    Lt += (size_t)cb * n_mt * BM * Kb;
    WA += (size_t)cb * Pp * Kb;
    mask += (size_t)cb * (n_mt * BM / 64) * Pp;
    partial += (size_t)cb * n_mt * Pp * KC;
    pbound += (size_t)cb * n_mt * Pp;
    if (dyn_start) {
        const int s0 = dyn_start[cb * STATUS_INTS];
        if (s0 < 0) return;
        if (dyn_hi_ptr) dyn_hi = dyn_hi_ptr[cb * STATUS_INTS];
        p0 = s0 / BN * BN;
        if (p0 + nt * BN >= dyn_hi) return;  // whole block: before any barrier
    }

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 31, fh = lane >> 5;
    const int pod_row = p0 + nt * BN + w * 32 + fr;  // this lane's pod (row of WA)
    const unsigned char *Ag = Lt + (size_t)mt * BM * Kb;
    const unsigned char *Bl = WA + (size_t)pod_row * Kb + 64 * fh;
    if constexpr (EPI == 3) {  // diagnostic: every block streams tile (0, 0)
        Ag = Lt;
        Bl = WA + (size_t)(w * 32 + fr) * Kb + 64 * fh;
    }

    // LDS-DMA piece j of wave w: rows (8j + w)*8 .. +8 of the stage, whole
    // 128-B lines, chunk swizzle chunk ^= (row >> 1) & 7 on the SOURCE side
    const int srow_in = lane >> 3, sq = lane & 7;
    auto stageA = [&](int buf, int k0) {
        unsigned char *base = lds + buf * TILE_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r0 = (j * 8 + w) * 8;
            const int row = r0 + srow_in;
            const int c = sq ^ ((row >> 1) & 7);
            glds16(Ag + (size_t)row * Kb + k0 + c * 16, base + r0 * BKB);
        }
    };
    // TB: WA pre-tiled in MFMA fragment order -- [pod group of 32][K-step]
    // [substep][64 lanes x 16 B] -- so each load is one contiguous 1 KiB
    // (8 full lines) instead of 32 rows x 32 B (timing only: same bytes)
    const unsigned char *Bt = WA + (size_t)(pod_row >> 5) * 32 * Kb + lane * 16;
    auto loadB = [&](v4i (&b)[4], int k0) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if constexpr (TB) b[s] = *reinterpret_cast<const v4i *>(Bt + k0 * 32 + 1024 * s);
            else b[s] = *reinterpret_cast<const v4i *>(Bl + k0 + 16 * s);
        }
    };

    // the epilogue's fit-mask words (4 per pod: nodes 64c .. 64c+63 of the tile)
    u64 mw[4];
    if constexpr (EPI == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) mw[c] = mask[(size_t)(mt * 4 + c) * Pp + pod_row];
    }
    acc_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = acc_t{};
    // ---- exact int32 traffic: the pod's entries outside the int8 plane,
    // e * L[m][n] over the tile's nodes, are the accumulators' initial value
    // (added before the K loop, while its operand registers are still free)
    if constexpr (DT == NAS_DT_I8 && EPI == 0) {
        if (ov.ptr) {
            const int r = pod_row;
            int beg = 0, end = 0;
            if (r < (ov.row_count ? *ov.row_count : 0x7fffffff)) {
                const int pod = (ov.row_pod ? ov.row_pod[r] : r) + cb * Pp;
                beg = ov.ptr[pod];
                end = ov.ptr[pod + 1];
            }
            const signed char *lr =
                ov.Lr + (size_t)cb * ov.N * (n_mt * BM) + mt * BM + 4 * fh;
            // node tile outermost: one tile's 16 accumulators live in the
            // entry loop at a time (the whole row at once spills)
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
                for (int j = beg; j < end; ++j) {
                    const int e = ov.e[j];
                    const signed char *row = lr + (size_t)ov.m[j] * (n_mt * BM) + mi * 32;
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        const int x = *reinterpret_cast<const int *>(row + 8 * g4);
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            acc[mi][4 * g4 + c] += e * (int)(signed char)(x >> (8 * c));
                    }
                }
        }
    }


    // one K-step from stage `buf` with this wave's B registers
    auto compute = [&](int buf, const v4i (&b)[4]) {
        const unsigned char *As = lds + buf * TILE_BYTES;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int c = 4 * fh + s;
            v4i a[8];
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                const int r = mi * 32 + fr;
                a[mi] = *reinterpret_cast<const v4i *>(As + r * BKB + ((c ^ ((r >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) acc[mi] = M::mma(a[mi], b[s], acc[mi]);
        }
    };

    const int nk = Kb / BKB;
    v4i b0[4], b1[4];
    if constexpr (EPI == 4) {
        // diagnostic: stage once, then the K loop on LDS + registers only
        stageA(0, 0);
        loadB(b0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int t = 0; t < nk; ++t) {
            compute(0, b0);
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    } else {
        // issue order: A(0) .. A(NST-2), B(0), B(1); step t: [wait A(t), B(t);
        // barrier] A(t+NST-1), compute t, B(t+2).  At the top of step t >= 1
        // the ops issued after B(t) are A(t+NST-2) and B(t+1) (each 4
        // instructions, when they exist): vmcnt(8 / 4 / 0) retires B(t) and,
        // older still, A(t).
        for (int t = 0; t < NST - 1; ++t)
            if (t < nk) stageA(t, t * BKB);
        loadB(b0, 0);
        if (nk > 1) loadB(b1, BKB);
        auto wait_step = [&](int t) {
            const int n = t == 0 ? (nk > 1 ? 4 : 0)
                                 : 4 * (t + NST - 2 < nk) + 4 * (t + 1 < nk);
            if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // every wave's pieces of A(t) landed;
            asm volatile("" ::: "memory");  // stage (t-1) % NST is free
        };
        // two K-steps per iteration, so the B register buffers have fixed names
        int t = 0;
        for (; t + 1 < nk; t += 2) {
            wait_step(t);
            if (t + NST - 1 < nk) stageA((t + NST - 1) % NST, (t + NST - 1) * BKB);
            compute(t % NST, b0);
            if (t + 2 < nk) loadB(b0, (t + 2) * BKB);
            wait_step(t + 1);
            if (t + NST < nk) stageA((t + NST) % NST, (t + NST) * BKB);
            compute((t + 1) % NST, b1);
            if (t + 3 < nk) loadB(b1, (t + 3) * BKB);
        }
        if (t < nk) {
            wait_step(t);
            compute(t % NST, b0);
        }
    }
    if constexpr (EPI != 0) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" ::"v"(acc[mi]));
#endif
        }
        return;
    }

    // ---- epilogue: per lane the top-4 of its pod's 128 (node, cost) values,
    // merged with lane ^ 32 (the same pod, the other 4 rows of each group)
    // into the pod's 8-list over the tile's 256 nodes
    unsigned u[8][16];
    unsigned kmin = 0xffffffffu, kmax = 0u;
    int smin = 0x7fffffff, smax = -0x7fffffff - 1;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            if constexpr (DT == NAS_DT_I8) {
                smin = min(smin, (int)acc[mi][reg]);
                smax = max(smax, (int)acc[mi][reg]);
            } else {
                u[mi][reg] = M::okey(acc[mi][reg]);
                kmin = min(kmin, u[mi][reg]);
                kmax = max(kmax, u[mi][reg]);
            }
        }
    if constexpr (DT == NAS_DT_I8) {
        kmin = M::okey(smin);
        kmax = M::okey(smax);
    }
    u64 k4[4];
    const unsigned nb = (unsigned)(node_base + mt * BM + 4 * fh);
    if (__all(kmax - kmin < (1u << 25) - 1u)) {
        // packed: (key - kmin) << 7 | i, i = mi * 16 + reg increasing in node
        // order; a non-fitting value is all-ones.  Sorted insert by med3.
        unsigned c0 = 0xffffffffu, c1 = c0, c2 = c0, c3 = c0;
        const unsigned nk7 = 0u - ((DT == NAS_DT_I8 ? (unsigned)smin : kmin) << 7);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
            const unsigned nbits = ~(unsigned)(mw[mi >> 1] >> (32 * (mi & 1)));
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = (reg & 3) + 8 * (reg >> 2) + 4 * fh;
                const unsigned raw = DT == NAS_DT_I8 ? (unsigned)(int)acc[mi][reg] : u[mi][reg];
                const unsigned x = ((raw << 7) + nk7) | (unsigned)(mi * 16 + reg) |
                                   (unsigned)__builtin_amdgcn_sbfe((int)nbits, row, 1);
                c3 = umed3(c2, c3, x);
                c2 = umed3(c1, c2, x);
                c1 = umed3(c0, c1, x);
                c0 = min(c0, x);
            }
        }
        const unsigned cc[4] = {c0, c1, c2, c3};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned i = cc[j] & 127u, r = i & 15u;
            const unsigned node = nb + (i >> 4) * 32u + (r & 3u) + 8u * (r >> 2);
            k4[j] = cc[j] == 0xffffffffu ? KEY_INVALID : ((u64)((cc[j] >> 7) + kmin) << 32) | node;
        }
    } else {
        Top4 t4;
        t4.init();
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
            const unsigned bits = (unsigned)(mw[mi >> 1] >> (32 * (mi & 1)));
            const unsigned node0 = nb + mi * 32;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = (reg & 3) + 8 * (reg >> 2);
                const unsigned key = DT == NAS_DT_I8 ? M::okey(acc[mi][reg]) : u[mi][reg];
                const unsigned x = key | ((((bits >> (row + 4 * fh)) & 1u) ^ 1u) * 0xffffffffu);
                t4.insert(x, node0 + row);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) k4[j] = t4.c[j] == 0xffffffffu ? KEY_INVALID : t4.key(j);
    }
    u64 o4[4], l8[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) o4[j] = shfl_xor64(k4[j], 32);
    merge44(k4, o4, l8);
    const u64 bnd = umin64(umin64(k4[3], o4[3]), l8[7]);
    // both halves hold the same list: half h stores keys 4h .. 4h+3
    u64 *dst = partial + ((size_t)mt * Pp + pod_row) * KC + 4 * fh;
    const u64 q0 = fh ? l8[4] : l8[0], q1 = fh ? l8[5] : l8[1];
    const u64 q2 = fh ? l8[6] : l8[2], q3 = fh ? l8[7] : l8[3];
    reinterpret_cast<ulonglong2 *>(dst)[0] = make_ulonglong2(q0, q1);
    reinterpret_cast<ulonglong2 *>(dst)[1] = make_ulonglong2(q2, q3);
    if (fh == 0) pbound[(size_t)mt * Pp + pod_row] = bnd;
}

// ---------------------------------------------------------------------------
// k_cost_topk3: k_cost_topk2's operand split at ONE wave per SIMD.  A
// 256-thread workgroup (4 waves) computes the 256-node x 256-pod tile; wave w
// owns pods 64w .. 64w+63 (2 pod tiles) x all 256 nodes = 16 MFMA tiles, 256
// accumulator registers of the 512 a lone wave may use.  Per k-substep: 8
// ds_read_b128 (the node tiles, shared by both pod tiles) for 16 MFMAs -- half
// the LDS reads per MFMA of k_cost_topk2 -- with the next substep's fragments
// read while the current MFMAs run, and WA rows streamed two K-steps ahead.
// ---------------------------------------------------------------------------
constexpr int THREADS3 = 256;
template <int DT, int EPI = 0, int NST = 4, int GM = COST_GM, bool TB = false>
__global__ void __launch_bounds__(THREADS3, 1)
k_cost_topk3(const unsigned char *__restrict__ Lt, const unsigned char *__restrict__ WA, int Kb,
             int n_mt, int n_nt, int p0, int Pp, const u64 *__restrict__ mask,
             u64 *__restrict__ partial, u64 *__restrict__ pbound, int node_base,
             const int *__restrict__ dyn_start, int dyn_hi, const int *__restrict__ dyn_hi_ptr,
             Ovf ov) {
    using M = Mma<DT>;
    using acc_t = typename M::acc_t;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int nwg = n_mt * n_nt;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int gsize = GM * n_nt;
    const int g = v / gsize;
    const int first_mt = g * GM;
    const int gm = min(n_mt - first_mt, GM);
    const int mt = first_mt + (v % gsize) % gm;
    const int nt = (v % gsize) / gm;
    const int cb = blockIdx.y;
    Lt += (size_t)cb * n_mt * BM * Kb;
    WA += (size_t)cb * Pp * Kb;
    mask += (size_t)cb * (n_mt * BM / 64) * Pp;
    partial += (size_t)cb * n_mt * Pp * KC;
    pbound += (size_t)cb * n_mt * Pp;
    if (dyn_start) {
        const int s0 = dyn_start[cb * STATUS_INTS];
        if (s0 < 0) return;
        if (dyn_hi_ptr) dyn_hi = dyn_hi_ptr[cb * STATUS_INTS];
        p0 = s0 / BN * BN;
        if (p0 + nt * BN >= dyn_hi) return;
    }

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int fr = lane & 31, fh = lane >> 5;
    const int prow0 = p0 + nt * BN + w * 64 + fr;  // pod of pod tile ni: prow0 + 32 * ni
    const unsigned char *Ag = Lt + (size_t)mt * BM * Kb;
    const unsigned char *B0 = WA + (size_t)prow0 * Kb + 64 * fh;
    const unsigned char *B1 = B0 + (size_t)32 * Kb;
    if constexpr (EPI == 3) {
        Ag = Lt;
        B0 = WA + (size_t)(w * 64 + fr) * Kb + 64 * fh;
        B1 = B0 + (size_t)32 * Kb;
    }
    const int srow_in = lane >> 3, sq = lane & 7;
    auto stageA = [&](int buf, int k0) {
        unsigned char *base = lds + buf * TILE_BYTES;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int r0 = (j * 4 + w) * 8;
            const int row = r0 + srow_in;
            const int c = sq ^ ((row >> 1) & 7);
            glds16(Ag + (size_t)row * Kb + k0 + c * 16, base + r0 * BKB);
        }
    };
    // WA rows by inline-asm loads retired by the explicit vmcnt of wait_step
    // (a compiler-visible load carried into the next loop iteration makes
    // hipcc put a vmcnt(0) in front of every step, draining the A prefetch)
    // TB: WA pre-tiled in fragment order (see k_cost_topk2): 1 KiB per load
    const unsigned char *T0 = WA + (size_t)(prow0 >> 5) * 32 * Kb + lane * 16;
    const unsigned char *T1 = T0 + (size_t)32 * Kb;
    auto loadB = [&](v4i (&b)[2][4], int k0) {
#pragma unroll
        for (int s = 0; s < 4; ++s) b[0][s] = gld16(TB ? T0 + k0 * 32 + 1024 * s : B0 + k0 + 16 * s);
#pragma unroll
        for (int s = 0; s < 4; ++s) b[1][s] = gld16(TB ? T1 + k0 * 32 + 1024 * s : B1 + k0 + 16 * s);
    };

    u64 mw[2][4];
    if constexpr (EPI == 0) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int c = 0; c < 4; ++c) mw[ni][c] = mask[(size_t)(mt * 4 + c) * Pp + prow0 + 32 * ni];
    }
    acc_t acc[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i][0] = acc[i][1] = acc_t{};

    // exact int32 traffic: overflow entries of the lane's two pods as the
    // accumulators' initial value (before the K loop's registers are live)
    if constexpr (DT == NAS_DT_I8 && EPI == 0) {
        if (ov.ptr) {
            const int lim = ov.row_count ? *ov.row_count : 0x7fffffff;
            const signed char *lr = ov.Lr + (size_t)cb * ov.N * (n_mt * BM) + mt * BM + 4 * fh;
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int r = prow0 + 32 * ni;
                int beg = 0, end = 0;
                if (r < lim) {
                    const int pod = (ov.row_pod ? ov.row_pod[r] : r) + cb * Pp;
                    beg = ov.ptr[pod];
                    end = ov.ptr[pod + 1];
                }
#pragma unroll
                for (int mi = 0; mi < 8; ++mi)
                    for (int j = beg; j < end; ++j) {
                        const int e = ov.e[j];
                        const signed char *row = lr + (size_t)ov.m[j] * (n_mt * BM) + mi * 32;
#pragma unroll
                        for (int g4 = 0; g4 < 4; ++g4) {
                            const int x = *reinterpret_cast<const int *>(row + 8 * g4);
#pragma unroll
                            for (int c = 0; c < 4; ++c)
                                acc[mi][ni][4 * g4 + c] += e * (int)(signed char)(x >> (8 * c));
                        }
                    }
            }
        }
    }

    // One K-step, hand-scheduled in inline asm (hipcc's scheduler otherwise
    // reads each fragment right before its MFMA pair and exposes the LDS
    // latency at one wave per SIMD): per k-substep two blocks of 8 MFMAs,
    // each interleaving the 4 fragment reads (ds_read_b128) of the NEXT
    // substep, one per MFMA pair; a block waits only for its own 4
    // fragments (lgkmcnt(4): the 4 reads issued after them stay in flight).
    // Node tile mi of the fragment image is 32 rows = 4096 B further, and
    // the row swizzle (row >> 1) & 7 does not depend on mi, so one address
    // per substep + immediate offsets.
    const unsigned lds_lane = (unsigned)(fr * BKB);
    const unsigned swz = (unsigned)((fr >> 1) & 7);
    auto faddr = [&](int buf, int s) -> unsigned {
        return (unsigned)(buf * TILE_BYTES) + lds_lane + ((((unsigned)(4 * fh + s)) ^ swz) << 4);
    };
    v4i fa[8], fb[8];
    auto read8 = [&](v4i (&f)[8], unsigned ad) {
        asm volatile(
            "ds_read_b128 %0, %8\n ds_read_b128 %1, %8 offset:4096\n"
            "ds_read_b128 %2, %8 offset:8192\n ds_read_b128 %3, %8 offset:12288\n"
            "ds_read_b128 %4, %8 offset:16384\n ds_read_b128 %5, %8 offset:20480\n"
            "ds_read_b128 %6, %8 offset:24576\n ds_read_b128 %7, %8 offset:28672\n"
            : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]), "=&v"(f[5]),
              "=&v"(f[6]), "=&v"(f[7])
            : "v"(ad)
            : "memory");
    };
    static_assert(DT == NAS_DT_I8, "k_cost_topk3 is written for the int8 MFMA");
#define NAS_MF(D, A, B) "v_mfma_i32_32x32x32_i8 " D ", " A ", " B ", " D "\n"
    // 8 MFMAs of node tiles h4*4 .. h4*4+3 on fragments cur[], reading next[]
    // (4 fragments at offsets of the same tiles) when ad is given
    auto block = [&](v4i(&cur)[8], v4i(&nxt)[8], int h4, const v4i &b0, const v4i &b1,
                     bool rd, unsigned ad, bool last) {
        const int o = h4 * 4;
        if (rd) {
            if (h4 == 0)
                asm volatile("s_waitcnt lgkmcnt(4)\n"
                             NAS_MF("%0", "%12", "%16") NAS_MF("%1", "%12", "%17")
                             "ds_read_b128 %8, %18\n"
                             NAS_MF("%2", "%13", "%16") NAS_MF("%3", "%13", "%17")
                             "ds_read_b128 %9, %18 offset:4096\n"
                             NAS_MF("%4", "%14", "%16") NAS_MF("%5", "%14", "%17")
                             "ds_read_b128 %10, %18 offset:8192\n"
                             NAS_MF("%6", "%15", "%16") NAS_MF("%7", "%15", "%17")
                             "ds_read_b128 %11, %18 offset:12288\n"
                             : "+a"(acc[o][0]), "+a"(acc[o][1]), "+a"(acc[o + 1][0]), "+a"(acc[o + 1][1]),
                               "+a"(acc[o + 2][0]), "+a"(acc[o + 2][1]), "+a"(acc[o + 3][0]),
                               "+a"(acc[o + 3][1]), "=&v"(nxt[o]), "=&v"(nxt[o + 1]),
                               "=&v"(nxt[o + 2]), "=&v"(nxt[o + 3])
                             : "v"(cur[o]), "v"(cur[o + 1]), "v"(cur[o + 2]), "v"(cur[o + 3]),
                               "v"(b0), "v"(b1), "v"(ad)
                             : "memory");
            else
                asm volatile("s_waitcnt lgkmcnt(4)\n"
                             NAS_MF("%0", "%12", "%16") NAS_MF("%1", "%12", "%17")
                             "ds_read_b128 %8, %18 offset:16384\n"
                             NAS_MF("%2", "%13", "%16") NAS_MF("%3", "%13", "%17")
                             "ds_read_b128 %9, %18 offset:20480\n"
                             NAS_MF("%4", "%14", "%16") NAS_MF("%5", "%14", "%17")
                             "ds_read_b128 %10, %18 offset:24576\n"
                             NAS_MF("%6", "%15", "%16") NAS_MF("%7", "%15", "%17")
                             "ds_read_b128 %11, %18 offset:28672\n"
                             : "+a"(acc[o][0]), "+a"(acc[o][1]), "+a"(acc[o + 1][0]), "+a"(acc[o + 1][1]),
                               "+a"(acc[o + 2][0]), "+a"(acc[o + 2][1]), "+a"(acc[o + 3][0]),
                               "+a"(acc[o + 3][1]), "=&v"(nxt[o]), "=&v"(nxt[o + 1]),
                               "=&v"(nxt[o + 2]), "=&v"(nxt[o + 3])
                             : "v"(cur[o]), "v"(cur[o + 1]), "v"(cur[o + 2]), "v"(cur[o + 3]),
                               "v"(b0), "v"(b1), "v"(ad)
                             : "memory");
        } else if (!last) {
            asm volatile("s_waitcnt lgkmcnt(4)\n"
                         NAS_MF("%0", "%8", "%12") NAS_MF("%1", "%8", "%13")
                         NAS_MF("%2", "%9", "%12") NAS_MF("%3", "%9", "%13")
                         NAS_MF("%4", "%10", "%12") NAS_MF("%5", "%10", "%13")
                         NAS_MF("%6", "%11", "%12") NAS_MF("%7", "%11", "%13")
                         : "+a"(acc[o][0]), "+a"(acc[o][1]), "+a"(acc[o + 1][0]), "+a"(acc[o + 1][1]),
                           "+a"(acc[o + 2][0]), "+a"(acc[o + 2][1]), "+a"(acc[o + 3][0]),
                           "+a"(acc[o + 3][1])
                         : "v"(cur[o]), "v"(cur[o + 1]), "v"(cur[o + 2]), "v"(cur[o + 3]), "v"(b0),
                           "v"(b1)
                         : "memory");
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)\n"
                         NAS_MF("%0", "%8", "%12") NAS_MF("%1", "%8", "%13")
                         NAS_MF("%2", "%9", "%12") NAS_MF("%3", "%9", "%13")
                         NAS_MF("%4", "%10", "%12") NAS_MF("%5", "%10", "%13")
                         NAS_MF("%6", "%11", "%12") NAS_MF("%7", "%11", "%13")
                         : "+a"(acc[o][0]), "+a"(acc[o][1]), "+a"(acc[o + 1][0]), "+a"(acc[o + 1][1]),
                           "+a"(acc[o + 2][0]), "+a"(acc[o + 2][1]), "+a"(acc[o + 3][0]),
                           "+a"(acc[o + 3][1])
                         : "v"(cur[o]), "v"(cur[o + 1]), "v"(cur[o + 2]), "v"(cur[o + 3]), "v"(b0),
                           "v"(b1)
                         : "memory");
        }
    };
#undef NAS_MF
    auto compute = [&](int buf, const v4i (&b)[2][4]) {
        read8(fa, faddr(buf, 0));
        block(fa, fb, 0, b[0][0], b[1][0], true, faddr(buf, 1), false);
        block(fa, fb, 1, b[0][0], b[1][0], true, faddr(buf, 1), false);
        block(fb, fa, 0, b[0][1], b[1][1], true, faddr(buf, 2), false);
        block(fb, fa, 1, b[0][1], b[1][1], true, faddr(buf, 2), false);
        block(fa, fb, 0, b[0][2], b[1][2], true, faddr(buf, 3), false);
        block(fa, fb, 1, b[0][2], b[1][2], true, faddr(buf, 3), false);
        block(fb, fa, 0, b[0][3], b[1][3], false, 0, false);
        block(fb, fa, 1, b[0][3], b[1][3], false, 0, true);
    };

    const int nk = Kb / BKB;
    v4i bA[2][4], bB[2][4];
    if constexpr (EPI == 4) {
        stageA(0, 0);
        loadB(bA, 0);
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(bA[0][0]), "+v"(bA[0][1]), "+v"(bA[0][2]),
                     "+v"(bA[0][3]), "+v"(bA[1][0]), "+v"(bA[1][1]), "+v"(bA[1][2]),
                     "+v"(bA[1][3])::"memory");
        __syncthreads();
        for (int t = 0; t < nk; ++t) {
            compute(0, bA);
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    } else {
        // Straight-line pipeline (nk even: the host pads K to 256 bytes).
        // Every step issues A(t+NST-1) and B(t+2) -- clamped to the last
        // K-step at the end, so the vmcnt count never changes and there is no
        // branch: at the wait for step t+1 the ops issued after B(t+1) are
        // exactly A(t+NST-1) and B(t+2), 8 + 8 instructions.
        for (int t = 0; t < NST - 1; ++t) stageA(t, min(t, nk - 1) * BKB);
        loadB(bA, 0);
        loadB(bB, BKB);
#define NAS_TIE_B(bb) "+v"(bb[0][0]), "+v"(bb[0][1]), "+v"(bb[0][2]), "+v"(bb[0][3]), \
                      "+v"(bb[1][0]), "+v"(bb[1][1]), "+v"(bb[1][2]), "+v"(bb[1][3])
        asm volatile("s_waitcnt vmcnt(8)" : NAS_TIE_B(bA)::"memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        for (int t = 0; t < nk; t += 2) {
            stageA((t + NST - 1) % NST, min(t + NST - 1, nk - 1) * BKB);
            compute(t % NST, bA);
            loadB(bA, min(t + 2, nk - 1) * BKB);
            asm volatile("s_waitcnt vmcnt(16)" : NAS_TIE_B(bB)::"memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            stageA((t + NST) % NST, min(t + NST, nk - 1) * BKB);
            compute((t + 1) % NST, bB);
            loadB(bB, min(t + 3, nk - 1) * BKB);
            asm volatile("s_waitcnt vmcnt(16)" : NAS_TIE_B(bA)::"memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
#undef NAS_TIE_B
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail loads
    }
    if constexpr (EPI != 0) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" ::"v"(acc[mi][0]), "v"(acc[mi][1]));
#endif
        }
        return;
    }

    // ---- epilogue, per pod tile: the lane's top-4 of its pod's 128 values,
    // merged with lane ^ 32 into the pod's 8-list over the tile's 256 nodes
    const unsigned nb = (unsigned)(node_base + mt * BM + 4 * fh);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        unsigned kmin = 0xffffffffu, kmax = 0u;
        int smin = 0x7fffffff, smax = -0x7fffffff - 1;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                if constexpr (DT == NAS_DT_I8) {
                    smin = min(smin, (int)acc[mi][ni][reg]);
                    smax = max(smax, (int)acc[mi][ni][reg]);
                } else {
                    const unsigned u = M::okey(acc[mi][ni][reg]);
                    kmin = min(kmin, u);
                    kmax = max(kmax, u);
                }
            }
        if constexpr (DT == NAS_DT_I8) {
            kmin = M::okey(smin);
            kmax = M::okey(smax);
        }
        u64 k4[4];
        if (__all(kmax - kmin < (1u << 25) - 1u)) {
            unsigned c0 = 0xffffffffu, c1 = c0, c2 = c0, c3 = c0;
            const unsigned nk7 = 0u - ((DT == NAS_DT_I8 ? (unsigned)smin : kmin) << 7);
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                const unsigned nbits = ~(unsigned)(mw[ni][mi >> 1] >> (32 * (mi & 1)));
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * fh;
                    const unsigned raw = DT == NAS_DT_I8 ? (unsigned)(int)acc[mi][ni][reg]
                                                         : M::okey(acc[mi][ni][reg]);
                    const unsigned x = ((raw << 7) + nk7) | (unsigned)(mi * 16 + reg) |
                                       (unsigned)__builtin_amdgcn_sbfe((int)nbits, row, 1);
                    c3 = umed3(c2, c3, x);
                    c2 = umed3(c1, c2, x);
                    c1 = umed3(c0, c1, x);
                    c0 = min(c0, x);
                }
            }
            const unsigned cc[4] = {c0, c1, c2, c3};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const unsigned i = cc[j] & 127u, r = i & 15u;
                const unsigned node = nb + (i >> 4) * 32u + (r & 3u) + 8u * (r >> 2);
                k4[j] = cc[j] == 0xffffffffu ? KEY_INVALID
                                             : ((u64)((cc[j] >> 7) + kmin) << 32) | node;
            }
        } else {
            Top4 t4;
            t4.init();
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                const unsigned bits = (unsigned)(mw[ni][mi >> 1] >> (32 * (mi & 1)));
                const unsigned node0 = nb + mi * 32;
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int row = (reg & 3) + 8 * (reg >> 2);
                    const unsigned x = M::okey(acc[mi][ni][reg]) |
                                       ((((bits >> (row + 4 * fh)) & 1u) ^ 1u) * 0xffffffffu);
                    t4.insert(x, node0 + row);
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) k4[j] = t4.c[j] == 0xffffffffu ? KEY_INVALID : t4.key(j);
        }
        u64 o4[4], l8[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = shfl_xor64(k4[j], 32);
        merge44(k4, o4, l8);
        const u64 bnd = umin64(umin64(k4[3], o4[3]), l8[7]);
        const int pod = prow0 + 32 * ni;
        u64 *dst = partial + ((size_t)mt * Pp + pod) * KC + 4 * fh;
        const u64 q0 = fh ? l8[4] : l8[0], q1 = fh ? l8[5] : l8[1];
        const u64 q2 = fh ? l8[6] : l8[2], q3 = fh ? l8[7] : l8[3];
        reinterpret_cast<ulonglong2 *>(dst)[0] = make_ulonglong2(q0, q1);
        reinterpret_cast<ulonglong2 *>(dst)[1] = make_ulonglong2(q2, q3);
        if (fh == 0) pbound[(size_t)mt * Pp + pod] = bnd;
    }
}


#ifdef NAS_DIAG_VARIANTS
#define NAS_INST2(E, S, G)                                                                         \
    template __global__ void k_cost_topk2<NAS_DT_I8, E, S, G>(                                     \
        const unsigned char *, const unsigned char *, int, int, int, int, int, const u64 *, u64 *,  \
        u64 *, int, const int *, int, const int *, Ovf);
NAS_INST2(0, 4, 4) NAS_INST2(1, 4, 4) NAS_INST2(3, 4, 4) NAS_INST2(4, 4, 4) NAS_INST2(0, 3, 4)
NAS_INST2(0, 4, 8) NAS_INST2(1, 3, 4)
#undef NAS_INST2
#define NAS_INST2T(E, S, G)                                                                        \
    template __global__ void k_cost_topk2<NAS_DT_I8, E, S, G, true>(                               \
        const unsigned char *, const unsigned char *, int, int, int, int, int, const u64 *, u64 *,  \
        u64 *, int, const int *, int, const int *, Ovf);
NAS_INST2T(0, 4, 4) NAS_INST2T(1, 4, 4) NAS_INST2T(0, 3, 4)
#undef NAS_INST2T
#define NAS_INST3(E, S, G)                                                                         \
    template __global__ void k_cost_topk3<NAS_DT_I8, E, S, G>(                                     \
        const unsigned char *, const unsigned char *, int, int, int, int, int, const u64 *, u64 *,  \
        u64 *, int, const int *, int, const int *, Ovf);
NAS_INST3(0, 4, 4) NAS_INST3(1, 4, 4) NAS_INST3(3, 4, 4) NAS_INST3(4, 4, 4) NAS_INST3(0, 4, 8)
#undef NAS_INST3
#define NAS_INST3T(E, S, G)                                                                        \
    template __global__ void k_cost_topk3<NAS_DT_I8, E, S, G, true>(                               \
        const unsigned char *, const unsigned char *, int, int, int, int, int, const u64 *, u64 *,  \
        u64 *, int, const int *, int, const int *, Ovf);
NAS_INST3T(0, 4, 4) NAS_INST3T(1, 4, 4)
#undef NAS_INST3T
#endif
// ---------------------------------------------------------------------------
// k_cost_wide (measured round 2, kept for the record): the same contraction with NI x 128 pods per workgroup tile
// (NI = 3: 256 nodes x 384 pods).  Every staged byte then feeds 1.2x the MACs
// of the 256 x 256 tile -- 17% fewer bytes through the L2 -> LDS fabric, which
// is what bounds k_cost_topk -- at the price of the whole LDS
// (two 80 KiB stages) and 192 accumulator registers per wave (8 waves as
// 2 node halves x 4 pod quarters, each 128 nodes x 32*NI pods).  PIPE 0
// staging, LDS-DMA with the source-side swizzle, double-buffered fragments;
// the epilogue writes each pod tile's 8-list to LDS as soon as it is built
// (the accumulators of that tile die there), then the node-half waves merge.
// Result (profiles/r02_mb_cost_wide.log): the main loop alone 4% faster than
// NI = 2 (8.3-8.4 vs 8.7 ms), not the 17% the byte count predicts, and the
// 3-tile epilogue at the 256-VGPR limit spills (10.2-10.3 ms in all) -- so the
// staging fabric is not bound by bytes alone; k_cost_topk stays at 256 x 256.
// ---------------------------------------------------------------------------
template <int DT, int EPI, bool RMAP, int NI>
__global__ void __launch_bounds__(THREADS, 1)
k_cost_wide(const unsigned char *__restrict__ Lt, const unsigned char *__restrict__ WA, int Kb,
            int n_mt, int n_nt, int p0, int Pp, const u64 *__restrict__ mask,
            u64 *__restrict__ partial, u64 *__restrict__ pbound, int node_base,
            const int *__restrict__ dyn_start, int dyn_hi, const int *__restrict__ dyn_hi_ptr,
            Ovf ov, const int *__restrict__ rowmap) {
    constexpr int BNW = 128 * NI;     // pods per tile
    constexpr int WP = 32 * NI;       // pods per wave
    constexpr int BPC = BNW / 64;     // B pieces per wave per stage
    constexpr int SB = (BM + BNW) * BKB;
    using M = Mma<DT>;
    using acc_t = typename M::acc_t;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int nwg = n_mt * n_nt;
    const int b = blockIdx.x;
    const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    int mt, nt;
    {  // pod-group major, groups of 4 pod tiles (k_cost_topk's COST_GM = -4)
        constexpr int PG = 4;
        const int gsize = PG * n_mt;
        const int g = v / gsize, r = v % gsize;
        const int first_nt = g * PG;
        const int pg = min(n_nt - first_nt, PG);
        mt = r / pg;
        nt = first_nt + r % pg;
    }
    const int cb = blockIdx.y;
    Lt += (size_t)cb * n_mt * BM * Kb;
    WA += (size_t)cb * Pp * Kb;
    mask += (size_t)cb * (n_mt * BM / 64) * Pp;
    partial += (size_t)cb * n_mt * Pp * KC;
    pbound += (size_t)cb * n_mt * Pp;
    if (dyn_start) {
        const int s = dyn_start[cb * STATUS_INTS];
        if (s < 0) return;
        if (dyn_hi_ptr) dyn_hi = dyn_hi_ptr[cb * STATUS_INTS];
        p0 = s / BNW * BNW;
        if (p0 + nt * BNW >= dyn_hi) return;
    }
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 2, wn = w & 3;
    const int fr = lane & 31, fh = lane >> 5;
    const int pod0 = p0 + nt * BNW;  // first pod (view row) of the tile
    const unsigned char *Ag = Lt + (size_t)mt * BM * Kb;
    const unsigned char *Bg = WA + (size_t)pod0 * Kb;
    const int srow_in = lane >> 3, sq = lane & 7;
    int bpod[BPC];
    if constexpr (RMAP) {
#pragma unroll
        for (int j = 0; j < BPC; ++j) bpod[j] = rowmap[min(pod0 + (j * 8 + w) * 8 + srow_in, dyn_hi - 1)];
    }
    auto stage = [&](int buf, int k0) {
        unsigned char *base = lds + buf * SB;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r0 = (j * 8 + w) * 8, row = r0 + srow_in;
            const int c = sq ^ ((row >> 1) & 7);
            glds16(Ag + (size_t)row * Kb + k0 + c * 16, base + r0 * BKB);
        }
#pragma unroll
        for (int j = 0; j < BPC; ++j) {
            const int r0 = (j * 8 + w) * 8, row = r0 + srow_in;
            const int c = sq ^ ((row >> 1) & 7);
            const unsigned char *src = RMAP ? WA + (size_t)bpod[j] * Kb : Bg + (size_t)row * Kb;
            glds16(src + k0 + c * 16, base + BM * BKB + r0 * BKB);
        }
    };
    u64 mwp[NI][2];
    if constexpr (EPI == 0) {
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
            for (int mi2 = 0; mi2 < 2; ++mi2) {
                const int pod = pod0 + wn * WP + ni * 32 + fr;
                const int chunk = (mt * BM + wm * 128 + mi2 * 64) >> 6;
                mwp[ni][mi2] = mask[(size_t)chunk * Pp + pod];
            }
    }
    acc_t acc[4][NI];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = acc_t{};
    if constexpr (DT == NAS_DT_I8 && EPI == 0) {
        if (ov.ptr) {  // exact traffic beyond int8: see k_cost_topk
            const int cnt_lim = ov.row_count ? *ov.row_count : 0x7fffffff;
            const signed char *lr = ov.Lr + (size_t)cb * ov.N * (n_mt * BM) + mt * BM + wm * 128 + 4 * fh;
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) {
                const int r = pod0 + wn * WP + ni * 32 + fr;
                int beg = 0, end = 0;
                if (r < cnt_lim) {
                    const int pod = (ov.row_pod ? ov.row_pod[r] : r) + cb * Pp;
                    beg = ov.ptr[pod];
                    end = ov.ptr[pod + 1];
                }
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
                    for (int j = beg; j < end; ++j) {
                        const int e = ov.e[j];
                        const signed char *row = lr + (size_t)ov.m[j] * (n_mt * BM) + mi * 32;
#pragma unroll
                        for (int g = 0; g < 4; ++g) {
                            const int x = *reinterpret_cast<const int *>(row + 8 * g);
#pragma unroll
                            for (int c = 0; c < 4; ++c)
                                acc[mi][ni][4 * g + c] += e * (int)(signed char)(x >> (8 * c));
                        }
                    }
            }
        }
    }
    auto compute = [&](int buf) {
        const unsigned char *As = lds + buf * SB;
        const unsigned char *Bs = As + BM * BKB;
        v4i a[2][4], bb[2][NI];
        auto read = [&](int kk, v4i (&ra)[4], v4i (&rb)[NI]) {
            const int c = kk * 2 + fh;
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int r = wm * 128 + mi * 32 + fr;
                ra[mi] = *reinterpret_cast<const v4i *>(As + r * BKB + ((c ^ ((r >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) {
                const int r = wn * WP + ni * 32 + fr;
                rb[ni] = *reinterpret_cast<const v4i *>(Bs + r * BKB + ((c ^ ((r >> 1) & 7)) << 4));
            }
        };
        read(0, a[0], bb[0]);
#pragma unroll
        for (int kk = 0; kk < BKB / 32; ++kk) {
            if (kk + 1 < BKB / 32) read(kk + 1, a[(kk + 1) & 1], bb[(kk + 1) & 1]);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < NI; ++ni)
                    acc[mi][ni] = M::mma(a[kk & 1][mi], bb[kk & 1][ni], acc[mi][ni]);
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
    if constexpr (EPI == 1) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) {
#if defined(__HIP_DEVICE_COMPILE__)
                asm volatile("" ::"v"(acc[mi][ni]));
#endif
            }
        return;
    }
    // ---- epilogue: per pod tile ni, the lane's top-4 -> lane^32 merge -> an
    // 8-list + bound, straight to LDS (staging is dead after the last barrier):
    // xk[wm][wn][ni][32][9]
    u64 *xk = reinterpret_cast<u64 *>(lds);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
        const u64 *mw = mwp[ni];
        unsigned u[4][16];
        unsigned kmin = 0xffffffffu, kmax = 0u;
        int smin = 0x7fffffff, smax = -0x7fffffff - 1;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                if constexpr (DT == NAS_DT_I8) {
                    smin = min(smin, (int)acc[mi][ni][reg]);
                    smax = max(smax, (int)acc[mi][ni][reg]);
                } else {
                    u[mi][reg] = M::okey(acc[mi][ni][reg]);
                    kmin = min(kmin, u[mi][reg]);
                    kmax = max(kmax, u[mi][reg]);
                }
            }
        if constexpr (DT == NAS_DT_I8) {
            kmin = M::okey(smin);
            kmax = M::okey(smax);
        }
        u64 k4[4];
        if (__all(kmax - kmin < (1u << 26) - 1u)) {
            unsigned c0 = 0xffffffffu, c1 = c0, c2 = c0, c3 = c0;
            const unsigned nk6 = 0u - ((DT == NAS_DT_I8 ? (unsigned)smin : kmin) << 6);
#pragma unroll
            for (int mi2 = 0; mi2 < 2; ++mi2)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int mi = mi2 * 2 + h;
                    const unsigned nbits = ~(unsigned)(mw[mi2] >> (32 * h));
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg) {
                        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * fh;
                        const unsigned raw = DT == NAS_DT_I8 ? (unsigned)(int)acc[mi][ni][reg]
                                                             : u[mi][reg];
                        const unsigned x = ((raw << 6) + nk6) | (unsigned)(mi * 16 + reg) |
                                           (unsigned)__builtin_amdgcn_sbfe((int)nbits, row, 1);
                        c3 = umed3(c2, c3, x);
                        c2 = umed3(c1, c2, x);
                        c1 = umed3(c0, c1, x);
                        c0 = min(c0, x);
                    }
                }
            const unsigned cc[4] = {c0, c1, c2, c3};
            const unsigned nb = (unsigned)(node_base + mt * BM + wm * 128 + 4 * fh);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const unsigned i = cc[j] & 63u, r = i & 15u;
                const unsigned node = nb + (i >> 4) * 32u + (r & 3u) + 8u * (r >> 2);
                k4[j] = cc[j] == 0xffffffffu ? KEY_INVALID
                                             : ((u64)((cc[j] >> 6) + kmin) << 32) | node;
            }
        } else {
            Top4 t4;
            t4.init();
#pragma unroll
            for (int mi2 = 0; mi2 < 2; ++mi2)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int mi = mi2 * 2 + h;
                    const unsigned bits = (unsigned)(mw[mi2] >> (32 * h));
                    const unsigned node0 = (unsigned)(node_base + mt * BM + wm * 128 + mi * 32);
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg) {
                        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * fh;
                        const unsigned key = DT == NAS_DT_I8 ? M::okey(acc[mi][ni][reg]) : u[mi][reg];
                        const unsigned x = key | ((((bits >> row) & 1u) ^ 1u) * 0xffffffffu);
                        t4.insert(x, node0 + row);
                    }
                }
#pragma unroll
            for (int j = 0; j < 4; ++j) k4[j] = t4.c[j] == 0xffffffffu ? KEY_INVALID : t4.key(j);
        }
        u64 o4[4], l8[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = shfl_xor64(k4[j], 32);
        merge44(k4, o4, l8);
        if (fh == 0) {
            u64 *d = xk + (((wm * 4 + wn) * NI + ni) * 32 + fr) * 9;
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = l8[j];
            d[8] = umin64(k4[3], o4[3]);
        }
    }
    __syncthreads();
    // the node-half waves' lists of each pod merged: waves wm = 0 take the
    // 4 * WP pods, lane l pods l and l + 64 (when < WP)
    if (wm == 0) {
#pragma unroll
        for (int q = 0; q < (WP + 63) / 64; ++q) {
            const int pp = q * 64 + lane;  // pod within the wave's WP pods
            if (pp < WP) {
                const int ni = pp >> 5, f = pp & 31;
                const u64 *s0 = xk + (((0 * 4 + wn) * NI + ni) * 32 + f) * 9;
                const u64 *s1 = xk + (((1 * 4 + wn) * NI + ni) * 32 + f) * 9;
                u64 mine[8], other[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    mine[j] = s0[j];
                    other[j] = s1[j];
                }
                merge88(mine, other);
                const u64 bd = umin64(umin64(s0[8], s1[8]), mine[7]);
                const int pod = pod0 + wn * WP + pp;
                store8(partial + ((size_t)mt * Pp + pod) * KC, mine);
                pbound[(size_t)mt * Pp + pod] = bd;
            }
        }
    }
}

#ifdef NAS_DIAG_VARIANTS
#define NAS_INSTW(E, NI)                                                                           \
    template __global__ void k_cost_wide<NAS_DT_I8, E, false, NI>(                                 \
        const unsigned char *, const unsigned char *, int, int, int, int, int, const u64 *, u64 *,  \
        u64 *, int, const int *, int, const int *, Ovf, const int *);
NAS_INSTW(0, 2) NAS_INSTW(1, 2) NAS_INSTW(0, 3) NAS_INSTW(1, 3)
#undef NAS_INSTW
#endif
}  // namespace
}  // namespace nas
