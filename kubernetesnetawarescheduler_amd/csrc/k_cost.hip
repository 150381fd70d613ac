// k_cost.hip -- network cost contraction on gfx950 MFMA with a fused
// fit-mask + per-pod top-k epilogue.
//
//   cost[p, n] = sum_m WA[p, m] * L[m, n]          (north star kernel (2))
//
// computed transposed, C^T[n, p] = sum_m Lt[n, m] * WA[p, m], so that the
// MFMA accumulator puts the NODE on the register axis and the POD on the
// lane axis: each lane then reduces its own pod's candidates in registers,
// with no cross-lane traffic until one lane^32 exchange (north star (3)).
// The cost matrix is never written to HBM.
//
//  * int8 path: v_mfma_i32_32x32x32_i8, int32 accumulation -- exact, so the
//    integer scores and the chosen nodes are bit-identical to the oracle.
//  * bf16 path: v_mfma_f32_32x32x16_bf16, fp32 accumulation.
//
// Tile: 256 nodes x 256 pods per 512-thread workgroup (8 wave64 as 2 x 4),
// each wave 128 nodes x 64 pods = 4 x 2 MFMA 32x32 tiles.  K is staged 128
// bytes per row per step into a double-buffered LDS image (2 x 64 KiB) with
// global_load_lds_dwordx4 (LDS-DMA); rows are 128 B with a 16-byte-chunk XOR
// swizzle (chunk ^= (row >> 1) & 7) applied to the SOURCE address, so the
// ds_read_b128 fragment reads are bank-conflict free.  Workgroup ids are
// remapped so the blocks sharing an XCD's L2 cover a 4 (node tiles) x 8
// (pod tiles) super-tile.
//
// Epilogue: per lane, 64 (node, cost) values per pod -> mask from the fit
// kernel (bit per node) -> packed key (orderable cost << 32 | node) -> sorted
// top-4 in registers -> merge with lane^32 -> merge across the two node-half
// waves through LDS -> partial[node_tile][pod][4] (32 B per pod per tile).
#include "nas_internal.h"

namespace nas {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned long long u64;

constexpr int THREADS = 512;
constexpr int BM = COST_BM;   // nodes per tile
constexpr int BN = COST_BN;   // pods per tile
constexpr int BKB = COST_BKB; // bytes of K per LDS stage (full 128-byte lines)
constexpr int STAGE_BYTES = (BM + BN) * BKB;  // 64 KiB
constexpr int LDS_BYTES = 2 * STAGE_BYTES;    // 128 KiB, double-buffered
constexpr int GM = 4;  // node tiles per L2 group

template <int DT>
struct Mma;

template <>
struct Mma<NAS_DT_I8> {
    using acc_t = v16i;
    static __device__ __forceinline__ acc_t mma(v4i a, v4i b, acc_t c) {
        return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ unsigned okey(int x) { return (unsigned)x ^ 0x80000000u; }
};

template <>
struct Mma<NAS_DT_BF16> {
    using acc_t = v16f;
    static __device__ __forceinline__ acc_t mma(v4i a, v4i b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                        __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ unsigned okey(float x) {
        x = x + 0.0f;  // -0 -> +0: the oracle compares costs, not sign bits
        const unsigned u = __float_as_uint(x);
        return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    }
};

__device__ __forceinline__ void glds16(const void *g, void *l) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)g,
                                     (void __attribute__((address_space(3))) *)l, 16, 0, 0);
}

__device__ __forceinline__ u64 umin(u64 a, u64 b) { return a < b ? a : b; }
__device__ __forceinline__ u64 umax(u64 a, u64 b) { return a < b ? b : a; }

// sorted 4-list insert (k0 <= k1 <= k2 <= k3)
__device__ __forceinline__ void insert4(u64 (&k)[4], u64 x) {
    k[3] = umin(k[3], x);
    u64 t = umin(k[2], k[3]); k[3] = umax(k[2], k[3]); k[2] = t;
    t = umin(k[1], k[2]); k[2] = umax(k[1], k[2]); k[1] = t;
    t = umin(k[0], k[1]); k[1] = umax(k[0], k[1]); k[0] = t;
}

// Per-lane running top-4 as separate (orderable cost, node) u32 words.
// A lane visits its nodes in ascending node order, so a new (x, n) sorts
// before entry j iff x < cost[j] strictly (an equal cost has the larger node):
// four independent 32-bit compares and a select network, no 64-bit compares.
struct Top4 {
    unsigned c[4], n[4];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = n[j] = 0xffffffffu;
    }
    __device__ __forceinline__ void insert(unsigned x, unsigned node) {
        const bool b0 = x < c[0], b1 = x < c[1], b2 = x < c[2], b3 = x < c[3];
        const unsigned c3 = b2 ? c[2] : (b3 ? x : c[3]), n3 = b2 ? n[2] : (b3 ? node : n[3]);
        const unsigned c2 = b1 ? c[1] : (b2 ? x : c[2]), n2 = b1 ? n[1] : (b2 ? node : n[2]);
        const unsigned c1 = b0 ? c[0] : (b1 ? x : c[1]), n1 = b0 ? n[0] : (b1 ? node : n[1]);
        c[0] = b0 ? x : c[0];
        n[0] = b0 ? node : n[0];
        c[1] = c1; n[1] = n1; c[2] = c2; n[2] = n2; c[3] = c3; n[3] = n3;
    }
    __device__ __forceinline__ u64 key(int j) const { return ((u64)c[j] << 32) | n[j]; }
};

// top-4 of two sorted 4-lists (bitonic: min against the reversed list, then a
// 4-element bitonic merge)
__device__ __forceinline__ void merge4(u64 (&a)[4], const u64 (&b)[4]) {
    u64 m0 = umin(a[0], b[3]), m1 = umin(a[1], b[2]), m2 = umin(a[2], b[1]), m3 = umin(a[3], b[0]);
    u64 t;
    t = umin(m0, m2); m2 = umax(m0, m2); m0 = t;
    t = umin(m1, m3); m3 = umax(m1, m3); m1 = t;
    t = umin(m0, m1); m1 = umax(m0, m1); m0 = t;
    t = umin(m2, m3); m3 = umax(m2, m3); m2 = t;
    a[0] = m0; a[1] = m1; a[2] = m2; a[3] = m3;
}

__device__ __forceinline__ u64 shfl_xor64(u64 x, int m) {
    const int lo = __shfl_xor((int)(unsigned)x, m);
    const int hi = __shfl_xor((int)(unsigned)(x >> 32), m);
    return ((u64)(unsigned)hi << 32) | (unsigned)lo;
}

// EPI != 0 are diagnostic variants for tools/mb_cost.hip: 1 = accumulators
// kept alive with an empty asm and no epilogue (times the main loop alone),
// 2 = per-lane top-1 instead of top-4.
template <int DT, int EPI = 0>
__global__ void __launch_bounds__(THREADS, 1)
k_cost_topk(const unsigned char *__restrict__ Lt, const unsigned char *__restrict__ WA, int Kb,
            int n_mt, int n_nt, int p0, int Pp, const u64 *__restrict__ mask,
            u64 *__restrict__ partial, int node_base) {
    using M = Mma<DT>;
    using acc_t = typename M::acc_t;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    // ---- XCD-aware tile order: blocks b, b+8, ... share an XCD (speed only)
    const int nwg = n_mt * n_nt;
    const int b = blockIdx.x;
    const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int gsize = GM * n_nt;
    const int g = v / gsize;
    const int first_mt = g * GM;
    const int gm = min(n_mt - first_mt, GM);
    const int mt = first_mt + (v % gsize) % gm;
    const int nt = (v % gsize) / gm;

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 2, wn = w & 3;

    const unsigned char *Ag = Lt + (size_t)mt * BM * Kb;
    const unsigned char *Bg = WA + (size_t)(p0 + nt * BN) * Kb;

    // LDS-DMA staging: piece j of wave w fills rows (8j + w)*8 .. +8 of A
    // and of B (1 KiB each, lane-linear: lane l -> row + l/8, 16-byte chunk
    // l%8; whole 128-byte lines per row -- 64-byte row pieces measured 12%
    // slower); the chunk swizzle chunk ^= (row >> 1) & 7 is applied on the
    // SOURCE address so fragment reads are bank-conflict free.
    const int srow_in = lane >> 3;
    const int sq = lane & 7;
    auto stage = [&](int buf, int k0) {
        unsigned char *As = lds + buf * STAGE_BYTES;
        unsigned char *Bs = As + BM * BKB;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r0 = (j * 8 + w) * 8;
            const int row = r0 + srow_in;
            const int c = sq ^ ((row >> 1) & 7);
            glds16(Ag + (size_t)row * Kb + k0 + c * 16, As + r0 * BKB);
            glds16(Bg + (size_t)row * Kb + k0 + c * 16, Bs + r0 * BKB);
        }
    };

    acc_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = acc_t{};

    const int fr = lane & 31, fh = lane >> 5;
    auto compute = [&](int buf) {
        const unsigned char *As = lds + buf * STAGE_BYTES;
        const unsigned char *Bs = As + BM * BKB;
#pragma unroll
        for (int kk = 0; kk < BKB / 32; ++kk) {
            const int c = kk * 2 + fh;
            v4i a[4], bb[2];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int r = wm * 128 + mi * 32 + fr;
                a[mi] = *reinterpret_cast<const v4i *>(As + r * BKB + ((c ^ ((r >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int r = wn * 64 + ni * 32 + fr;
                bb[ni] = *reinterpret_cast<const v4i *>(Bs + r * BKB + ((c ^ ((r >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = M::mma(a[mi], bb[ni], acc[mi][ni]);
        }
    };

    // two-stage pipeline: stage t+1 streams in (LDS-DMA) while stage t is read
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
            for (int ni = 0; ni < 2; ++ni) {
#if defined(__HIP_DEVICE_COMPILE__)
                asm volatile("" ::"v"(acc[mi][ni]));
#endif
            }
        return;
    }
    // ---- epilogue: fit mask + per-pod top-4
    u64 key[2][4];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        Top4 t4;
        t4.init();
        unsigned best1 = 0xffffffffu, bnode1 = 0xffffffffu;
        const int pod = p0 + nt * BN + wn * 64 + ni * 32 + fr;
#pragma unroll
        for (int mi2 = 0; mi2 < 2; ++mi2) {
            const int chunk = (mt * BM + wm * 128 + mi2 * 64) >> 6;
            const u64 mw = mask[(size_t)chunk * Pp + pod];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int mi = mi2 * 2 + h;
                const unsigned bits = (unsigned)(mw >> (32 * h));
                const unsigned node0 = (unsigned)(node_base + mt * BM + wm * 128 + mi * 32);
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * fh;
                    // not fitting -> cost all-ones, never inserted (branch-free)
                    const unsigned x = M::okey(acc[mi][ni][reg]) | ((((bits >> row) & 1u) ^ 1u) * 0xffffffffu);
                    if constexpr (EPI == 2) {
                        const bool b = x < best1;
                        best1 = b ? x : best1;
                        bnode1 = b ? node0 + row : bnode1;
                    } else {
                        t4.insert(x, node0 + row);
                    }
                }
            }
        }
        if constexpr (EPI == 2) t4.c[0] = best1, t4.n[0] = bnode1;
#pragma unroll
        for (int j = 0; j < 4; ++j) key[ni][j] = t4.c[j] == 0xffffffffu ? KEY_INVALID : t4.key(j);
        // lanes l and l^32 hold the same pod, complementary node rows
        u64 o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = shfl_xor64(key[ni][j], 32);
        merge4(key[ni], o);
    }

    // merge the two node-half waves (wm = 0, 1) through LDS
    u64 *xk = reinterpret_cast<u64 *>(lds);  // [wn][ni][32][4], staging is dead
    if (wm == 1 && fh == 0) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j) xk[((wn * 2 + ni) * 32 + fr) * 4 + j] = key[ni][j];
    }
    __syncthreads();
    if (wm == 0) {
        const int ni = fh;  // lane < 32 -> pods wn*64 + 0..31, lane >= 32 -> +32..63
        u64 mine[4], other[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            mine[j] = ni ? key[1][j] : key[0][j];
            other[j] = xk[((wn * 2 + ni) * 32 + fr) * 4 + j];
        }
        merge4(mine, other);
        const int pod = p0 + nt * BN + wn * 64 + lane;
        u64 *dst = partial + ((size_t)mt * Pp + pod) * KC;
        *reinterpret_cast<ulonglong2 *>(dst) = make_ulonglong2(mine[0], mine[1]);
        *reinterpret_cast<ulonglong2 *>(dst + 2) = make_ulonglong2(mine[2], mine[3]);
    }
}

// merge n_lists sorted 4-lists per pod: src[l * stride + p * 4 + j]
__global__ void k_merge(const u64 *__restrict__ src, int n_lists, long long stride, int src_p0,
                        int p0, int np, u64 *__restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const int p = p0 + i;
    const size_t ps = (size_t)(p - src_p0) * KC;
    u64 a[4], bb[4];
    const ulonglong2 *s = reinterpret_cast<const ulonglong2 *>(src + ps);
    ulonglong2 x = s[0], y = s[1];
    a[0] = x.x; a[1] = x.y; a[2] = y.x; a[3] = y.y;
    for (int l = 1; l < n_lists; ++l) {
        const ulonglong2 *t = reinterpret_cast<const ulonglong2 *>(src + l * stride + ps);
        x = t[0]; y = t[1];
        bb[0] = x.x; bb[1] = x.y; bb[2] = y.x; bb[3] = y.y;
        merge4(a, bb);
    }
    ulonglong2 *d = reinterpret_cast<ulonglong2 *>(dst + (size_t)p * KC);
    d[0] = make_ulonglong2(a[0], a[1]);
    d[1] = make_ulonglong2(a[2], a[3]);
}

__global__ void k_unpack(const u64 *__restrict__ keys, int p0, int np, int *__restrict__ node,
                         int *__restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const int p = p0 + i;
    int c = 0;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
        const u64 k = keys[(size_t)p * KC + j];
        const bool ok = k != KEY_INVALID;
        node[(size_t)p * KC + j] = ok ? (int)(unsigned)k : -1;
        c += ok;
    }
    cnt[p] = c;
}

#ifdef NAS_DIAG_VARIANTS
template __global__ void k_cost_topk<NAS_DT_I8, 1>(const unsigned char *, const unsigned char *, int,
                                                   int, int, int, int, const u64 *, u64 *, int);
template __global__ void k_cost_topk<NAS_DT_I8, 2>(const unsigned char *, const unsigned char *, int,
                                                   int, int, int, int, const u64 *, u64 *, int);
#endif

template <int DT>
hipError_t launch_cost_t(hipStream_t st, const void *Lt, const void *WA, int Mp, int Kb, int Pp,
                         int p0, int np, const uint64_t *mask, uint64_t *partial, int node_base) {
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_cost_topk<DT>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const int n_mt = Mp / BM, n_nt = np / BN;
    k_cost_topk<DT><<<n_mt * n_nt, THREADS, LDS_BYTES, st>>>(
        static_cast<const unsigned char *>(Lt), static_cast<const unsigned char *>(WA), Kb, n_mt,
        n_nt, p0, Pp, reinterpret_cast<const u64 *>(mask), reinterpret_cast<u64 *>(partial),
        node_base);
    return hipGetLastError();
}

}  // namespace

// Kp: padded contraction length in ELEMENTS; np: pods, multiple of BN,
// p0 + np <= Pp; Mp multiple of BM.
hipError_t launch_cost_topk(hipStream_t st, int dtype, const void *Lt, const void *WA, int Mp,
                            int Kp, int Pp, int p0, int np, const uint64_t *mask,
                            uint64_t *partial, int node_base) {
    if (np <= 0) return hipSuccess;
    if (Mp % BM || np % BN || p0 + np > Pp) return hipErrorInvalidValue;
    if (dtype == NAS_DT_I8) {
        if (Kp % BKB) return hipErrorInvalidValue;
        return launch_cost_t<NAS_DT_I8>(st, Lt, WA, Mp, Kp, Pp, p0, np, mask, partial, node_base);
    }
    if ((2 * Kp) % BKB) return hipErrorInvalidValue;
    return launch_cost_t<NAS_DT_BF16>(st, Lt, WA, Mp, 2 * Kp, Pp, p0, np, mask, partial, node_base);
}

hipError_t launch_merge(hipStream_t st, const uint64_t *partial, int n_lists, int64_t list_stride,
                        int src_p0, int p0, int np, uint64_t *cand_key) {
    if (np <= 0) return hipSuccess;
    k_merge<<<(np + 255) / 256, 256, 0, st>>>(reinterpret_cast<const u64 *>(partial), n_lists,
                                                list_stride, src_p0, p0, np,
                                                reinterpret_cast<u64 *>(cand_key));
    return hipGetLastError();
}

hipError_t launch_unpack(hipStream_t st, const uint64_t *cand_key, int p0, int np, int dtype,
                         int32_t *cand_node, int32_t *cand_cnt) {
    (void)dtype;
    if (np <= 0) return hipSuccess;
    k_unpack<<<(np + 255) / 256, 256, 0, st>>>(reinterpret_cast<const u64 *>(cand_key), p0, np,
                                                 cand_node, cand_cnt);
    return hipGetLastError();
}

}  // namespace nas
