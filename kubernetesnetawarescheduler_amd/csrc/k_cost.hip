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
//  * bf16 path: v_mfma_f32_16x16x32_bf16 (the 16x16 shape: 3.5% faster than
//    32x32x16 here, see mfma16()), fp32 accumulation; also the fp32 path,
//    whose operands are split into three bf16 planes each and laid out along
//    a six-fold K (k_misc.hip k_split6: products to 2^-24 relative).
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
// Epilogue: per lane, 64 (node, cost) values per pod (32 with the 16x16
// shape) -> mask from the fit kernel (bit per node) -> sorted top-4 of
// (orderable cost, node) in registers -> merged with the lanes holding the
// same pod (lane^32; 16x16: lane^16, then lane^32) into an 8-list with an
// exactness bound (klist.h) -> merged across the two node-half waves through
// LDS -> partial[node_tile][pod][8] + pbound[node_tile][pod] (72 B per pod
// per tile).
#include "klist.h"

#include <type_traits>

namespace nas {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BM = COST_BM;   // nodes per tile
constexpr int BN = COST_BN;   // pods per tile
constexpr int BKB = COST_BKB; // bytes of K per LDS stage (full 128-byte lines)
// XCD tile order, pod-group major: PG pod tiles x every node tile per group,
// so an XCD keeps one pod group's traffic rows hot in the memory-side cache
// while it sweeps the node tiles.  256 x 256: groups of 4 (32 concurrent
// workgroups per XCD = 8 node tiles x 4 pod tiles), 2.0-2.5% faster than
// node-group-major 4 (profiles/r02_mb_cost_order.log); the wide tile: groups
// of 2, C3 pass 8.04-8.09 vs 8.09-8.12 ms for groups of 4 (launch equal;
// groups of 1 / 3 / 8 and node-group-major 2 / 8 slower,
// profiles/r02_s4_ab_gm.txt, r03_ab_gm_wide.txt).  The measured-and-rejected
// variants of this kernel (other pipelines, schedules, one wave per SIMD,
// cache policies) live in tools/k_cost_diag.hip.
constexpr int PG_NARROW = 4;
constexpr int PG_WIDE = 2;
// wave layouts: NWN = 4 -> 256 x 256 per 8-wave workgroup (2 node halves x 4
// pod quarters, each wave 128 nodes x 64 pods = 4 x 2 MFMA 32x32 tiles, 128
// accumulator registers, two waves per SIMD, 128 KiB LDS double buffer);
// NWN = 6 -> the wide tile, 256 x 384 per 12-wave workgroup (3 waves per
// SIMD of the same 128 x 64 shape, 160 KiB LDS double buffer), 17% fewer
// staged bytes per MAC, for the main scoring pass of one large cluster
constexpr int WIDE_PODS = 384;
// (8 waves of 128 x 96 per wave for the wide tile -- two per SIMD, 22% fewer
// LDS fragment reads per MAC -- measured 0.3% slower per C3 launch and 2%
// per pass in int8, 2.5% slower in bf16, 3-5% slower on C5:
// profiles/r05b_ab_mfma_shape.txt)
// MFMA shape per dtype (same box, alternating, profiles/r05b_ab_mfma_shape.txt):
// bf16 runs v_mfma_f32_16x16x32_bf16 -- the C3 launch 13.40 -> 12.95 ms (0.593
// -> 0.614 of the bf16 peak): the chip holds a higher clock on the 16x16
// shape under this power-limited loop (MI355X_MICROARCH.md, DVFS give-back
// item 7) -- while int8 stays on v_mfma_i32_32x32x32_i8 (16x16x64: launch
// 6.91 -> 7.26 ms, C5 0.45 -> 0.40)
template <int DT>
constexpr bool mfma16() { return DT == NAS_DT_BF16; }
template <int DT>
struct Mma;

template <>
struct Mma<NAS_DT_I8> {
    using acc_t = v16i;
    using acc4_t = v4i;
    static __device__ __forceinline__ acc_t mma(v4i a, v4i b, acc_t c) {
        return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ acc4_t mma16(v4i a, v4i b, acc4_t c) {
        return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ unsigned okey(int x) { return (unsigned)x ^ 0x80000000u; }
};

template <>
struct Mma<NAS_DT_BF16> {
    using acc_t = v16f;
    using acc4_t = v4f;
    static __device__ __forceinline__ acc_t mma(v4i a, v4i b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                        __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ acc4_t mma16(v4i a, v4i b, acc4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                        __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ unsigned okey(float x) {
        x = x + 0.0f;  // -0 -> +0: the oracle compares costs, not sign bits
        const unsigned u = __float_as_uint(x);
        return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    }
};

// 16-byte LDS-DMA (global_load_lds_dwordx4), default cache policy (sc1,
// sc0 sc1 measured equal; nt slower: tools/k_cost_diag.hip COST_AUX_*)
__device__ __forceinline__ void glds16(const void *g, void *l) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)g,
                                     (void __attribute__((address_space(3))) *)l, 16, 0, 0);
}

// The same 16-byte LDS-DMA in its saddr form: a wave-uniform 64-bit base in
// SGPRs plus a 32-bit per-lane offset, so every piece of a wave shares ONE
// offset VGPR (the builtin keeps a 64-bit VGPR address per piece live across
// the loop).  M0 (the LDS destination, wave-uniform) is saved and restored in
// the statement.  hipcc does not count these loads: the K-loop retires them
// with its explicit vmcnt(0) before each barrier.
__device__ __forceinline__ unsigned lds_off(const void *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void glds16_s(const void *sbase, unsigned voff, unsigned ldsa) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(ldsa)
                 : "memory");
}

__device__ __forceinline__ unsigned umed3(unsigned a, unsigned b, unsigned c) {
    unsigned d;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// Instantiations (launch_cost_t): NWN = 4 (256 x 256) with the k_fit mask
// (node shards, rescore windows), with the fused fit (FUSE: main pod ranges at
// world 1, batches) or with a row map (RMAP); NWN = 6 (the wide tile, always
// fused).  The k-substep schedule is hipcc's own (pinned interleaves,
// setprio and iglp_opt measured within +-1%: tools/k_cost_diag.hip SCHED).
// RMAP: a gathered rescore view -- view row q's traffic is WA row rowmap[q]
// (read in place by the LDS-DMA source addresses; rows past the view's count
// read its last row and are never merged)
template <int DT, bool RMAP, int NWN, bool FUSE>
__global__ void __launch_bounds__(128 * NWN, 1)
k_cost_topk(const unsigned char *__restrict__ Lt, const unsigned char *__restrict__ WA, int Kb,
            int n_mt, int n_nt, int p0, int Pp, const u64 *__restrict__ mask,
            u64 *__restrict__ partial, u64 *__restrict__ pbound, int node_base,
            const int *__restrict__ dyn_start, int dyn_hi, const int *__restrict__ dyn_hi_ptr,
            Ovf ov, const int *__restrict__ rowmap, FitSrc fs, unsigned *__restrict__ cc) {
    static_assert(NWN == 4 || NWN == 6, "the 8- and 12-wave layouts");
    constexpr int NW = 2 * NWN;              // waves
    constexpr int NI = 2;                    // 32-pod columns per wave
    constexpr int WPODS = 32 * NI;           // pods per wave
    constexpr int BNK = NWN * WPODS;         // pods per tile (256; the wide tile 384)
    constexpr bool WIDE = BNK > BN;
    static_assert(!WIDE || (!RMAP && FUSE), "the wide tile serves the main pass only");
    static_assert(!FUSE || !RMAP, "the fused fit: main-range launches");
    constexpr int STG = (BM + BNK) * BKB;    // bytes per LDS stage
    constexpr int PG = WIDE ? PG_WIDE : PG_NARROW;
    constexpr int PPWA = (BM / 8 + NW - 1) / NW;   // 1 KiB LDS-DMA pieces of A per wave per stage
    constexpr int PPWB = (BNK / 8 + NW - 1) / NW;  // ... of B
    constexpr int PPW = PPWB;
    using M = Mma<DT>;
    using acc_t = typename M::acc_t;
    // accumulator blocks of a wave's 128 nodes x 64 pods: 4 x 2 blocks of
    // 32 x 32 (16 registers each), or with the 16x16 shape 8 x 4 blocks of
    // 16 x 16 (4 registers each); the pod is the block's column = the lane
    // (mod PB), the node its row = register (+ lane group)
    constexpr bool M16 = mfma16<DT>();
    constexpr int AM = M16 ? 8 : 4;
    constexpr int AN = M16 ? 2 * NI : NI;
    constexpr int AR = M16 ? 4 : 16;
    constexpr int PB = M16 ? 16 : 32;  // pods per block
    using accb_t = std::conditional_t<M16, typename M::acc4_t, acc_t>;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // the fused fit's words after the main loop: behind the cross-wave merge's
    // lists ([NWN][NI][32][9] u64), inside the smallest staging image
    constexpr int FIT_LDS_OFF = 32768;
    static_assert(FIT_LDS_OFF >= NWN * NI * 32 * 9 * 8 &&
                  FIT_LDS_OFF + NW * AN * 2 * 64 * 8 <= 2 * STG, "fused-fit LDS words");

    // ---- XCD-aware tile order: blocks b, b+8, ... share an XCD (speed only)
    const int nwg = n_mt * n_nt;
    const int b = blockIdx.x;
    const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    // pod-group major: PG pod tiles x every node tile per group
    const int gsize = PG * n_mt;
    const int g = v / gsize, r = v % gsize;
    const int first_nt = g * PG;
    const int pg = min(n_nt - first_nt, PG);
    const int mt = r / pg;
    const int nt = first_nt + r % pg;
    const int cb = blockIdx.y;  // cluster of a batched launch
    if constexpr (FUSE) {
        fs.cap += (size_t)cb * 3 * fs.N;
        fs.req += (size_t)cb * 3 * Pp;
    }
    Lt += (size_t)cb * n_mt * BM * Kb;  // (tile order above: speed only)
    WA += (size_t)cb * Pp * Kb;
    mask += (size_t)cb * (n_mt * BM / 64) * Pp;
    partial += (size_t)cb * n_mt * Pp * KC;
    pbound += (size_t)cb * n_mt * Pp;
    if (dyn_start) {  // rescore slot: pod tiles from the window start in device memory
        const int s = dyn_start[cb * STATUS_INTS];
        if (s < 0) return;
        if (dyn_hi_ptr) dyn_hi = dyn_hi_ptr[cb * STATUS_INTS];
        p0 = s / BN * BN;
        if (p0 + nt * BNK >= dyn_hi) return;  // whole block: before any barrier
    }
    // the wide tile (BNK = 384 over a launch of 256-pod units): pods at and
    // past p_end (= dyn_hi, the launch's end) read rows past it (the next
    // launch's, or the WA_PAD_ROWS padding) and are never written
    const int p_end = (BNK != BN && !dyn_start) ? dyn_hi : 0x7fffffff;

    // (the wide tile: the wave index wave-uniform in SGPRs, and the lane index
    // re-derived after the main loop -- see below -- so that nothing per-lane
    // outlives the loop beside the 128 accumulators: at three waves per SIMD
    // the loop fills the 168 registers, and values held across it spilled)
    const int tid = threadIdx.x;
    int lane = tid & 63;
    const int w = WIDE ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
    const int wm = w / NWN, wn = w % NWN;

    const unsigned char *Ag = Lt + (size_t)mt * BM * Kb;
    const unsigned char *Bg = WA + (size_t)(p0 + nt * BNK) * Kb;

    // LDS-DMA staging: piece j of wave w fills rows (NW*j + w)*8 .. +8 of A
    // and of B (1 KiB each, lane-linear: lane l -> row + l/8, 16-byte chunk
    // l%8; whole 128-byte lines per row -- 64-byte row pieces measured 12%
    // slower); the chunk swizzle chunk ^= (row >> 1) & 7 is applied on the
    // SOURCE address so fragment reads are bank-conflict free.
    const int srow_in = lane >> 3;
    const int sq = lane & 7;
    // stage b of the double buffer: the A (latency) rows, then the B (traffic) rows
    auto abuf = [&](int b) -> unsigned char * { return lds + b * STG; };
    auto bbuf = [&](int b) -> unsigned char * { return lds + b * STG + BM * BKB; };
    // one 1 KiB LDS-DMA piece (8 rows x 128 B) of operand A / B: piece j of
    // wave w fills rows (NW*j + w)*8 .. +8
    // (saddr form: rows r0 + l/8 of a piece all swizzle by
    // (4 * (r0 / 8) + l / 16) & 7 = (4 * (w & 1) + l / 16) & 7 -- NW is even --,
    // so one lane offset serves every piece of the wave, A and B alike)
    const unsigned loffn = (unsigned)(srow_in * Kb) +
                           ((unsigned)(sq ^ ((4 * (w & 1) + (srow_in >> 1)) & 7)) << 4);
    auto pieceA = [&](int buf, int k0, int j) {
        if (BM / 8 % NW && j * NW + w >= BM / 8) return;
        const int r0 = (j * NW + w) * 8;
        const int ru = __builtin_amdgcn_readfirstlane(r0);
        glds16_s(Ag + (size_t)ru * Kb + k0, loffn,
                 __builtin_amdgcn_readfirstlane(lds_off(abuf(buf) + r0 * BKB)));
    };
    int bpod[PPW];  // RMAP: the WA rows of this lane's B pieces
    if constexpr (RMAP) {
#pragma unroll
        for (int j = 0; j < PPW; ++j)
            bpod[j] = rowmap[min(p0 + nt * BNK + (j * NW + w) * 8 + srow_in, dyn_hi - 1)];
    }
    auto pieceB = [&](int buf, int k0, int j) {
        if (BNK / 8 % NW && j * NW + w >= BNK / 8) return;
        const int r0 = (j * NW + w) * 8;
        if constexpr (!RMAP) {
            const int ru = __builtin_amdgcn_readfirstlane(r0);
            glds16_s(Bg + (size_t)ru * Kb + k0, loffn,
                     __builtin_amdgcn_readfirstlane(lds_off(bbuf(buf) + r0 * BKB)));
            return;
        }
        const int row = r0 + srow_in;
        const int c = sq ^ ((row >> 1) & 7);
        const unsigned char *src = RMAP ? WA + (size_t)bpod[j] * Kb : Bg + (size_t)row * Kb;
        glds16(src + k0 + c * 16, bbuf(buf) + r0 * BKB);
    };
    // the wide tile stages A rows then B rows as one run of 80 pieces (the
    // B image follows the A image in LDS); piece pj of wave wu is 8 rows at
    // pj * 8, and since pj = 12 j + wu has the parity of wu, every piece of a
    // wave has the same swizzled lane offset: one VGPR, the row base uniform
    // (3 waves per SIMD leave 168 registers, 128 of them accumulators)
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const unsigned loff = (unsigned)(srow_in * Kb) +
                          ((unsigned)(sq ^ ((4 * (wu & 1) + (srow_in >> 1)) & 7)) << 4);
    auto piece6 = [&](int buf, int k0, int j) {
        const int pj = j * NW + wu;
        if (pj >= (BM + BNK) / 8) return;
        const unsigned char *base = pj < BM / 8 ? Ag + (size_t)pj * 8 * Kb
                                                : Bg + (size_t)(pj - BM / 8) * 8 * Kb;
        glds16_s(base + k0, loff, __builtin_amdgcn_readfirstlane(lds_off(lds + buf * STG + pj * 8 * BKB)));
    };
    auto stageA = [&](int buf, int k0) {
        if constexpr (WIDE) {
#pragma unroll
            for (int j = 0; j < ((BM + BNK) / 8 + NW - 1) / NW; ++j) piece6(buf, k0, j);
        } else {
#pragma unroll
            for (int j = 0; j < PPWA; ++j) pieceA(buf, k0, j);
        }
    };
    auto stageB = [&](int buf, int k0) {
        if constexpr (!WIDE) {  // (the wide tile's stageA stages both)
#pragma unroll
            for (int j = 0; j < PPW; ++j) pieceB(buf, k0, j);
        }
    };

    // Fused fit (main-range launches: the pass's chunks launch back to back
    // with no k_fit between them -- a fit launch in front of every cost
    // launch could not start until a wide workgroup drained its CU, and the
    // cost launch behind it then waited too).  The workgroup decides the fit
    // words itself, exactly as k_fit does, after its main loop: per 64-node
    // chunk the minima / maxima of the free capacity (read then -- after the
    // previous chunks' commits and possibly during this chunk's predecessor's;
    // capacity only shrinks, so a "does not fit" read at any earlier time
    // still holds at the pod's turn) decide every pod that fits all valid
    // nodes or none; the rest compare against the lanes' capacities (three
    // ballots).  The words land where the k_fit mask words would (mwp).
    int rq[FUSE ? AN : 1][3];
    int fcap[2][3];
    auto fit_issue = [&]() {  // the requests of the lane's pods, its nodes' capacities
#pragma unroll
        for (int ni = 0; ni < AN; ++ni) {
            const int pod = min(p0 + nt * BNK + wn * WPODS + ni * PB + (lane & (PB - 1)), p_end - 1);
#pragma unroll
            for (int r = 0; r < 3; ++r) rq[ni][r] = fs.req[(size_t)r * Pp + pod];
        }
#pragma unroll
        for (int mi2 = 0; mi2 < 2; ++mi2) {
            const int nl = mt * BM + wm * 128 + mi2 * 64 + lane;
#pragma unroll
            for (int r = 0; r < 3; ++r)
                fcap[mi2][r] = nl < fs.nloc ? __hip_atomic_load(const_cast<int *>(fs.cap) + (size_t)r * fs.N + fs.n0 + nl,
                                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                            : -1;
        }
    };
    // fit words: bit j of word (ni, mi2) = the lane's pod of group ni fits
    // node wm*128 + mi2*64 + j of the tile; each lane stores its own words in
    // LDS (fit_slot, past the cross-wave merge's region) and reads them back
    // per pod group in the epilogue (held in registers beside the 128
    // accumulators they spilled: 24 B of scratch per lane)
    auto fit_slot = [&](int ni, int mi2) -> u64 * {
        return reinterpret_cast<u64 *>(lds + FIT_LDS_OFF) + ((w * AN + ni) * 2 + mi2) * 64 + lane;
    };
    auto fit_words = [&]() {
#pragma unroll
        for (int mi2 = 0; mi2 < 2; ++mi2) {
            const bool real = mt * BM + wm * 128 + mi2 * 64 + lane < fs.nloc;
            const u64 valid = __builtin_amdgcn_ballot_w64(real);
            int mn[3], mx[3];
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                int a = real ? fcap[mi2][r] : 0x7fffffff, x = real ? fcap[mi2][r] : (int)0x80000000;
#pragma unroll
                for (int o = 32; o; o >>= 1) {
                    a = min(a, __shfl_xor(a, o));
                    x = max(x, __shfl_xor(x, o));
                }
                mn[r] = __builtin_amdgcn_readfirstlane(a);
                mx[r] = __builtin_amdgcn_readfirstlane(x);
            }
#pragma unroll
            for (int ni = 0; ni < AN; ++ni) {
                const int a = rq[ni][0], bq = rq[ni][1], d = rq[ni][2];
                const bool all = a <= mn[0] && bq <= mn[1] && d <= mn[2];
                const bool none = a > mx[0] || bq > mx[1] || d > mx[2];
                u64 word = all ? valid : 0ull;
                // lanes l and l + PB (+ 2 PB, 3 PB) hold the same pod: decide
                // lanes 0..PB-1
                u64 rest = __builtin_amdgcn_ballot_w64(!all && !none) & ((1ull << PB) - 1);
                while (rest) {
                    const int i = (int)__builtin_ctzll(rest);
                    rest &= rest - 1;
                    const int ra = __builtin_amdgcn_readlane(a, i), rb = __builtin_amdgcn_readlane(bq, i);
                    const int rd = __builtin_amdgcn_readlane(d, i);
                    const u64 m = __builtin_amdgcn_ballot_w64(ra <= fcap[mi2][0]) &
                                  __builtin_amdgcn_ballot_w64(rb <= fcap[mi2][1]) &
                                  __builtin_amdgcn_ballot_w64(rd <= fcap[mi2][2]);
                    if ((lane & (PB - 1)) == i) word = m;
                }
                *fit_slot(ni, mi2) = word;
            }
        }
    };

    // the epilogue's fit-mask words, loaded now so their latency hides
    // under the main loop (k_fit wrote them before this launch)
    // (issued after the overflow seeding, whose loop they would otherwise
    // stay live across)
    u64 mwp[AN][2];
    auto load_mask = [&]() __attribute__((always_inline)) {
        if constexpr (!FUSE) {
#pragma unroll
            for (int ni = 0; ni < AN; ++ni)
#pragma unroll
                for (int mi2 = 0; mi2 < 2; ++mi2) {
                    const int pod = min(p0 + nt * BNK + wn * WPODS + ni * PB + (lane & (PB - 1)), p_end - 1);
                    const int chunk = (mt * BM + wm * 128 + mi2 * 64) >> 6;
                    mwp[ni][mi2] = mask[(size_t)chunk * Pp + pod];
                }
        }
    };
    accb_t acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) acc[i][j] = accb_t{};
    // fr: the lane's pod within a block; fh: its row group (rows 4 fh ..)
    int fr = lane & (PB - 1), fh = lane / PB;
    // ---- exact int32 traffic: the entries outside the int8 plane (nas::Ovf):
    // e * L[m][n] for the lane's 64 nodes per pod are the accumulators'
    // initial value (4 dwords of Lr per 32-node tile: rows (reg & 3) +
    // 8 * (reg >> 2) + 4 * fh are 4 groups of 4 consecutive nodes).  Both pod
    // groups' list bounds load together, and an entry's 16 row dwords (all
    // four 32-node tiles) in one round, so an entry costs two dependent
    // loads, not eight; the two-stage pipeline runs this behind its first
    // stage's LDS-DMA (the prologue waits once for both)
    // (the layout of rounds 1-2, inline: the wide tile, whose registers allow
    // one tile's row dwords at a time, and the 256 x 256 launches without the
    // fused fit -- node shards, rescore windows -- which must stay at <= 192
    // VGPRs: a node shard's merge / all-gather / commit kernels run beside a
    // cost workgroup only while its two waves per SIMD leave registers free
    // (at 256 VGPRs the G = 8 rehearsal pass rose from 1.39 to 1.50 ms:
    // profiles/r03_bisect_g8.txt))
    constexpr bool OVF_ROUND2 = WIDE || !FUSE;
    if constexpr (OVF_ROUND2 && DT == NAS_DT_I8) {
        if (ov.ptr) {
            const int cnt_lim = ov.row_count ? *ov.row_count : 0x7fffffff;
            const signed char *lr = ov.Lr + (size_t)cb * ov.N * (n_mt * BM) + mt * BM + wm * 128 + 4 * fh;
#pragma unroll
            for (int ni = 0; ni < AN; ++ni) {
                const int r = p0 + nt * BNK + wn * WPODS + ni * PB + fr;
                int beg = 0, end = 0;
                if (r < cnt_lim && r < p_end) {
                    const int pod = (ov.row_pod ? ov.row_pod[r] : r) + cb * Pp;
                    beg = ov.ptr[pod];
                    end = ov.ptr[pod + 1];
                }
#pragma unroll
                for (int mi = 0; mi < AM; ++mi)
                    for (int j = beg; j < end; ++j) {
                        const int e = ov.e[j];
                        const signed char *row = lr + (size_t)ov.m[j] * (n_mt * BM) + mi * (128 / AM);
#pragma unroll
                        for (int g = 0; g < AR / 4; ++g) {
                            const int v = *reinterpret_cast<const int *>(row + 8 * g);
#pragma unroll
                            for (int c = 0; c < 4; ++c)
                                acc[mi][ni][4 * g + c] += e * (int)(signed char)(v >> (8 * c));
                        }
                    }
            }
        }
    }
    auto seed_ovf = [&]() __attribute__((always_inline)) {
        if constexpr (!OVF_ROUND2 && DT == NAS_DT_I8) {
            if (ov.ptr) {
                const int cnt_lim = ov.row_count ? *ov.row_count : 0x7fffffff;
                const signed char *lr = ov.Lr + (size_t)cb * ov.N * (n_mt * BM) + mt * BM + wm * 128 + 4 * fh;
                // pod group ni's entries [beg, end)
                auto bounds = [&](int ni, int &beg, int &end) {
                    const int r = p0 + nt * BNK + wn * WPODS + ni * PB + fr;
                    beg = end = 0;
                    if (r < cnt_lim && r < p_end) {
                        const int pod = (ov.row_pod ? ov.row_pod[r] : r) + cb * Pp;
                        beg = ov.ptr[pod];
                        end = ov.ptr[pod + 1];
                    }
                };
                {
                    int beg[AN], end[AN];
#pragma unroll
                    for (int ni = 0; ni < AN; ++ni) bounds(ni, beg[ni], end[ni]);
#pragma unroll
                    for (int ni = 0; ni < AN; ++ni)
                        for (int j = beg[ni]; j < end[ni]; ++j) {
                            const int e = ov.e[j];
                            const signed char *row = lr + (size_t)ov.m[j] * (n_mt * BM);
                            int v[AM][AR / 4];
#pragma unroll
                            for (int mi = 0; mi < AM; ++mi)
#pragma unroll
                                for (int g = 0; g < AR / 4; ++g)
                                    v[mi][g] = *reinterpret_cast<const int *>(row + mi * (128 / AM) + 8 * g);
#pragma unroll
                            for (int mi = 0; mi < AM; ++mi)
#pragma unroll
                                for (int g = 0; g < AR / 4; ++g)
#pragma unroll
                                    for (int c = 0; c < 4; ++c)
                                        acc[mi][ni][4 * g + c] += e * (int)(signed char)(v[mi][g] >> (8 * c));
                        }
                }
            }
        }
    };
    if constexpr (WIDE) load_mask();

    // fragments of k-substep kk+1 are read from LDS while the 8 MFMAs of kk
    // run (register double buffer)
    auto compute = [&](int buf) {
        const unsigned char *As = abuf(buf);
        const unsigned char *Bs = bbuf(buf);
        if constexpr (M16) {
            // 16x16x64 (i8) / 16x16x32 (bf16): a fragment is 16 rows x 64 B of
            // K, lane l holding row l & 15, bytes 16 (l >> 4) .. +16 of the
            // substep's 64 (the same map on both operands, so the product
            // sums every k once); chunk 4 kk + fh swizzled by (row >> 1) & 7,
            // i.e. ((fh ^ s) << 4) ^ (kk << 6) past the row base: conflict-free
            // ds_read_b128 in its 16-lane groups (rows 0-3/12-15 of one chunk
            // with rows 4-11 of the next)
            const unsigned sw = (unsigned)((fh ^ ((fr >> 1) & 7)) << 4);
            const unsigned ao0 = (unsigned)((wm * 128 + fr) * BKB) + sw;
            const unsigned bo0 = (unsigned)((wn * WPODS + fr) * BKB) + sw;
#pragma unroll
            for (int kk = 0; kk < BKB / 64; ++kk) {
                const unsigned ao = ao0 ^ (unsigned)(kk << 6), bo = bo0 ^ (unsigned)(kk << 6);
                v4i bq[AN];
#pragma unroll
                for (int ni = 0; ni < AN; ++ni)
                    bq[ni] = *reinterpret_cast<const v4i *>(Bs + bo + ni * 16 * BKB);
#pragma unroll
                for (int mi = 0; mi < AM; ++mi) {
                    const v4i aq = *reinterpret_cast<const v4i *>(As + ao + mi * 16 * BKB);
#pragma unroll
                    for (int ni = 0; ni < AN; ++ni) acc[mi][ni] = M::mma16(aq, bq[ni], acc[mi][ni]);
                }
            }
            return;
        } else {
        v4i a[2][4], bb[2][NI];
        // fragment (kk, mi) of row r = base + mi * 32 + fr sits at r * BKB +
        // ((2 kk + fh) ^ ((r >> 1) & 7)) * 16 = (row0 * BKB + ((fh ^ s) << 4)) ^
        // (kk << 5) + mi * 4096 with s = (fr >> 1) & 7 (the same for every mi,
        // ni and both operands): one lane offset per operand, an XOR per
        // substep and immediate offsets
        auto read = [&](int kk, v4i (&ra)[4], v4i (&rb)[NI]) {
            const unsigned ao = ((unsigned)((wm * 128 + fr) * BKB) + (unsigned)((fh ^ ((fr >> 1) & 7)) << 4)) ^ (unsigned)(kk << 5);
            const unsigned bo = ((unsigned)((wn * WPODS + fr) * BKB) + (unsigned)((fh ^ ((fr >> 1) & 7)) << 4)) ^ (unsigned)(kk << 5);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
                ra[mi] = *reinterpret_cast<const v4i *>(As + ao + mi * 32 * BKB);
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
                rb[ni] = *reinterpret_cast<const v4i *>(Bs + bo + ni * 32 * BKB);
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
        }
    };

    // two-stage pipeline: stage t+1 streams in (LDS-DMA) while t is read
    const int nk = Kb / BKB;
    stageA(0, 0);
    stageB(0, 0);
    seed_ovf();
    if constexpr (!WIDE) load_mask();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        if (t + 1 < nk) {
            stageA(cur ^ 1, (t + 1) * BKB);
            stageB(cur ^ 1, (t + 1) * BKB);
        }
        compute(cur);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    if constexpr (WIDE) {
        // the lane index afresh (volatile: not CSE'd with the prologue's), so
        // the old one dies in the loop
        int l;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
        lane = l;
        fr = l & (PB - 1);
        fh = l / PB;
    }
    if (cc) {
        // the cost-row cache (gathered rescores of a herd read it instead of
        // recomputing the contraction, k_rescore.hip k_rescore_cached): every
        // (pod, local node) value as its orderable 32-bit key, row-major
        // [cluster][Pp][Mp]; a lane's four consecutive nodes per 16-byte
        // store, and the lanes of one pod (l, l ^ 32; 16x16 also l ^ 16,
        // l ^ 48) fill whole 128-byte lines of its row between them, which
        // the L2 combines before they go to HBM
        unsigned *crow = cc + (size_t)cb * Pp * (n_mt * BM) + mt * BM + wm * 128;
#pragma unroll
        for (int ni = 0; ni < AN; ++ni) {
            const int pod = p0 + nt * BNK + wn * WPODS + ni * PB + fr;
            if (pod >= p_end) continue;
            unsigned *d = crow + (size_t)pod * (n_mt * BM);
#pragma unroll
            for (int mi = 0; mi < AM; ++mi)
#pragma unroll
                for (int g = 0; g < AR / 4; ++g) {
                    uint4 v;
                    v.x = M::okey(acc[mi][ni][4 * g + 0]);
                    v.y = M::okey(acc[mi][ni][4 * g + 1]);
                    v.z = M::okey(acc[mi][ni][4 * g + 2]);
                    v.w = M::okey(acc[mi][ni][4 * g + 3]);
                    *reinterpret_cast<uint4 *>(d + (M16 ? mi * 16 + 4 * fh : mi * 32 + 8 * g + 4 * fh)) = v;
                }
        }
    }
    if constexpr (FUSE) {
        // the fused fit, after the main loop: nothing of it is live across
        // the loop (held there, its registers pushed the loop's LDS-DMA
        // addresses into scratch: the launch ran 12-24% slower); the loads'
        // latency (~1 us of L2) is exposed once per workgroup
        fit_issue();
        fit_words();
    }
    // ---- epilogue: fit mask + per-pod candidate list
    // per lane: top-4 of its 64 (32 with the 16x16 shape) (node, cost) values
    // per pod; the lanes holding the same pod (complementary rows: l, l^32;
    // 16x16: l, l^16, l^32, l^48) merge into a sorted 8-list whose bound is
    // the smallest of the 4th keys (every key <= bound is in the list)
    // value (mi, reg) of the lane: node offset within the wave's 128 (in
    // increasing order of the slot mi * AR + reg), and its fit bit = that
    // offset's bit of fit word off >> 6
    auto noff = [&](int mi, int reg) -> int {
        return M16 ? mi * 16 + 4 * fh + reg : mi * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * fh;
    };
    // 16x16: each pod block's merged list goes to LDS as soon as it is made
    // (lists of both node halves, [wm][wn][pod][9] u64, past the fused fit's
    // words: the second staging image is dead), so no block's list stays in
    // registers beside the accumulators (held there, they spilled)
    constexpr int XL_OFF = FIT_LDS_OFF + NW * AN * 2 * 64 * 8;
    static_assert(!M16 || XL_OFF + 2 * NWN * WPODS * 9 * 8 <= 2 * STG, "16x16 list image");
    u64 *xl = reinterpret_cast<u64 *>(lds + XL_OFF);
    u64 key[M16 ? 1 : AN][8], bnd[M16 ? 1 : AN];
#pragma unroll
    for (int ni = 0; ni < AN; ++ni) {
        u64 (&kl)[8] = key[M16 ? 0 : ni];
        u64 &bl = bnd[M16 ? 0 : ni];
        u64 mwf[2];
        if constexpr (FUSE) {
#pragma unroll
            for (int mi2 = 0; mi2 < 2; ++mi2) mwf[mi2] = *fit_slot(ni, mi2);
        }
        const u64 *mw = FUSE ? mwf : mwp[ni];
        // orderable keys of the lane's (node, cost) values and their range
        // (int8: the range of the raw int32 costs -- the key is x ^ 2^31, so
        // key differences are cost differences)
        unsigned u[AM][AR];
        unsigned kmin = 0xffffffffu, kmax = 0u;
        int smin = 0x7fffffff, smax = -0x7fffffff - 1;
#pragma unroll
        for (int mi = 0; mi < AM; ++mi)
#pragma unroll
            for (int reg = 0; reg < AR; ++reg) {
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
        // the lane's fit bits of block mi, bit (M16: reg; else row(reg)) of a
        // 32-bit word: M16 the lane's nibble, else the block's 32-node half
        auto block_bits = [&](int mi) -> unsigned {
            if constexpr (M16)
                return (unsigned)(mw[mi >> 2] >> ((mi & 3) * 16 + 4 * fh)) & 0xfu;
            else
                return (unsigned)(mw[mi >> 1] >> (32 * (mi & 1)));
        };
        constexpr unsigned ALL_BITS = M16 ? 0xfu : 0xffffffffu;
        auto bitpos = [&](int reg) -> int { return M16 ? reg : (reg & 3) + 8 * (reg >> 2) + 4 * fh; };
        u64 k4[4];
        if (__all(kmax - kmin < (1u << 26) - 1u)) {
            // packed path (every lane's keys span < 2^26 - 1): one u32 per
            // value, (key - kmin) << 6 | i with i = mi*AR + reg increasing in
            // node order, so u32 order = (cost, node) order; a non-fitting
            // value is all-ones (never < a fitting one, < 2^32 - 1).  Sorted
            // insert of x into c0 <= .. <= c3: c3 = med3(c2, c3, x), c2 =
            // med3(c1, c2, x), c1 = med3(c0, c1, x), c0 = min(c0, x).
            unsigned c0 = 0xffffffffu, c1 = c0, c2 = c0, c3 = c0;
            // int8 with every lane's costs in [0, 2^26 - 1) (the common case:
            // non-negative traffic and latency): x = cost << 6 | i directly
            // (key base = okey(0)); otherwise relative to the lane's base
            // (int8: raw = cost bits, base = min cost; bf16: raw = key, base =
            // kmin).  Epilogue VALU per value 8 -> 5 (direct, every node of the
            // block fitting every lane's pod: one v_lshl_or_b32) / 7
            // (PMC: the epilogue is VALU-issue-bound, 1,377 instructions per
            // wave = ~10% of a C5 launch, profiles/r03_pmc_epilogue.txt)
            const bool direct = DT == NAS_DT_I8 && __all(smin >= 0 && smax < (1 << 26) - 1);
            const unsigned kbase = direct ? 0x80000000u : kmin;
            const unsigned nk6 = 0u - ((DT == NAS_DT_I8 ? (unsigned)smin : kmin) << 6);
            auto insert = [&](unsigned x) {
                c3 = umed3(c2, c3, x);
                c2 = umed3(c1, c2, x);
                c1 = umed3(c0, c1, x);
                c0 = min(c0, x);
            };
#pragma unroll
            for (int mi = 0; mi < AM; ++mi) {
                const unsigned bitsw = block_bits(mi);
                const unsigned nbits = ~bitsw;
                if (direct && __all(bitsw == ALL_BITS)) {
#pragma unroll
                    for (int reg = 0; reg < AR; ++reg)
                        insert(((unsigned)(int)acc[mi][ni][reg] << 6) | (unsigned)(mi * AR + reg));
                } else {
#pragma unroll
                    for (int reg = 0; reg < AR; ++reg) {
                        const unsigned raw = DT == NAS_DT_I8 ? (unsigned)(int)acc[mi][ni][reg]
                                                             : u[mi][reg];
                        // (raw << 6) - (base << 6) in one v_lshl_add (hipcc
                        // otherwise emits a subtract and a shift); slot and
                        // the sign-extended not-fit bit (v_bfe_i32) OR'ed in
                        unsigned y;
                        if (direct) {
                            y = raw << 6;
                        } else {
                            asm("v_lshl_add_u32 %0, %1, 6, %2" : "=v"(y) : "v"(raw), "v"(nk6));
                        }
                        insert(y | (unsigned)(mi * AR + reg) |
                               (unsigned)__builtin_amdgcn_sbfe((int)nbits, bitpos(reg), 1));
                    }
                }
            }
            const unsigned cc[4] = {c0, c1, c2, c3};
            const unsigned nb = (unsigned)(node_base + mt * BM + wm * 128 + 4 * fh);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const unsigned i = cc[j] & 63u;
                unsigned node;
                if constexpr (M16) {
                    node = nb + (i >> 2) * 16u + (i & 3u);
                } else {
                    const unsigned r = i & 15u;
                    node = nb + (i >> 4) * 32u + (r & 3u) + 8u * (r >> 2);
                }
                k4[j] = cc[j] == 0xffffffffu ? KEY_INVALID
                                             : ((u64)((cc[j] >> 6) + kbase) << 32) | node;
            }
        } else {
            Top4 t4;
            t4.init();
            const unsigned node0 = (unsigned)(node_base + mt * BM + wm * 128);
#pragma unroll
            for (int mi = 0; mi < AM; ++mi) {
                const unsigned bits = block_bits(mi);
#pragma unroll
                for (int reg = 0; reg < AR; ++reg) {
                    // not fitting -> cost all-ones, never inserted (branch-free)
                    const unsigned key = DT == NAS_DT_I8 ? M::okey(acc[mi][ni][reg]) : u[mi][reg];
                    const unsigned x = key | ((((bits >> bitpos(reg)) & 1u) ^ 1u) * 0xffffffffu);
                    t4.insert(x, node0 + noff(mi, reg));
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) k4[j] = t4.c[j] == 0xffffffffu ? KEY_INVALID : t4.key(j);
        }
        u64 o4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = shfl_xor64(k4[j], M16 ? 16 : 32);
        merge44(k4, o4, kl);
        bl = umin64(k4[3], o4[3]);
        if constexpr (M16) {  // the other two row groups (lanes l ^ 32)
            u64 o8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o8[j] = shfl_xor64(kl[j], 32);
            const u64 ob = shfl_xor64(bl, 32);
            merge88(kl, o8);
            bl = umin64(umin64(bl, ob), kl[7]);
            // the four row groups now hold the same list: group ni & 3 stores it
            if (fh == (ni & 3)) {
                u64 *d = xl + ((size_t)(wm * NWN + wn) * WPODS + ni * 16 + fr) * 9;
#pragma unroll
                for (int j = 0; j < 8; ++j) d[j] = kl[j];
                d[8] = bl;
            }
        }
    }

    // merge the two node-half waves (wm = 0, 1) through LDS
    u64 *xk = reinterpret_cast<u64 *>(lds);  // [wn][64 pods][9], staging is dead
    if constexpr (M16) {
        // lane l of a wm = 0 wave merges pod 64 rr + l's two node-half lists
        __syncthreads();
        if (wm == 0) {
#pragma unroll
            for (int rr = 0; rr < (WPODS + 63) / 64; ++rr) {
                if (rr * 64 + lane >= WPODS) continue;
                const u64 *d0 = xl + ((size_t)wn * WPODS + rr * 64 + lane) * 9;
                const u64 *d1 = d0 + (size_t)NWN * WPODS * 9;
                u64 mine[8], other[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    mine[j] = d0[j];
                    other[j] = d1[j];
                }
                merge88(mine, other);
                const u64 bb = umin64(umin64(d0[8], d1[8]), mine[7]);
                const int pod = p0 + nt * BNK + wn * WPODS + rr * 64 + lane;
                if (pod < p_end) {
                    store8(partial + ((size_t)mt * Pp + pod) * KC, mine);
                    pbound[(size_t)mt * Pp + pod] = bb;
                }
            }
        }
        return;
    } else {
    if (wm == 1 && fh == 0) {
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
            u64 *d = xk + ((wn * NI + ni) * 32 + fr) * 9;
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = key[ni][j];
            d[8] = bnd[ni];
        }
    }
    __syncthreads();
    if (wm == 0) {
        // round rr: lane < 32 -> pods wn*WPODS + 64rr + 0..31 (ni = 2rr), lane >=
        // 32 -> +32..63 (ni = 2rr + 1); constant-index branches, not key[fh][j]
        // (a runtime index puts the lists in scratch)
        auto finish = [&](u64 (&mine)[8], u64 b, int ni, int rr) {
            u64 other[8];
            const u64 *s = xk + ((wn * NI + ni) * 32 + fr) * 9;
#pragma unroll
            for (int j = 0; j < 8; ++j) other[j] = s[j];
            merge88(mine, other);
            b = umin64(umin64(b, s[8]), mine[7]);
            const int pod = p0 + nt * BNK + wn * WPODS + rr * 64 + lane;
            if (pod >= p_end) return;
            store8(partial + ((size_t)mt * Pp + pod) * KC, mine);
            pbound[(size_t)mt * Pp + pod] = b;
        };
#pragma unroll
        for (int rr = 0; rr < (NI + 1) / 2; ++rr) {
            if (fh == 0) finish(key[2 * rr], bnd[2 * rr], 2 * rr, rr);
            else if (2 * rr + 1 < NI) finish(key[2 * rr + 1], bnd[2 * rr + 1], 2 * rr + 1, rr);
        }
    }
    }
}

// merge n_lists candidate lists per pod (list l of pod p at
// keys[l * stride + (p - src_p0) * KC], bound[l * bstride + p - src_p0]).
// MERGE_LANES lanes per pod: lane s folds lists s, s + MERGE_LANES, ... in
// registers, then three xor-shuffle rounds merge the lanes' lists.  The 8
// smallest keys of the union do not depend on the merge tree, and neither
// does the bound: every intermediate kept[7] is >= the final kept[7], so the
// result is min(all list bounds, final kept[7]) -- identical to a serial fold.
constexpr int MERGE_LANES = 8;
// 64 pods per workgroup (2 waves per SIMD at 56 VGPRs): still co-resides
// with a 256 x 256 cost workgroup (2 waves per SIMD at 192 VGPRs) on a node
// shard; 1,024-thread blocks do not, and measured 7% slower at G = 8 (the
// wide tile admits nothing beside it either way: C3 within noise for 256 /
// 512 / 1,024, profiles/r03_ab_merge_block.txt)
constexpr int MERGE_BLOCK = 512;

__global__ void __launch_bounds__(MERGE_BLOCK)
k_merge(const u64 *__restrict__ keys, const u64 *__restrict__ bounds, int n_lists,
        long long stride, long long bstride, int src_p0, int p0, int np,
        u64 *__restrict__ dst, u64 *__restrict__ dst_bound, int dst_p0,
        const int *__restrict__ dyn_start, int dyn_hi, int dyn_flags, long long dst_cs,
        const int *__restrict__ dyn_hi_ptr, const int *__restrict__ dst_idx,
        int *__restrict__ init_status) {
    // a one-stream pass's status words start here (k_pass_init's duty, one
    // kernel and one boundary fewer; nothing before the commit reads them)
    if (init_status && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 2 * STATUS_INTS)
        init_status[threadIdx.x] = threadIdx.x == 0 ? -1 : 0;
    const int cb = blockIdx.y;  // cluster of a batched launch (dst_cs pods apart)
    keys += (size_t)cb * n_lists * stride;
    bounds += (size_t)cb * n_lists * bstride;
    dst += (size_t)cb * dst_cs * KC;
    dst_bound += (size_t)cb * dst_cs;
    if (dyn_start) {  // rescore slot: pods [s, min(s + np, hi)); source / destination
        const int s = dyn_start[cb * STATUS_INTS];  // indexed from s when flagged (staging)
        if (s < 0) return;
        if (dyn_hi_ptr) dyn_hi = dyn_hi_ptr[cb * STATUS_INTS];
        p0 = s;
        np = min(np, dyn_hi - s);
        if (dyn_flags & MERGE_SRC_WINDOW) src_p0 = s;
        if (dyn_flags & MERGE_DST_WINDOW) dst_p0 = s;
    }
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = t / MERGE_LANES, s = t % MERGE_LANES;
    const bool live = i < np;  // the whole 8-lane group shares i: shuffles stay in-group
    const size_t ps = (size_t)(p0 + (live ? i : 0) - src_p0);
    u64 a[8], bb[8];
    u64 bound = KEY_INVALID;
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = KEY_INVALID;
    if (live) {
        for (int l = s; l < n_lists; l += MERGE_LANES) {
            load8(keys + l * stride + ps * KC, bb);
            merge88(a, bb);
            bound = umin64(bound, bounds[l * bstride + ps]);
        }
    }
#pragma unroll
    for (int m = 1; m < MERGE_LANES; m <<= 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = shfl_xor64(a[j], m);
        bound = umin64(bound, shfl_xor64(bound, m));
        merge88(a, bb);
    }
    if (!live || s != 0) return;
    // dst_idx (gathered rescore view, one cluster): row r's lists go straight
    // back to pod dst_idx[r]'s slots -- the scatter fused into the store
    const int r = p0 + i - dst_p0;
    const int p = dst_idx ? dst_idx[r] : r;
    store8(dst + (size_t)p * KC, a);
    dst_bound[p] = umin64(bound, a[7]);
}

template <int DT, bool RMAP, int NWN = 4, bool FUSE = (NWN == 6)>
hipError_t launch_cost_t(hipStream_t st, const void *Lt, const void *WA, int Mp, int Kb, int Pp,
                         int p0, int np, const uint64_t *mask, uint64_t *partial,
                         uint64_t *pbound, int node_base, const Dyn *dyn, int batch,
                         const Ovf &ov, const int32_t *rowmap, const FitSrc &fs = FitSrc{},
                         uint32_t *cache = nullptr) {
    constexpr int BNK = NWN * 64;
    constexpr bool WIDE = BNK > BN;
    const void *fn = reinterpret_cast<const void *>(&k_cost_topk<DT, RMAP, NWN, FUSE>);
    constexpr int lds = 2 * (BM + BNK) * BKB;
    static std::atomic<unsigned long long> attr_set{0};
    hipError_t e = set_lds_once(fn, lds, attr_set);
    if (e != hipSuccess) return e;
    const int n_mt = Mp / BM, n_nt = (np + BNK - 1) / BNK;
    // the wide tile's last pod tile reads up to WA_PAD_ROWS rows past the
    // launch; past the last cluster's Pp rows only the padding is allocated
    if (WIDE && (int64_t)p0 + (int64_t)n_nt * BNK > (int64_t)Pp + WA_PAD_ROWS)
        return hipErrorInvalidValue;
    // the fused fit (the wide tile always): capacity and requests
    if (FUSE && (!fs.cap || !fs.req || fs.nloc > Mp || fs.n0 + fs.nloc > fs.N || dyn))
        return hipErrorInvalidValue;
    auto *lt = static_cast<const unsigned char *>(Lt);
    auto *wa = static_cast<const unsigned char *>(WA);
    auto *mk = reinterpret_cast<const u64 *>(mask);
    auto *pa = reinterpret_cast<u64 *>(partial);
    auto *pb = reinterpret_cast<u64 *>(pbound);
    const int *ds = dyn ? dyn->start : nullptr;
    const int dh = dyn ? dyn->hi : 0;
    const int *dhp = dyn ? dyn->hi_ptr : nullptr;
    // the wide tile's launch end rides in dyn_hi (unused without a window)
    const int dhi = WIDE ? p0 + np : dh;
    k_cost_topk<DT, RMAP, NWN, FUSE><<<dim3(n_mt * n_nt, batch), 128 * NWN, lds, st>>>(
        lt, wa, Kb, n_mt, n_nt, p0, Pp, mk, pa, pb, node_base, ds, dhi, dhp, ov, rowmap, fs,
        reinterpret_cast<unsigned *>(cache));
    return hipGetLastError();
}

}  // namespace

int cost_tile_pods(int) { return WIDE_PODS; }

// Kp: padded contraction length in ELEMENTS; np: pods, multiple of BN,
// p0 + np <= Pp; Mp multiple of BM.
hipError_t launch_cost_topk(hipStream_t st, int dtype, const void *Lt, const void *WA, int Mp,
                            int Kp, int Pp, int p0, int np, const uint64_t *mask,
                            uint64_t *partial, uint64_t *pbound, int node_base, const Dyn *dyn,
                            int batch, const Ovf *ovf, const int32_t *rowmap, bool wide,
                            const FitSrc *fit, uint32_t *cache) {
    if (fit && (dyn || rowmap)) return hipErrorInvalidValue;  // windows keep the k_fit mask
    if (cache && (dyn || rowmap)) return hipErrorInvalidValue;  // the cache: main pod ranges
    if (!fit && wide && !dyn && !rowmap) return hipErrorInvalidValue;  // the wide tile fuses
    const Ovf ov = ovf ? *ovf : Ovf{};
    if (rowmap && (!dyn || batch != 1)) return hipErrorInvalidValue;
#define NAS_COST_DISPATCH(DTV, KB, OVV)                                                            \
    (rowmap ? launch_cost_t<DTV, true>(st, Lt, WA, Mp, KB, Pp, p0, np, mask, partial, pbound,     \
                                       node_base, dyn, batch, OVV, rowmap)                        \
     : (!dyn && wide)                                                                             \
            ? launch_cost_t<DTV, false, 6>(st, Lt, WA, Mp, KB, Pp, p0, np, mask, partial, pbound, \
                                           node_base, dyn, batch, OVV, nullptr, *fit, cache)      \
     : fit ? launch_cost_t<DTV, false, 4, true>(st, Lt, WA, Mp, KB, Pp, p0, np,     \
                                                             mask, partial, pbound, node_base,    \
                                                             dyn, batch, OVV, nullptr, *fit,      \
                                                             cache)                               \
            : launch_cost_t<DTV, false>(st, Lt, WA, Mp, KB, Pp, p0, np, mask, partial, pbound,    \
                                        node_base, dyn, batch, OVV, nullptr, FitSrc{}, cache))
    if (dyn) {  // tiles covering any window [s, s + win) clipped to hi: one extra for the offset
        p0 = 0;
        np = (int)round_up(dyn->win, BN) + BN;
        if (!dyn->hi_ptr && dyn->hi > Pp) return hipErrorInvalidValue;
    }
    if (np <= 0) return hipSuccess;
    if (Mp % BM || np % BN || (!dyn && p0 + np > Pp)) return hipErrorInvalidValue;
    if (dtype == NAS_DT_I8) {
        if (Kp % BKB) return hipErrorInvalidValue;
        return NAS_COST_DISPATCH(NAS_DT_I8, Kp, ov);
    }
    // (NAS_DT_F32 operands arrive here as their bf16 six-segment splits,
    // dtype NAS_DT_BF16: nas_api.hip launch_cost)
    if (dtype != NAS_DT_BF16) return hipErrorInvalidValue;
    if ((2 * Kp) % BKB) return hipErrorInvalidValue;
    return NAS_COST_DISPATCH(NAS_DT_BF16, 2 * Kp, Ovf{});
#undef NAS_COST_DISPATCH
}

hipError_t launch_merge(hipStream_t st, const uint64_t *keys, const uint64_t *bounds, int n_lists,
                        int64_t stride, int64_t bstride, int src_p0, int p0, int np,
                        uint64_t *cand_key, uint64_t *cand_bound, int dst_p0, const Dyn *dyn,
                        int dyn_flags, int batch, int64_t dst_cluster_pods,
                        const int32_t *dst_idx, int32_t *init_status) {
    if (dyn) np = dyn->win;
    if (np <= 0) return hipSuccess;
    if (dst_idx && batch != 1) return hipErrorInvalidValue;
    if (init_status && (dyn || batch != 1)) return hipErrorInvalidValue;
    k_merge<<<dim3((int)(((int64_t)np * MERGE_LANES + MERGE_BLOCK - 1) / MERGE_BLOCK), batch),
              MERGE_BLOCK, 0, st>>>(
        reinterpret_cast<const u64 *>(keys), reinterpret_cast<const u64 *>(bounds), n_lists, stride,
        bstride, src_p0, p0, np, reinterpret_cast<u64 *>(cand_key),
        reinterpret_cast<u64 *>(cand_bound), dst_p0, dyn ? dyn->start : nullptr, dyn ? dyn->hi : 0,
        dyn_flags, (long long)dst_cluster_pods, dyn ? dyn->hi_ptr : nullptr, dst_idx, init_status);
    return hipGetLastError();
}

}  // namespace nas
