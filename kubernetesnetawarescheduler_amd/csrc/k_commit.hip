// k_commit.hip -- conflict-resolving greedy commit with capacity update.
//
// Sequential semantics (the extended-mode oracle, oracle/oracle.c or_place):
// pods in order take the (cost, node)-smallest node that still fits the
// remaining capacity, which is then decremented.  Each pod arrives with a
// candidate list (klist.h): keys <= its bound are exactly the best nodes that
// fit some EARLIER capacity state.  Capacity only shrinks, so the pod's
// sequential choice is its first usable candidate that fits now -- every
// better node is either ahead of it in the list and does not fit, or never
// fit.  If no usable candidate fits: a complete list (bound = KEY_INVALID)
// means no node fits (NAS_EMPTY); otherwise the pod needs a rescore against
// the current capacity (host loop in nas_api.hip).
//
// Parallel form: one 1024-thread workgroup, one pod per thread, a window of
// 1024 consecutive pods per round.
//   1. Every pending pod picks its first fitting usable candidate against the
//      capacity at the start of the round and RESERVES it per resource (a
//      fetch-and-subtract undone on failure, or for huge requests a
//      compare-and-swap loop that never goes below zero; see reserve()).
//   2. A pod is BAD if a reservation failed or it needs a rescore; s = the
//      lowest bad pod (LDS atomicMin).
//   3. Every pod below s is exactly what the sequential walk does: for the
//      pods below s on any node c, the last of them to reserve (in atomic
//      order) still found its request available after all the others that
//      reserved before it, so their total fits c, hence every prefix of them
//      in pod order does; and nothing below s changed its mind.  They commit.
//   4. Pods >= s release their reservations.  Pod s re-checks its pick
//      against the capacity now (= start minus the committed pods): if it
//      fits it commits too.  The round ends; the next one re-runs the same
//      window with the pods not yet committed (the first of them always
//      commits, so every round makes progress).
// A round with no bad pod costs two barriers; the next window's lists are
// prefetched into registers while the current one runs.  A rescore pod
// halts the launch (halt word) after the pods below it commit; a launch with
// p_begin < 0 resumes from the halted pod after a rescore slot (nas_api.hip).
// The working capacity lives in LDS (3 x N int32) when it fits, else in L2.
// The L2 form's speculative reservations can dip below the committed state, so
// it also subtracts each committed pod from `pub` (when given): a published
// capacity that is always >= the working one, for concurrent scoring to read.
//
// Zero-traffic pods (zrow[p] = 1: no traffic to any bound peer, so every cost
// is exactly 0 and key order is node order): the list holds the lowest-index
// nodes that fitted when it was scored, and every node up to the bound's node
// is either in the list or did not fit then (capacity only shrinks).  When
// none of its usable candidates fits, such a pod's sequential choice is the
// first node ABOVE the bound's node that fits now -- found by a scan of the
// capacity instead of a rescore; a scan that reaches the last node without a
// fit means no node fits (NAS_EMPTY).  A herd of such pods (pods with no
// placed peers) fills the nodes in index order, and without the scan drains
// one 8-node list per rescore slot (C2: 5 slots, 1,087 of its 1,654
// zero-traffic pods land outside their first list).
#include "klist.h"

namespace nas {
namespace {

constexpr int THREADS = 1024;  // one window of pods per round
constexpr int LDS_DYN_MAX = 160 * 1024 - 512;  // leaves room for the static LDS
// k_commit_w's prefetch ring of candidate lists in LDS (after the capacity):
// PF_SLOTS windows of 64 pods, PF_SLOT bytes each -- keys [64][8] u64 at 0,
// bounds [128] u64 from the even pod at or below the window at 4096, requests
// [3][64] int32 at 5120, zero-traffic flags [256] bytes from the multiple of 4
// at or below the window at 5888
constexpr int PF_SLOT = 6144;
constexpr int PF_SLOTS = 4;
constexpr int PF_BYTES = PF_SLOT * PF_SLOTS;
constexpr int PF_LOADS = 9;  // LDS-DMA instructions per window
// windows in flight beyond the walked one (1 vs 3 measured equal)
constexpr int COMMIT_AHEAD = 3;
static_assert(COMMIT_AHEAD >= 1 && COMMIT_AHEAD < PF_SLOTS, "ring depth");
template <int N>
__device__ __forceinline__ void retire_window();
// retire the oldest window in flight while `younger` (0..3) later ones stay
__device__ __forceinline__ void retire_oldest(int younger);
constexpr int LDS_CAP_MAX_NODES = (LDS_DYN_MAX - PF_BYTES - 256) / 12;  // + cap_to_lds padding
constexpr int NO_POD = 0x7fffffff;

// k_commit_w's side-by-side capacity image: 16 B per node beside the ring
constexpr int AOS_MAX_NODES = (LDS_DYN_MAX - PF_BYTES - 256) / 16;
// walks of up to this many pods run in one wave (k_commit_w): fewer, exact
// stops for herds on small clusters (C2: 0.67 -> 0.62 ms per pass; with the
// zero-traffic scan and no rescore left, 0.55 vs 0.63 ms for k_commit); longer
// walks keep the 1024-pod windows of k_commit, whose conflict-free rounds
// commit 16x more pods each (C3: 0.8 vs 2.4 ms of commit per pass).
// Cluster batches walk with k_commit (1,024 threads) even when a cluster is
// short enough for one wave: C5's 64 x 5,000-pod walks 7.93 -> 7.77 ms per
// pass (profiles/r04_ab_batch_commit.txt); one cluster keeps the one-wave
// walk below ONE_WAVE_MAX_PODS (C2's herds)
constexpr int ONE_WAVE_MAX_PODS = 16384;

// Requests up to this size reserve with one fetch-and-subtract (undone on
// failure) instead of a compare-and-swap loop: a herd of m pods picking one
// node then costs m atomics, not ~m^2 retries.  The dips of failed
// subtractions are transient and can only make a concurrent reservation fail
// spuriously (one more round), never succeed wrongly; THREADS of them stay
// above INT_MIN (1024 * 2^21 = 2^31).  Larger requests keep the CAS loop,
// which never takes a resource below zero.
constexpr int FETCH_SUB_MAX = 1 << 21;

// the orderable encoding of cost 0 (int8: 0 ^ 2^31; bf16 / fp32: +0 with the
// sign bit set), the high word of every key of a zero-traffic pod
constexpr unsigned ZERO_COST_KEY = 0x80000000u;
// nodes a zero-traffic pick scans past its list (capacity in LDS / in L2);
// a longer walk falls back to a rescore
constexpr int ZSCAN_LDS = 1024;
constexpr int ZSCAN_L2 = 16;

// A zero-traffic pod whose usable candidates are all full: the first node
// above its bound's node that fits the capacity read by `ld`.  Returns the
// node, -1 when no node fits at all (the scan reached N), or -2 when the scan
// limit ran out first (rescore).
// `from` (per pod, -1 at first): where this pod's previous scan stopped -- the
// nodes below it did not fit then and capacity only shrinks between picks
// (a round's failed reservations are undone before the next round picks)
template <bool LDS_CAP, typename LD3>
__device__ __forceinline__ int zero_row_scan(u64 bound, int r0, int r1, int r2, int N, LD3 &&ld3,
                                             int &from) {
    const int nb = (int)(unsigned)bound + 1;
    const int n0 = max(nb, from);
    const int n1 = min(N, nb + (LDS_CAP ? ZSCAN_LDS : ZSCAN_L2));
    // 8 nodes per step, their 24 reads in flight together (a node past n1
    // re-reads n1 - 1 and is never taken)
    for (int n = n0; n < n1; n += 8) {
        unsigned fit = 0;
        int4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ld3(min(n + j, n1 - 1));
        // the 8 reads issue back to back (hipcc otherwise waits for each
        // before the next: 8 LDS round trips per step)
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            fit |= (unsigned)((r0 <= v[j].x) & (r1 <= v[j].y) & (r2 <= v[j].z) & (n + j < n1)) << j;
        if (fit) {
            from = n + __builtin_ctz(fit);
            return from;
        }
    }
    from = n1;
    return n1 == N ? -1 : -2;
}

// reserve r from *c iff *c >= r; returns success
template <bool LDS_CAP>
__device__ __forceinline__ bool reserve(int *c, int r) {
    if (r == 0) return true;
    int old = LDS_CAP ? *c : __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old < r) return false;
    if (r <= FETCH_SUB_MAX) {
        const int prev = atomicSub(c, r);
        if (prev >= r) return true;
        atomicAdd(c, r);
        return false;
    }
    while (old >= r) {
        const int prev = atomicCAS(c, old, old - r);
        if (prev == old) return true;
        old = prev;
    }
    return false;
}

// A barrier inside the walk.  With the capacity in LDS every value the next
// step reads is in LDS, so waiting for this wave's LDS operations is enough; a
// full __syncthreads would also drain the next window's prefetch loads (and
// the output stores) at every round.  The L2 form keeps the full fence: its
// capacity updates are global atomics.
template <bool LDS_CAP>
__device__ __forceinline__ void round_barrier() {
    if constexpr (LDS_CAP) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    } else {
        __syncthreads();
    }
}

// all three resources of a pick: with small requests the three
// fetch-and-subtracts are in flight together (no load before them: a request
// that plainly does not fit dips and undoes like any failed one)
template <bool LDS_CAP>
__device__ __forceinline__ void reserve3(int *c0, int *c1, int *c2, int r0, int r1, int r2,
                                         bool &g0, bool &g1, bool &g2) {
    if (r0 <= FETCH_SUB_MAX && r1 <= FETCH_SUB_MAX && r2 <= FETCH_SUB_MAX) {
        // all three subtractions in flight together (a zero request subtracts
        // nothing and is granted whatever it reads)
        const int p0 = atomicSub(c0, r0);
        const int p1 = atomicSub(c1, r1);
        const int p2 = atomicSub(c2, r2);
        __builtin_amdgcn_sched_group_barrier(0x80, 3, 0);
        g0 = r0 == 0 || p0 >= r0;
        g1 = r1 == 0 || p1 >= r1;
        g2 = r2 == 0 || p2 >= r2;
        if (!g0) atomicAdd(c0, r0);
        if (!g1) atomicAdd(c1, r1);
        if (!g2) atomicAdd(c2, r2);
        return;
    }
    g0 = reserve<LDS_CAP>(c0, r0);
    g1 = reserve<LDS_CAP>(c1, r1);
    g2 = reserve<LDS_CAP>(c2, r2);
}

// The working capacity into LDS by LDS-DMA: one `global_load_lds_dword` per
// 64 ints (lane-linear), all in flight together, one vmcnt(0) at the end.
// (A register copy loop, even with 8 loads per thread in flight, made hipcc
// branch around each load and wait between them: ~30 dependent L2 round trips
// per thread at 10k nodes for every commit launch.)  Lanes past 3n re-read
// the last element into the padding of the LDS image (the launch rounds its
// LDS size up to a 256-byte piece).
__device__ __forceinline__ void cap_to_lds(const int *g, int *l, int n3, int wave, int n_waves) {
    const int lane = threadIdx.x & 63;
    for (int j = wave; j * 64 < n3; j += n_waves) {
        const int i = min(j * 64 + lane, n3 - 1);
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(g + i),
                                         (void __attribute__((address_space(3))) *)(l + j * 64), 4,
                                         0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The launch's placements [p_begin, p_end) (and their raw keys) into the
// host's pinned stage, for the host to unpack while later chunks still run:
// a launch of its own per array behind every commit (copy kernels) waited
// 100-170 us each for a CU beside the wide cost workgroups and put four more
// dependent launches into the pass's tail.  Pods past a halt carry stale
// values here exactly as the copies did; the host re-reads everything then.
__device__ __forceinline__ void to_stage(const int *out_node, const unsigned *out_cost,
                                         int *stage_node, unsigned *stage_cost, int p_begin,
                                         int p_end, int t, int nt) {
    if (!stage_node) return;
    // 16-byte stores while both stage arrays are aligned: a quarter of the
    // store instructions over the host link
    auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
    if (al(stage_node + p_begin) && al(out_node + p_begin) &&
        (!stage_cost || (al(stage_cost + p_begin) && al(out_cost + p_begin)))) {
        const int nv = (p_end - p_begin) >> 2;
        for (int v = t; v < nv; v += nt) {
            const int i = p_begin + 4 * v;
            *reinterpret_cast<int4 *>(stage_node + i) = *reinterpret_cast<const int4 *>(out_node + i);
            if (stage_cost)
                *reinterpret_cast<uint4 *>(stage_cost + i) =
                    *reinterpret_cast<const uint4 *>(out_cost + i);
        }
        p_begin += 4 * nv;
    }
    for (int i = p_begin + t; i < p_end; i += nt) {
        stage_node[i] = out_node[i];
        if (stage_cost) stage_cost[i] = out_cost[i];
    }
}

// the status words (after this walk's updates, by the thread that made them)
// into the host's pinned status area: the pass's last commit, so the host's
// wait for it brings the status with the results
__device__ __forceinline__ void status_to_stage(const int *halt, int *stage_status) {
    if (!stage_status) return;
#pragma unroll
    for (int j = 0; j < COMMIT_STATUS_WORDS; ++j) stage_status[j] = halt[j];
}

template <bool LDS_CAP>
__global__ void __launch_bounds__(THREADS)
k_commit(const u64 *__restrict__ cand_key, const u64 *__restrict__ cand_bound,
         const int *__restrict__ req, int Pp, int p_begin, int p_end, int *__restrict__ cap_g,
         int N, int *__restrict__ out_node, unsigned *__restrict__ out_cost,
         int *__restrict__ halt, int *__restrict__ pub, const unsigned char *__restrict__ zrow,
         int *__restrict__ stage_node, unsigned *__restrict__ stage_cost, int *__restrict__ stage_status) {
    // one workgroup per cluster of a batched launch
    const int cb = blockIdx.x;
    cand_key += (size_t)cb * Pp * KC;
    cand_bound += (size_t)cb * Pp;
    req += (size_t)cb * 3 * Pp;
    cap_g += (size_t)cb * 3 * N;
    out_node += (size_t)cb * Pp;
    out_cost += (size_t)cb * Pp;
    halt += cb * STATUS_INTS;
    if (pub) pub += (size_t)cb * 3 * N;
    if (zrow) zrow += (size_t)cb * Pp;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    __shared__ int first_bad[3];  // round r uses slot r % 3
    __shared__ int s_rescore;     // the round's lowest bad pod needs a rescore
    int *capl = smem;
    const int tid = threadIdx.x;
    // an earlier commit launch on this stream stopped at a pod that needs a
    // rescore: every later pod must wait for it (sequential semantics)
    // p_begin < 0: a rescore slot's resume -- continue from the halted pod
    // (nothing to do unless a walk halted), clearing the halt word
    const int h = __hip_atomic_load(halt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool resume = p_begin < 0;
    // (a halt word past the walk's end is not a pod: FLAG_TIMEOUT_HALT, the
    // tail's failed wait for the commit stream -- never resumed from, and it
    // stays for the host to report)
    if (resume ? (h < 0 || h >= p_end) : h >= 0) {  // nothing to walk (the status still goes out)
        if (threadIdx.x == 0) status_to_stage(halt, stage_status);
        return;
    }
    if (resume) p_begin = h;
    if (LDS_CAP) cap_to_lds(cap_g, capl, 3 * N, tid >> 6, THREADS / 64);
    int *cap = LDS_CAP ? capl : cap_g;
    if (tid == 0) first_bad[0] = first_bad[1] = first_bad[2] = NO_POD;

    struct Pod {
        u64 k[KC];
        u64 bound;
        int r0, r1, r2;
    };
    // branch-free fill: pods past p_end read a clamped, in-bounds row; they
    // are `done` from the start of their window, so nothing reads their
    // values -- no select on the loaded registers here, which would make the
    // prefetch of the next window wait for its loads on the spot
    auto load = [&](int base, Pod &c) {
        const int ii = min(base + tid, Pp - 1);
        load8(cand_key + (size_t)ii * KC, c.k);
        c.bound = cand_bound[ii];
        c.r0 = req[ii];
        c.r1 = req[Pp + ii];
        c.r2 = req[2 * Pp + ii];
    };
    auto publish = [&](int n, const Pod &c) {
        if (LDS_CAP || !pub || n < 0) return;
        atomicSub(pub + n, c.r0);
        atomicSub(pub + N + n, c.r1);
        atomicSub(pub + 2 * N + n, c.r2);
    };
    auto ld = [&](int idx) -> int {
        if (LDS_CAP) return cap[idx];
        return __hip_atomic_load(cap + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };

    Pod cur, nxt;
    load(p_begin, cur);
    __syncthreads();  // every thread has read the halt word
    if (tid == 0 && h >= 0) {
        halt[0] = -1;
        // device-side rescores, reported in nas_timings; the first resume's
        // pod (the pass's first halt) tells the host which pods' copies were
        // final before it
        if (resume) {
            if (halt[1] == 0) halt[3] = h;
            halt[1] += 1;
        }
    }
    int round = 0;
    int stop = p_end;
    for (int base = p_begin; base < p_end; base += THREADS) {
        if (base + THREADS < p_end) load(base + THREADS, nxt);  // prefetch the next window
        const int i = base + tid;
        bool done = i >= p_end;
        int zfrom = -1;  // zero-traffic scan resume point (zero_row_scan)
        while (true) {
            // slot (round + 1) % 3 was last read before the previous round's
            // first barrier and is next written after this round's: reset it
            if (tid == 0) first_bad[(round + 1) % 3] = NO_POD;
            // 1. pick against the capacity at the start of the round, reserve
            // candidates in list order, stopping at the first that fits (most
            // pods stop at their first): 3 LDS reads per candidate looked at
            int choice = -1;
            unsigned ccost = 0;
            if (!done) {
#pragma unroll
                for (int j = 0; j < KC; ++j) {
                    const u64 k = cur.k[j];
                    if (k == KEY_INVALID || k > cur.bound) break;  // end of the usable prefix
                    const int n = (int)(unsigned)k;
                    const int a = ld(n), b = ld(N + n), c = ld(2 * N + n);
                    if (cur.r0 <= a && cur.r1 <= b && cur.r2 <= c) {
                        choice = n;
                        ccost = (unsigned)(k >> 32);
                        break;
                    }
                }
            }
            if (done) choice = -1;
            bool rescore = !done && choice < 0 && cur.bound != KEY_INVALID;
            if (rescore && zrow && zrow[i] && (unsigned)(cur.bound >> 32) == ZERO_COST_KEY) {
                auto ld3 = [&](int n) { return make_int4(ld(n), ld(N + n), ld(2 * N + n), 0); };
                const int z = zero_row_scan<LDS_CAP>(cur.bound, cur.r0, cur.r1, cur.r2, N, ld3, zfrom);
                if (z != -2) {
                    rescore = false;
                    choice = z;  // -1: nothing fits (NAS_EMPTY)
                    ccost = ZERO_COST_KEY;
                }
            }
            // every pick must see the capacity at the START of the round: a
            // later pod's reservation must not push an earlier pod off a node
            round_barrier<LDS_CAP>();
            bool g0 = false, g1 = false, g2 = false;
            if (choice >= 0)
                reserve3<LDS_CAP>(cap + choice, cap + N + choice, cap + 2 * N + choice, cur.r0,
                                  cur.r1, cur.r2, g0, g1, g2);
            const bool bad = rescore || (choice >= 0 && !(g0 && g1 && g2));
            int *fb = &first_bad[round % 3];
            if (bad) atomicMin(fb, i);
            round_barrier<LDS_CAP>();
            // 2. the lowest bad pod
            const int s = *fb;
            ++round;
            if (s == NO_POD) {
                // 3. no conflict: every pending pod of the window commits
                if (!done) {
                    out_node[i] = choice >= 0 ? choice : NAS_EMPTY;
                    out_cost[i] = ccost;
                    publish(choice, cur);
                }
                break;
            }
            // 4. pods >= s release what they reserved; pods < s commit
            if (!done && i >= s && choice >= 0) {
                if (g0) atomicAdd(cap + choice, cur.r0);
                if (g1) atomicAdd(cap + N + choice, cur.r1);
                if (g2) atomicAdd(cap + 2 * N + choice, cur.r2);
            }
            if (!done && i < s) {
                out_node[i] = choice >= 0 ? choice : NAS_EMPTY;
                out_cost[i] = ccost;
                publish(choice, cur);
                done = true;
            }
            if (i == s) s_rescore = rescore;
            round_barrier<LDS_CAP>();
            // a rescore pod ends the launch: everything below it is committed
            if (s_rescore) {
                stop = s;
                break;
            }
            if (i == s) {
                // pod s against the capacity left by the pods below it
                const int n = choice;
                if (cur.r0 <= ld(n) && cur.r1 <= ld(N + n) && cur.r2 <= ld(2 * N + n)) {
                    if (LDS_CAP) {
                        cap[n] -= cur.r0; cap[N + n] -= cur.r1; cap[2 * N + n] -= cur.r2;
                    } else {
                        atomicSub(cap + n, cur.r0); atomicSub(cap + N + n, cur.r1);
                        atomicSub(cap + 2 * N + n, cur.r2);
                    }
                    out_node[i] = n;
                    out_cost[i] = ccost;
                    publish(n, cur);
                    done = true;
                }
            }
            // the next round's picks must see pod s's update (a bare s_barrier
            // does not wait for the store: round_barrier waits for it)
            round_barrier<LDS_CAP>();
            // pods below s are done; s itself is done unless it must re-pick
        }
        if (stop < p_end) break;
        if (base + THREADS < p_end) cur = nxt;
    }
    if (tid == 0) {
        if (stop < p_end) *halt = stop;
        halt[2] += round;  // rounds walked, reported in nas_timings
        status_to_stage(halt, stage_status);
    }
    __syncthreads();
    to_stage(out_node, out_cost, stage_node ? stage_node + (size_t)cb * p_end : nullptr,
             stage_cost ? stage_cost + (size_t)cb * p_end : nullptr, p_begin, p_end, tid, THREADS);
    if (LDS_CAP)
        for (int i = tid; i < 3 * N; i += THREADS) cap_g[i] = capl[i];
}

// ---------------------------------------------------------------------------
// k_commit_w: the same walk in ONE wave (a window of 64 pods per round).
// No barriers at all -- a wave's LDS operations execute in order, so every
// step sees the previous one -- and the lowest bad pod is a ballot.  The
// reservations of one wave instruction are applied one lane after another,
// so within a window the first failing pod is (in practice) the first pod
// whose request truly does not fit after the pods below it: herds of pods
// wanting the same node no longer stop at a spurious failure of an early
// member, as they do across the 16 waves of k_commit.  Correctness never
// depends on that order (the argument of step 3 holds for any atomic order);
// only the number of rounds does.
// ---------------------------------------------------------------------------
// The lists of windows k+1 .. k+3 stream into an LDS ring (LDS-DMA) while
// window k walks: a window's lists were written by k_merge on other XCDs, so
// every load is a trip beyond L2 (~1-2 us), longer than a window's rounds.
// LDS-DMA keeps the in-flight data out of registers (a register prefetch
// across loop iterations lets the compiler copy a pending load's destination
// before its wait).  The retire waits only for the window it takes.
template <int N>
__device__ __forceinline__ void retire_window() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
    __builtin_amdgcn_s_barrier();  // (one wave: orders its own LDS-DMA before its reads)
    asm volatile("" ::: "memory");
}
// LDS-DMA hipcc does not count (cdna_hip_programming.md §5.7 recipe): with the
// builtin, hipcc drains every outstanding LDS-DMA (vmcnt(0)) before each LDS
// atomic of the walk, as it cannot tell the ring from the capacity.  `lds` is
// the wave-uniform LDS byte address; M0 is saved and restored in the statement.
__device__ __forceinline__ unsigned lds_addr(const void *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void retire_oldest(int younger) {
    if (younger >= 3) retire_window<3 * PF_LOADS>();
    else if (younger == 2) retire_window<2 * PF_LOADS>();
    else if (younger == 1) retire_window<PF_LOADS>();
    else retire_window<0>();
}
template <int SZ>
__device__ __forceinline__ void glds(const void *g, unsigned lds) {
    unsigned keep;
    if constexpr (SZ == 16)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(g), "s"(lds)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(g), "s"(lds)
                     : "memory");
}

// AOS (capacity in LDS only): node n's three resources side by side,
// {cpu, mem, pods, 0} at capl + 4 n, so a candidate check is ONE 16-byte LDS
// read instead of three (up to 8,656 nodes beside the prefetch ring)
template <bool LDS_CAP, bool AOS = false>
__global__ void __launch_bounds__(64)
k_commit_w(const u64 *__restrict__ cand_key, const u64 *__restrict__ cand_bound,
           const int *__restrict__ req, int Pp, int p_begin, int p_end, int *__restrict__ cap_g,
           int N, int *__restrict__ out_node, unsigned *__restrict__ out_cost,
           int *__restrict__ halt, int *__restrict__ pub, const unsigned char *__restrict__ zrow,
           int *__restrict__ stage_node, unsigned *__restrict__ stage_cost, int *__restrict__ stage_status) {
    const int cb = blockIdx.x;
    cand_key += (size_t)cb * Pp * KC;
    cand_bound += (size_t)cb * Pp;
    req += (size_t)cb * 3 * Pp;
    cap_g += (size_t)cb * 3 * N;
    out_node += (size_t)cb * Pp;
    out_cost += (size_t)cb * Pp;
    halt += cb * STATUS_INTS;
    if (pub) pub += (size_t)cb * 3 * N;
    if (zrow) zrow += (size_t)cb * Pp;
    extern __shared__ __attribute__((aligned(16))) int smem[];
    int *capl = smem;
    const int lane = threadIdx.x;
    const int h = __hip_atomic_load(halt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool resume = p_begin < 0;
    // (a halt word past the walk's end is not a pod: FLAG_TIMEOUT_HALT, the
    // tail's failed wait for the commit stream -- never resumed from, and it
    // stays for the host to report)
    if (resume ? (h < 0 || h >= p_end) : h >= 0) {  // nothing to walk (the status still goes out)
        if (threadIdx.x == 0) status_to_stage(halt, stage_status);
        return;
    }
    if (resume) p_begin = h;
    static_assert(!AOS || LDS_CAP, "the side-by-side layout is an LDS image");
    if constexpr (AOS) {
        for (int i = lane; i < N; i += 64)
            *reinterpret_cast<int4 *>(capl + 4 * i) = make_int4(cap_g[i], cap_g[N + i], cap_g[2 * N + i], 0);
    } else if (LDS_CAP) {
        cap_to_lds(cap_g, capl, 3 * N, 0, 1);
    }
    int *cap = LDS_CAP ? capl : cap_g;
    // resource r of node n
    auto ci = [&](int r, int n) { return AOS ? 4 * n + r : r * N + n; };
    struct Pod {
        u64 k[KC];
        u64 bound;
        int r0, r1, r2;
        int z;  // zero-traffic pod (zrow)
    };
    auto publish = [&](int n, const Pod &c) {
        if (LDS_CAP || !pub || n < 0) return;
        atomicSub(pub + n, c.r0);
        atomicSub(pub + N + n, c.r1);
        atomicSub(pub + 2 * N + n, c.r2);
    };
    auto ld = [&](int idx) -> int {
        if (LDS_CAP) return cap[idx];
        return __hip_atomic_load(cap + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto ld3 = [&](int n) -> int4 {
        if constexpr (AOS) return *reinterpret_cast<const int4 *>(cap + 4 * n);
        return make_int4(ld(n), ld(N + n), ld(2 * N + n), 0);
    };
    Pod cur;
    if (lane == 0 && h >= 0) {
        halt[0] = -1;
        if (resume) {
            if (halt[1] == 0) halt[3] = h;
            halt[1] += 1;
        }
    }
    unsigned char *pf = reinterpret_cast<unsigned char *>(smem) +
                        (AOS ? (16 * N + 255) / 256 * 256 : LDS_CAP ? (3 * N * 4 + 255) / 256 * 256 : 0);
    const unsigned char *zsrc = zrow ? zrow : reinterpret_cast<const unsigned char *>(req);
    // window wbase's lists into ring slot `slot` (9 LDS-DMA instructions; lanes
    // past the data re-read its last bytes into the slot's idle space)
    auto issue = [&](int wbase, int slot) {
        if (wbase >= p_end) return;
        const unsigned d = __builtin_amdgcn_readfirstlane(lds_addr(pf + slot * PF_SLOT));
        const auto *kb = reinterpret_cast<const unsigned char *>(cand_key);
        const size_t kmax = (size_t)Pp * KC * 8 - 16;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            glds<16>(kb + min((size_t)wbase * KC * 8 + j * 1024 + lane * 16, kmax), d + j * 1024);
        // bounds and flags from aligned starts (a window may begin at any pod
        // after a halt): 16-byte pieces from the even pod below, dwords from
        // the multiple of 4 below; take() skips the leading entries
        glds<16>(reinterpret_cast<const unsigned char *>(cand_bound) +
                     min((size_t)(wbase & ~1) * 8 + lane * 16, (size_t)Pp * 8 - 16),
                 d + 4096);
#pragma unroll
        for (int r = 0; r < 3; ++r) glds<4>(req + (size_t)r * Pp + min(wbase + lane, Pp - 1), d + 5120 + r * 256);
        glds<4>(zsrc + min((wbase & ~3) + 4 * lane, Pp - 4), d + 5888);
    };
    auto take = [&](int slot, int wbase) {
        const unsigned char *d = pf + slot * PF_SLOT;
        load8(reinterpret_cast<const u64 *>(d) + lane * KC, cur.k);
        cur.bound = reinterpret_cast<const u64 *>(d + 4096)[lane + (wbase & 1)];
        cur.r0 = reinterpret_cast<const int *>(d + 5120)[lane];
        cur.r1 = reinterpret_cast<const int *>(d + 5120 + 256)[lane];
        cur.r2 = reinterpret_cast<const int *>(d + 5120 + 512)[lane];
        cur.z = zrow ? (int)d[5888 + lane + (wbase & 3)] : 0;
    };
    // windows 0..3 into slots 0..3; window w always sits in slot w % 4
    int younger = 0;
    for (int j = 0; j <= COMMIT_AHEAD; ++j) {
        issue(p_begin + 64 * j, j);
        younger += j > 0 && p_begin + 64 * j < p_end;
    }
    retire_oldest(younger);
    take(0, p_begin);
    int round = 0;
    int stop = p_end;
    for (int base = p_begin, w = 0;; ++w) {
        const int i = base + lane;
        bool done = i >= p_end;
        int zfrom = -1;  // zero-traffic scan resume point (zero_row_scan)
        while (true) {
            int choice = -1;
            unsigned ccost = 0;
            if (!done) {
                // every usable candidate's capacity in one LDS round trip (8
                // independent reads), the lowest fitting one is the sequential
                // choice (keys ascend; unusable ones come last).  Candidate 0
                // first and the other 7 only for the lanes whose first was full
                // took two round trips: C2 0.467 -> 0.457 ms
                // (profiles/r04_ab_c2_commit.txt)
                int4 v[KC];
#pragma unroll
                for (int j = 0; j < KC; ++j) {
                    const u64 k = cur.k[j];
                    const bool usable = k != KEY_INVALID && k <= cur.bound;
                    v[j] = ld3(usable ? (int)(unsigned)k : 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x100, KC, 0);
                unsigned okm = 0;
#pragma unroll
                for (int j = 0; j < KC; ++j) {
                    const u64 k = cur.k[j];
                    const bool usable = k != KEY_INVALID && k <= cur.bound;
                    okm |= (unsigned)(usable & (cur.r0 <= v[j].x) & (cur.r1 <= v[j].y) & (cur.r2 <= v[j].z))
                           << j;
                }
#pragma unroll
                for (int j = KC - 1; j >= 0; --j)  // constant indices (no scratch array)
                    if ((okm >> j) & 1u) {
                        choice = (int)(unsigned)cur.k[j];
                        ccost = (unsigned)(cur.k[j] >> 32);
                    }
            }
            bool rescore = !done && choice < 0 && cur.bound != KEY_INVALID;
            if (rescore && cur.z && (unsigned)(cur.bound >> 32) == ZERO_COST_KEY) {
                const int z = zero_row_scan<LDS_CAP>(cur.bound, cur.r0, cur.r1, cur.r2, N, ld3, zfrom);
                if (z != -2) {
                    rescore = false;
                    choice = z;  // -1: nothing fits (NAS_EMPTY)
                    ccost = ZERO_COST_KEY;
                }
            }
            bool g0 = false, g1 = false, g2 = false;
            if (choice >= 0)
                reserve3<LDS_CAP>(cap + ci(0, choice), cap + ci(1, choice), cap + ci(2, choice), cur.r0,
                                  cur.r1, cur.r2, g0, g1, g2);
            const bool bad = rescore || (choice >= 0 && !(g0 && g1 && g2));
            const u64 bm = __ballot(bad);
            ++round;
            if (bm == 0) {  // no conflict: every pending pod of the window commits
                if (!done) {
                    out_node[i] = choice >= 0 ? choice : NAS_EMPTY;
                    out_cost[i] = ccost;
                    publish(choice, cur);
                }
                break;
            }
            const int sl = (int)__builtin_ctzll(bm);
            const int s = base + sl;
            if (!done && lane >= sl && choice >= 0) {
                if (g0) atomicAdd(cap + ci(0, choice), cur.r0);
                if (g1) atomicAdd(cap + ci(1, choice), cur.r1);
                if (g2) atomicAdd(cap + ci(2, choice), cur.r2);
            }
            if (!done && lane < sl) {
                out_node[i] = choice >= 0 ? choice : NAS_EMPTY;
                out_cost[i] = ccost;
                publish(choice, cur);
                done = true;
            }
            if (__builtin_amdgcn_readlane((int)rescore, sl)) {
                stop = s;
                break;
            }
            if (!LDS_CAP) __threadfence_block();  // the releases above before the re-check
            if (lane == sl) {
                // pod s against the capacity left by the pods below it
                const int n = choice;
                const int4 v = ld3(n);
                if (cur.r0 <= v.x && cur.r1 <= v.y && cur.r2 <= v.z) {
                    atomicSub(cap + ci(0, n), cur.r0);
                    atomicSub(cap + ci(1, n), cur.r1);
                    atomicSub(cap + ci(2, n), cur.r2);
                    out_node[i] = n;
                    out_cost[i] = ccost;
                    publish(n, cur);
                    done = true;
                }
            }
        }
        if (stop < p_end || base + 64 >= p_end) break;
        // window w+1 (slot (w+1) % 4): windows w+2, w+3 may stay in flight
        younger = 0;
        for (int j = 2; j <= COMMIT_AHEAD; ++j) younger += base + 64 * j < p_end;
        retire_oldest(younger);
        take((w + 1) & 3, base + 64);
        base += 64;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot w % 4's reads done
        issue(base + 64 * COMMIT_AHEAD, (w + 1 + COMMIT_AHEAD) & 3);  // window w+1+AHEAD
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no untracked load outlives the walk
    if (lane == 0) {
        if (stop < p_end) *halt = stop;
        halt[2] += round;
        status_to_stage(halt, stage_status);
    }
    __syncthreads();  // (one wave: every lane's placements written)
    to_stage(out_node, out_cost, stage_node ? stage_node + (size_t)cb * p_end : nullptr,
             stage_cost ? stage_cost + (size_t)cb * p_end : nullptr, p_begin, p_end, lane, 64);
    if constexpr (AOS) {
        for (int i = lane; i < N; i += 64) {
            const int4 v = *reinterpret_cast<const int4 *>(capl + 4 * i);
            cap_g[i] = v.x;
            cap_g[N + i] = v.y;
            cap_g[2 * N + i] = v.z;
        }
    } else if (LDS_CAP) {
        for (int i = lane; i < 3 * N; i += 64) cap_g[i] = capl[i];
    }
}

}  // namespace

bool commit_in_lds(int N) { return N <= LDS_CAP_MAX_NODES; }

hipError_t launch_commit(hipStream_t st, const uint64_t *cand_key, const uint64_t *cand_bound,
                         const int32_t *req, int Pp, int p_begin, int p_end, int32_t *cap, int N,
                         int32_t *out_node, int32_t *out_cost, int32_t *halt, int batch,
                         int32_t *pub, const uint8_t *zrow, int32_t *stage_node,
                         int32_t *stage_cost, int32_t *stage_status) {
    if (p_begin >= 0 && p_end <= p_begin) return hipSuccess;
    // a batch stages whole clusters, [cluster][p_end] rows from pod 0
    if (stage_node && (p_begin < 0 || (batch != 1 && p_begin != 0))) return hipErrorInvalidValue;
    if (stage_status && batch != 1) return hipErrorInvalidValue;
    auto *sc = reinterpret_cast<unsigned *>(stage_cost);
    const auto *ck = reinterpret_cast<const u64 *>(cand_key);
    const auto *cb = reinterpret_cast<const u64 *>(cand_bound);
    auto *oc = reinterpret_cast<unsigned *>(out_cost);
    if (Pp <= ONE_WAVE_MAX_PODS && batch == 1) {
        if (N <= AOS_MAX_NODES) {
            const size_t lds = round_up(16 * (size_t)N, 256) + PF_BYTES;
            static std::atomic<unsigned long long> attr{0};
            hipError_t e = set_lds_once(reinterpret_cast<const void *>(&k_commit_w<true, true>),
                                        LDS_DYN_MAX, attr);
            if (e != hipSuccess) return e;
            k_commit_w<true, true><<<batch, 64, lds, st>>>(ck, cb, req, Pp, p_begin, p_end, cap, N,
                                                           out_node, oc, halt, nullptr, zrow, stage_node,
                                                           sc, stage_status);
        } else if (N <= LDS_CAP_MAX_NODES) {
            const size_t lds = round_up(3 * (size_t)N * 4, 256) + PF_BYTES;  // cap_to_lds pieces + ring
            static std::atomic<unsigned long long> attr{0};
            hipError_t e = set_lds_once(reinterpret_cast<const void *>(&k_commit_w<true>),
                                        LDS_DYN_MAX, attr);
            if (e != hipSuccess) return e;
            k_commit_w<true><<<batch, 64, lds, st>>>(ck, cb, req, Pp, p_begin, p_end, cap, N,
                                                     out_node, oc, halt, nullptr, zrow, stage_node, sc, stage_status);
        } else {
            k_commit_w<false><<<batch, 64, PF_BYTES, st>>>(ck, cb, req, Pp, p_begin, p_end, cap, N,
                                                           out_node, oc, halt, pub, zrow, stage_node, sc, stage_status);
        }
        return hipGetLastError();
    }
    if (N <= LDS_CAP_MAX_NODES) {
        const size_t lds = round_up(3 * (size_t)N * 4, 256);  // cap_to_lds pieces
        static std::atomic<unsigned long long> attr{0};
        hipError_t e = set_lds_once(reinterpret_cast<const void *>(&k_commit<true>), LDS_DYN_MAX, attr);
        if (e != hipSuccess) return e;
        k_commit<true><<<batch, THREADS, lds, st>>>(ck, cb, req, Pp, p_begin, p_end, cap, N, out_node,
                                                oc, halt, nullptr, zrow, stage_node, sc, stage_status);
    } else {
        k_commit<false><<<batch, THREADS, 0, st>>>(ck, cb, req, Pp, p_begin, p_end, cap, N, out_node,
                                               oc, halt, pub, zrow, stage_node, sc, stage_status);
    }
    return hipGetLastError();
}

}  // namespace nas
