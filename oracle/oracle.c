/*
 * oracle.c -- CPU restatement of the placement decision path of
 * pablojara/kubernetesNetAwareScheduler (scheduler/scheduler.go).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: it may be linked or
 * executed only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  The product path (kubernetesnetawarescheduler_amd/)
 * never calls it, and must fail loudly rather than fall back to it.
 *
 * Two families of functions:
 *
 *  (1) REFERENCE MODE -- the vote scorer, bit-exact restatement of
 *      scheduler.go:248-394.  Go map iteration order is randomised, so the
 *      two map walks are explicit inputs:
 *        order1[N]   -- iteration order of `range nodeMetricsMap` (:334)
 *        order2[N+1] -- iteration order of `range priorities` (:387); the
 *                       value N stands for the "none" key that :364 creates.
 *      or_vote_literal() follows the Go statements one by one;
 *      or_vote_closed() is the associative (value, position) restatement the
 *      GPU kernel uses and is cross-checked against
 *      the literal loop exhaustively at N = 5.
 *      Parity pinning: the reference ships no tests or golden vectors
 *       and cannot be built here (Go is absent, and the
 *      file does not compile as shipped: scheduler.go:214, :235).  The
 *      literal loop is pinned by the hand-derived known-answer vectors of
 *      SURVEY.md Appendix A (tests/golden/vote_kat.json).
 *
 *  (2) EXTENDED MODE -- build-defined (no reference counterpart; parity vs
 *      the reference is "unpinned"):
 *        fit      req[p,r] <= free[n,r] for every resource r
 *        cost     cost[p,n] = sum_m WA[p,m] * L[m,n]   (int64, exact, for
 *                 int8 latency with int32 traffic -- the aggregated traffic is
 *                 never saturated; double for bf16 inputs)
 *        choose   argmin over fitting n of (cost, n) lexicographic
 *        commit   sequential greedy in pod order, free[n] -= req[p]
 *
 * Output codes follow include/nas.h: NAS_NONE (-2) = the "none" pseudo-node,
 * NAS_EMPTY (-1) = the empty string findBestNode returns when no score > 0
 * (reference mode) or "unschedulable" (extended mode).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_NONE (-2)
#define OR_EMPTY (-1)

/* winner slots, in the order of the += statements at scheduler.go:360-365 */
enum { W_CPU = 0, W_MEM = 1, W_NETSENT = 2, W_NETREC = 3, W_BW = 4, W_DISK = 5 };

/* sentinels: scheduler.go:258-265 (networkBandwith omitted -> 0.0) */
static const double SENT_CPU = 99999999999.0;
static const double SENT_MEM = 99999999999.0;
static const int64_t SENT_RX = 99999999999LL;
static const int64_t SENT_TX = 99999999999LL;
static const double SENT_BW = 0.0;
static const int64_t SENT_DISK = 999;

/* weights: scheduler.go:360-365 */
static const int WEIGHT[6] = {3, 2, 1, 1, 3, 1};

static void vote_accumulate(int n, const int32_t winners[6], const int32_t *order2,
                            int64_t *scores /* n+1, slot n = "none" */,
                            int32_t *best_out) {
    for (int i = 0; i <= n; ++i) scores[i] = 0;
    for (int w = 0; w < 6; ++w) {
        int key = winners[w] == OR_NONE ? n : winners[w];
        scores[key] += WEIGHT[w]; /* nodePriorities[bestX] += weight */
    }
    /* findBestNode, scheduler.go:384-394: maxP = 0, strict >, map order */
    int64_t maxp = 0;
    int32_t best = OR_EMPTY; /* bestNode = "" */
    for (int i = 0; i <= n; ++i) {
        int key = order2[i];
        if (scores[key] > maxp) {
            maxp = scores[key];
            best = key == n ? OR_NONE : key;
        }
    }
    *best_out = best;
}

/*
 * Literal restatement of scheduler.go:250-394 for one snapshot.
 * Returns 0, or -1 if an order is not a permutation.
 */
int or_vote_literal(int n, const double *cpu, const double *mem, const int64_t *rx,
                    const int64_t *tx, const double *bw, const int64_t *disk,
                    const int32_t *order1, const int32_t *order2, int32_t *best_out,
                    int32_t *winners_out /* 6 */, int64_t *scores_out /* n+1 or NULL */) {
    /* sampleMetrics, :258-265 */
    double s_cpu = SENT_CPU, s_mem = SENT_MEM, s_bw = SENT_BW;
    int64_t s_rx = SENT_RX, s_tx = SENT_TX, s_disk = SENT_DISK;
    /* best*Node := "none", :267-272 */
    int32_t b_cpu = OR_NONE, b_mem = OR_NONE, b_sent = OR_NONE, b_rec = OR_NONE;
    int32_t b_bw = OR_NONE, b_disk = OR_NONE;
    for (int i = 0; i < n; ++i) { /* for node, nodeStats := range nodeMetricsMap, :334 */
        int node = order1[i];
        if (node < 0 || node >= n) return -1;
        if (cpu[node] < s_cpu) { s_cpu = cpu[node]; b_cpu = node; }          /* :335-338 */
        if (mem[node] < s_mem) { s_mem = mem[node]; b_mem = node; }          /* :339-342 */
        if (rx[node] < s_rx) { s_rx = rx[node]; b_rec = node; }              /* :343-346 */
        if (tx[node] < s_tx) { s_tx = tx[node]; b_sent = node; }             /* :347-350 */
        if (bw[node] > s_bw) { s_bw = bw[node]; b_sent = node; }             /* :351-354, sic */
        if (disk[node] < s_disk && disk[node] != 0) { s_disk = disk[node]; b_disk = node; } /* :355 */
    }
    int32_t w[6];
    w[W_CPU] = b_cpu; w[W_MEM] = b_mem; w[W_NETSENT] = b_sent; w[W_NETREC] = b_rec;
    w[W_BW] = b_bw; /* never assigned: always "none" (:271, :364) */
    w[W_DISK] = b_disk;
    int64_t *scores = scores_out ? scores_out : (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    for (int i = 0; i <= n; ++i)
        if (order2[i] < 0 || order2[i] > n) { if (!scores_out) free(scores); return -1; }
    vote_accumulate(n, w, order2, scores, best_out);
    if (!scores_out) free(scores);
    if (winners_out) memcpy(winners_out, w, sizeof(w));
    return 0;
}

/*
 * Closed-form restatement: every winner is the first
 * position in order1 attaining the extremum among values that beat the
 * sentinel; net-sent is whichever of (argmin tx, argmax bw) sits later in
 * order1.  Works from pos1 = inverse(order1), visiting nodes in storage
 * order -- the same associative formulation the HIP vote kernel reduces.
 */
int or_vote_closed(int n, const double *cpu, const double *mem, const int64_t *rx,
                   const int64_t *tx, const double *bw, const int64_t *disk,
                   const int32_t *order1, const int32_t *order2, int32_t *best_out,
                   int32_t *winners_out) {
    int32_t *pos = (int32_t *)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) pos[i] = -1;
    for (int i = 0; i < n; ++i) {
        if (order1[i] < 0 || order1[i] >= n || pos[order1[i]] != -1) { free(pos); return -1; }
        pos[order1[i]] = i;
    }
    /* (value, pos) candidates; pos = INT32_MAX means "none" */
    double v_cpu = 0, v_mem = 0, v_bw = 0;
    int64_t v_rx = 0, v_tx = 0, v_disk = 0;
    int32_t p_cpu = INT32_MAX, p_mem = INT32_MAX, p_rx = INT32_MAX, p_tx = INT32_MAX;
    int32_t p_bw = INT32_MAX, p_disk = INT32_MAX;
    for (int node = 0; node < n; ++node) {
        int32_t q = pos[node];
        if (cpu[node] < SENT_CPU &&
            (p_cpu == INT32_MAX || cpu[node] < v_cpu || (!(v_cpu < cpu[node]) && q < p_cpu))) {
            v_cpu = cpu[node]; p_cpu = q;
        }
        if (mem[node] < SENT_MEM &&
            (p_mem == INT32_MAX || mem[node] < v_mem || (!(v_mem < mem[node]) && q < p_mem))) {
            v_mem = mem[node]; p_mem = q;
        }
        if (rx[node] < SENT_RX && (p_rx == INT32_MAX || rx[node] < v_rx || (rx[node] == v_rx && q < p_rx))) {
            v_rx = rx[node]; p_rx = q;
        }
        if (tx[node] < SENT_TX && (p_tx == INT32_MAX || tx[node] < v_tx || (tx[node] == v_tx && q < p_tx))) {
            v_tx = tx[node]; p_tx = q;
        }
        if (bw[node] > SENT_BW &&
            (p_bw == INT32_MAX || bw[node] > v_bw || (!(v_bw > bw[node]) && q < p_bw))) {
            v_bw = bw[node]; p_bw = q;
        }
        if (disk[node] != 0 && disk[node] < SENT_DISK &&
            (p_disk == INT32_MAX || disk[node] < v_disk || (disk[node] == v_disk && q < p_disk))) {
            v_disk = disk[node]; p_disk = q;
        }
    }
    int32_t w[6];
#define NODE_AT(p) ((p) == INT32_MAX ? OR_NONE : order1[(p)])
    w[W_CPU] = NODE_AT(p_cpu);
    w[W_MEM] = NODE_AT(p_mem);
    {
        int32_t ps = INT32_MAX;
        if (p_tx != INT32_MAX) ps = p_tx;
        if (p_bw != INT32_MAX && (ps == INT32_MAX || p_bw > ps)) ps = p_bw;
        w[W_NETSENT] = NODE_AT(ps);
    }
    w[W_NETREC] = NODE_AT(p_rx);
    w[W_BW] = OR_NONE;
    w[W_DISK] = NODE_AT(p_disk);
#undef NODE_AT
    free(pos);
    for (int i = 0; i <= n; ++i)
        if (order2[i] < 0 || order2[i] > n) return -1;
    int64_t *scores = (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    vote_accumulate(n, w, order2, scores, best_out);
    free(scores);
    if (winners_out) memcpy(winners_out, w, sizeof(w));
    return 0;
}

/*
 * Batched reference mode, the shape nas_score_reference() takes:
 * snapshots are SoA blocks of n nodes; snapshot s uses order set
 * (n_orders == 1 ? 0 : s); pod p uses snapshot pod_snapshot[p] (or p).
 */
int or_vote_batch(int n, int n_snapshots, const double *cpu, const double *mem,
                  const int64_t *rx, const int64_t *tx, const double *bw, const int64_t *disk,
                  const int32_t *order1, const int32_t *order2, int n_orders,
                  const int32_t *pod_snapshot, int P, int32_t *best_out, int32_t *winners_out) {
    int err = 0;
    /* pods are independent (one Schedule call each); OMP_NUM_THREADS=1 is the
     * reference's single goroutine */
#pragma omp parallel for schedule(dynamic, 16) reduction(| : err)
    for (int p = 0; p < P; ++p) {
        int s = pod_snapshot ? pod_snapshot[p] : p;
        if (s < 0 || s >= n_snapshots) {
            err |= 1;
            continue;
        }
        int o = n_orders == 1 ? 0 : s;
        size_t b = (size_t)s * n;
        int rc = or_vote_literal(n, cpu + b, mem + b, rx + b, tx + b, bw + b, disk + b,
                                 order1 + (size_t)o * n, order2 + (size_t)o * (n + 1),
                                 best_out + p, winners_out ? winners_out + (size_t)6 * p : NULL,
                                 NULL);
        if (rc) err |= 1;
    }
    return err ? -1 : 0;
}

/* ------------------------------------------------------------------------ */
/* Extended mode (build-defined)                                             */
/* ------------------------------------------------------------------------ */

static inline double bf16_to_f64(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return (double)f;
}

static inline int fits(int32_t rc, int32_t rm, int32_t rp, int32_t fc, int32_t fm, int32_t fp) {
    return rc <= fc && rm <= fm && rp <= fp;
}

/* resource-fit filter: mask[p*W + n/32] bit (n%32) set iff pod p fits node n */
void or_fit(int P, int N, const int32_t *rc, const int32_t *rm, const int32_t *rp,
            const int32_t *fc, const int32_t *fm, const int32_t *fp, uint32_t *mask) {
    int W = (N + 31) / 32;
    for (int p = 0; p < P; ++p) {
        uint32_t *row = mask + (size_t)p * W;
        for (int w = 0; w < W; ++w) row[w] = 0;
        for (int n = 0; n < N; ++n)
            if (fits(rc[p], rm[p], rp[p], fc[n], fm[n], fp[n])) row[n >> 5] |= 1u << (n & 31);
    }
}

/* one cost row, int32 traffic x int8 latency: exact int64 */
static void cost_row_i8(int N, const int32_t *wa_row, const int8_t *L, int64_t *out) {
    for (int n = 0; n < N; ++n) out[n] = 0;
    for (int m = 0; m < N; ++m) {
        int64_t w = wa_row[m];
        if (!w) continue;
        const int8_t *lr = L + (size_t)m * N;
        for (int n = 0; n < N; ++n) out[n] += w * lr[n];
    }
}

/* one cost row, bf16 inputs: double accumulation (products of two bf16 are exact in double) */
static void cost_row_bf16(int N, const uint16_t *wa_row, const uint16_t *L, double *out) {
    for (int n = 0; n < N; ++n) out[n] = 0.0;
    for (int m = 0; m < N; ++m) {
        double w = bf16_to_f64(wa_row[m]);
        if (w == 0.0) continue;
        const uint16_t *lr = L + (size_t)m * N;
        for (int n = 0; n < N; ++n) out[n] += w * bf16_to_f64(lr[n]);
    }
}

/* one cost row, fp32 inputs: double accumulation (products of two floats are
 * exact in double; the sum's rounding is ~1e-16 relative) */
static void cost_row_f32(int N, const float *wa_row, const float *L, double *out) {
    for (int n = 0; n < N; ++n) out[n] = 0.0;
    for (int m = 0; m < N; ++m) {
        double w = wa_row[m];
        if (w == 0.0) continue;
        const float *lr = L + (size_t)m * N;
        for (int n = 0; n < N; ++n) out[n] += w * (double)lr[n];
    }
}

void or_cost_f32(int P, int N, const float *WA, const float *L, double *cost) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int p = 0; p < P; ++p) cost_row_f32(N, WA + (size_t)p * N, L, cost + (size_t)p * N);
}

void or_cost_i8(int P, int N, const int32_t *WA, const int8_t *L, int64_t *cost) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int p = 0; p < P; ++p) cost_row_i8(N, WA + (size_t)p * N, L, cost + (size_t)p * N);
}

void or_cost_bf16(int P, int N, const uint16_t *WA, const uint16_t *L, double *cost) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int p = 0; p < P; ++p) cost_row_bf16(N, WA + (size_t)p * N, L, cost + (size_t)p * N);
}

/*
 * Top-k candidates per pod among nodes set in mask, ordered by (cost, node)
 * ascending.  count[p] = number of valid entries (< k iff fewer nodes fit).
 * cost given as int64 (i8 path) or double (bf16 path; pass one of them).
 */
void or_topk(int P, int N, int k, const int64_t *cost_i, const double *cost_d,
             const uint32_t *mask, int32_t *cand_node, int64_t *cand_cost_i,
             double *cand_cost_d, int32_t *count) {
    int W = (N + 31) / 32;
#pragma omp parallel for schedule(dynamic, 8)
    for (int p = 0; p < P; ++p) {
        int32_t *cn = cand_node + (size_t)p * k;
        int c = 0;
        for (int n = 0; n < N; ++n) {
            if (!(mask[(size_t)p * W + (n >> 5)] >> (n & 31) & 1)) continue;
            /* insert (cost, n) into sorted list of length c (<= k) */
            int j = c < k ? c : k;
            if (cost_i) {
                int64_t v = cost_i[(size_t)p * N + n];
                int64_t *cc = cand_cost_i + (size_t)p * k;
                if (c == k && !(v < cc[k - 1])) continue; /* ties: lower n already present */
                while (j > 0 && v < cc[j - 1]) {
                    if (j < k) { cc[j] = cc[j - 1]; cn[j] = cn[j - 1]; }
                    --j;
                }
                if (j < k) { cc[j] = v; cn[j] = n; }
            } else {
                double v = cost_d[(size_t)p * N + n];
                double *cc = cand_cost_d + (size_t)p * k;
                if (c == k && !(v < cc[k - 1])) continue;
                while (j > 0 && v < cc[j - 1]) {
                    if (j < k) { cc[j] = cc[j - 1]; cn[j] = cn[j - 1]; }
                    --j;
                }
                if (j < k) { cc[j] = v; cn[j] = n; }
            }
            if (c < k) ++c;
        }
        count[p] = c;
        for (int j = c; j < k; ++j) {
            cn[j] = -1;
            if (cost_i) cand_cost_i[(size_t)p * k + j] = 0;
            else cand_cost_d[(size_t)p * k + j] = 0.0;
        }
    }
}

/*
 * Sequential greedy placement, the extended-mode oracle proper.  free_* are
 * updated in place.  Cost rows are computed in parallel blocks (they do not
 * depend on capacity); the commit walk is strictly sequential in pod order.
 * dtype: 1 = int32 traffic x int8 latency (exact int64 costs), 2 = bf16
 * (double costs), 3 = fp32 (double costs).
 */
int or_place(int P, int N, int dtype, const void *WA, const void *L, const int32_t *rc,
             const int32_t *rm, const int32_t *rp, int32_t *fc, int32_t *fm, int32_t *fp,
             int32_t *node_out, int64_t *cost_i_out, double *cost_d_out) {
    const int B = 64;
    int64_t *ci = NULL;
    double *cd = NULL;
    if (dtype == 1) ci = (int64_t *)malloc(sizeof(int64_t) * (size_t)B * N);
    else if (dtype == 2 || dtype == 3) cd = (double *)malloc(sizeof(double) * (size_t)B * N);
    else return -1;
    for (int p0 = 0; p0 < P; p0 += B) {
        int nb = P - p0 < B ? P - p0 : B;
#pragma omp parallel for schedule(dynamic, 1)
        for (int i = 0; i < nb; ++i) {
            if (ci) cost_row_i8(N, (const int32_t *)WA + (size_t)(p0 + i) * N, (const int8_t *)L,
                                ci + (size_t)i * N);
            else if (dtype == 3) cost_row_f32(N, (const float *)WA + (size_t)(p0 + i) * N,
                                              (const float *)L, cd + (size_t)i * N);
            else cost_row_bf16(N, (const uint16_t *)WA + (size_t)(p0 + i) * N,
                               (const uint16_t *)L, cd + (size_t)i * N);
        }
        for (int i = 0; i < nb; ++i) {
            int p = p0 + i, best = -1;
            for (int n = 0; n < N; ++n) {
                if (!fits(rc[p], rm[p], rp[p], fc[n], fm[n], fp[n])) continue;
                if (best < 0) { best = n; continue; }
                if (ci ? ci[(size_t)i * N + n] < ci[(size_t)i * N + best]
                       : cd[(size_t)i * N + n] < cd[(size_t)i * N + best])
                    best = n;
            }
            node_out[p] = best < 0 ? OR_EMPTY : best;
            if (best >= 0) {
                fc[best] -= rc[p]; fm[best] -= rm[p]; fp[best] -= rp[p];
                if (cost_i_out) cost_i_out[p] = ci ? ci[(size_t)i * N + best] : 0;
                if (cost_d_out) cost_d_out[p] = ci ? (double)ci[(size_t)i * N + best] : cd[(size_t)i * N + best];
            } else {
                if (cost_i_out) cost_i_out[p] = 0;
                if (cost_d_out) cost_d_out[p] = 0.0;
            }
        }
    }
    free(ci);
    free(cd);
    return 0;
}

/*
 * Commit from candidate lists (what the GPU commit kernel does): pods in
 * order take their first candidate (of the count[p] usable ones) that still
 * fits.  A pod whose usable candidates all fail while its list is not
 * complete (complete[p] == 0; NULL means complete iff count < k) needs a
 * rescore: return its index in *stop (and commit nothing for it); *stop = P
 * when all pods were committed.  A complete list whose candidates all fail
 * means the pod is unschedulable (NAS_EMPTY).
 */
void or_commit(int P, int k, const int32_t *cand_node, const int32_t *count,
               const int32_t *complete, const int32_t *rc, const int32_t *rm, const int32_t *rp,
               int32_t *fc, int32_t *fm, int32_t *fp, int32_t *node_out, int32_t *slot_out,
               int *stop) {
    for (int p = 0; p < P; ++p) {
        int chosen = -1, slot = -1;
        for (int j = 0; j < count[p]; ++j) {
            int n = cand_node[(size_t)p * k + j];
            if (fits(rc[p], rm[p], rp[p], fc[n], fm[n], fp[n])) { chosen = n; slot = j; break; }
        }
        if (chosen < 0 && !(complete ? complete[p] : count[p] < k)) { *stop = p; return; }
        node_out[p] = chosen < 0 ? OR_EMPTY : chosen;
        if (slot_out) slot_out[p] = slot;
        if (chosen >= 0) { fc[chosen] -= rc[p]; fm[chosen] -= rm[p]; fp[chosen] -= rp[p]; }
    }
    *stop = P;
}
