// k_misc.hip -- layout kernels (latency transpose, sparse traffic
// aggregation) and seeded synthetic input generators that write straight
// into HBM (benchmarks; SURVEY.md §8(d) workload shapes).
#include "nas_internal.h"

#include <algorithm>

namespace nas {
namespace {

// ---------------------------------------------------------------- transpose
// Lt[i][m] = L[m][n0 + i] for i < nloc, m < N; zero padding up to Mp x Kp.
template <typename T>
__global__ void k_transpose(const T *__restrict__ L, int N, int n0, int nloc, int Mp, int Kp,
                            T *__restrict__ Lt) {
    __shared__ T tile[64][65];
    const int m0 = blockIdx.x * 64;  // source row block (contraction index m)
    const int i0 = blockIdx.y * 64;  // destination row block (local node i)
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    for (int r = ty; r < 64; r += 4) {
        const int m = m0 + r, i = i0 + tx;
        tile[r][tx] = (m < N && i < nloc) ? L[(size_t)m * N + n0 + i] : T(0);
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int i = i0 + r, m = m0 + tx;
        if (i < Mp && m < Kp) Lt[(size_t)i * Kp + m] = tile[tx][r];
    }
}

// --------------------------------------------------------- CSR aggregation
// bf16 traffic: WA[p][m] = sum of weights of p's peers bound to node m (row
// zeroed before), in fp32, rounded once.  One thread per pod; peers per pod
// are few, so the O(nnz_p^2) dedupe walk is cheap and needs no atomics.  (The
// int8 path aggregates exactly on the host: nas_upload_traffic_csr.)
__global__ void k_csr_bf16(const int *__restrict__ row_ptr, const int *__restrict__ peer,
                           const unsigned short *__restrict__ w, int P, int N, int Kp,
                           unsigned short *__restrict__ WA) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int b = row_ptr[p], e = row_ptr[p + 1];
    for (int x = b; x < e; ++x) {
        const int m = peer[x];
        if (m < 0 || m >= N) continue;
        bool seen = false;
        for (int y = b; y < x && !seen; ++y) seen = peer[y] == m;
        if (seen) continue;
        float s = 0.f;
        for (int y = x; y < e; ++y)
            if (peer[y] == m) s += __uint_as_float((unsigned)w[y] << 16);
        // round to nearest even bf16 (s is finite)
        const unsigned u = __float_as_uint(s);
        WA[(size_t)p * Kp + m] = (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
}

// ---------------------------------------------------------------- synthetic
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long hsh(unsigned long long seed, unsigned long long a,
                                                  unsigned long long b, unsigned long long c) {
    return mix64(seed ^ mix64(a * 0x9e3779b97f4a7c15ull ^ mix64(b + 0x632be59bd9b4e019ull) ^
                              (c << 48)));
}
__device__ __forceinline__ double unit(unsigned long long h) {  // [0, 1)
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

// Reference-mode snapshots, SURVEY.md §8(d) C1: cpu = mean of 4 per-core
// frequencies in {0.6, 1.2, 1.5, 1.8} GHz (float32-rounded like
// strconv.ParseFloat(s, 32), scheduler.go:423-441); mem% = 100 - avail*100/total
// (:444-460) on float32-rounded byte counts; rx/tx ~ U[0, 1e6) with 10% zeros
// (Atoi failures, :474-478); bw 0 for node 0 ("ubuntu", :287) and 20% of the
// rest, else U(8e7, 9.5e7) bit/s; disk 0 in 30%, else U[1, 1000].
__global__ void k_synth_snap(unsigned long long seed, int lo, int nl, long long ns, int S,
                             double *__restrict__ cpu, double *__restrict__ mem,
                             double *__restrict__ bw, long long *__restrict__ rx,
                             long long *__restrict__ tx, long long *__restrict__ disk) {
    const long long total = (long long)S * ns;
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const long long s = t / ns;
        const int local = (int)(t - s * ns);
        const int node = lo + local;  // node index in the whole cluster
        if (local >= nl) {  // padding: never wins any comparison
            cpu[t] = __longlong_as_double(0x7ff8000000000000ll);
            mem[t] = cpu[t];
            bw[t] = cpu[t];
            rx[t] = 0x7fffffffffffffffll;
            tx[t] = rx[t];
            disk[t] = 0;
            continue;
        }
        const unsigned long long h0 = hsh(seed, s, node, 1), h1 = hsh(seed, s, node, 2);
        const unsigned long long h2 = hsh(seed, s, node, 3);
        const float freqs[4] = {6e8f, 1.2e9f, 1.5e9f, 1.8e9f};
        double f = 0;
        for (int c = 0; c < 4; ++c) f += (double)freqs[(h0 >> (8 * c)) & 3];
        cpu[t] = f / 4;
        const float totalb = (float)(1073741824.0 * (1 + ((h0 >> 40) & 7)));
        const float avail = (float)(unit(h1) * (double)totalb);
        mem[t] = 100.0 - (((double)avail * 100.0) / (double)totalb);
        rx[t] = ((h2 & 1023) < 102) ? 0 : (long long)((h2 >> 10) % 1000000);
        tx[t] = (((h2 >> 30) & 1023) < 102) ? 0 : (long long)((h2 >> 40) % 1000000);
        const unsigned long long h3 = hsh(seed, s, node, 4);
        bw[t] = (node == 0 || (h3 & 1023) < 205) ? 0.0 : 8e7 + unit(h3 * 0x2545f4914f6cdd1dull) * 1.5e7;
        disk[t] = ((h3 >> 12) % 100 < 30) ? 0 : (long long)(1 + (h3 >> 20) % 1000);
    }
}

// Extended-mode cluster (build-defined):
// nodes in racks of 32, racks in zones of 16; symmetric latency by distance
// class (0 self, 2-4 same rack, 12-19 same zone, 40-105 cross zone);
// traffic: dense background 0..2 to every node (thinned past 10k nodes, see
// k_synth_bg) plus `peers` heavy bound peers
// (16..127) in the pod's home rack / zone, saturated at 127;
// capacity cpu {4000, 8000} m, memory {4, 8} GiB, 110 pods; requests
// log-uniform over the clusterloader2 ranges (cpu 0.000213-0.5376 cores, mem
// 7.6-311 MB, datasets/clusterloader2/*/*.json), 1 pod slot.
__device__ __forceinline__ int lat(unsigned long long seed, int a, int b) {
    if (a == b) return 0;
    const int lo = min(a, b), hi = max(a, b);
    const unsigned long long h = hsh(seed, lo, hi, 7);
    if ((lo >> 5) == (hi >> 5)) return 2 + (int)(h % 3);
    if ((lo >> 9) == (hi >> 9)) return 12 + (int)(h % 8);
    return 40 + (int)((((hi >> 9) - (lo >> 9)) * 7) % 50) + (int)(h % 16);
}

// Profile 1 (NAS_OPT_SYNTH_PROFILE): SURVEY.md §8(d)'s C3
// operand distribution, uniform over the whole int8 range -- latency
// U{1..127} (the int8 form of U[1, 1000] us: ~7.9 us per step), symmetric,
// zero diagonal; traffic U{0..127} (the int8 form of U[0, 1)) to every node,
// no locality, no bound-peer structure
__device__ __forceinline__ int lat_uniform(unsigned long long seed, int a, int b) {
    if (a == b) return 0;
    return 1 + (int)(hsh(seed, min(a, b), max(a, b), 31) % 127);
}
__device__ __forceinline__ int latv(unsigned long long seed, int a, int b, int profile) {
    return profile == 1 ? lat_uniform(seed, a, b) : lat(seed, a, b);
}

template <typename T>
__device__ __forceinline__ T from_int(int v);
template <>
__device__ __forceinline__ signed char from_int<signed char>(int v) { return (signed char)v; }
template <>
__device__ __forceinline__ float from_int<float>(int v) { return (float)v; }
template <>
__device__ __forceinline__ unsigned short from_int<unsigned short>(int v) {
    // round to nearest even (exact for |v| <= 256)
    const unsigned u = __float_as_uint((float)v);
    return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// dense background traffic 0..2 to every node (every pod talks a little to
// everything: the contraction is genuinely dense), zero padding past N.
// Clusters larger than BG_NODES thin it out so that it does not swamp the
// peer traffic (at 50k nodes a full background would be ~50 GB per pod
// against ~0.6 GB to its peers, and every pod would rank nodes alike).
constexpr int BG_NODES = 10000;
// background traffic of pod p < P to node m < N (element t = p * Kp + m)
__device__ __forceinline__ int bg_value(unsigned long long seed, int N, long long t) {
    const unsigned long long h = mix64(seed ^ ((unsigned long long)t * 0x9e3779b97f4a7c15ull));
    // past BG_NODES nodes each entry is kept with probability BG_NODES / N: a
    // pod's total background volume stays that of a BG_NODES-node cluster
    // instead of growing with N
    const bool keep = N <= BG_NODES || (int)((h >> 32) % (unsigned)N) < BG_NODES;
    return keep ? (int)(h % 3) : 0;
}
template <typename T>
__global__ void k_synth_bg(unsigned long long seed, int N, int P, int Kp, long long total,
                           T *__restrict__ WA) {
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(t / Kp), m = (int)(t - (long long)p * Kp);
        WA[t] = from_int<T>(p < P && m < N ? bg_value(seed, N, t) : 0);
    }
}

// profile 1: uniform traffic U{0..127} to every node (zero padding past N)
template <typename T>
__global__ void k_synth_uniform(unsigned long long seed, int N, int P, int Kp, long long total,
                                T *__restrict__ WA) {
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(t / Kp), m = (int)(t - (long long)p * Kp);
        const unsigned long long h = mix64(seed ^ 0x5bd1e9955bd1e995ull ^
                                           ((unsigned long long)t * 0x9e3779b97f4a7c15ull));
        WA[t] = from_int<T>(p < P && m < N ? (int)(h >> 57) : 0);
    }
}

template <typename T>
__global__ void k_synth_lt(unsigned long long seed, int N, int n0, int nloc, int Mp, int Kp,
                           T *__restrict__ Lt, int profile) {
    const long long total = (long long)Mp * Kp;
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int i = (int)(t / Kp), m = (int)(t - (long long)i * Kp);
        Lt[t] = (i < nloc && m < N) ? from_int<T>(latv(seed, m, n0 + i, profile)) : T(0);
    }
}

template <typename T>
__global__ void k_synth_lfull(unsigned long long seed, int N, T *__restrict__ L, int profile) {
    const long long total = (long long)N * N;
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int m = (int)(t / N), n = (int)(t - (long long)m * N);
        L[t] = from_int<T>(latv(seed, m, n, profile));
    }
}

// The heavy peers of pod p: nodes[j], wts[j] for j < min(peers, 16) -- in the
// home rack (all but 2) and in the zone.
__device__ __forceinline__ int synth_peers(unsigned long long seed, int N, int p, int peers,
                                           int (&nodes)[16], int (&wts)[16]) {
    const int n_racks = (N + 31) / 32;
    const unsigned long long hp = hsh(seed, p, 0, 11);
    const int rack = (int)(hp % n_racks);
    const int np = min(peers, 16);
    for (int j = 0; j < np; ++j) {
        const unsigned long long h = hsh(seed, p, j + 1, 12);
        // uniform over the racks of the zone and the nodes of the rack (the
        // last zone / rack may be partial)
        int r = rack;
        if (!(j < np - 2 || np <= 2)) {  // another rack of the same zone
            const int zone0 = (rack >> 4) << 4;
            r = zone0 + (int)((h >> 20) % (unsigned)min(16, n_racks - zone0));
        }
        const int node = r * 32 + (int)(h % (unsigned)min(32, N - r * 32));
        nodes[j] = min(node, N - 1);
        wts[j] = 16 + (int)((h >> 40) % 112);
    }
    return np;
}

// one thread per pod: the heavy peers added on top of the background (exact
// sums; the int8 plane holds them clamped to [-128, 127], the excess goes to
// the overflow lists of launch_synth_overflow), and the pod's requests
template <typename T>
__global__ void k_synth_pods(unsigned long long seed, int N, int P, int peers, int Kp, int Pp,
                             T *__restrict__ WA, int *__restrict__ req) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= Pp) return;
    if (p >= P) { req[p] = 0; req[Pp + p] = 0; req[2 * Pp + p] = 0; return; }
    int nodes[16], wts[16];
    const int np = synth_peers(seed, N, p, peers, nodes, wts);
    for (int j = 0; j < np; ++j) {
        bool seen = false;
        for (int y = 0; y < j; ++y) seen |= nodes[y] == nodes[j];
        if (seen) continue;
        const long long t = (long long)p * Kp + nodes[j];
        int s = bg_value(seed, N, t);
        for (int y = j; y < np; ++y) s += nodes[y] == nodes[j] ? wts[y] : 0;
        if constexpr (sizeof(T) == 1) s = min(s, 127);  // the plane; the rest is overflow
        WA[t] = from_int<T>(s);
    }
    const unsigned long long hr = hsh(seed, p, 0, 13);
    const double lc0 = -3.6716, lc1 = -0.2695;  // log10 of 0.000213, 0.5376 cores
    const double lm0 = 6.8833, lm1 = 8.4928;    // log10 of 7.64e6, 3.11e8 bytes
    const double cores = pow(10.0, lc0 + (lc1 - lc0) * unit(hr));
    const double bytes = pow(10.0, lm0 + (lm1 - lm0) * unit(mix64(hr)));
    req[p] = max(1, (int)ceil(cores * 1000.0));
    req[Pp + p] = (int)ceil(bytes / 1024.0);
    req[2 * Pp + p] = 1;
}

// int8 overflow lists of the synthetic traffic (see launch_synth_overflow)
__global__ void k_synth_ovf(unsigned long long seed, int N, int P, int peers, int Kp, int pass,
                            int *__restrict__ cnt, const int *__restrict__ ptr,
                            int *__restrict__ om, int *__restrict__ oe) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    int nodes[16], wts[16];
    const int np = synth_peers(seed, N, p, peers, nodes, wts);
    int c = 0;
    const int base = pass ? ptr[p] : 0;
    for (int j = 0; j < np; ++j) {
        bool seen = false;
        for (int y = 0; y < j; ++y) seen |= nodes[y] == nodes[j];
        if (seen) continue;
        int s = bg_value(seed, N, (long long)p * Kp + nodes[j]);
        for (int y = j; y < np; ++y) s += nodes[y] == nodes[j] ? wts[y] : 0;
        if (s > 127) {
            if (pass) {
                om[base + c] = nodes[j];
                oe[base + c] = s - 127;
            }
            ++c;
        }
    }
    if (!pass) cnt[p] = c;
}

__global__ void k_synth_cap(unsigned long long seed, int N, int *__restrict__ cap) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const unsigned long long h = hsh(seed, n, 0, 21);
    cap[n] = (h & 1) ? 8000 : 4000;
    cap[N + n] = ((h >> 1) & 1) ? 8 * 1048576 : 4 * 1048576;
    cap[2 * N + n] = 110;
}

inline int grid_for(long long total, int threads) {
    long long g = (total + threads - 1) / threads;
    return (int)(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

// WA[pod[i]][node[i]] = val[i]
__global__ void k_plane_scatter(const int *__restrict__ pod, const int *__restrict__ node,
                                const signed char *__restrict__ val, long long n, int Kp,
                                signed char *__restrict__ WA) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        WA[(size_t)pod[i] * Kp + node[i]] = val[i];
}

__global__ void k_scatter_f32(const int *__restrict__ pod, const int *__restrict__ node,
                              const float *__restrict__ val, long long n, int Kp,
                              float *__restrict__ WA) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        WA[(size_t)pod[i] * Kp + node[i]] = val[i];
}

// Lr[m][i] = Lt[i][m], m < N, i < Mp: 64 x 64 tiles through LDS
__global__ void k_make_lr(const signed char *__restrict__ Lt, int N, int Mp, int Kp,
                          signed char *__restrict__ Lr) {
    __shared__ signed char tile[64][65];
    const int i0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int i = i0 + r, m = m0 + tx;
        tile[r][tx] = (i < Mp && m < Kp) ? Lt[(size_t)i * Kp + m] : 0;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int m = m0 + r, i = i0 + tx;
        if (m < N && i < Mp) Lr[(size_t)m * Mp + i] = tile[tx][r];
    }
}

// one wave per row: sum_k |plane[r][k]|, corrected by the row's overflow
// entries (|plane + e| - |plane|), max over rows into *out
__global__ void k_row_abs_max(const signed char *__restrict__ WA, long long rows, int Kp,
                              const int *__restrict__ optr, const int *__restrict__ om,
                              const int *__restrict__ oe, unsigned long long *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const long long w0 = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
    const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
    for (long long r = w0; r < rows; r += nw) {
        const signed char *row = WA + (size_t)r * Kp;
        long long s = 0;
        for (int k = lane * 4; k < Kp; k += 256) {
            const int v = *reinterpret_cast<const int *>(row + k);
            s += abs((signed char)(v & 0xff)) + abs((signed char)((v >> 8) & 0xff)) +
                 abs((signed char)((v >> 16) & 0xff)) + abs((signed char)(v >> 24));
        }
        if (optr)
            for (int j = optr[r] + lane; j < optr[r + 1]; j += 64) {
                const long long pl = row[om[j]];
                s += llabs(pl + oe[j]) - llabs(pl);
            }
        for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) atomicMax(out, (unsigned long long)s);
    }
}

__global__ void k_abs_max_i8(const signed char *__restrict__ a, long long n,
                             unsigned *__restrict__ out) {
    unsigned m = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        m = max(m, (unsigned)abs((int)a[i]));
    for (int o = 32; o; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

// NAS_OPT_INJECT_STALL_MS: one lane spins on the 100 MHz real-time counter
__global__ void k_stall(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

__global__ void k_pass_init(int *__restrict__ status, const int *__restrict__ cap,
                            int *__restrict__ cap_snap, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 2 * STATUS_INTS) status[t] = t == 0 ? -1 : 0;
    if (cap_snap)
        for (int i = t; i < n; i += gridDim.x * blockDim.x) cap_snap[i] = cap[i];
}

// device-to-device copy of n int32 (nas_reset_capacity): a kernel launch
// costs the host ~5 us where hipMemcpyAsync's device-to-device path cost
// 15-36 us per call (the marker trace of a reset-then-place cycle,
// gpurun_out/r06r/prof/trace_place)
__global__ void k_copy_i32(int *__restrict__ dst, const int *__restrict__ src, long long n,
                           int vec) {
    const long long n4 = vec ? n >> 2 : 0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride)
        reinterpret_cast<int4 *>(dst)[i] = reinterpret_cast<const int4 *>(src)[i];
    for (long long i = 4 * n4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = src[i];
}

__global__ void k_rehearse_replicate(unsigned long long *__restrict__ a, long long n, int G, int N) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long k = a[i];
        for (int r = 1; r < G; ++r)
            a[r * n + i] = k == ~0ull ? k : k + (unsigned long long)((long long)r * N / G);
    }
}

// In-process all-gather (nas_comm_init_local): dst[r][i] = src_r[i] for the
// G ranks' send buffers, pulled by the receiving rank on its own stream.
// blockIdx.y = source rank; 16-byte units when every pointer and the size
// allow it, else 8-byte units (every exchanged record is a multiple of 8 B).
template <typename U>
__global__ void k_local_gather(LocalSrcs srcs, U *__restrict__ dst, long long n) {
    const U *__restrict__ s = static_cast<const U *>(srcs.p[blockIdx.y]);
    U *__restrict__ d = dst + (long long)blockIdx.y * n;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        d[i] = s[i];
}

// fp32 -> bf16, round to nearest even (finite inputs)
__device__ __forceinline__ unsigned short bf16_rne(float x) {
    const unsigned u = __float_as_uint(x);
    return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }

// The fp32 contraction as a bf16 one (nas_api.hip prepare_split): x = h + m +
// l with h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) (each residual is
// exact in fp32), and the K axis extended six-fold so that sum_k A'[k] B'[k]
// = sum_k (Ah Bh + Ah Bm + Am Bh + Ah Bl + Al Bh + Am Bm): every term of the
// exact product down to 2^-24 relative; the dropped Am Bl + Al Bm + Al Bl are
// below 2^-23 of it.  Products of bf16 pairs are exact in the MFMA's fp32
// accumulation.  Segment s of a row holds plane A_PAT[s] (latency, pattern
// 0) or B_PAT[s] (traffic, pattern 1) of that row's K values.
__global__ void k_split6(const float *__restrict__ src, unsigned short *__restrict__ dst,
                         long long rows, int Kp, int pattern) {
    const long long n = rows * Kp;
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n;
         t += (long long)gridDim.x * blockDim.x) {
        const long long r = t / Kp;
        const int k = (int)(t - r * Kp);
        const float x = src[t];
        const unsigned short h = bf16_rne(x);
        const float r1 = x - bf16_f(h);
        const unsigned short m = bf16_rne(r1);
        const unsigned short l = bf16_rne(r1 - bf16_f(m));
        // A: h h m h l m     B: h m h l h m
        unsigned short *d = dst + (size_t)r * 6 * Kp + k;
        if (pattern == 0) {
            d[0] = h; d[(size_t)Kp] = h; d[(size_t)2 * Kp] = m;
            d[(size_t)3 * Kp] = h; d[(size_t)4 * Kp] = l; d[(size_t)5 * Kp] = m;
        } else {
            d[0] = h; d[(size_t)Kp] = m; d[(size_t)2 * Kp] = h;
            d[(size_t)3 * Kp] = l; d[(size_t)4 * Kp] = h; d[(size_t)5 * Kp] = m;
        }
    }
}

// The pass's commits run in chunk order on two streams -- the commit stream,
// then the tail chunk's own stream -- ordered by a device word instead of a
// stream-wait packet (~10-20 us on the pass's critical path even when the
// awaited event had long completed): after each commit the commit stream
// stores the commit's sequence number (a kernel boundary behind the commit,
// so its capacity and status writes are released first), and the tail
// stream's commit is preceded by a wait until the word reaches the last one.
// The wait is bounded: after `ticks` of the 100 MHz real-time clock (the
// caller's budget: the communicator deadline when the pass issued
// collectives, 2 s otherwise) it stores FLAG_TIMEOUT_HALT into the halt word,
// which the pass reports as its own error (NAS_ERR_COMM, communicators
// aborted, when collectives are involved) instead of hanging.
__global__ void k_flag_set(unsigned long long *flag, unsigned long long v) {
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_flag_wait(const unsigned long long *flag, unsigned long long v, int *halt,
                            unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < v) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            __hip_atomic_store(halt, FLAG_TIMEOUT_HALT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

}  // namespace

hipError_t launch_flag_set(hipStream_t st, uint64_t *flag, uint64_t v) {
    k_flag_set<<<1, 1, 0, st>>>(reinterpret_cast<unsigned long long *>(flag), v);
    return hipGetLastError();
}

hipError_t launch_flag_wait(hipStream_t st, const uint64_t *flag, uint64_t v, int32_t *halt,
                            int64_t budget_ms) {
    // 100 MHz real-time clock: 1e5 ticks per ms
    const unsigned long long ticks = (unsigned long long)std::max<int64_t>(budget_ms, 0) * 100000ull;
    k_flag_wait<<<1, 1, 0, st>>>(reinterpret_cast<const unsigned long long *>(flag), v, halt, ticks);
    return hipGetLastError();
}

hipError_t launch_pass_init(hipStream_t st, int32_t *status, const int32_t *cap, int32_t *cap_snap,
                            int n) {
    k_pass_init<<<cap_snap ? grid_for(n, 256) : 1, 256, 0, st>>>(status, cap, cap_snap, n);
    return hipGetLastError();
}

hipError_t launch_copy_i32(hipStream_t st, int32_t *dst, const int32_t *src, int64_t n) {
    if (n <= 0) return hipSuccess;
    // 16-byte moves when both buffers are 16-byte aligned (hipMalloc's), else dwords
    const bool vec = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
    k_copy_i32<<<grid_for(vec ? (n + 3) / 4 : n, 256), 256, 0, st>>>(dst, src, (long long)n, vec);
    return hipGetLastError();
}

hipError_t launch_rehearse_replicate(hipStream_t st, uint64_t *buf, size_t n, int G, int N) {
    k_rehearse_replicate<<<grid_for((long long)n, 256), 256, 0, st>>>(
        reinterpret_cast<unsigned long long *>(buf), (long long)n, G, N);
    return hipGetLastError();
}

hipError_t launch_local_gather(hipStream_t st, const LocalSrcs &srcs, int G, void *dst,
                               size_t bytes) {
    if (G < 1 || G > LOCAL_MAX_WORLD || bytes % 8) return hipErrorInvalidValue;
    if (bytes == 0) return hipSuccess;
    bool v16 = bytes % 16 == 0 && reinterpret_cast<uintptr_t>(dst) % 16 == 0;
    for (int r = 0; r < G; ++r) v16 = v16 && reinterpret_cast<uintptr_t>(srcs.p[r]) % 16 == 0;
    const long long n = (long long)(bytes / (v16 ? 16 : 8));
    const dim3 grid((unsigned)std::min<long long>((n + 255) / 256, 1024), G);
    if (v16)
        k_local_gather<uint4><<<grid, 256, 0, st>>>(srcs, static_cast<uint4 *>(dst), n);
    else
        k_local_gather<unsigned long long><<<grid, 256, 0, st>>>(
            srcs, static_cast<unsigned long long *>(dst), n);
    return hipGetLastError();
}

hipError_t launch_transpose_L(hipStream_t st, const void *L_dev, int dtype, int N, int n0,
                              int nloc, int Mp, int Kp, void *Lt) {
    dim3 grid((Kp + 63) / 64, (Mp + 63) / 64);
    if (dtype == NAS_DT_I8)
        k_transpose<signed char><<<grid, 256, 0, st>>>(static_cast<const signed char *>(L_dev), N,
                                                       n0, nloc, Mp, Kp,
                                                       static_cast<signed char *>(Lt));
    else if (dtype == NAS_DT_F32)
        k_transpose<float><<<grid, 256, 0, st>>>(static_cast<const float *>(L_dev), N, n0, nloc, Mp,
                                                 Kp, static_cast<float *>(Lt));
    else
        k_transpose<unsigned short><<<grid, 256, 0, st>>>(
            static_cast<const unsigned short *>(L_dev), N, n0, nloc, Mp, Kp,
            static_cast<unsigned short *>(Lt));
    return hipGetLastError();
}

hipError_t launch_csr_aggregate_bf16(hipStream_t st, const int32_t *row_ptr, const int32_t *peer,
                                     const uint16_t *w, int P, int N, int Kp, uint16_t *WA) {
    if (P <= 0) return hipSuccess;
    k_csr_bf16<<<(P + 255) / 256, 256, 0, st>>>(row_ptr, peer, w, P, N, Kp, WA);
    return hipGetLastError();
}

hipError_t launch_plane_scatter(hipStream_t st, const int32_t *pod, const int32_t *node,
                                const signed char *val, int64_t n, int Kp, signed char *WA) {
    if (n <= 0) return hipSuccess;
    k_plane_scatter<<<grid_for(n, 256), 256, 0, st>>>(pod, node, val, (long long)n, Kp, WA);
    return hipGetLastError();
}

hipError_t launch_scatter_f32(hipStream_t st, const int32_t *pod, const int32_t *node,
                              const float *val, int64_t n, int Kp, float *WA) {
    if (n <= 0) return hipSuccess;
    k_scatter_f32<<<grid_for(n, 256), 256, 0, st>>>(pod, node, val, (long long)n, Kp, WA);
    return hipGetLastError();
}

hipError_t launch_split6(hipStream_t st, const float *src, uint16_t *dst, int64_t rows, int Kp,
                         int pattern) {
    if (rows <= 0) return hipSuccess;
    const long long n = rows * (long long)Kp;
    k_split6<<<(int)std::min<long long>((n + 255) / 256, 65536), 256, 0, st>>>(
        src, reinterpret_cast<unsigned short *>(dst), (long long)rows, Kp, pattern);
    return hipGetLastError();
}

hipError_t launch_make_lr(hipStream_t st, const signed char *Lt, int N, int Mp, int Kp,
                          signed char *Lr) {
    k_make_lr<<<dim3((Mp + 63) / 64, (N + 63) / 64), 256, 0, st>>>(Lt, N, Mp, Kp, Lr);
    return hipGetLastError();
}

hipError_t launch_row_abs_max(hipStream_t st, const signed char *WA, int64_t rows, int Kp,
                              const int32_t *ovf_ptr, const int32_t *ovf_m, const int32_t *ovf_e,
                              unsigned long long *out) {
    if (rows <= 0) return hipSuccess;
    if (Kp % 4) return hipErrorInvalidValue;
    k_row_abs_max<<<grid_for(rows * 64, 256), 256, 0, st>>>(WA, (long long)rows, Kp, ovf_ptr,
                                                            ovf_m, ovf_e, out);
    return hipGetLastError();
}

hipError_t launch_abs_max_i8(hipStream_t st, const signed char *a, int64_t n, unsigned *out) {
    if (n <= 0) return hipSuccess;
    k_abs_max_i8<<<std::min(grid_for(n, 256), 4096), 256, 0, st>>>(a, (long long)n, out);
    return hipGetLastError();
}

hipError_t launch_stall(hipStream_t st, int64_t ms) {
    if (ms <= 0) return hipSuccess;
    k_stall<<<1, 64, 0, st>>>((unsigned long long)ms * 100000ull);
    return hipGetLastError();
}

hipError_t launch_synth_snapshots(hipStream_t st, uint64_t seed, int n, int lo, int nl,
                                  int64_t ns, int S, double *cpu, double *mem, double *bw,
                                  int64_t *rx, int64_t *tx, int64_t *disk) {
    (void)n;  // the generator is per (snapshot, node): a slice needs only its bounds
    k_synth_snap<<<grid_for((long long)S * ns, 256), 256, 0, st>>>(
        seed, lo, nl, ns, S, cpu, mem, bw, reinterpret_cast<long long *>(rx),
        reinterpret_cast<long long *>(tx), reinterpret_cast<long long *>(disk));
    return hipGetLastError();
}

template <typename T>
hipError_t synth_cluster_t(hipStream_t st, uint64_t seed, int N, int P, int peers, int n0, int nloc,
                           int Mp, int Kp, int Pp, void *Lt, void *WA, int32_t *req, void *L_full,
                           int profile) {
    hipError_t e;
    if (Lt) {
        k_synth_lt<T><<<grid_for((long long)Mp * Kp, 256), 256, 0, st>>>(seed, N, n0, nloc, Mp, Kp,
                                                                         static_cast<T *>(Lt), profile);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (L_full) {
        k_synth_lfull<T><<<grid_for((long long)N * N, 256), 256, 0, st>>>(
            seed, N, static_cast<T *>(L_full), profile);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (WA) {
        const long long tot = (long long)Pp * Kp;
        if (profile == 1)
            k_synth_uniform<T><<<grid_for(tot, 256), 256, 0, st>>>(seed, N, P, Kp, tot,
                                                                   static_cast<T *>(WA));
        else
            k_synth_bg<T><<<grid_for(tot, 256), 256, 0, st>>>(seed, N, P, Kp, tot, static_cast<T *>(WA));
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // (profile 1: no bound peers -- the launch writes the requests only)
        k_synth_pods<T><<<(Pp + 255) / 256, 256, 0, st>>>(seed, N, P, profile == 1 ? 0 : peers, Kp,
                                                           Pp, static_cast<T *>(WA), req);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_synth_cluster(hipStream_t st, uint64_t seed, int N, int P, int dtype, int peers,
                                int n0, int nloc, int Mp, int Kp, int Pp, void *Lt, void *WA,
                                int32_t *cap, int32_t *req, void *L_full, int profile) {
    hipError_t e = dtype == NAS_DT_I8
                       ? synth_cluster_t<signed char>(st, seed, N, P, peers, n0, nloc, Mp, Kp, Pp,
                                                      Lt, WA, req, L_full, profile)
                   : dtype == NAS_DT_F32
                       ? synth_cluster_t<float>(st, seed, N, P, peers, n0, nloc, Mp, Kp, Pp, Lt, WA,
                                                req, L_full, profile)
                       : synth_cluster_t<unsigned short>(st, seed, N, P, peers, n0, nloc, Mp, Kp,
                                                         Pp, Lt, WA, req, L_full, profile);
    if (e != hipSuccess) return e;
    if (cap) {
        k_synth_cap<<<(N + 255) / 256, 256, 0, st>>>(seed, N, cap);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_synth_overflow(hipStream_t st, uint64_t seed, int N, int P, int peers, int Kp,
                                 int pass, const signed char *WA, int32_t *ovf_cnt,
                                 const int32_t *ovf_ptr, int32_t *ovf_m, int32_t *ovf_e) {
    (void)WA;  // the aggregates are recomputed from the seed
    k_synth_ovf<<<(P + 255) / 256, 256, 0, st>>>(seed, N, P, peers, Kp, pass, ovf_cnt, ovf_ptr,
                                                  ovf_m, ovf_e);
    return hipGetLastError();
}


// zrow[r] = 1 iff row r of WA is all zero bytes and has no overflow entries:
// one wave per row, 16 bytes per lane per load (row_bytes is a multiple of 128)
__global__ void __launch_bounds__(256)
k_zero_rows(const unsigned char *__restrict__ WA, int64_t rows, int64_t row_bytes,
            const int32_t *__restrict__ ovf_ptr, uint8_t *__restrict__ zrow) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const uint4 *p = reinterpret_cast<const uint4 *>(WA + r * row_bytes);
    unsigned acc = 0;
    for (int64_t i = lane; i < row_bytes / 16; i += 64) {
        const uint4 v = p[i];
        acc |= v.x | v.y | v.z | v.w;
    }
    const bool nz = __ballot(acc != 0) != 0;
    if (lane == 0) zrow[r] = (!nz && (!ovf_ptr || ovf_ptr[r + 1] == ovf_ptr[r])) ? 1 : 0;
}

hipError_t launch_zero_rows(hipStream_t st, const void *WA, int64_t rows, int64_t row_bytes,
                            const int32_t *ovf_ptr, uint8_t *zrow) {
    if (rows <= 0) return hipSuccess;
    if (row_bytes % 16) return hipErrorInvalidValue;
    k_zero_rows<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(
        static_cast<const unsigned char *>(WA), rows, row_bytes, ovf_ptr, zrow);
    return hipGetLastError();
}

}  // namespace nas
