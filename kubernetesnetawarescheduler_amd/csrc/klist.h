// klist.h -- sorted candidate lists of packed keys (orderable cost << 32 |
// node) in registers: compare-exchange networks shared by the cost epilogue,
// the per-pod merge and the commit.
//
// A list is the KC = 8 smallest keys of some node subset plus a BOUND: every
// key of that subset that is <= bound is in the list (keys above it may have
// been dropped).  bound == KEY_INVALID means nothing was dropped, i.e. the
// list holds every fitting node of the subset.  Merging two lists keeps the
// 8 smallest keys and bound = min(bound_a, bound_b, kept[7]).
#pragma once

#include "nas_internal.h"

namespace nas {

typedef unsigned long long u64;
static_assert(KC == 8, "list networks are written for 8 candidates");

__device__ __forceinline__ u64 umin64(u64 a, u64 b) { return a < b ? a : b; }
__device__ __forceinline__ u64 umax64(u64 a, u64 b) { return a < b ? b : a; }
__device__ __forceinline__ void cex(u64 &a, u64 &b) {
    const u64 lo = umin64(a, b);
    b = umax64(a, b);
    a = lo;
}

// sort a bitonic sequence of 8 ascending
__device__ __forceinline__ void bitonic8(u64 (&x)[8]) {
    cex(x[0], x[4]); cex(x[1], x[5]); cex(x[2], x[6]); cex(x[3], x[7]);
    cex(x[0], x[2]); cex(x[1], x[3]); cex(x[4], x[6]); cex(x[5], x[7]);
    cex(x[0], x[1]); cex(x[2], x[3]); cex(x[4], x[5]); cex(x[6], x[7]);
}

// two sorted 4-lists -> one sorted 8-list
__device__ __forceinline__ void merge44(const u64 (&a)[4], const u64 (&b)[4], u64 (&out)[8]) {
    out[0] = a[0]; out[1] = a[1]; out[2] = a[2]; out[3] = a[3];
    out[4] = b[3]; out[5] = b[2]; out[6] = b[1]; out[7] = b[0];
    bitonic8(out);
}

// the 8 smallest of two sorted 8-lists, sorted, into a
__device__ __forceinline__ void merge88(u64 (&a)[8], const u64 (&b)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = umin64(a[i], b[7 - i]);
    bitonic8(a);
}

__device__ __forceinline__ u64 shfl_xor64(u64 x, int m) {
    const int lo = __shfl_xor((int)(unsigned)x, m);
    const int hi = __shfl_xor((int)(unsigned)(x >> 32), m);
    return ((u64)(unsigned)hi << 32) | (unsigned)lo;
}

// Per-lane running top-4 as separate (orderable cost, node) u32 words.
// A lane visits its nodes in ascending node order, so a new (x, n) sorts
// before entry j iff x < cost[j] strictly (an equal cost has the larger node):
// four independent 32-bit compares and a select network, no 64-bit compares.
// (cost all-ones is never inserted: the "does not fit" value of the callers)
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

__device__ __forceinline__ void load8(const u64 *p, u64 (&k)[8]) {
    const ulonglong2 *s = reinterpret_cast<const ulonglong2 *>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const ulonglong2 v = s[i];
        k[2 * i] = v.x;
        k[2 * i + 1] = v.y;
    }
}

__device__ __forceinline__ void store8(u64 *p, const u64 (&k)[8]) {
    ulonglong2 *d = reinterpret_cast<ulonglong2 *>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = make_ulonglong2(k[2 * i], k[2 * i + 1]);
}

}  // namespace nas
