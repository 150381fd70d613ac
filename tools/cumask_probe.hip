// cumask_probe.hip -- DIAGNOSTIC: how hipExtStreamCreateWithCUMask's bits map
// to the CUs of the 8 XCDs, and whether a kernel on a stream confined to a
// few reserved CUs starts at once while a LDS-filling kernel occupies every
// other CU (the node-shard pass's merge / commit chain beside the wide cost
// tile).
//   build: hipcc -O3 --offload-arch=gfx950 tools/cumask_probe.hip -o tools/cumask_probe
//   run:   tools/cumask_probe            (prints one JSON object)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <set>
#include <utility>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                           \
        }                                                                       \
    } while (0)

// one record per workgroup: XCC id and HW_ID (CU / SH / SE fields)
__global__ void where(unsigned *out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

// a workgroup that holds its CU's whole LDS for `ticks` of the 100 MHz clock
__global__ void hog(unsigned long long ticks, int *sink) {
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    if (threadIdx.x == 0 && lds[5] == -1) *sink = 1;
}

__global__ void tiny(int *p) {
    if (threadIdx.x == 0) p[blockIdx.x] = 1;
}

int main() {
    int ncu = 0;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    ncu = prop.multiProcessorCount;
    const int words = (ncu + 31) / 32;
    unsigned *rec;
    CK(hipMalloc(&rec, 2 * 4096 * 4));
    std::vector<unsigned> h(2 * 4096);
    printf("{\"cus\": %d", ncu);
    // which (xcc, se, sh, cu) does each single mask bit select?
    auto run_mask = [&](const std::vector<uint32_t> &mask, const char *name) -> int {
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
        where<<<2048, 64, 0, s>>>(rec);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), rec, 2 * 2048 * 4, hipMemcpyDeviceToHost));
        std::set<std::pair<unsigned, unsigned>> used;
        for (int i = 0; i < 2048; ++i) {
            const unsigned hw = h[2 * i + 1];
            const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            used.insert({h[2 * i], (se << 5) | (sh << 4) | cu});
        }
        printf(", \"%s\": [", name);
        bool first = true;
        for (auto &u : used) {
            printf("%s[%u,%u,%u,%u]", first ? "" : ",", u.first, u.second >> 5, (u.second >> 4) & 1,
                   u.second & 15);
            first = false;
        }
        printf("]");
        CK(hipStreamDestroy(s));
        return 0;
    };
    std::vector<uint32_t> m(words, 0);
    for (int b : {0, 1, 7, 8, 9, 31, 32, 255}) {
        if (b >= ncu) continue;
        std::fill(m.begin(), m.end(), 0u);
        m[b / 32] = 1u << (b % 32);
        char nm[32];
        snprintf(nm, sizeof nm, "bit%d", b);
        if (run_mask(m, nm)) return 1;
    }
    // latency of a tiny kernel on the reserved CUs (bits 0..R-1) while a hog
    // occupies the others (mask = the complement), vs both unmasked
    int *sink;
    CK(hipMalloc(&sink, 4096 * 4));
    CK(hipFuncSetAttribute((const void *)hog, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    for (int R : {0, 8, 16}) {
        std::vector<uint32_t> mh(words, 0xffffffffu), mt(words, 0u);
        for (int b = 0; b < R; ++b) {
            mh[b / 32] &= ~(1u << (b % 32));
            mt[b / 32] |= 1u << (b % 32);
        }
        if (R == 0) std::fill(mt.begin(), mt.end(), 0xffffffffu);
        hipStream_t sh, stt;
        CK(hipExtStreamCreateWithCUMask(&sh, words, mh.data()));
        CK(hipExtStreamCreateWithCUMask(&stt, words, mt.data()));
        hipEvent_t a, b, c, d;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventCreate(&c));
        CK(hipEventCreate(&d));
        // hog: 4 waves of ncu workgroups of 200 us each
        CK(hipEventRecord(a, sh));
        hog<<<4 * ncu, 256, 160 * 1024, sh>>>(20000, sink);
        CK(hipEventRecord(b, sh));
        // tiny kernels launched 100 us into the hog
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(100)) {
        }
        CK(hipEventRecord(c, stt));
        for (int i = 0; i < 8; ++i) tiny<<<64, 64, 0, stt>>>(sink);
        CK(hipEventRecord(d, stt));
        CK(hipDeviceSynchronize());
        float hog_ms = 0, tiny_ms = 0;
        CK(hipEventElapsedTime(&hog_ms, a, b));
        CK(hipEventElapsedTime(&tiny_ms, c, d));
        printf(", \"reserve%d\": {\"hog_ms\": %.3f, \"tiny8_ms\": %.3f}", R, hog_ms, tiny_ms);
        CK(hipStreamDestroy(sh));
        CK(hipStreamDestroy(stt));
    }
    printf("}\n");
    return 0;
}
