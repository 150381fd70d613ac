// stage_order_probe.hip -- diagnostic for DESIGN.md §5 "pinned stage
// ordering" (VERDICT r4 item 7): the round-4 TAIL_SDMA variant moved the last
// chunk's results to the host with hipMemcpyAsync(D2H) behind the commit
// kernel on the same stream and returned stale rows.  This probe repeats that
// shape outside the engine and tells the candidate mechanisms apart:
//   a one-workgroup kernel writes n ints (values new every iteration) ->
//   hipMemcpyAsync D2H into pinned memory on the same stream -> event ->
//   the host polls the event (as wait_event does) and checks the rows;
//   then, after a full device synchronise, checks them again.
// Rows wrong at the event but right after the synchronise: the event
// completed before the copy's data landed (host-side ordering).  Rows wrong
// both times: the copy read the source before the kernel's stores were
// visible to it.  Streams: a plain non-blocking one and a CU-masked one
// (hipExtStreamCreateWithCUMask, as set_stream_masks makes on node shards),
// and the kernel-written stage of the kept path (the kernel stores straight
// into the pinned rows) as the control.
//   hipcc -O3 --offload-arch=gfx950 tools/stage_order_probe.hip -o tools/stage_order_probe
//   ./tools/stage_order_probe [iterations]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(2);                                                            \
        }                                                                            \
    } while (0)

// one workgroup, as k_commit: every thread writes its rows of `out`
// (and, for the control, the pinned rows directly)
__global__ void __launch_bounds__(1024) k_write(int *out, int *pinned, int n, int it) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int v = it * 1000003 + i;
        out[i] = v;
        if (pinned) pinned[i] = v;
    }
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int n = 8480;  // the C4 G = 2 tail chunk's pods
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    int *dev = nullptr, *pin = nullptr;
    CK(hipMalloc(&dev, n * 4));
    CK(hipHostMalloc(reinterpret_cast<void **>(&pin), n * 4, hipHostMallocDefault));
    hipStream_t plain, masked;
    CK(hipStreamCreateWithFlags(&plain, hipStreamNonBlocking));
    std::vector<uint32_t> mask((ncu + 31) / 32, 0);
    for (int b = 16; b < ncu; ++b) mask[b / 32] |= 1u << (b % 32);  // all but 2 CUs per XCD
    CK(hipExtStreamCreateWithCUMask(&masked, (uint32_t)mask.size(), mask.data()));
    hipEvent_t ev;
    CK(hipEventCreate(&ev));
    struct Mode {
        const char *name;
        hipStream_t st;
        bool kernel_writes_stage;
    } modes[] = {{"copy/plain", plain, false},
                 {"copy/cu-masked", masked, false},
                 {"kernel-stage/plain", plain, true},
                 {"kernel-stage/cu-masked", masked, true}};
    int bad_total = 0;
    for (const Mode &m : modes) {
        long long bad_ev = 0, bad_sync = 0;
        int iters_bad = 0;
        for (int it = 1; it <= iters; ++it) {
            k_write<<<1, 1024, 0, m.st>>>(dev, m.kernel_writes_stage ? pin : nullptr, n, it);
            if (!m.kernel_writes_stage) CK(hipMemcpyAsync(pin, dev, n * 4, hipMemcpyDeviceToHost, m.st));
            CK(hipEventRecord(ev, m.st));
            hipError_t q;
            while ((q = hipEventQuery(ev)) == hipErrorNotReady) {
            }
            CK(q);
            int b1 = 0;
            for (int i = 0; i < n; ++i) b1 += pin[i] != it * 1000003 + i;
            CK(hipDeviceSynchronize());
            int b2 = 0;
            for (int i = 0; i < n; ++i) b2 += pin[i] != it * 1000003 + i;
            bad_ev += b1;
            bad_sync += b2;
            iters_bad += b1 > 0;
        }
        std::printf("{\"mode\": \"%s\", \"iterations\": %d, \"iterations_with_stale_rows_at_event\": %d, "
                    "\"stale_rows_at_event\": %lld, \"stale_rows_after_sync\": %lld}\n",
                    m.name, iters, iters_bad, bad_ev, bad_sync);
        bad_total += iters_bad;
    }
    CK(hipEventDestroy(ev));
    CK(hipStreamDestroy(plain));
    CK(hipStreamDestroy(masked));
    CK(hipFree(dev));
    CK(hipHostFree(pin));
    return bad_total ? 1 : 0;
}
