// rccl_init_probe.cpp -- probe behind nas_comm_init's design (profiles/r03_rccl_init_abort_probe.txt):
// rank 0 of a 2-rank communicator whose rank 1 never joins, init on a helper
// thread; the main thread reads the communicator handle RCCL publishes and
// aborts it after 3 s.  Does the helper return?  argv[1]: config.blocking (0 / 1).
// build: hipcc -O1 -std=c++17 tools/rccl_init_probe.cpp -o rccl_init_probe -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <dirent.h>
#include <thread>
#include <unistd.h>

static double now() {
    using namespace std::chrono;
    static const auto t0 = steady_clock::now();
    return duration<double>(steady_clock::now() - t0).count();
}
static int threads() {
    int n = 0;
    DIR *d = opendir("/proc/self/task");
    while (d && readdir(d)) ++n;
    if (d) closedir(d);
    return n - 2;
}

int main(int argc, char **argv) {
    const int blocking = argc > 1 ? atoi(argv[1]) : 0;
    (void)hipSetDevice(0);
    ncclUniqueId id;
    ncclGetUniqueId(&id);
    fprintf(stderr, "[%.3f] blocking=%d unique id done, threads %d\n", now(), blocking, threads());
    static ncclComm_t c = nullptr;
    std::atomic<int> done{0};
    std::atomic<int> rc{-1};
    std::thread h([&] {
        (void)hipSetDevice(0);
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = blocking;
        ncclResult_t r = ncclCommInitRankConfig(&c, 2, id, 0, &cfg);
        rc = (int)r;
        done = 1;
    });
    ncclComm_t seen = nullptr;
    for (int i = 0; i < 30 && !done; ++i) {
        seen = __atomic_load_n(&c, __ATOMIC_ACQUIRE);
        if (i % 10 == 0)
            fprintf(stderr, "[%.3f] handle %p done %d threads %d\n", now(), (void *)seen, done.load(),
                    threads());
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    seen = __atomic_load_n(&c, __ATOMIC_ACQUIRE);
    fprintf(stderr, "[%.3f] after 3 s: handle %p done %d rc %d\n", now(), (void *)seen, done.load(),
            rc.load());
    if (seen) {
        fprintf(stderr, "[%.3f] abort from main thread\n", now());
        ncclResult_t r = ncclCommAbort(seen);
        fprintf(stderr, "[%.3f] abort returned %d, helper done %d rc %d\n", now(), (int)r,
                done.load(), rc.load());
    }
    for (int i = 0; i < 50 && !done; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    fprintf(stderr, "[%.3f] helper done %d rc %d threads %d\n", now(), done.load(), rc.load(),
            threads());
    if (done) {
        h.join();
        std::this_thread::sleep_for(std::chrono::milliseconds(300));
        fprintf(stderr, "[%.3f] joined, threads %d\n", now(), threads());
        return 0;
    }
    h.detach();
    fprintf(stderr, "[%.3f] helper stuck\n", now());
    _exit(3);
}
