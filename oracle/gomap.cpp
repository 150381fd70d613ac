/*
 * gomap.cpp -- TEST INFRASTRUCTURE ONLY (bench.py's reference-mode CPU
 * baseline; see oracle.c's header for the rules).  The reference's per-pod
 * scoring with Go's data structures restated in C++ (Go is absent here):
 *
 *   nodeMetricsMap := map[string]PrometheusNodeMetrics{...}   scheduler.go:281-331
 *       (the struct fill, from in-memory snapshots instead of the scrapes)
 *   for node, nodeStats := range nodeMetricsMap { ... }         :334-359
 *   nodePriorities map[string]int, += 3/2/1/1/3/1               :250-256, :360-365
 *   findBestNode: for node, p := range priorities, maxP = 0      :384-394
 *
 * Go randomises map iteration; std::unordered_map walks its buckets.  The
 * orders actually walked are returned (order1 for the :334 loop, order2 for
 * the :387 loop, node index n = "none"), so the GPU can be checked on exactly
 * the orders this run used.  fill_ns / loop_ns split the time between building
 * the map (:281-331 minus the I/O) and the loops (:334-394).
 */
#include <chrono>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

struct Rec {  // PrometheusNodeMetrics (:24-32) + the node's index
    double cpu, mem;
    int64_t rx, tx;
    double bw;
    int64_t disk;
    int32_t idx;
};

}  // namespace

extern "C" int or_vote_gomap(int n, int P, const double *cpu, const double *mem, const int64_t *rx,
                             const int64_t *tx, const double *bw, const int64_t *disk,
                             int32_t *best_out, int32_t *order1_out, int32_t *order2_out,
                             int64_t *fill_ns, int64_t *loop_ns) {
    using clk = std::chrono::steady_clock;
    std::vector<std::string> names(n);
    for (int i = 0; i < n; ++i) names[i] = "node-" + std::to_string(i);
    const std::string none = "none";
    int64_t tf = 0, tl = 0;
    for (int p = 0; p < P; ++p) {
        const size_t b = (size_t)p * n;
        const auto t0 = clk::now();
        std::unordered_map<std::string, Rec> metrics;  // :281-331
        metrics.reserve(n);
        for (int i = 0; i < n; ++i)
            metrics.emplace(names[i], Rec{cpu[b + i], mem[b + i], rx[b + i], tx[b + i], bw[b + i],
                                          disk[b + i], i});
        const auto t1 = clk::now();
        // sentinels :258-265, winners "none" :267-272
        double s_cpu = 99999999999.0, s_mem = 99999999999.0, s_bw = 0.0;
        int64_t s_rx = 99999999999LL, s_tx = 99999999999LL, s_disk = 999;
        const std::string *b_cpu = &none, *b_mem = &none, *b_sent = &none, *b_rec = &none;
        const std::string *b_bw = &none, *b_disk = &none;
        int32_t *o1 = order1_out + b;
        int k = 0;
        for (const auto &kv : metrics) {  // :334
            const Rec &s = kv.second;
            o1[k++] = s.idx;
            if (s.cpu < s_cpu) { s_cpu = s.cpu; b_cpu = &kv.first; }       // :335-338
            if (s.mem < s_mem) { s_mem = s.mem; b_mem = &kv.first; }       // :339-342
            if (s.rx < s_rx) { s_rx = s.rx; b_rec = &kv.first; }           // :343-346
            if (s.tx < s_tx) { s_tx = s.tx; b_sent = &kv.first; }          // :347-350
            if (s.bw > s_bw) { s_bw = s.bw; b_sent = &kv.first; }          // :351-354 (sic)
            if (s.disk < s_disk && s.disk != 0) { s_disk = s.disk; b_disk = &kv.first; }  // :355
        }
        std::unordered_map<std::string, int> pri;  // :250-256 (every listed node at 0)
        pri.reserve(n + 1);
        for (int i = 0; i < n; ++i) pri.emplace(names[i], 0);
        pri[*b_cpu] += 3;   // :360
        pri[*b_mem] += 2;   // :361
        pri[*b_sent] += 1;  // :362
        pri[*b_rec] += 1;   // :363
        pri[*b_bw] += 3;    // :364 (always "none")
        pri[*b_disk] += 1;  // :365
        // findBestNode :384-394
        int maxp = 0;
        const std::string *best = nullptr;
        int32_t *o2 = order2_out + (size_t)p * (n + 1);
        k = 0;
        for (const auto &kv : pri) {
            o2[k++] = kv.first == none ? n : metrics.at(kv.first).idx;
            if (kv.second > maxp) { maxp = kv.second; best = &kv.first; }
        }
        if (k != n + 1) return -1;  // "none" is always created at :364
        best_out[p] = !best ? -1 : *best == none ? -2 : metrics.at(*best).idx;
        const auto t2 = clk::now();
        tf += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        tl += std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
    }
    if (fill_ns) *fill_ns = tf;
    if (loop_ns) *loop_ns = tl;
    return 0;
}
