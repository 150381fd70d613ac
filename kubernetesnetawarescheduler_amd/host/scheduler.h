// scheduler.h -- C++ mirror of the reference's Go host (scheduler/scheduler.go
// CustomScheduler), calling the MI355X engine through include/nas.h.  Go is
// absent from this image, so the host side the north star wants in Go is
// here in C++ with the same structure, names, argument meanings and error
// behaviour; INTEGRATION.md shows the cgo binding a Go host would use instead.
//
//   Reference (scheduler.go)            Mirror
//   informer AddFunc filter :166-176    CustomScheduler::enqueue
//   podQueue (chan, cap 300) :129       bounded deque, kQueueCap
//   Schedule :189-237                   schedule_one (Bind, then Event)
//   findNodesThatFit :239-246           find_nodes_that_fit
//   prioritize :248-368                 prioritize: ingest (ingest.h) on the
//                                       host, the vote on the GPU
//                                       (nas_score_reference)
//   findBestNode :384-394               find_best_node (GPU result; the host
//                                       restatement is used only for the
//                                       priorities map it returns)
//   bindPod :370-382                    ClusterApi::bind
// Extensions (the north star's network-aware path, no reference counterpart):
//   schedule_batch: one metrics scrape for a batch of pods, one GPU call;
//   place_pending: fit + network cost + greedy commit for every queued pod
//   (nas_place) against node capacities, a pairwise latency matrix and the
//   pods' traffic to already-bound peers.
#pragma once

#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "ingest.h"

struct nas_ctx;

namespace nas_host {

constexpr const char *kSchedulerName = "netAwareScheduler";  // :121
constexpr size_t kQueueCap = 300;                              // make(chan *v1.Pod, 300)

struct Peer {
    std::string pod;  // "namespace/name" of a peer pod
    int weight;       // traffic volume (MB), any int32 (aggregated exactly)
};

// the fields of *v1.Pod the scheduler reads
struct Pod {
    std::string ns, name, uid, scheduler_name, node_name;
    int32_t cpu_milli = 0, mem_kib = 0;  // requests (network-aware path)
    std::vector<Peer> peers;             // communication graph (network-aware path)
};

// The API-server side (client-go in the reference).  Non-empty string = error.
struct ClusterApi {
    virtual ~ClusterApi() = default;
    virtual std::string list_nodes(std::vector<std::string> &names) = 0;    // nodeLister.List
    virtual std::string bind(const Pod &p, const std::string &node) = 0;    // Pods().Bind
    virtual std::string create_event(const Pod &p, const std::string &message) = 0;  // Events().Create
    // network-aware path: free capacity of a node, and where a pod is bound ("" = not bound)
    virtual bool node_capacity(const std::string &node, int32_t &cpu_milli, int32_t &mem_kib,
                               int32_t &pods) = 0;
    virtual std::string pod_node(const std::string &ns_name) = 0;
};

// Node-exporter scrapes and iperf report files (net/http and os in the reference)
struct MetricsSource {
    virtual ~MetricsSource() = default;
    virtual bool http_get(const std::string &url, std::string &body) = 0;  // false: transport error
    virtual bool read_file(const std::string &path, std::string &bytes) = 0;  // false: os.Open error
};

// Go's randomised map iteration, made explicit: the order of
// `range nodeMetricsMap` (:334, a permutation of the scraped nodes) and of
// `range priorities` (:387, a permutation of those nodes plus "none" = index n)
struct MapOrder {
    virtual ~MapOrder() = default;
    virtual void orders(int n, int32_t *order1, int32_t *order2) = 0;
};

// One scraped node: name (the getters branch on "ubuntu"), metrics URL, and
// the bandwidth source (:287 hard-codes 0.0 for "ubuntu").
struct Endpoint {
    std::string name, url;
};
std::vector<Endpoint> reference_topology();  // :275-279

struct Outcome {
    enum Kind { BOUND, NO_POD, LIST_ERROR, BIND_ERROR, EVENT_ERROR, PANIC, UNSCHEDULABLE } kind;
    std::string node, message;
};

class CustomScheduler {
public:
    CustomScheduler(nas_ctx *ctx, ClusterApi &api, MetricsSource &src, MapOrder &order);

    // informer AddFunc (:166-176): queue unbound pods that name this scheduler.
    // Returns false when filtered out; throws when the queue is full (the Go
    // channel send would block the informer).
    bool enqueue(const Pod &p);
    size_t queued() const { return queue_.size(); }

    // Schedule (:189-237): one pod, one scrape, one GPU vote, Bind, Event.
    Outcome schedule_one(Pod *popped = nullptr);
    // Batched: up to max_pods queued pods against ONE scrape (the reference
    // scrapes per pod), each with its own Go map orders, one GPU call.
    std::vector<std::pair<Pod, Outcome>> schedule_batch(int max_pods);

    // findNodesThatFit (:239-246); throws GoPanic as the reference panics
    std::string find_nodes_that_fit(const Pod &p, std::string &err);
    // prioritize (:248-368): the reference's map[string]int, keys in the
    // order `range` would visit them (order2)
    std::vector<std::pair<std::string, int>> prioritize(const Pod &p);

    // Network-aware placement of every queued pod (north star): returns
    // (pod, node or "" when nothing fits) in queue order, binding each placed pod.
    // costs on the latency set last: int8 ms (set_latency, exact integer
    // scores) or fp32 us (set_latency_f32, unquantised measurements)
    std::vector<std::pair<Pod, Outcome>> place_pending();
    // pairwise latency matrix for place_pending, indexed like `names`
    void set_latency(const std::vector<std::string> &names, const std::vector<int8_t> &L);
    void set_latency_f32(const std::vector<std::string> &names, const std::vector<float> &L);

    void set_topology(std::vector<Endpoint> t) { topo_ = std::move(t); }
    // replaces the reference's node -> report map (:505-510) entry by entry
    void add_iperf_path(const std::string &node, const std::string &path) {
        if (use_ref_iperf_) iperf_.clear();
        iperf_[node] = path;
        use_ref_iperf_ = false;
    }

    // the metric records of the last scrape (for tests / tracing)
    const std::vector<NodeMetrics> &last_metrics() const { return metrics_; }

private:
    void scrape();  // :275-331, throws GoPanic
    int vote(int P, const std::vector<int32_t> &o1, const std::vector<int32_t> &o2,
             std::vector<int32_t> &best, std::vector<int32_t> &winners);
    Outcome bind_and_event(const Pod &p, const std::string &node);

    nas_ctx *ctx_;
    ClusterApi &api_;
    MetricsSource &src_;
    MapOrder &order_;
    std::deque<Pod> queue_;
    std::vector<Endpoint> topo_;
    std::map<std::string, std::string> iperf_;
    bool use_ref_iperf_ = true;
    std::vector<NodeMetrics> metrics_;
    std::vector<int32_t> pod_snap_;  // vote(): every pod on snapshot 0
    std::vector<std::string> lat_names_;
    std::vector<int8_t> lat_;
    std::vector<float> lat_f_;
    bool lat_f32_ = false;  // place_pending on lat_f_ (NAS_DT_F32)
};

}  // namespace nas_host
