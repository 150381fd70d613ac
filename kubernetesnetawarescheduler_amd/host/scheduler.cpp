// scheduler.cpp -- see scheduler.h.
#include "scheduler.h"

#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "nas.h"

namespace nas_host {
namespace {

void check(nas_ctx *ctx, int rc, const char *what) {
    if (rc != NAS_OK)
        throw std::runtime_error(std::string(what) + ": " + nas_last_error(ctx));
}

// nas_score_reference winner slots -> the += lines of :360-365
constexpr int kWeight[6] = {3, 2, 1, 1, 3, 1};  // NAS_W_CPU .. NAS_W_DISK

}  // namespace

std::vector<Endpoint> reference_topology() {
    return {{"ubuntu", "http://192.168.1.137:9100/metrics"},
            {"raspiworker0", "http://192.168.1.132:9100/metrics"},
            {"raspiworker1", "http://192.168.1.135:9100/metrics"},
            {"raspiworker2", "http://192.168.1.133:9100/metrics"},
            {"raspiworker3", "http://192.168.1.134:9100/metrics"}};
}

CustomScheduler::CustomScheduler(nas_ctx *ctx, ClusterApi &api, MetricsSource &src, MapOrder &order)
    : ctx_(ctx), api_(api), src_(src), order_(order), topo_(reference_topology()) {}

bool CustomScheduler::enqueue(const Pod &p) {
    if (!(p.node_name.empty() && p.scheduler_name == kSchedulerName)) return false;
    if (queue_.size() >= kQueueCap)
        throw std::runtime_error("pod queue full (the informer would block on the channel send)");
    queue_.push_back(p);
    return true;
}

void CustomScheduler::scrape() {
    // :275-279: every body first; a transport error leaves resp nil and
    // resp.Body dereferences it
    std::vector<std::string> bodies(topo_.size());
    for (size_t i = 0; i < topo_.size(); ++i)
        if (!src_.http_get(topo_[i].url, bodies[i]))
            throw GoPanic("runtime error: invalid memory address or nil pointer dereference");
    auto path = [&](std::string_view node) -> std::string {
        if (use_ref_iperf_) return reference_iperf_path(node);
        auto it = iperf_.find(std::string(node));
        return it == iperf_.end() ? std::string() : it->second;
    };
    auto read = [&](const std::string &p, std::string &b) { return src_.read_file(p, b); };
    metrics_.assign(topo_.size(), NodeMetrics{});
    // :281-331, struct-literal field order
    for (size_t i = 0; i < topo_.size(); ++i) {
        const std::string &name = topo_[i].name;
        const std::string &body = bodies[i];
        NodeMetrics m;
        m.cpu_frequency_hertz = get_current_cpu_usage(body);
        m.occupied_memory_percentage = get_occupied_memory_percentage(body);
        m.network_packets_received = get_network_packets_received(body, name);
        m.network_packets_sent = get_network_packets_sent(body, name);
        m.network_bandwidth = name == "ubuntu" ? 0.0 : get_network_bandwidth(name, path, read);
        m.disk_io_now = get_disk_io_now(body, name);
        metrics_[i] = m;
    }
}

int CustomScheduler::vote(int P, const std::vector<int32_t> &o1, const std::vector<int32_t> &o2,
                          std::vector<int32_t> &best, std::vector<int32_t> &winners) {
    const int n = (int)metrics_.size();
    // ONE snapshot (the scrape every pod of the batch sees); each pod walks
    // its own map orders (nas_upload_pod_orders), pod p -> snapshot 0
    std::vector<double> cpu(n), mem(n), bw(n);
    std::vector<int64_t> rx(n), tx(n), disk(n);
    for (int i = 0; i < n; ++i) {
        const NodeMetrics &m = metrics_[i];
        cpu[i] = m.cpu_frequency_hertz;
        mem[i] = m.occupied_memory_percentage;
        rx[i] = m.network_packets_received;
        tx[i] = m.network_packets_sent;
        bw[i] = m.network_bandwidth;
        disk[i] = m.disk_io_now;
    }
    check(ctx_, nas_upload_snapshot(ctx_, cpu.data(), mem.data(), rx.data(), tx.data(), bw.data(),
                                    disk.data(), n, 1),
          "nas_upload_snapshot");
    check(ctx_, nas_upload_pod_orders(ctx_, o1.data(), o2.data(), P), "nas_upload_pod_orders");
    pod_snap_.assign(P, 0);
    best.assign(P, 0);
    winners.assign((size_t)P * 6, 0);
    check(ctx_, nas_score_reference(ctx_, nullptr, nullptr, pod_snap_.data(), P, best.data(),
                                    winners.data()),
          "nas_score_reference");
    return n;
}

std::vector<std::pair<std::string, int>> CustomScheduler::prioritize(const Pod &) {
    scrape();
    const int n = (int)topo_.size();
    std::vector<int32_t> o1(n), o2(n + 1), best, win;
    order_.orders(n, o1.data(), o2.data());
    vote(1, o1, o2, best, win);
    // nodePriorities: the five names at 0 (:251-256), "none" created by the
    // always-"none" bandwidth winner (:364)
    std::vector<int> score(n + 1, 0);
    for (int s = 0; s < 6; ++s) score[win[s] < 0 ? n : win[s]] += kWeight[s];
    std::vector<std::pair<std::string, int>> out;
    for (int k = 0; k <= n; ++k) {
        const int key = o2[k];
        out.emplace_back(key == n ? std::string("none") : topo_[key].name, score[key]);
    }
    return out;
}

std::string CustomScheduler::find_nodes_that_fit(const Pod &, std::string &err) {
    std::vector<std::string> nodes;
    err = api_.list_nodes(nodes);  // :240-243 (the listed nodes are not used further)
    if (!err.empty()) return "";
    scrape();
    const int n = (int)topo_.size();
    std::vector<int32_t> o1(n), o2(n + 1), best, win;
    order_.orders(n, o1.data(), o2.data());
    vote(1, o1, o2, best, win);
    if (best[0] == NAS_NONE) return "none";
    if (best[0] == NAS_EMPTY) return "";
    return topo_[best[0]].name;
}

Outcome CustomScheduler::bind_and_event(const Pod &p, const std::string &node) {
    std::string err = api_.bind(p, node);  // :196-206
    if (!err.empty()) return {Outcome::BIND_ERROR, node, err};
    char msg[1024];
    std::snprintf(msg, sizeof msg, "Assigned pod %s to %s\n", p.name.c_str(), node.c_str());  // :212
    err = api_.create_event(p, msg);
    if (!err.empty()) return {Outcome::EVENT_ERROR, node, err};
    return {Outcome::BOUND, node, msg};
}

Outcome CustomScheduler::schedule_one(Pod *popped) {
    if (queue_.empty()) return {Outcome::NO_POD, "", "queue empty"};
    const Pod p = queue_.front();
    queue_.pop_front();
    if (popped) *popped = p;
    std::string err, node;
    try {
        node = find_nodes_that_fit(p, err);
    } catch (const GoPanic &e) {
        return {Outcome::PANIC, "", e.what()};
    }
    if (!err.empty()) return {Outcome::LIST_ERROR, "", err};  // :193-195: pod dropped
    return bind_and_event(p, node);
}

std::vector<std::pair<Pod, Outcome>> CustomScheduler::schedule_batch(int max_pods) {
    std::vector<std::pair<Pod, Outcome>> out;
    std::vector<Pod> pods;
    while (!queue_.empty() && (int)pods.size() < max_pods) {
        pods.push_back(queue_.front());
        queue_.pop_front();
    }
    if (pods.empty()) return out;
    std::vector<std::string> nodes;
    std::string err = api_.list_nodes(nodes);
    if (!err.empty()) {
        for (auto &p : pods) out.push_back({p, {Outcome::LIST_ERROR, "", err}});
        return out;
    }
    try {
        scrape();
    } catch (const GoPanic &e) {
        for (auto &p : pods) out.push_back({p, {Outcome::PANIC, "", e.what()}});
        return out;
    }
    const int n = (int)topo_.size(), P = (int)pods.size();
    std::vector<int32_t> o1((size_t)P * n), o2((size_t)P * (n + 1)), best, win;
    for (int p = 0; p < P; ++p) order_.orders(n, o1.data() + (size_t)p * n, o2.data() + (size_t)p * (n + 1));
    vote(P, o1, o2, best, win);
    for (int p = 0; p < P; ++p) {
        const std::string node = best[p] == NAS_NONE ? "none" : best[p] == NAS_EMPTY ? "" : topo_[best[p]].name;
        out.push_back({pods[p], bind_and_event(pods[p], node)});
    }
    return out;
}

void CustomScheduler::set_latency(const std::vector<std::string> &names, const std::vector<int8_t> &L) {
    if (L.size() != names.size() * names.size()) throw std::invalid_argument("latency matrix size");
    lat_names_ = names;
    lat_ = L;
    lat_f32_ = false;
}

void CustomScheduler::set_latency_f32(const std::vector<std::string> &names,
                                      const std::vector<float> &L) {
    if (L.size() != names.size() * names.size()) throw std::invalid_argument("latency matrix size");
    lat_names_ = names;
    lat_f_ = L;
    lat_f32_ = true;
}

std::vector<std::pair<Pod, Outcome>> CustomScheduler::place_pending() {
    std::vector<std::pair<Pod, Outcome>> out;
    std::vector<Pod> pods(queue_.begin(), queue_.end());
    queue_.clear();
    if (pods.empty()) return out;
    std::vector<std::string> nodes;
    std::string err = api_.list_nodes(nodes);
    if (!err.empty()) {
        for (auto &p : pods) out.push_back({p, {Outcome::LIST_ERROR, "", err}});
        return out;
    }
    const int n = (int)nodes.size(), P = (int)pods.size();
    std::map<std::string, int> lat_idx, node_idx;
    for (size_t i = 0; i < lat_names_.size(); ++i) lat_idx[lat_names_[i]] = (int)i;
    for (int i = 0; i < n; ++i) node_idx[nodes[i]] = i;
    // L over the listed nodes (every listed node must have been measured)
    std::vector<int8_t> L(lat_f32_ ? 0 : (size_t)n * n);
    std::vector<float> Lf(lat_f32_ ? (size_t)n * n : 0);
    for (int a = 0; a < n; ++a)
        for (int b = 0; b < n; ++b) {
            auto ia = lat_idx.find(nodes[a]), ib = lat_idx.find(nodes[b]);
            if (ia == lat_idx.end() || ib == lat_idx.end())
                throw std::runtime_error("no latency measured for node " +
                                         (ia == lat_idx.end() ? nodes[a] : nodes[b]));
            const size_t src = (size_t)ia->second * lat_names_.size() + ib->second;
            if (lat_f32_) Lf[(size_t)a * n + b] = lat_f_[src];
            else L[(size_t)a * n + b] = lat_[src];
        }
    std::vector<int32_t> cc(n), cm(n), cp(n);
    for (int i = 0; i < n; ++i)
        if (!api_.node_capacity(nodes[i], cc[i], cm[i], cp[i]))
            throw std::runtime_error("no capacity for node " + nodes[i]);
    std::vector<int32_t> rc(P), rm(P), rp(P, 1), row_ptr(P + 1, 0), peer_node;
    std::vector<int32_t> weight;  // exact: aggregated per node in int64 by the engine
    std::vector<float> weight_f;  // fp32 path: aggregated in fp64, rounded once
    for (int p = 0; p < P; ++p) {
        rc[p] = pods[p].cpu_milli;
        rm[p] = pods[p].mem_kib;
        for (const Peer &q : pods[p].peers) {
            const std::string where = api_.pod_node(q.pod);
            auto it = node_idx.find(where);
            peer_node.push_back(it == node_idx.end() ? -1 : it->second);  // unbound: skipped
            weight.push_back(q.weight);
            weight_f.push_back((float)q.weight);
        }
        row_ptr[p + 1] = (int32_t)peer_node.size();
    }
    if (lat_f32_) check(ctx_, nas_upload_latency(ctx_, Lf.data(), NAS_DT_F32, n), "nas_upload_latency");
    else check(ctx_, nas_upload_latency(ctx_, L.data(), NAS_DT_I8, n), "nas_upload_latency");
    check(ctx_, nas_upload_capacity(ctx_, cc.data(), cm.data(), cp.data(), n), "nas_upload_capacity");
    check(ctx_, nas_upload_pods(ctx_, rc.data(), rm.data(), rp.data(), P), "nas_upload_pods");
    check(ctx_, nas_upload_traffic_csr(ctx_, row_ptr.data(), peer_node.data(),
                                       lat_f32_ ? (const void *)weight_f.data() : weight.data(),
                                       lat_f32_ ? NAS_DT_F32 : NAS_DT_I32, P, n,
                                       (int64_t)peer_node.size()),
          "nas_upload_traffic_csr");
    std::vector<int32_t> node_out(P);
    check(ctx_, nas_place(ctx_, node_out.data(), nullptr, nullptr), "nas_place");
    for (int p = 0; p < P; ++p) {
        if (node_out[p] < 0) {
            out.push_back({pods[p], {Outcome::UNSCHEDULABLE, "", "no node fits the pod's requests"}});
            continue;
        }
        out.push_back({pods[p], bind_and_event(pods[p], nodes[node_out[p]])});
    }
    return out;
}

}  // namespace nas_host
