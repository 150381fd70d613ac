// capi.cpp -- extern "C" surface of the host mirror (include/nas_host.h):
// adapts the callback table to the C++ interfaces of scheduler.h and keeps
// every exception on this side of the ABI.
#include <algorithm>
#include <cstring>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "go_json.h"
#include "go_semantics.h"
#include "ingest.h"
#include "latency.h"
#include "nas_host.h"
#include "scheduler.h"

struct nas_host_buf {
    std::string s;
};

using namespace nas_host;

namespace {

void copy_str(char *dst, size_t cap, const std::string &s) {
    if (!dst || cap == 0) return;
    const size_t n = std::min(cap - 1, s.size());
    std::memcpy(dst, s.data(), n);
    dst[n] = 0;
}

struct CbApi : ClusterApi {
    nas_host_io io;
    std::string list_nodes(std::vector<std::string> &names) override {
        nas_host_buf b, e;
        if (!io.list_nodes) return "list_nodes callback missing";
        if (io.list_nodes(io.user, &b, &e) != 0) return e.s.empty() ? "list nodes failed" : e.s;
        names.clear();
        size_t a = 0;
        while (a < b.s.size()) {
            size_t z = b.s.find('\n', a);
            if (z == std::string::npos) z = b.s.size();
            if (z > a) names.push_back(b.s.substr(a, z - a));
            a = z + 1;
        }
        return "";
    }
    std::string bind(const Pod &p, const std::string &node) override {
        nas_host_buf e;
        if (!io.bind) return "bind callback missing";
        if (io.bind(io.user, p.ns.c_str(), p.name.c_str(), node.c_str(), &e) != 0)
            return e.s.empty() ? "bind failed" : e.s;
        return "";
    }
    std::string create_event(const Pod &p, const std::string &msg) override {
        nas_host_buf e;
        if (!io.create_event) return "";
        if (io.create_event(io.user, p.ns.c_str(), p.name.c_str(), p.uid.c_str(), msg.c_str(), &e) != 0)
            return e.s.empty() ? "event create failed" : e.s;
        return "";
    }
    bool node_capacity(const std::string &node, int32_t &c, int32_t &m, int32_t &p) override {
        return io.node_capacity && io.node_capacity(io.user, node.c_str(), &c, &m, &p) == 0;
    }
    std::string pod_node(const std::string &ns_name) override {
        nas_host_buf b;
        if (!io.pod_node || io.pod_node(io.user, ns_name.c_str(), &b) != 0) return "";
        return b.s;
    }
};

struct CbSource : MetricsSource {
    nas_host_io io;
    bool http_get(const std::string &url, std::string &body) override {
        nas_host_buf b;
        if (!io.http_get || io.http_get(io.user, url.c_str(), &b) != 0) return false;
        body = std::move(b.s);
        return true;
    }
    bool read_file(const std::string &path, std::string &bytes) override {
        nas_host_buf b;
        if (!io.read_file || io.read_file(io.user, path.c_str(), &b) != 0) return false;
        bytes = std::move(b.s);
        return true;
    }
};

struct CbOrder : MapOrder {
    nas_host_io io;
    void orders(int n, int32_t *o1, int32_t *o2) override {
        for (int i = 0; i < n; ++i) o1[i] = i;
        for (int i = 0; i <= n; ++i) o2[i] = i;
        if (io.map_order) io.map_order(io.user, n, o1, o2);
    }
};

void fill(nas_host_outcome &o, const Pod &p, const Outcome &r) {
    static const int32_t kind[] = {NAS_HOST_BOUND,      NAS_HOST_NO_POD,      NAS_HOST_LIST_ERROR,
                                   NAS_HOST_BIND_ERROR, NAS_HOST_EVENT_ERROR, NAS_HOST_PANICKED,
                                   NAS_HOST_UNSCHEDULABLE};
    o.kind = kind[r.kind];
    copy_str(o.pod, sizeof o.pod, p.ns + "/" + p.name);
    copy_str(o.node, sizeof o.node, r.node);
    copy_str(o.message, sizeof o.message, r.message);
}

}  // namespace

struct nas_host_sched {
    CbApi api;
    CbSource src;
    CbOrder order;
    std::unique_ptr<CustomScheduler> s;
    std::string err;
};

#define GUARD(s, body)                                  \
    try {                                               \
        body                                            \
    } catch (const GoPanic &e) {                        \
        if (s) (s)->err = e.what();                     \
        return NAS_HOST_PANIC;                          \
    } catch (const std::invalid_argument &e) {          \
        if (s) (s)->err = e.what();                     \
        return NAS_ERR_ARG;                             \
    } catch (const std::exception &e) {                 \
        if (s) (s)->err = e.what();                     \
        return NAS_ERR_STATE;                           \
    }

extern "C" {

void nas_host_buf_append(nas_host_buf *b, const char *data, size_t n) {
    if (b && data) b->s.append(data, n);
}

int nas_host_parse_float(const char *s, size_t n, int32_t bits, double *value, int32_t *go_err) {
    if ((!s && n) || !value || (bits != 32 && bits != 64)) return NAS_ERR_ARG;
    const GoFloat f = go_parse_float(std::string_view(s ? s : "", n), bits);
    *value = f.value;
    if (go_err) *go_err = f.err;
    return NAS_OK;
}

int nas_host_atoi(const char *s, size_t n, int64_t *value, int32_t *go_err) {
    if ((!s && n) || !value) return NAS_ERR_ARG;
    const GoInt v = go_atoi(std::string_view(s ? s : "", n));
    *value = v.value;
    if (go_err) *go_err = v.err;
    return NAS_OK;
}

int nas_host_node_metrics(const char *body, size_t n, const char *node, double *cpu, double *mem,
                          int64_t *rx, int64_t *tx, int64_t *disk, char *panic_msg,
                          size_t panic_cap) {
    if ((!body && n) || !node || !cpu || !mem || !rx || !tx || !disk) return NAS_ERR_ARG;
    const std::string_view b(body ? body : "", n);
    try {
        *cpu = get_current_cpu_usage(b);
        *mem = get_occupied_memory_percentage(b);
        *rx = get_network_packets_received(b, node);
        *tx = get_network_packets_sent(b, node);
        *disk = get_disk_io_now(b, node);
    } catch (const GoPanic &e) {
        copy_str(panic_msg, panic_cap, e.what());
        return NAS_HOST_PANIC;
    }
    return NAS_OK;
}

int nas_host_snapshot_from_bodies(int32_t n, const char *const *bodies, const size_t *body_len,
                                  const char *const *names, double *cpu, double *mem, int64_t *rx,
                                  int64_t *tx, int64_t *disk, int32_t *status, int32_t threads) {
    if (n < 0 || (n > 0 && (!bodies || !body_len || !names || !cpu || !mem || !rx || !tx ||
                            !disk || !status)))
        return NAS_ERR_ARG;
    for (int32_t i = 0; i < n; ++i)
        if ((!bodies[i] && body_len[i]) || !names[i]) return NAS_ERR_ARG;
    // any exception stays inside its node: a worker thread must not reach
    // std::terminate, and nothing may cross the extern "C" boundary
    std::atomic<bool> other_error{false};
    auto one = [&](int32_t i) {
        const std::string_view b(bodies[i] ? bodies[i] : "", body_len[i]);
        int st = NAS_OK;
        try {
            const double c = get_current_cpu_usage(b);
            const double m = get_occupied_memory_percentage(b);
            const int64_t r = get_network_packets_received(b, names[i]);
            const int64_t t = get_network_packets_sent(b, names[i]);
            const int64_t d = get_disk_io_now(b, names[i]);
            cpu[i] = c, mem[i] = m, rx[i] = r, tx[i] = t, disk[i] = d;
        } catch (const GoPanic &) {
            st = NAS_HOST_PANIC;
        } catch (...) {  // bad_alloc and the like: not a reference behaviour
            st = NAS_ERR_STATE;
            other_error.store(true, std::memory_order_relaxed);
        }
        if (st != NAS_OK) {
            cpu[i] = mem[i] = 0;
            rx[i] = tx[i] = disk[i] = 0;
        }
        status[i] = st;
    };
    int w = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    w = std::max(1, std::min<int>(w, n / 64 + 1));  // >= 64 nodes per worker
    auto range = [&](int k) {
        const int32_t lo = (int32_t)((int64_t)n * k / w), hi = (int32_t)((int64_t)n * (k + 1) / w);
        for (int32_t i = lo; i < hi; ++i) one(i);
    };
    std::vector<std::thread> pool;
    int started = 0;
    if (w > 1) {
        try {
            pool.reserve(w);
            for (; started < w; ++started) pool.emplace_back(range, started);
        } catch (...) {  // could not start a worker: this thread does the rest
        }
    }
    for (int k = started; k < w; ++k) range(k);
    for (auto &t : pool) t.join();
    return other_error.load() ? NAS_ERR_STATE : NAS_OK;
}

int nas_host_iperf_receiver(const char *json, size_t n, double *receiver_bps, double *sender_bps,
                            int32_t *n_streams, int32_t *valid_json) {
    if (!json && n) return NAS_ERR_ARG;
    const IperfReceiver r = go_unmarshal_iperf(std::string_view(json ? json : "", n));
    if (receiver_bps) *receiver_bps = r.receiver_bps;
    if (sender_bps) *sender_bps = r.sender_bps;
    if (n_streams) *n_streams = r.n_streams;
    if (valid_json) *valid_json = r.valid_json;
    return NAS_OK;
}

int32_t nas_host_latency_from_bps(double bps) { return latency_from_bps(bps); }

int nas_host_latency_matrix(int32_t n, const char *const *reports, const size_t *report_len,
                            int8_t *L_out) {
    if (n <= 0 || !reports || !report_len || !L_out) return NAS_ERR_ARG;
    const std::vector<int8_t> L = latency_matrix(n, [&](int i, int j, std::string &bytes) {
        const size_t k = (size_t)i * n + j;
        if (!reports[k]) return false;
        bytes.assign(reports[k], report_len[k]);
        return true;
    });
    std::memcpy(L_out, L.data(), L.size());
    return NAS_OK;
}

float nas_host_latency_us_from_bps(double bps) { return latency_us_from_bps(bps); }

int nas_host_latency_matrix_us(int32_t n, const char *const *reports, const size_t *report_len,
                               float *L_out) {
    if (n <= 0 || !reports || !report_len || !L_out) return NAS_ERR_ARG;
    const std::vector<float> L = latency_matrix_us(n, [&](int i, int j, std::string &bytes) {
        const size_t k = (size_t)i * n + j;
        if (!reports[k]) return false;
        bytes.assign(reports[k], report_len[k]);
        return true;
    });
    std::memcpy(L_out, L.data(), L.size() * sizeof(float));
    return NAS_OK;
}

int nas_host_create(nas_host_sched **out, nas_ctx *ctx, const nas_host_io *io) {
    if (!out || !ctx || !io) return NAS_ERR_ARG;
    auto *s = new (std::nothrow) nas_host_sched;
    if (!s) return NAS_ERR_NOMEM;
    s->api.io = s->src.io = s->order.io = *io;
    s->s.reset(new CustomScheduler(ctx, s->api, s->src, s->order));
    *out = s;
    return NAS_OK;
}

void nas_host_destroy(nas_host_sched *s) { delete s; }

const char *nas_host_last_error(nas_host_sched *s) { return s ? s->err.c_str() : "null scheduler"; }

int nas_host_set_topology(nas_host_sched *s, const char *const *names, const char *const *urls,
                          int32_t n) {
    if (!s || !names || !urls || n <= 0) return NAS_ERR_ARG;
    std::vector<Endpoint> t;
    for (int i = 0; i < n; ++i) {
        if (!names[i] || !urls[i]) return NAS_ERR_ARG;
        t.push_back({names[i], urls[i]});
    }
    s->s->set_topology(std::move(t));
    return NAS_OK;
}

int nas_host_set_iperf_path(nas_host_sched *s, const char *node, const char *path) {
    if (!s || !node || !path) return NAS_ERR_ARG;
    s->s->add_iperf_path(node, path);
    return NAS_OK;
}

int nas_host_set_latency(nas_host_sched *s, const char *const *names, const int8_t *L, int32_t n) {
    if (!s || !names || !L || n <= 0) return NAS_ERR_ARG;
    GUARD(s, {
        std::vector<std::string> nm;
        for (int i = 0; i < n; ++i) nm.push_back(names[i] ? names[i] : "");
        s->s->set_latency(nm, std::vector<int8_t>(L, L + (size_t)n * n));
        return NAS_OK;
    })
}

int nas_host_set_latency_f32(nas_host_sched *s, const char *const *names, const float *L,
                             int32_t n) {
    if (!s || !names || !L || n <= 0) return NAS_ERR_ARG;
    GUARD(s, {
        std::vector<std::string> nm;
        for (int i = 0; i < n; ++i) nm.push_back(names[i] ? names[i] : "");
        s->s->set_latency_f32(nm, std::vector<float>(L, L + (size_t)n * n));
        return NAS_OK;
    })
}

int nas_host_enqueue(nas_host_sched *s, const nas_host_pod *p) {
    if (!s || !p || !p->ns || !p->name) return NAS_ERR_ARG;
    if (p->n_peers < 0 || (p->n_peers > 0 && (!p->peers || !p->peer_weight))) return NAS_ERR_ARG;
    Pod pod;
    pod.ns = p->ns;
    pod.name = p->name;
    pod.uid = p->uid ? p->uid : "";
    pod.scheduler_name = p->scheduler_name ? p->scheduler_name : "";
    pod.node_name = p->node_name ? p->node_name : "";
    pod.cpu_milli = p->cpu_milli;
    pod.mem_kib = p->mem_kib;
    for (int i = 0; i < p->n_peers; ++i) pod.peers.push_back({p->peers[i] ? p->peers[i] : "", p->peer_weight[i]});
    GUARD(s, { return s->s->enqueue(pod) ? 1 : 0; })
}

int32_t nas_host_queued(nas_host_sched *s) { return s ? (int32_t)s->s->queued() : 0; }

int nas_host_schedule_one(nas_host_sched *s, nas_host_outcome *out) {
    if (!s || !out) return NAS_ERR_ARG;
    GUARD(s, {
        Pod p;
        const Outcome r = s->s->schedule_one(&p);
        fill(*out, p, r);
        return NAS_OK;
    })
}

int nas_host_schedule_batch(nas_host_sched *s, int32_t max_pods, nas_host_outcome *out,
                            int32_t *n_out) {
    if (!s || !out || !n_out || max_pods <= 0) return NAS_ERR_ARG;
    GUARD(s, {
        auto rs = s->s->schedule_batch(max_pods);
        for (size_t i = 0; i < rs.size(); ++i) fill(out[i], rs[i].first, rs[i].second);
        *n_out = (int32_t)rs.size();
        return NAS_OK;
    })
}

int nas_host_place_pending(nas_host_sched *s, nas_host_outcome *out, int32_t *n_out) {
    if (!s || !out || !n_out) return NAS_ERR_ARG;
    GUARD(s, {
        auto rs = s->s->place_pending();
        for (size_t i = 0; i < rs.size(); ++i) fill(out[i], rs[i].first, rs[i].second);
        *n_out = (int32_t)rs.size();
        return NAS_OK;
    })
}

}  // extern "C"
