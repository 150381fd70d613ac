// san_driver.cpp -- the CPU code of this repo under AddressSanitizer +
// UndefinedBehaviorSanitizer (tests/test_sanitize_cpu.py builds it with
// -fsanitize=address,undefined -fno-sanitize-recover=all and runs it).
//
// Host mirror (kubernetesnetawarescheduler_amd/host/): the node-exporter
// getters, iperf3 JSON decoding, Go strconv/slicing and the latency matrices
// -- the code that parses untrusted cluster text -- on fixture inputs and on
// every prefix and thousands of byte mutations of them.  Oracle (oracle/):
// every entry point on random small inputs, with internal consistency checks
// (literal vs closed-form vote, Go-map vote vs literal on the walked orders,
// place vs cost + fit + top-k + commit).  Exit status 0 and "SAN OK" on
// success; any sanitizer report aborts with a nonzero status.
//
// usage: san_driver METRICS_BODY_FILE NODE_NAME IPERF_REPORT_FILE
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "go_json.h"
#include "go_semantics.h"
#include "ingest.h"
#include "latency.h"

extern "C" {
int or_vote_literal(int n, const double *cpu, const double *mem, const int64_t *rx,
                    const int64_t *tx, const double *bw, const int64_t *disk,
                    const int32_t *order1, const int32_t *order2, int32_t *best_out,
                    int32_t *winners_out, int64_t *scores_out);
int or_vote_closed(int n, const double *cpu, const double *mem, const int64_t *rx,
                   const int64_t *tx, const double *bw, const int64_t *disk,
                   const int32_t *order1, const int32_t *order2, int32_t *best_out,
                   int32_t *winners_out);
int or_vote_batch(int n, int n_snapshots, const double *cpu, const double *mem, const int64_t *rx,
                  const int64_t *tx, const double *bw, const int64_t *disk, const int32_t *order1,
                  const int32_t *order2, int n_orders, const int32_t *pod_snapshot, int P,
                  int32_t *best_out, int32_t *winners_out);
int or_vote_gomap(int n, int P, const double *cpu, const double *mem, const int64_t *rx,
                  const int64_t *tx, const double *bw, const int64_t *disk, int32_t *best_out,
                  int32_t *order1_out, int32_t *order2_out, int64_t *fill_ns, int64_t *loop_ns);
void or_fit(int P, int N, const int32_t *rc, const int32_t *rm, const int32_t *rp,
            const int32_t *fc, const int32_t *fm, const int32_t *fp, uint32_t *mask);
void or_cost_i8(int P, int N, const int32_t *WA, const int8_t *L, int64_t *cost);
void or_cost_f32(int P, int N, const float *WA, const float *L, double *cost);
void or_cost_bf16(int P, int N, const uint16_t *WA, const uint16_t *L, double *cost);
void or_topk(int P, int N, int k, const int64_t *cost_i, const double *cost_d, const uint32_t *mask,
             int32_t *cand_node, int64_t *cand_cost_i, double *cand_cost_d, int32_t *count);
int or_place(int P, int N, int dtype, const void *WA, const void *L, const int32_t *rc,
             const int32_t *rm, const int32_t *rp, int32_t *fc, int32_t *fm, int32_t *fp,
             int32_t *node_out, int64_t *cost_i_out, double *cost_d_out);
void or_commit(int P, int k, const int32_t *cand_node, const int32_t *count,
               const int32_t *complete, const int32_t *rc, const int32_t *rm, const int32_t *rp,
               int32_t *fc, int32_t *fm, int32_t *fp, int32_t *node_out, int32_t *slot_out,
               int *stop);
}

namespace {

using namespace nas_host;

int failures = 0;
void expect(bool ok, const char *what) {
    if (!ok) {
        std::fprintf(stderr, "CHECK FAILED: %s\n", what);
        ++failures;
    }
}

std::string slurp(const char *path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

double sink = 0;  // keeps results observable

// every getter of one scrape (scheduler.go:281-331); Go panics are exceptions
void ingest_all(std::string_view body, std::string_view node) {
    try { sink += get_current_cpu_usage(body); } catch (const GoPanic &) {}
    try { sink += get_occupied_memory_percentage(body); } catch (const GoPanic &) {}
    try { sink += (double)get_network_packets_sent(body, node); } catch (const GoPanic &) {}
    try { sink += (double)get_network_packets_received(body, node); } catch (const GoPanic &) {}
    try { sink += (double)get_disk_io_now(body, node); } catch (const GoPanic &) {}
}

void fuzz_host(const std::string &body, const std::string &node, const std::string &report,
               std::mt19937_64 &rng) {
    ingest_all(body, node);
    for (size_t n = 0; n <= body.size(); n += 3) ingest_all(std::string(body, 0, n), node);
    for (int it = 0; it < 3000; ++it) {
        std::string b = body;
        const int flips = 1 + (int)(rng() % 4);
        for (int f = 0; f < flips && !b.empty(); ++f) b[rng() % b.size()] = (char)(rng() & 0xff);
        ingest_all(b, node);
    }
    const IperfReceiver r0 = go_unmarshal_iperf(report);
    expect(r0.valid_json && r0.n_streams == 1, "fixture iperf report decodes");
    for (size_t n = 0; n <= report.size(); ++n) {
        const IperfReceiver r = go_unmarshal_iperf(std::string_view(report).substr(0, n));
        sink += r.receiver_bps;
    }
    static const char alphabet[] = "{}[]\":,.-+eE0123456789 \\ntfaulsr";
    for (int it = 0; it < 5000; ++it) {
        std::string j = report;
        const int flips = 1 + (int)(rng() % 6);
        for (int f = 0; f < flips; ++f) j[rng() % j.size()] = alphabet[rng() % (sizeof(alphabet) - 1)];
        if (rng() % 4 == 0) j.insert(rng() % j.size(), std::string(1 + rng() % 64, '['));
        const IperfReceiver r = go_unmarshal_iperf(j);
        sink += r.sender_bps + r.n_streams;
    }
    // strconv on random short strings, slicing out of range
    static const char num[] = "0123456789.eE+-_xXpPabcdfinINFtyn ";
    for (int it = 0; it < 20000; ++it) {
        std::string s(rng() % 24, ' ');
        for (char &c : s) c = num[rng() % (sizeof(num) - 1)];
        const GoFloat f = go_parse_float(s, (rng() & 1) ? 32 : 64);
        const GoInt i = go_atoi(s);
        sink += (std::isfinite(f.value) ? f.value : 0.0) + (double)(i.value & 0xff) + f.err + i.err;
        try {
            sink += (double)go_slice(s, (int64_t)(rng() % 40) - 8, (int64_t)(rng() % 40) - 8).size();
        } catch (const GoPanic &) {}
        sink += (double)go_index(s, std::string_view(num + rng() % 8, rng() % 3));
    }
    // latency matrices from reports that exist, are corrupt or are missing
    for (int n : {1, 2, 5, 9}) {
        auto report_of = [&](int i, int j, std::string &out) {
            const unsigned h = (unsigned)(i * 31 + j * 7);
            if (h % 5 == 0) return false;
            out = report;
            if (h % 3 == 0) out.resize(out.size() / 2);
            return true;
        };
        const std::vector<int8_t> L = latency_matrix(n, report_of);
        const std::vector<float> Lu = latency_matrix_us(n, report_of);
        expect((int)L.size() == n * n && (int)Lu.size() == n * n, "latency matrix sizes");
        for (int i = 0; i < n; ++i) expect(L[i * n + i] == 0 && Lu[i * n + i] == 0.0f, "zero diagonal");
    }
    for (double bps : {0.0, -1.0, 1.0, 1e3, 9.4e7, 1e12, (double)INFINITY, (double)NAN, 1e308})
        sink += latency_from_bps(bps) + latency_us_from_bps(bps);
}

// ---- oracle

struct Snap {
    std::vector<double> cpu, mem, bw;
    std::vector<int64_t> rx, tx, disk;
};

Snap random_snaps(int n, int S, std::mt19937_64 &rng) {
    Snap s;
    const size_t t = (size_t)n * S;
    s.cpu.resize(t); s.mem.resize(t); s.bw.resize(t); s.rx.resize(t); s.tx.resize(t); s.disk.resize(t);
    for (size_t i = 0; i < t; ++i) {
        const int ties = (int)(rng() % 4);  // small value sets force ties
        s.cpu[i] = ties ? (double)(rng() % 3) * 1e9 : (double)(rng() % 2000000000);
        s.mem[i] = (rng() % 17 == 0) ? NAN : (double)(rng() % 100);
        s.bw[i] = (rng() % 13 == 0) ? -0.0 : (double)(rng() % 1000) * 1e5;
        s.rx[i] = ties ? (int64_t)(rng() % 3) : (int64_t)(rng() % 1000000);
        s.tx[i] = (int64_t)(rng() % 1000000);
        s.disk[i] = (int64_t)(rng() % 4);
    }
    return s;
}

std::vector<int32_t> perm(int n, std::mt19937_64 &rng) {
    std::vector<int32_t> p(n);
    for (int i = 0; i < n; ++i) p[i] = i;
    for (int i = n - 1; i > 0; --i) std::swap(p[i], p[rng() % (i + 1)]);
    return p;
}

void fuzz_vote(std::mt19937_64 &rng) {
    for (int n : {1, 2, 5, 17, 64, 301}) {
        const int S = 24;
        const Snap s = random_snaps(n, S, rng);
        std::vector<int32_t> o1, o2;
        for (int k = 0; k < S; ++k) {
            const auto a = perm(n, rng), b = perm(n + 1, rng);
            o1.insert(o1.end(), a.begin(), a.end());
            o2.insert(o2.end(), b.begin(), b.end());
        }
        std::vector<int32_t> best(S), win(6 * S), pods(3 * S);
        for (auto &p : pods) p = (int32_t)(rng() % S);
        expect(or_vote_batch(n, S, s.cpu.data(), s.mem.data(), s.rx.data(), s.tx.data(), s.bw.data(),
                             s.disk.data(), o1.data(), o2.data(), S, nullptr, S, best.data(),
                             win.data()) == 0, "or_vote_batch");
        for (int k = 0; k < S; ++k) {
            const size_t b = (size_t)k * n;
            int32_t bl, bc, wl[6], wc[6];
            std::vector<int64_t> scores(n + 1);
            or_vote_literal(n, &s.cpu[b], &s.mem[b], &s.rx[b], &s.tx[b], &s.bw[b], &s.disk[b],
                            &o1[b], &o2[(size_t)k * (n + 1)], &bl, wl, scores.data());
            or_vote_closed(n, &s.cpu[b], &s.mem[b], &s.rx[b], &s.tx[b], &s.bw[b], &s.disk[b],
                           &o1[b], &o2[(size_t)k * (n + 1)], &bc, wc);
            expect(bl == bc && bl == best[k] && !std::memcmp(wl, wc, sizeof wl), "literal == closed");
        }
        std::vector<int32_t> bpod(pods.size()), wpod(6 * pods.size());
        or_vote_batch(n, S, s.cpu.data(), s.mem.data(), s.rx.data(), s.tx.data(), s.bw.data(),
                      s.disk.data(), o1.data(), o2.data(), S, pods.data(), (int)pods.size(),
                      bpod.data(), wpod.data());
        for (size_t p = 0; p < pods.size(); ++p) expect(bpod[p] == best[pods[p]], "pod_snapshot gather");
        // the Go-map restatement against the literal loop on the orders it walked
        std::vector<int32_t> bg(S), g1((size_t)S * n), g2((size_t)S * (n + 1));
        int64_t fill = 0, loop = 0;
        expect(or_vote_gomap(n, S, s.cpu.data(), s.mem.data(), s.rx.data(), s.tx.data(), s.bw.data(),
                             s.disk.data(), bg.data(), g1.data(), g2.data(), &fill, &loop) == 0,
               "or_vote_gomap");
        std::vector<int32_t> bl(S), wl(6 * S);
        or_vote_batch(n, S, s.cpu.data(), s.mem.data(), s.rx.data(), s.tx.data(), s.bw.data(),
                      s.disk.data(), g1.data(), g2.data(), S, nullptr, S, bl.data(), wl.data());
        expect(bl == bg, "gomap == literal on walked orders");
    }
}

void fuzz_place(std::mt19937_64 &rng) {
    for (int trial = 0; trial < 12; ++trial) {
        const int P = 1 + (int)(rng() % 200), N = 1 + (int)(rng() % 150), K = 8;
        std::vector<int32_t> WA((size_t)P * N), rc(P), rm(P), rp(P), fc(N), fm(N), fp(N);
        std::vector<int8_t> L((size_t)N * N);
        std::vector<float> WAf((size_t)P * N), Lf((size_t)N * N);
        std::vector<uint16_t> WAb((size_t)P * N), Lb((size_t)N * N);
        for (size_t i = 0; i < WA.size(); ++i) {
            WA[i] = (rng() % 9 == 0) ? (int32_t)(rng() % 200000) - 1000 : (int32_t)(rng() % 256) - 128;
            WAf[i] = (float)WA[i] * 0.25f;
            WAb[i] = (uint16_t)(0x3f80 + rng() % 0x400);
        }
        for (size_t i = 0; i < L.size(); ++i) {
            L[i] = (int8_t)((int)(rng() % 256) - 128);
            Lf[i] = (float)L[i] * 1.5f;
            Lb[i] = (uint16_t)(0x3f80 + rng() % 0x400);
        }
        for (int p = 0; p < P; ++p) {
            rc[p] = (int32_t)(rng() % 600);
            rm[p] = (int32_t)(rng() % 300000);
            rp[p] = 1;
        }
        for (int n = 0; n < N; ++n) {
            fc[n] = (int32_t)(rng() % 4000);
            fm[n] = (int32_t)(rng() % 3000000);
            fp[n] = (int32_t)(rng() % 12);
        }
        const int W = (N + 31) / 32;
        std::vector<uint32_t> mask((size_t)P * W);
        or_fit(P, N, rc.data(), rm.data(), rp.data(), fc.data(), fm.data(), fp.data(), mask.data());
        std::vector<int64_t> ci((size_t)P * N);
        std::vector<double> cd((size_t)P * N);
        or_cost_i8(P, N, WA.data(), L.data(), ci.data());
        or_cost_f32(P, N, WAf.data(), Lf.data(), cd.data());
        or_cost_bf16(P, N, WAb.data(), Lb.data(), cd.data());
        std::vector<int32_t> cn((size_t)P * K), cnt(P);
        std::vector<int64_t> cc((size_t)P * K);
        std::vector<double> ccd((size_t)P * K);
        or_topk(P, N, K, ci.data(), nullptr, mask.data(), cn.data(), cc.data(), nullptr, cnt.data());
        or_topk(P, N, K, nullptr, cd.data(), mask.data(), cn.data(), nullptr, ccd.data(), cnt.data());
        or_topk(P, N, K, ci.data(), nullptr, mask.data(), cn.data(), cc.data(), nullptr, cnt.data());
        // sequential greedy vs commit-from-lists on the same inputs: equal
        // up to the first pod whose list runs dry
        std::vector<int32_t> f1 = fc, m1 = fm, p1 = fp, f2 = fc, m2 = fm, p2 = fp;
        std::vector<int32_t> node1(P), node2(P), slot(P);
        std::vector<int64_t> cost1(P);
        std::vector<double> costd(P);
        expect(or_place(P, N, 1, WA.data(), L.data(), rc.data(), rm.data(), rp.data(), f1.data(),
                        m1.data(), p1.data(), node1.data(), cost1.data(), costd.data()) == 0,
               "or_place i8");
        int stop = -1;
        or_commit(P, K, cn.data(), cnt.data(), nullptr, rc.data(), rm.data(), rp.data(), f2.data(),
                  m2.data(), p2.data(), node2.data(), slot.data(), &stop);
        expect(stop >= 0 && stop <= P, "or_commit stop");
        for (int p = 0; p < stop; ++p) expect(node1[p] == node2[p], "commit == place before stop");
        std::vector<int32_t> f3 = fc, m3 = fm, p3 = fp;
        or_place(P, N, 3, WAf.data(), Lf.data(), rc.data(), rm.data(), rp.data(), f3.data(),
                 m3.data(), p3.data(), node1.data(), nullptr, costd.data());
        f3 = fc; m3 = fm; p3 = fp;
        or_place(P, N, 2, WAb.data(), Lb.data(), rc.data(), rm.data(), rp.data(), f3.data(),
                 m3.data(), p3.data(), node1.data(), nullptr, costd.data());
        expect(or_place(P, N, 9, WA.data(), L.data(), rc.data(), rm.data(), rp.data(), f3.data(),
                        m3.data(), p3.data(), node1.data(), nullptr, nullptr) == -1,
               "or_place rejects a bad dtype");
    }
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s METRICS_BODY NODE IPERF_REPORT\n", argv[0]);
        return 2;
    }
    const std::string body = slurp(argv[1]), node = argv[2], report = slurp(argv[3]);
    std::mt19937_64 rng(0x5A17);
    fuzz_host(body, node, report, rng);
    fuzz_vote(rng);
    fuzz_place(rng);
    std::printf("SAN %s (checksum %g)\n", failures ? "FAILED" : "OK", std::isfinite(sink) ? sink : 0.0);
    return failures ? 1 : 0;
}
