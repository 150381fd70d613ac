// latency.cpp -- see latency.h.
#include "latency.h"

#include <algorithm>
#include <cmath>

#include "go_json.h"

namespace nas_host {

int8_t latency_from_bps(double bps) {
    if (!(bps > 0) || std::isinf(bps)) return bps > 0 ? 1 : 127;  // +Inf bps: fastest; <= 0 / NaN: unusable
    const double ms = std::ceil(8e9 / bps);  // 8e6 bits at bps bits/s, in ms
    return (int8_t)std::max(1.0, std::min(127.0, ms));
}

std::vector<int8_t> latency_matrix(int n, const std::function<bool(int, int, std::string &)> &report) {
    std::vector<int8_t> dir((size_t)n * n, 127), L((size_t)n * n, 0);
    std::string bytes;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            if (i == j) continue;
            bytes.clear();
            if (!report(i, j, bytes)) continue;
            const IperfReceiver r = go_unmarshal_iperf(bytes);
            if (r.n_streams > 0) dir[(size_t)i * n + j] = latency_from_bps(r.receiver_bps);
        }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            if (i != j) L[(size_t)i * n + j] = std::max(dir[(size_t)i * n + j], dir[(size_t)j * n + i]);
    return L;
}

float latency_us_from_bps(double bps) {
    if (!(bps > 0)) return kUnusableUs;  // <= 0 / NaN
    if (std::isinf(bps)) return 0.0f;
    return (float)std::min<double>(kUnusableUs, 8e12 / bps);  // 8e6 bits at bps bits/s, in us
}

std::vector<float> latency_matrix_us(int n,
                                     const std::function<bool(int, int, std::string &)> &report) {
    std::vector<float> dir((size_t)n * n, kUnusableUs), L((size_t)n * n, 0.0f);
    std::string bytes;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            if (i == j) continue;
            bytes.clear();
            if (!report(i, j, bytes)) continue;
            const IperfReceiver r = go_unmarshal_iperf(bytes);
            if (r.n_streams > 0) dir[(size_t)i * n + j] = latency_us_from_bps(r.receiver_bps);
        }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            if (i != j) L[(size_t)i * n + j] = std::max(dir[(size_t)i * n + j], dir[(size_t)j * n + i]);
    return L;
}

}  // namespace nas_host
