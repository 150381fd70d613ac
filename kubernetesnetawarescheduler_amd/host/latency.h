// latency.h -- pairwise network measurements -> the N x N cost matrix L that
// nas_upload_latency takes.
//
// The reference measures a star: every node's iperf3 client against ONE
// server pod (netperfScript/run.sh:3-14, deployment.yaml), keeping the
// receiver bits/s of End.Streams[0] (scheduler.go:528).  The engine needs all
// pairs, so a pairwise run (tools/pairwise_iperf.sh) leaves one iperf3 -J
// report per ordered pair (client i -> server j), decoded here with the same
// Go semantics as the reference (go_json.h).
//
// L is int8, in milliseconds to move 1 MB: ceil(8e9 / bps), i.e.
// ceil(8000 / Mbit/s), clamped to [1, 127] off the diagonal, 0 on it.  A
// pair is the slower of its two directions (L symmetric); a pair with no
// usable report (unreadable, invalid, no streams, bps <= 0) is 127.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace nas_host {

int8_t latency_from_bps(double bps);

// report(i, j, bytes) -> false when there is no report for client i -> server j
std::vector<int8_t> latency_matrix(int n,
                                   const std::function<bool(int, int, std::string &)> &report);

// The unquantised form for the fp32 path (NAS_DT_F32): microseconds to move
// 1 MB, 8e12 / bps, as float; an unusable pair (no report, bps <= 0 or NaN)
// costs kUnusableUs, +Inf bps costs 0.  Symmetric (the slower direction),
// 0 on the diagonal.
constexpr float kUnusableUs = 1e7f;  // 10 s per MB: never preferred, never Inf/NaN
float latency_us_from_bps(double bps);
std::vector<float> latency_matrix_us(int n,
                                     const std::function<bool(int, int, std::string &)> &report);

}  // namespace nas_host
