// ingest.h -- host metric ingest: node-exporter /metrics text and iperf3
// reports -> one PrometheusNodeMetrics record (scheduler/scheduler.go:24-32),
// with the reference's exact values, including its error paths
// (SURVEY.md §8(f) next-1 and next-2).
//
// Each getter restates the reference function it names, statement by
// statement: fixed-offset slicing between two strings.Index results (a Go
// slice-bounds panic when a marker is missing -- GoPanic), then
// strconv.ParseFloat(s, 32) or strconv.Atoi with the reference's handling of
// the error (ignored for floats, 0 for ints, cpu3 := cpu2 for the fourth
// core).
#pragma once

#include <functional>
#include <string>
#include <string_view>

#include "go_semantics.h"

namespace nas_host {

// scheduler.go:24-32 (nodeName kept by the caller)
struct NodeMetrics {
    double cpu_frequency_hertz = 0;
    double occupied_memory_percentage = 0;
    int64_t network_packets_received = 0;
    int64_t network_packets_sent = 0;
    double network_bandwidth = 0;
    int64_t disk_io_now = 0;
};

double get_current_cpu_usage(std::string_view body);                        // :409-442
double get_occupied_memory_percentage(std::string_view body);               // :444-461
int64_t get_network_packets_sent(std::string_view body, std::string_view node);      // :463-481
int64_t get_network_packets_received(std::string_view body, std::string_view node);  // :482-501
int64_t get_disk_io_now(std::string_view body, std::string_view node);      // :532-549

// :503-530.  `iperf_path` maps a node name to its report file (the map of
// :505-510; "" for an unmapped node, as Go's map lookup gives); `read_file`
// returns false when os.Open fails.  An unreadable or undecodable report
// leaves End.Streams empty and Streams[0] panics, as in the reference.
double get_network_bandwidth(std::string_view node,
                             const std::function<std::string(std::string_view)> &iperf_path,
                             const std::function<bool(const std::string &, std::string &)> &read_file);

// the reference's map of :505-510
std::string reference_iperf_path(std::string_view node);

}  // namespace nas_host
