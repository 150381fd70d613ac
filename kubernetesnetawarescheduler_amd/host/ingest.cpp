// ingest.cpp -- see ingest.h.  Offsets are the reference's (+42, +33, +37,
// +55/+51, +54/+50, +31/+35), which are the lengths of the metric names they
// skip plus the separating space.
#include "ingest.h"

#include "go_json.h"

namespace nas_host {
namespace {

// body[Index(body, a) + off : Index(body, b) - 1]
std::string_view between(std::string_view body, std::string_view a, int64_t off,
                         std::string_view b) {
    return go_slice(body, go_index(body, a) + off, go_index(body, b) - 1);
}

double parse_float32(std::string_view s, bool *failed = nullptr) {
    const GoFloat f = go_parse_float(s, 32);
    if (failed) *failed = f.err != GO_OK;
    return f.value;  // the reference prints the error and uses the value anyway
}

int64_t atoi_or_zero(std::string_view s) {
    const GoInt v = go_atoi(s);
    return v.err == GO_OK ? v.value : 0;  // "Error while parsing integer!" -> return 0
}

}  // namespace

double get_current_cpu_usage(std::string_view body) {
    const char *c0 = "node_cpu_scaling_frequency_hertz{cpu=\"0\"}";
    const char *c1 = "node_cpu_scaling_frequency_hertz{cpu=\"1\"}";
    const char *c2 = "node_cpu_scaling_frequency_hertz{cpu=\"2\"}";
    const char *c3 = "node_cpu_scaling_frequency_hertz{cpu=\"3\"}";
    const std::string_view s0 = between(body, c0, 42, c1);
    const std::string_view s1 = between(body, c1, 42, c2);
    const std::string_view s2 = between(body, c2, 42, c3);
    const std::string_view s3 = between(body, c3, 42, "# HELP node_cpu_scaling_frequency_max_hrts");
    const double i0 = parse_float32(s0), i1 = parse_float32(s1), i2 = parse_float32(s2);
    bool bad3 = false;
    double i3 = parse_float32(s3, &bad3);
    if (bad3) i3 = i2;  // :436-439
    return (i0 + i1 + i2 + i3) / 4;
}

double get_occupied_memory_percentage(std::string_view body) {
    const std::string_view s = between(body, "gauge\nnode_memory_MemTotal_bytes", 33,
                                       "# HELP node_memory_Mlocked_bytes");
    const std::string_view s1 = between(body, "gauge\nnode_memory_MemAvailable_bytes", 37,
                                        "# HELP node_memory_MemFree_bytes");
    const double i = parse_float32(s), i1 = parse_float32(s1);
    return 100 - ((i1 * 100) / i);
}

int64_t get_network_packets_sent(std::string_view body, std::string_view node) {
    const char *end = "node_network_transmit_packets_total{device=\"flannel.1\"}";
    if (node == "ubuntu")
        return atoi_or_zero(
            between(body, "node_network_transmit_packets_total{device=\"enp3s0f1\"}", 55, end));
    return atoi_or_zero(between(body, "node_network_transmit_packets_total{device=\"eth0\"}", 51, end));
}

int64_t get_network_packets_received(std::string_view body, std::string_view node) {
    const char *end = "node_network_receive_packets_total{device=\"flannel.1\"}";
    if (node == "ubuntu")
        return atoi_or_zero(
            between(body, "node_network_receive_packets_total{device=\"enp3s0f1\"}", 54, end));
    return atoi_or_zero(between(body, "node_network_receive_packets_total{device=\"eth0\"}", 50, end));
}

int64_t get_disk_io_now(std::string_view body, std::string_view node) {
    if (node == "ubuntu")
        return atoi_or_zero(
            between(body, "node_disk_io_now{device=\"sda\"}", 31, "node_disk_io_now{device=\"sr0\"}"));
    return atoi_or_zero(between(body, "node_disk_io_now{device=\"mmcblk0\"}", 35,
                                "node_disk_io_now{device=\"mmcblk0p1\"}"));
}

std::string reference_iperf_path(std::string_view node) {
    if (node == "raspimaster") return "/home/192.168.1.133.json";
    if (node == "raspiworker0") return "/home/192.168.1.135.json";
    if (node == "raspiworker1") return "/home/192.168.1.133.json";
    if (node == "raspiworker2") return "/home/192.168.1.134.json";
    return "";
}

double get_network_bandwidth(std::string_view node,
                             const std::function<std::string(std::string_view)> &iperf_path,
                             const std::function<bool(const std::string &, std::string &)> &read_file) {
    std::string bytes;
    // os.Open error: jsonFile is nil, ReadAll returns no bytes
    if (!read_file(iperf_path(node), bytes)) bytes.clear();
    const IperfReceiver r = go_unmarshal_iperf(bytes);
    if (r.n_streams == 0)
        throw GoPanic("runtime error: index out of range [0] with length 0");
    return r.receiver_bps;
}

}  // namespace nas_host
