// go_json.h -- the part of Go's encoding/json that getNetworkBandwith
// (scheduler/scheduler.go:503-530) depends on: json.Unmarshal of an iperf3
// -J report into the Iperf struct (:34-117), then
// End.Streams[0].Receiver.BitsPerSecond (:528).
//
// Restated from Go's encoding/json (Go >= 1.21; Go is absent here, so this is
// a restatement of the published behaviour, parity pinned by the hand-made
// fixtures in tests/test_host_ingest.py):
//   * the whole input is validated first (checkValid: RFC 8259 grammar as
//     Go's scanner has it, control bytes rejected in strings, invalid UTF-8
//     accepted, nesting depth <= 10000); an invalid document leaves the
//     struct zero (the error itself is ignored by the reference);
//   * object keys are unescaped and matched to field tags exactly, else
//     case-insensitively with Go's name folding (ASCII case plus U+017F,
//     U+212A, U+0130, U+0131, which fold onto 'S', 'K', 'I', 'I');
//     repeated keys decode in order, so scalars take the last value and
//     objects merge into the existing struct;
//   * arrays decode into the existing slice elements (merging), grow with
//     zero elements, truncate at the end, and become empty for [];
//     null resets a slice to nil and leaves structs / numbers unchanged;
//   * a value of the wrong JSON type for a field, or a number that
//     overflows float64, leaves the field unchanged (UnmarshalTypeError,
//     ignored by the reference).
#pragma once

#include <string_view>

namespace nas_host {

struct IperfReceiver {
    bool valid_json;      // checkValid passed
    int n_streams;        // len(End.Streams) after decoding
    double receiver_bps;  // End.Streams[0].Receiver.BitsPerSecond (0 when n_streams == 0)
    double sender_bps;    // End.Streams[0].Sender.BitsPerSecond
};

IperfReceiver go_unmarshal_iperf(std::string_view data);

}  // namespace nas_host
