// go_semantics.h -- the Go runtime / stdlib behaviour the reference's host
// code leans on, restated in C++ (Go is not installed in this image).
//
// scheduler/scheduler.go parses node-exporter text with strings.Index +
// slicing and strconv.ParseFloat(s, 32) / strconv.Atoi, ignoring errors
// except to print them.  The VALUES it goes on to use on error paths are part
// of its behaviour (a failed Atoi gives 0, which then wins the rx/tx
// arg-min), so this file reproduces them exactly:
//   * go_parse_float: strconv.ParseFloat(s, bitSize) of Go >= 1.13 (decimal
//     and hexadecimal literals, '_' separators checked by underscoreOK, the
//     case-insensitive "inf"/"infinity"/"nan" specials, whole-string match),
//     returning Go's value on error too (0 on a syntax error, +-Inf on
//     overflow with ErrRange; underflow is not an error);
//   * go_atoi: strconv.Atoi on a 64-bit platform (sign + decimal digits only,
//     no '_', range-checked to int64);
//   * go_index / go_slice: strings.Index and s[lo:hi] with Go's bounds panic.
// A Go panic is a C++ exception (GoPanic) carrying Go's runtime message.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>

namespace nas_host {

struct GoPanic : std::runtime_error {
    using std::runtime_error::runtime_error;
};

enum GoErr { GO_OK = 0, GO_ERR_SYNTAX = 1, GO_ERR_RANGE = 2 };

struct GoFloat {
    double value;  // float32-rounded when bits == 32, widened to float64 (Go's return type)
    int err;       // GoErr
};
GoFloat go_parse_float(std::string_view s, int bits);

struct GoInt {
    int64_t value;  // Go's value on error: 0 for syntax, the clamped bound for range
    int err;
};
GoInt go_atoi(std::string_view s);

// strings.Index: byte offset of the first occurrence of sub, or -1
int64_t go_index(std::string_view s, std::string_view sub);
// s[lo:hi]; panics like the Go runtime when !(0 <= lo <= hi <= len(s))
std::string_view go_slice(std::string_view s, int64_t lo, int64_t hi);

}  // namespace nas_host
