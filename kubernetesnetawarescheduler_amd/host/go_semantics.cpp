// go_semantics.cpp -- see go_semantics.h.  Grammar checks follow Go's
// strconv/atof.go (special, readFloat), strconv/atoi.go (underscoreOK,
// ParseUint, ParseInt, Atoi); the rounding itself is delegated to the C
// library's correctly rounded strtof_l / strtod_l in the "C" locale, which
// agree with Go's correctly rounded conversion for every well-formed input.
#include "go_semantics.h"

#include <cerrno>
#include <clocale>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <locale.h>

namespace nas_host {
namespace {

inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? char(c - 'A' + 'a') : c; }

size_t common_prefix_ci(std::string_view s, std::string_view prefix) {
    size_t n = 0;
    while (n < s.size() && n < prefix.size() && lower(s[n]) == prefix[n]) ++n;
    return n;
}

// atof.go special(): returns consumed length (0 = not special)
size_t special(std::string_view s, double &f) {
    if (s.empty()) return 0;
    int sign = 1;
    size_t nsign = 0;
    switch (s[0]) {
        case '+':
        case '-':
            if (s[0] == '-') sign = -1;
            nsign = 1;
            s = s.substr(1);
            [[fallthrough]];
        case 'i':
        case 'I': {
            size_t n = common_prefix_ci(s, "infinity");
            if (3 < n && n < 8) n = 3;  // "inf" is the longest shorter match
            if (n == 3 || n == 8) {
                f = sign * std::numeric_limits<double>::infinity();
                return nsign + n;
            }
            break;
        }
        case 'n':
        case 'N':
            if (common_prefix_ci(s, "nan") == 3) {
                f = std::numeric_limits<double>::quiet_NaN();
                return 3;
            }
            break;
        default:
            break;
    }
    return 0;
}

// atoi.go underscoreOK
bool underscore_ok(std::string_view s) {
    char saw = '^';
    size_t i = 0;
    if (!s.empty() && (s[0] == '-' || s[0] == '+')) s = s.substr(1);
    bool hex = false;
    if (s.size() >= 2 && s[0] == '0' &&
        (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
        i = 2;
        saw = '0';
        hex = lower(s[1]) == 'x';
    }
    for (; i < s.size(); ++i) {
        const char c = s[i];
        if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) {
            saw = '0';
            continue;
        }
        if (c == '_') {
            if (saw != '0') return false;
            saw = '_';
            continue;
        }
        if (saw == '_') return false;
        saw = '!';
    }
    return saw != '_';
}

// atof.go readFloat, grammar only: returns the length of the longest valid
// prefix, or 0 when there is none
size_t read_float(std::string_view s, bool &underscores) {
    size_t i = 0;
    underscores = false;
    if (i >= s.size()) return 0;
    if (s[i] == '+' || s[i] == '-') ++i;
    bool base16 = false;
    char exp_char = 'e';
    if (i + 2 < s.size() && s[i] == '0' && lower(s[i + 1]) == 'x') {
        base16 = true;
        exp_char = 'p';
        i += 2;
    }
    bool sawdot = false, sawdigits = false;
    for (; i < s.size(); ++i) {
        const char c = s[i];
        if (c == '_') {
            underscores = true;
            continue;
        }
        if (c == '.') {
            if (sawdot) break;
            sawdot = true;
            continue;
        }
        if (c >= '0' && c <= '9') {
            sawdigits = true;
            continue;
        }
        if (base16 && lower(c) >= 'a' && lower(c) <= 'f') {
            sawdigits = true;
            continue;
        }
        break;
    }
    if (!sawdigits) return 0;
    if (i < s.size() && lower(s[i]) == exp_char) {
        ++i;
        if (i >= s.size()) return 0;
        if (s[i] == '+' || s[i] == '-') ++i;
        if (i >= s.size() || s[i] < '0' || s[i] > '9') return 0;
        for (; i < s.size() && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); ++i)
            if (s[i] == '_') underscores = true;
    } else if (base16) {
        return 0;  // a hexadecimal mantissa needs a 'p' exponent
    }
    if (underscores && !underscore_ok(s.substr(0, i))) return 0;
    return i;
}

locale_t c_locale() {
    static locale_t loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    return loc;
}

}  // namespace

GoFloat go_parse_float(std::string_view s, int bits) {
    double f = 0;
    const size_t ns = special(s, f);
    if (ns) {
        if (ns != s.size()) return {0.0, GO_ERR_SYNTAX};
        return {f, GO_OK};
    }
    bool underscores = false;
    const size_t n = read_float(s, underscores);
    if (n == 0 || n != s.size()) return {0.0, GO_ERR_SYNTAX};
    std::string buf;
    buf.reserve(s.size());
    for (char c : s)
        if (c != '_') buf.push_back(c);
    errno = 0;
    char *end = nullptr;
    double v;
    if (bits == 32)
        v = (double)strtof_l(buf.c_str(), &end, c_locale());
    else
        v = strtod_l(buf.c_str(), &end, c_locale());
    if (end != buf.c_str() + buf.size()) return {0.0, GO_ERR_SYNTAX};  // not reached for valid input
    if (std::isinf(v)) return {v, GO_ERR_RANGE};  // overflow: +-Inf with ErrRange
    return {v, GO_OK};  // underflow rounds to a denormal or zero without error
}

GoInt go_atoi(std::string_view s) {
    const size_t len = s.size();
    if (len > 0 && len < 19) {  // Atoi's fast path (intSize == 64)
        std::string_view t = s;
        if (t[0] == '-' || t[0] == '+') {
            t = t.substr(1);
            if (t.empty()) return {0, GO_ERR_SYNTAX};
        }
        int64_t n = 0;
        for (char c : t) {
            if (c < '0' || c > '9') return {0, GO_ERR_SYNTAX};
            n = n * 10 + (c - '0');
        }
        return {s[0] == '-' ? -n : n, GO_OK};
    }
    // ParseInt(s, 10, 0)
    if (len == 0) return {0, GO_ERR_SYNTAX};
    std::string_view t = s;
    bool neg = false;
    if (t[0] == '+' || t[0] == '-') {
        neg = t[0] == '-';
        t = t.substr(1);
    }
    // ParseUint(t, 10, 64): base 10 given explicitly, so no '_'
    if (t.empty()) return {0, GO_ERR_SYNTAX};
    const uint64_t max_u = std::numeric_limits<uint64_t>::max();
    uint64_t un = 0;
    bool range = false;
    for (char c : t) {
        if (c < '0' || c > '9') return {0, GO_ERR_SYNTAX};
        const uint64_t d = uint64_t(c - '0');
        if (un > max_u / 10 || un * 10 > max_u - d) {
            range = true;  // ParseUint stops at the first overflow: ErrRange
            break;
        }
        un = un * 10 + d;
    }
    const uint64_t cutoff = uint64_t(1) << 63;
    if (range) return {neg ? std::numeric_limits<int64_t>::min() : std::numeric_limits<int64_t>::max(), GO_ERR_RANGE};
    if (!neg && un >= cutoff) return {std::numeric_limits<int64_t>::max(), GO_ERR_RANGE};
    if (neg && un > cutoff) return {std::numeric_limits<int64_t>::min(), GO_ERR_RANGE};
    return {neg ? (int64_t)(0 - un) : (int64_t)un, GO_OK};
}

int64_t go_index(std::string_view s, std::string_view sub) {
    const size_t p = s.find(sub);
    return p == std::string_view::npos ? -1 : (int64_t)p;
}

std::string_view go_slice(std::string_view s, int64_t lo, int64_t hi) {
    const int64_t len = (int64_t)s.size();
    if (hi < 0 || hi > len)
        throw GoPanic("runtime error: slice bounds out of range [:" + std::to_string(hi) +
                      "] with length " + std::to_string(len));
    if (lo < 0 || lo > hi)
        throw GoPanic("runtime error: slice bounds out of range [" + std::to_string(lo) + ":" +
                      std::to_string(hi) + "]");
    return s.substr((size_t)lo, (size_t)(hi - lo));
}

}  // namespace nas_host
