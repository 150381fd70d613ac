// go_json.cpp -- see go_json.h.  A validating parser into a small DOM, then a
// decoder that walks only the fields on the path to bits_per_second with
// Go's decoding rules.
#include "go_json.h"

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "go_semantics.h"

namespace nas_host {
namespace {

constexpr int MAX_DEPTH = 10000;  // encoding/json scanner maxNestingDepth

struct Value {
    enum Kind { NUL, BOOL, NUMBER, STRING, ARRAY, OBJECT } kind = NUL;
    std::string text;  // NUMBER: literal; STRING: unescaped UTF-8
    std::vector<Value> items;                          // ARRAY
    std::vector<std::pair<std::u32string, Value>> members;  // OBJECT: unescaped keys (code points)
};

struct Parser {
    std::string_view s;
    size_t i = 0;
    bool ok = true;

    void ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool lit(const char *w, size_t n) {
        if (s.substr(i, n) != std::string_view(w, n)) return false;
        i += n;
        return true;
    }
    static int hexv(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    // one UTF-8 sequence at s[i]: the code point (U+FFFD and 1 byte when invalid)
    char32_t utf8(size_t &k) const {
        const unsigned char c = (unsigned char)s[k];
        auto cont = [&](size_t j) {
            return j < s.size() && ((unsigned char)s[j] & 0xC0) == 0x80;
        };
        if (c < 0x80) { ++k; return c; }
        if (c >= 0xC2 && c <= 0xDF && cont(k + 1)) {
            char32_t r = ((c & 0x1F) << 6) | ((unsigned char)s[k + 1] & 0x3F);
            k += 2;
            return r;
        }
        if (c >= 0xE0 && c <= 0xEF && cont(k + 1) && cont(k + 2)) {
            char32_t r = ((c & 0x0F) << 12) | (((unsigned char)s[k + 1] & 0x3F) << 6) |
                         ((unsigned char)s[k + 2] & 0x3F);
            if (r >= 0x800 && (r < 0xD800 || r > 0xDFFF)) { k += 3; return r; }
        }
        if (c >= 0xF0 && c <= 0xF4 && cont(k + 1) && cont(k + 2) && cont(k + 3)) {
            char32_t r = ((c & 0x07) << 18) | (((unsigned char)s[k + 1] & 0x3F) << 12) |
                         (((unsigned char)s[k + 2] & 0x3F) << 6) | ((unsigned char)s[k + 3] & 0x3F);
            if (r >= 0x10000 && r <= 0x10FFFF) { k += 4; return r; }
        }
        ++k;
        return 0xFFFD;
    }
    // a string literal at s[i] == '"': validates and unescapes to code points
    bool str(std::u32string &out) {
        ++i;
        while (true) {
            if (i >= s.size()) return false;
            const unsigned char c = (unsigned char)s[i];
            if (c == '"') { ++i; return true; }
            if (c < 0x20) return false;
            if (c != '\\') { out.push_back(utf8(i)); continue; }
            if (++i >= s.size()) return false;
            const char e = s[i++];
            switch (e) {
                case '"': out.push_back('"'); break;
                case '\\': out.push_back('\\'); break;
                case '/': out.push_back('/'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    auto hex4 = [&](size_t at, char32_t &v) {
                        if (at + 4 > s.size()) return false;
                        v = 0;
                        for (int j = 0; j < 4; ++j) {
                            const int h = hexv(s[at + j]);
                            if (h < 0) return false;
                            v = v * 16 + h;
                        }
                        return true;
                    };
                    char32_t r;
                    if (!hex4(i, r)) return false;
                    i += 4;
                    if (r >= 0xD800 && r < 0xDC00) {
                        // a high surrogate pairs only with an immediately following \uDC00-\uDFFF
                        char32_t r2;
                        if (i + 1 < s.size() && s[i] == '\\' && s[i + 1] == 'u' && hex4(i + 2, r2) &&
                            r2 >= 0xDC00 && r2 < 0xE000) {
                            i += 6;
                            r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
                        } else {
                            r = 0xFFFD;
                        }
                    } else if (r >= 0xDC00 && r < 0xE000) {
                        r = 0xFFFD;
                    }
                    out.push_back(r);
                    break;
                }
                default: return false;
            }
        }
    }
    bool number(std::string &out) {
        const size_t b = i;
        if (i < s.size() && s[i] == '-') ++i;
        if (i >= s.size()) return false;
        if (s[i] == '0') {
            ++i;
        } else if (s[i] >= '1' && s[i] <= '9') {
            while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
        } else {
            return false;
        }
        if (i < s.size() && s[i] == '.') {
            ++i;
            if (i >= s.size() || s[i] < '0' || s[i] > '9') return false;
            while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
        }
        if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
            ++i;
            if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
            if (i >= s.size() || s[i] < '0' || s[i] > '9') return false;
            while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
        }
        out.assign(s.substr(b, i - b));
        return true;
    }
    bool value(Value &v, int depth) {
        ws();
        if (i >= s.size()) return false;
        const char c = s[i];
        if (c == '{' || c == '[') {
            if (depth + 1 > MAX_DEPTH) return false;
            ++i;
            ws();
            const char close = c == '{' ? '}' : ']';
            v.kind = c == '{' ? Value::OBJECT : Value::ARRAY;
            if (i < s.size() && s[i] == close) { ++i; return true; }
            while (true) {
                if (v.kind == Value::OBJECT) {
                    ws();
                    if (i >= s.size() || s[i] != '"') return false;
                    std::u32string key;
                    if (!str(key)) return false;
                    ws();
                    if (i >= s.size() || s[i] != ':') return false;
                    ++i;
                    v.members.emplace_back(std::move(key), Value());
                    if (!value(v.members.back().second, depth + 1)) return false;
                } else {
                    v.items.emplace_back();
                    if (!value(v.items.back(), depth + 1)) return false;
                }
                ws();
                if (i >= s.size()) return false;
                if (s[i] == ',') { ++i; continue; }
                if (s[i] == close) { ++i; return true; }
                return false;
            }
        }
        if (c == '"') {
            std::u32string t;
            v.kind = Value::STRING;
            return str(t);
        }
        if (c == 't') { v.kind = Value::BOOL; return lit("true", 4); }
        if (c == 'f') { v.kind = Value::BOOL; return lit("false", 5); }
        if (c == 'n') { v.kind = Value::NUL; return lit("null", 4); }
        v.kind = Value::NUMBER;
        return number(v.text);
    }
};

// Go's field-name folding (encoding/json appendFoldedName): ASCII upper
// case; non-ASCII runes r -> ToUpper(ToLower(r)), of which only these four
// land on ASCII letters
char32_t fold(char32_t r) {
    if (r >= 'a' && r <= 'z') return r - 'a' + 'A';
    switch (r) {
        case 0x017F: return 'S';  // LATIN SMALL LETTER LONG S
        case 0x212A: return 'K';  // KELVIN SIGN
        case 0x0130: return 'I';  // LATIN CAPITAL LETTER I WITH DOT ABOVE (ToLower -> 'i')
        case 0x0131: return 'I';  // LATIN SMALL LETTER DOTLESS I
        default: return r;
    }
}

bool key_is(const std::u32string &key, const char *name) {
    // exact match first, else folded; our field names are distinct under folding
    size_t n = 0;
    while (name[n]) ++n;
    if (key.size() != n) return false;
    bool exact = true;
    for (size_t j = 0; j < n; ++j) exact &= key[j] == (char32_t)(unsigned char)name[j];
    if (exact) return true;
    for (size_t j = 0; j < n; ++j)
        if (fold(key[j]) != fold((char32_t)(unsigned char)name[j])) return false;
    return true;
}

struct SumReceived {
    double bits_per_second = 0;
};
struct Stream {
    SumReceived sender, receiver;
};
struct StreamSlice {  // a Go slice: backing array contents (its capacity) + length
    std::vector<Stream> backing;
    size_t len = 0;
};

void decode_float(const Value &v, double &f) {
    if (v.kind != Value::NUMBER) return;  // null: unchanged; other kinds: type error
    const GoFloat g = go_parse_float(v.text, 64);
    if (g.err != GO_OK) return;  // overflow: UnmarshalTypeError, field unchanged
    f = g.value;
}

void decode_sum(const Value &v, SumReceived &r) {
    if (v.kind != Value::OBJECT) return;
    for (const auto &m : v.members)
        if (key_is(m.first, "bits_per_second")) decode_float(m.second, r.bits_per_second);
}

void decode_stream(const Value &v, Stream &st) {
    if (v.kind != Value::OBJECT) return;
    for (const auto &m : v.members) {
        if (key_is(m.first, "sender")) decode_sum(m.second, st.sender);
        else if (key_is(m.first, "receiver")) decode_sum(m.second, st.receiver);
    }
}

void decode_streams(const Value &v, StreamSlice &sl) {
    if (v.kind == Value::NUL) {  // v.SetZero(): nil slice
        sl.backing.clear();
        sl.len = 0;
        return;
    }
    if (v.kind != Value::ARRAY) return;
    size_t i = 0;
    for (const Value &e : v.items) {
        if (i >= sl.len) {
            // grow: a reallocation copies the whole (full) backing array and
            // zero-fills the rest, so growing by one zero element is exact
            if (i >= sl.backing.size()) sl.backing.emplace_back();
            sl.len = i + 1;
        }
        decode_stream(e, sl.backing[i]);  // merge into the existing element
        ++i;
    }
    if (i < sl.len) sl.len = i;  // truncate (the backing array keeps the tail)
    if (i == 0) {                 // reflect.MakeSlice(t, 0, 0)
        sl.backing.clear();
        sl.len = 0;
    }
}

void decode_end(const Value &v, StreamSlice &streams) {
    if (v.kind != Value::OBJECT) return;
    for (const auto &m : v.members)
        if (key_is(m.first, "streams")) decode_streams(m.second, streams);
}

}  // namespace

IperfReceiver go_unmarshal_iperf(std::string_view data) {
    IperfReceiver out{false, 0, 0.0, 0.0};
    Parser p{data};
    Value top;
    bool ok = p.value(top, 0);
    if (ok) {
        p.ws();
        ok = p.i == data.size();
    }
    if (!ok) return out;  // checkValid failed: the struct stays zero
    out.valid_json = true;
    StreamSlice streams;
    if (top.kind == Value::OBJECT)
        for (const auto &m : top.members)
            if (key_is(m.first, "end")) decode_end(m.second, streams);
    out.n_streams = (int)streams.len;
    if (streams.len > 0) {
        out.receiver_bps = streams.backing[0].receiver.bits_per_second;
        out.sender_bps = streams.backing[0].sender.bits_per_second;
    }
    return out;
}

}  // namespace nas_host
