// ks_ingest.cpp — host ingest (include/ks_ingest.h): Quantity strings, the simSpec annotation and
// the cluster config YAML, into the engine's int64 / bitmask records.
//
// Quantities are parsed exactly (a small decimal bignum: no float, no int64 overflow), following
// resource.ParseQuantity (vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go:146-377):
// the scanner parseQuantityString (:146-260), the suffixes of suffix.go (decimal SI n u m "" k M G
// T P E, binary SI Ki..Ei, e/E exponents), non-zero values rounded up to the nano scale (:354-360)
// and binary-SI values capped at 2^63 - 1 (:363-366).  The YAML reader is the subset the
// reference's files use (block mappings and sequences, plain and quoted scalars, comments, empty
// flow collections); yaml.v2 hands map values to a map[string]string as their literal text
// (vendor/gopkg.in/yaml.v2/decode.go:420-428), which is what a scalar keeps here.
#include <algorithm>
#include <array>
#include <cctype>
#include <cerrno>
#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/ks_ingest.h"

namespace {

// ------------------------------------------------------------------------------------------
// Quantity
// ------------------------------------------------------------------------------------------
// Unsigned decimal bignum, base 1e9 limbs, little endian.
struct Big {
    std::vector<uint32_t> d;
    static constexpr uint32_t kBase = 1000000000u;
    bool zero() const { return d.empty(); }
    void trim() { while (!d.empty() && d.back() == 0) d.pop_back(); }
    void mul(uint32_t m) {
        uint64_t c = 0;
        for (auto& x : d) {
            const uint64_t v = (uint64_t)x * m + c;
            x = (uint32_t)(v % kBase);
            c = v / kBase;
        }
        while (c) { d.push_back((uint32_t)(c % kBase)); c /= kBase; }
        trim();
    }
    void add(uint32_t a) {
        uint64_t c = a;
        for (size_t i = 0; i < d.size() && c; i++) {
            const uint64_t v = (uint64_t)d[i] + c;
            d[i] = (uint32_t)(v % kBase);
            c = v / kBase;
        }
        if (c) d.push_back((uint32_t)c);
    }
    uint32_t divmod(uint32_t m) {  // this /= m, returns the remainder
        uint64_t r = 0;
        for (size_t i = d.size(); i-- > 0;) {
            const uint64_t v = r * kBase + d[i];
            d[i] = (uint32_t)(v / m);
            r = v % m;
        }
        trim();
        return (uint32_t)r;
    }
    bool fits_u63(uint64_t* out) const {  // value < 2^63
        unsigned __int128 v = 0;
        for (size_t i = d.size(); i-- > 0;) {
            v = v * kBase + d[i];
            if (v >> 63) return false;
        }
        *out = (uint64_t)v;
        return true;
    }
};

enum class QErr { kOk, kFormat, kSuffix, kRange };

// value of s in nano-units, rounded up to an integer count of nano-units (quantity.go:354-360);
// sign separately
QErr parse_quantity_nano(const char* str, bool* negative, Big* nano) {
    const size_t end = std::strlen(str);
    if (end == 0) return QErr::kFormat;
    *negative = false;
    nano->d.clear();
    if (std::strcmp(str, "0") == 0) return QErr::kOk;
    size_t pos = 0;
    if (str[0] == '-') { *negative = true; pos = 1; }
    else if (str[0] == '+') pos = 1;
    while (pos < end && str[pos] == '0') pos++;  // leading zeros
    if (pos >= end) return QErr::kOk;            // "-000": zero
    std::string num, denom, suffix;
    size_t i = pos;
    while (i < end && std::isdigit((unsigned char)str[i])) i++;
    num = std::string(str + pos, str + i);
    pos = i;
    if (pos < end && str[pos] == '.') {
        pos++;
        i = pos;
        while (i < end && std::isdigit((unsigned char)str[i])) i++;
        denom = std::string(str + pos, str + i);
        pos = i;
    }
    const size_t suf_start = pos;
    i = pos;
    while (i < end && std::strchr("eEinumkKMGTP", str[i])) i++;
    pos = i;
    if (pos < end && (str[pos] == '-' || str[pos] == '+')) pos++;
    while (pos < end) {
        if (!std::isdigit((unsigned char)str[pos])) return QErr::kFormat;  // ErrFormatWrong
        pos++;
    }
    suffix = std::string(str + suf_start, str + end);
    // suffix.go: base 10 exponent or base 2 exponent
    int e10 = 0, e2 = 0;
    bool binary = false, huge = false;  // huge: |exponent| > 10^6 (only a zero value stays exact)
    static const std::pair<const char*, int> dec[] = {{"", 0}, {"n", -9}, {"u", -6}, {"m", -3}, {"k", 3},
                                                      {"M", 6}, {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
    static const std::pair<const char*, int> bin[] = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
    bool found = false;
    for (const auto& x : dec)
        if (suffix == x.first) { e10 = x.second; found = true; }
    for (const auto& x : bin)
        if (suffix == x.first) { e2 = x.second; binary = true; found = true; }
    if (!found) {
        if (suffix.size() > 1 && (suffix[0] == 'e' || suffix[0] == 'E')) {
            const char* p = suffix.c_str() + 1;
            char* q = nullptr;
            errno = 0;
            const long long v = std::strtoll(p, &q, 10);
            if (*p == 0 || *q != 0) return QErr::kSuffix;  // strconv.ParseInt fails
            if (errno == ERANGE || v > 1000000 || v < -1000000) huge = true;
            else e10 = (int)v;
        } else {
            return QErr::kSuffix;  // ErrSuffix
        }
    }
    // value = int(num denom) * 10^(e10 - len(denom)) * 2^e2; nano = value * 10^9, rounded up
    Big v;
    for (const char* s : {num.c_str(), denom.c_str()})
        for (const char* c = s; *c; c++) { v.mul(10); v.add((uint32_t)(*c - '0')); }
    if (v.zero()) return QErr::kOk;
    if (huge) return QErr::kRange;  // astronomically large, or below 1 nano (rounds to 1 nano)
    const long long k = (long long)e10 - (long long)denom.size() + 9;
    if (k > 200) return QErr::kRange;  // far beyond any int64 milli count
    for (int b = 0; b < e2; b++) v.mul(2);
    bool inexact = false;
    if (k >= 0) {
        for (long long t = 0; t < k; t++) v.mul(10);
    } else {
        for (long long t = 0; t < -k && !v.zero(); t++) inexact |= v.divmod(10) != 0;
        if (-k > 400) inexact = true;
    }
    if (inexact) v.add(1);  // RoundUp (away from zero) to the nano scale
    // binary SI values are capped at 2^63 - 1 (quantity.go:363-366): beyond it the milli count
    // overflows anyway, so the cap only matters for the range check below
    (void)binary;
    *nano = v;
    return QErr::kOk;
}

ks_status quantity_milli(const char* s, int64_t* milli) {
    bool neg = false;
    Big nano;
    const QErr e = parse_quantity_nano(s, &neg, &nano);
    if (e == QErr::kFormat || e == QErr::kSuffix) return KS_EINVAL;
    if (e == QErr::kRange) return KS_ERANGE;
    if (nano.zero()) { *milli = 0; return KS_OK; }
    if (neg) return KS_ERANGE;
    if (nano.divmod(1000000) != 0) return KS_ERANGE;  // not a whole number of milli-units
    uint64_t m = 0;
    if (!nano.fits_u63(&m)) return KS_ERANGE;
    *milli = (int64_t)m;
    return KS_OK;
}

// ceil of the quantity's value (Quantity.Value(), quantity.go:684-686), for `pods`
ks_status quantity_value_ceil(const char* s, int64_t* out) {
    bool neg = false;
    Big nano;
    const QErr e = parse_quantity_nano(s, &neg, &nano);
    if (e == QErr::kFormat || e == QErr::kSuffix) return KS_EINVAL;
    if (e == QErr::kRange) return KS_ERANGE;
    if (nano.zero()) { *out = 0; return KS_OK; }
    if (neg) return KS_ERANGE;
    const bool frac = nano.divmod(1000000000u) != 0;
    if (frac) nano.add(1);
    uint64_t v = 0;
    if (!nano.fits_u63(&v)) return KS_ERANGE;
    *out = (int64_t)v;
    return KS_OK;
}

// ------------------------------------------------------------------------------------------
// YAML subset
// ------------------------------------------------------------------------------------------
struct YNode {
    enum Kind { kScalar, kMap, kSeq, kNull } kind = kNull;
    std::string scalar;
    bool quoted = false;  // a quoted scalar is always a string (yaml.v2: no implicit resolution)
    std::vector<std::pair<std::string, std::unique_ptr<YNode>>> map;
    std::vector<std::unique_ptr<YNode>> seq;
    const YNode* get(const std::string& k, bool nocase = false) const {
        for (const auto& kv : map) {
            if (kv.first == k) return kv.second.get();
            if (nocase && kv.first.size() == k.size() &&
                std::equal(k.begin(), k.end(), kv.first.begin(),
                           [](char a, char b) { return std::tolower((unsigned char)a) == std::tolower((unsigned char)b); }))
                return kv.second.get();
        }
        return nullptr;
    }
};

struct Line {
    int indent;
    std::string text;  // without indentation and comment
    int no;
};

struct YamlError {
    std::string msg;
};

std::string rstrip(const std::string& s) {
    size_t e = s.size();
    while (e > 0 && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r')) e--;
    return s.substr(0, e);
}

// strip a comment that is not inside quotes ('#' at line start or after whitespace)
std::string strip_comment(const std::string& s) {
    char q = 0;
    for (size_t i = 0; i < s.size(); i++) {
        const char c = s[i];
        if (q) {
            if (c == q) q = 0;
        } else if (c == '"' || c == '\'') {
            if (i == 0 || s[i - 1] == ' ' || s[i - 1] == ':' || s[i - 1] == '-') q = c;
        } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
            return s.substr(0, i);
        }
    }
    return s;
}

std::vector<Line> split_lines(const char* text) {
    std::vector<Line> out;
    const char* p = text;
    int no = 0;
    while (*p) {
        const char* e = std::strchr(p, '\n');
        std::string raw = e ? std::string(p, e) : std::string(p);
        no++;
        p = e ? e + 1 : p + raw.size();
        if (raw.find('\t') != std::string::npos && raw.find_first_not_of(" \t") != std::string::npos &&
            raw.find_first_not_of(' ') < raw.size() && raw[raw.find_first_not_of(' ')] == '\t')
            throw YamlError{"line " + std::to_string(no) + ": tab indentation"};
        std::string t = rstrip(strip_comment(raw));
        const size_t ind = t.find_first_not_of(' ');
        if (ind == std::string::npos) continue;
        if (t.compare(ind, 3, "---") == 0 && t.size() == ind + 3) continue;  // document marker
        out.push_back({(int)ind, t.substr(ind), no});
    }
    return out;
}

std::string unquote(const std::string& s, int no) {
    if (s.size() >= 2 && s.front() == '"' && s.back() == '"') {
        std::string o;
        for (size_t i = 1; i + 1 < s.size(); i++) {
            if (s[i] == '\\' && i + 2 < s.size()) {
                const char c = s[++i];
                o += c == 'n' ? '\n' : c == 't' ? '\t' : c;
            } else {
                o += s[i];
            }
        }
        return o;
    }
    if (s.size() >= 2 && s.front() == '\'' && s.back() == '\'') {
        std::string o;
        for (size_t i = 1; i + 1 < s.size(); i++) {
            o += s[i];
            if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') i++;
        }
        return o;
    }
    if (!s.empty() && (s.front() == '"' || s.front() == '\'')) throw YamlError{"line " + std::to_string(no) + ": unterminated quote"};
    return s;
}

// position of the "key: " separator of a mapping line (outside quotes), or npos
size_t key_sep(const std::string& t) {
    char q = 0;
    for (size_t i = 0; i < t.size(); i++) {
        const char c = t[i];
        if (q) {
            if (c == q) q = 0;
            continue;
        }
        if ((c == '"' || c == '\'') && i == 0) { q = c; continue; }
        if (c == ':' && (i + 1 == t.size() || t[i + 1] == ' ')) return i;
    }
    return std::string::npos;
}

std::unique_ptr<YNode> scalar_node(const std::string& v, int no) {
    auto n = std::make_unique<YNode>();
    if (v == "{}") { n->kind = YNode::kMap; return n; }
    if (v == "[]") { n->kind = YNode::kSeq; return n; }
    if (v == "~" || v == "null") { n->kind = YNode::kNull; return n; }
    if (!v.empty() && (v.front() == '{' || v.front() == '[' || v.front() == '&' || v.front() == '*' || v.front() == '|' ||
                       v.front() == '>' || v.front() == '!'))
        throw YamlError{"line " + std::to_string(no) + ": unsupported YAML construct '" + v + "'"};
    n->kind = YNode::kScalar;
    n->quoted = !v.empty() && (v.front() == '"' || v.front() == '\'');
    n->scalar = unquote(v, no);
    return n;
}

std::unique_ptr<YNode> parse_block(const std::vector<Line>& L, size_t& i, int indent);

// the mapping whose first key is on line i at column `indent` (first entry text may be given)
std::unique_ptr<YNode> parse_map(const std::vector<Line>& L, size_t& i, int indent, std::string first, int first_no) {
    auto m = std::make_unique<YNode>();
    m->kind = YNode::kMap;
    bool have_first = !first.empty();
    while (true) {
        std::string t;
        int no;
        if (have_first) {
            t = first;
            no = first_no;
            have_first = false;
        } else {
            if (i >= L.size() || L[i].indent != indent) break;
            if (L[i].text.compare(0, 2, "- ") == 0 || L[i].text == "-") break;
            t = L[i].text;
            no = L[i].no;
            i++;
        }
        const size_t sep = key_sep(t);
        if (sep == std::string::npos) throw YamlError{"line " + std::to_string(no) + ": expected 'key: value'"};
        std::string key = unquote(rstrip(t.substr(0, sep)), no);
        std::string rest = sep + 1 < t.size() ? t.substr(sep + 1) : "";
        const size_t vs = rest.find_first_not_of(' ');
        rest = vs == std::string::npos ? "" : rest.substr(vs);
        for (const auto& kv : m->map)
            if (kv.first == key) throw YamlError{"line " + std::to_string(no) + ": duplicate key '" + key + "'"};
        std::unique_ptr<YNode> v;
        if (!rest.empty()) {
            v = scalar_node(rest, no);
        } else if (i < L.size() && (L[i].indent > indent ||
                                    (L[i].indent == indent && (L[i].text.compare(0, 2, "- ") == 0 || L[i].text == "-")))) {
            v = parse_block(L, i, L[i].indent);
        } else {
            v = std::make_unique<YNode>();  // null
        }
        m->map.emplace_back(std::move(key), std::move(v));
    }
    return m;
}

std::unique_ptr<YNode> parse_seq(const std::vector<Line>& L, size_t& i, int indent) {
    auto s = std::make_unique<YNode>();
    s->kind = YNode::kSeq;
    while (i < L.size() && L[i].indent == indent && (L[i].text.compare(0, 2, "- ") == 0 || L[i].text == "-")) {
        const Line& ln = L[i++];
        std::string rest = ln.text.size() > 2 ? ln.text.substr(2) : "";
        const size_t vs = rest.find_first_not_of(' ');
        const int item_indent = indent + 2 + (vs == std::string::npos ? 0 : (int)vs);
        rest = vs == std::string::npos ? "" : rest.substr(vs);
        if (rest.empty()) {
            if (i < L.size() && L[i].indent > indent) s->seq.push_back(parse_block(L, i, L[i].indent));
            else s->seq.push_back(std::make_unique<YNode>());
        } else if (key_sep(rest) != std::string::npos) {
            s->seq.push_back(parse_map(L, i, item_indent, rest, ln.no));  // "- key: v" + more keys below
        } else {
            s->seq.push_back(scalar_node(rest, ln.no));
        }
    }
    return s;
}

std::unique_ptr<YNode> parse_block(const std::vector<Line>& L, size_t& i, int indent) {
    if (i >= L.size()) return std::make_unique<YNode>();
    if (L[i].text.compare(0, 2, "- ") == 0 || L[i].text == "-") return parse_seq(L, i, indent);
    if (key_sep(L[i].text) != std::string::npos) return parse_map(L, i, indent, "", 0);
    auto n = scalar_node(L[i].text, L[i].no);
    i++;
    return n;
}

std::unique_ptr<YNode> yaml_parse(const char* text) {
    const std::vector<Line> L = split_lines(text);
    size_t i = 0;
    if (L.empty()) return std::make_unique<YNode>();
    auto root = parse_block(L, i, L[0].indent);
    if (i < L.size()) throw YamlError{"line " + std::to_string(L[i].no) + ": unexpected indentation"};
    return root;
}

void set_err(char* err, int32_t len, const char* fmt, ...) {
    if (!err || len <= 0) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err, (size_t)len, fmt, ap);
    va_end(ap);
}

// strconv.ParseInt(s, 0, 64) of Go 1.11 (the reference's pinned toolchain, .travis.yml): optional
// sign, then "0x"/"0X" hex, a leading "0" octal, else decimal.  Returns false on a syntax error;
// *big = true when the magnitude does not fit int64 (ErrRange).
bool go_parse_int(const std::string& s0, __int128* v, bool* big) {
    *big = false;
    if (s0.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s0[0] == '+' || s0[0] == '-') { neg = s0[0] == '-'; i = 1; }
    std::string s = s0.substr(i);
    if (s.empty()) return false;
    int base = 10;
    if (s[0] == '0' && s.size() > 1 && (s[1] == 'x' || s[1] == 'X')) {
        if (s.size() < 3) return false;
        base = 16;
        s = s.substr(2);
    } else if (s[0] == '0') {
        base = 8;
        s = s.substr(1);
    }
    unsigned __int128 n = 0;
    for (char c : s) {
        int d;
        if (c >= '0' && c <= '9') d = c - '0';
        else if (c >= 'a' && c <= 'z') d = c - 'a' + 10;
        else if (c >= 'A' && c <= 'Z') d = c - 'A' + 10;
        else return false;
        if (d >= base) return false;
        if (n <= ((unsigned __int128)1 << 70)) n = n * base + d;  // saturates far above 2^64
    }
    const unsigned __int128 lim = (unsigned __int128)1 << 63;
    if (neg ? n > lim : n >= lim) *big = true;
    *v = neg ? -(__int128)n : (__int128)n;
    return true;
}

// An int32 struct field decoded by yaml.v2 v2.2.2 (vendor/gopkg.in/yaml.v2/resolve.go:86-196,
// decode.go:443-465): null -> 0; a quoted scalar is a string (type error); a plain scalar
// resolves by its first character: digits / sign -> underscores dropped, ParseInt(base 0), then
// ParseUint (too big for int32 anyway), then a YAML-style float (truncated toward zero), then
// 0b / -0b binary; '.' -> a float; the resolve map (bools, nulls, .inf, .nan) and anything else
// -> not an int32.  The result must fit int32 (OverflowInt).
bool yaml_int32(const YNode* n, int32_t* out) {
    *out = 0;
    if (!n || n->kind == YNode::kNull) return true;
    if (n->kind != YNode::kScalar || n->quoted) return false;
    const std::string& in = n->scalar;
    static const char* kNulls[] = {"", "~", "null", "Null", "NULL"};
    for (const char* z : kNulls)
        if (in == z) return true;
    if (in.empty()) return true;
    auto fits = [&](__int128 v) {
        if (v < INT32_MIN || v > INT32_MAX) return false;
        *out = (int32_t)v;
        return true;
    };
    auto from_float = [&](double f) {  // decode.go: resolved <= MaxInt64 && !OverflowInt(int64(f))
        if (!(f <= 9223372036854775807.0) || f < -2147483649.0) return false;
        return fits((__int128)(int64_t)f);
    };
    auto float_syntax = [](const std::string& t, size_t i) {  // ^[-+]?[0-9]*\.?[0-9]+([eE][-+][0-9]+)?$
        if (i < t.size() && (t[i] == '+' || t[i] == '-')) i++;
        size_t a = i;
        while (i < t.size() && std::isdigit((unsigned char)t[i])) i++;
        const size_t int_digits = i - a;
        if (i < t.size() && t[i] == '.') {
            i++;
            size_t b = i;
            while (i < t.size() && std::isdigit((unsigned char)t[i])) i++;
            if (i == b) return false;
        } else if (int_digits == 0) {
            return false;
        }
        if (i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
            i++;
            if (i >= t.size() || (t[i] != '+' && t[i] != '-')) return false;
            i++;
            size_t b = i;
            while (i < t.size() && std::isdigit((unsigned char)t[i])) i++;
            if (i == b) return false;
        }
        return i == t.size();
    };
    const char c0 = in[0];
    if (c0 == '.') {  // ParseFloat(in): ".5", ".5e3", ".5E-2" (".inf" / ".nan" are map entries: no int)
        size_t i = 1, b = 1;
        while (i < in.size() && std::isdigit((unsigned char)in[i])) i++;
        if (i == b) return false;
        if (i < in.size() && (in[i] == 'e' || in[i] == 'E')) {
            i++;
            if (i < in.size() && (in[i] == '+' || in[i] == '-')) i++;
            size_t e = i;
            while (i < in.size() && std::isdigit((unsigned char)in[i])) i++;
            if (i == e) return false;
        }
        if (i != in.size()) return false;
        return from_float(std::strtod(in.c_str(), nullptr));
    }
    if (!(std::isdigit((unsigned char)c0) || c0 == '+' || c0 == '-')) return false;  // bools, words: strings
    {  // a timestamp (four digits then '-') never decodes into an int
        size_t i = 0;
        while (i < in.size() && std::isdigit((unsigned char)in[i])) i++;
        if (i == 4 && i < in.size() && in[i] == '-') return false;
    }
    std::string plain;
    for (char c : in)
        if (c != '_') plain += c;
    __int128 v = 0;
    bool big = false;
    if (go_parse_int(plain, &v, &big)) return !big && fits(v);  // ParseUint only adds >= 2^63
    if (float_syntax(plain, 0)) return from_float(std::strtod(plain.c_str(), nullptr));
    if (plain.compare(0, 2, "0b") == 0 || plain.compare(0, 3, "-0b") == 0) {
        const bool neg = plain[0] == '-';
        const std::string d = plain.substr(neg ? 3 : 2);
        if (d.empty()) return false;
        unsigned __int128 n = 0;
        for (char c : d) {
            if (c != '0' && c != '1') return false;
            if (n <= ((unsigned __int128)1 << 70)) n = n * 2 + (c - '0');
        }
        return fits(neg ? -(__int128)n : (__int128)n);
    }
    return false;
}

int resource_index(const std::string& name) {
    if (name == "cpu") return 0;
    if (name == "memory") return 1;
    if (name == "nvidia.com/gpu") return 2;
    return -1;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Cluster
// ------------------------------------------------------------------------------------------
struct ks_cluster {
    using Taint = std::tuple<std::string, std::string, std::string>;  // key, value, effect
    using Pair = std::pair<std::string, std::string>;
    using Tol = std::array<std::string, 4>;                            // key, operator, value, effect
    int32_t tick = 10;
    std::string start_clock;
    std::vector<std::string> names;
    std::vector<int64_t> alloc;  // [n][4]
    std::vector<uint64_t> taint, label;
    // every NoSchedule/NoExecute taint and label pair the nodes carry (sorted), and each node's
    std::vector<Taint> all_taints;
    std::vector<Pair> all_pairs;
    std::vector<std::vector<int32_t>> node_taints, node_pairs;
    // the encoding ks_cluster_seal chose: taint -> bit (its toleration class) and label pair -> bit
    bool sealed = false;
    std::vector<int32_t> taint_bit;
    int32_t n_taint_bits = 0;
    std::map<Pair, int> label_dict;
    // pods noted before sealing (the two-phase form): distinct toleration lists, referenced pairs
    std::set<std::vector<Tol>> noted_tols;
    std::set<Pair> noted_pairs;
};

namespace {

bool tolerates(const ks_cluster::Tol& t, const ks_cluster::Taint& x) {
    const auto& [tk, tv, te] = x;
    bool ok = t[3].empty() || t[3] == te;                                  // toleration.go:38-40
    ok = ok && (t[0].empty() || t[0] == tk);                               // :42-44
    return ok && ((t[1].empty() || t[1] == "Equal") ? t[2] == tv : t[1] == "Exists");  // :47-55
}

/* Choose the masks' bits and build the node masks.  One bit per taint and per label pair while
 * the cluster fits one 64-bit mask (the cluster alone decides: ks_cluster_parse).  Past that
 * (VERDICT r5 item 5), with the pods noted: only label pairs some noted nodeSelector references get
 * bits (no other pair can change a placement — per-node hostname labels need none), and taints
 * that exactly the same noted toleration lists tolerate share one bit (a node is feasible for a pod
 * iff the pod tolerates each of its taints, so interchangeable taints decide identically). */
ks_status seal(ks_cluster* c, bool wide, char* err, int32_t err_len) {
    const size_t T = c->all_taints.size(), L = c->all_pairs.size();
    c->taint_bit.assign(T, 0);
    if (T <= 64 || !wide) {
        for (size_t t = 0; t < T; t++) c->taint_bit[t] = (int32_t)t;
        c->n_taint_bits = (int32_t)T;
    } else {
        std::map<std::vector<bool>, int32_t> cls;
        for (size_t t = 0; t < T; t++) {
            std::vector<bool> sig;
            sig.reserve(c->noted_tols.size());
            for (const auto& tl : c->noted_tols) {
                bool any = false;
                for (const auto& x : tl) any = any || tolerates(x, c->all_taints[t]);
                sig.push_back(any);
            }
            const auto it = cls.emplace(std::move(sig), (int32_t)cls.size()).first;
            c->taint_bit[t] = it->second;
        }
        c->n_taint_bits = (int32_t)cls.size();
    }
    c->label_dict.clear();
    int li = 0;
    for (const auto& l : c->all_pairs)
        if (L <= 63 || !wide || c->noted_pairs.count(l)) c->label_dict[l] = li++;
    if (c->n_taint_bits > 64 || li > 63) {
        set_err(err, err_len, "%d taint classes / %d label pairs exceed one 64-bit mask%s", c->n_taint_bits, li,
                wide ? "" : " (note the pods and seal: ks_cluster_parse_ex)");
        return KS_ERANGE;
    }
    const size_t n = c->names.size();
    c->taint.assign(n, 0);
    c->label.assign(n, 0);
    for (size_t i = 0; i < n; i++) {
        for (int32_t t : c->node_taints[i]) c->taint[i] |= 1ull << c->taint_bit[t];
        for (int32_t l : c->node_pairs[i]) {
            const auto it = c->label_dict.find(c->all_pairs[l]);
            if (it != c->label_dict.end()) c->label[i] |= 1ull << it->second;
        }
    }
    c->sealed = true;
    return KS_OK;
}

std::string cstr(const char* s) { return std::string(s ? s : ""); }

}  // namespace

extern "C" {

ks_status ks_parse_quantity(const char* s, int64_t* milli_out) {
    if (!s || !milli_out) return KS_EINVAL;
    return quantity_milli(s, milli_out);
}

ks_status ks_parse_simspec(const char* yaml, int32_t max_phases, int32_t* n_phases, int32_t* seconds,
                           int64_t* usage, uint8_t* usage_mask, char* err, int32_t err_len) {
    if (!yaml || !n_phases || max_phases < 0 || (max_phases > 0 && (!seconds || !usage || !usage_mask)))
        return KS_EINVAL;
    *n_phases = 0;
    std::unique_ptr<YNode> doc;
    try {
        doc = yaml_parse(yaml);
    } catch (const YamlError& e) {
        set_err(err, err_len, "%s", e.msg.c_str());
        return KS_EINVAL;
    }
    if (doc->kind == YNode::kNull) return KS_OK;  // an empty document: no phases
    if (doc->kind != YNode::kSeq) {
        set_err(err, err_len, "simSpec is not a YAML list");
        return KS_EINVAL;
    }
    int32_t n = 0;
    for (const auto& ph : doc->seq) {
        const YNode* ru = ph->kind == YNode::kMap ? ph->get("resourceUsage") : nullptr;
        if (ru && ru->kind != YNode::kNull && ru->kind != YNode::kMap) {  // yaml.v2: cannot unmarshal into a map
            set_err(err, err_len, "resourceUsage is not a mapping");
            return KS_EINVAL;
        }
        if (!ru || ru->kind == YNode::kNull) {  // spec.go:48-50
            set_err(err, err_len, "Invalid spec.resoruceUsage field");
            return KS_EINVAL;
        }
        int32_t sec = 0;
        if (!yaml_int32(ph->get("seconds"), &sec)) {  // yaml.v2 int32 field decoding
            const YNode* s = ph->get("seconds");
            set_err(err, err_len, "cannot unmarshal seconds %s%s%s into int32", s && s->quoted ? "\"" : "",
                    s && s->kind == YNode::kScalar ? s->scalar.c_str() : "(non-scalar)", s && s->quoted ? "\"" : "");
            return KS_EINVAL;
        }
        int64_t use[3] = {0, 0, 0};
        uint8_t mask = 0;
        for (const auto& kv : ru->map) {
            const std::string v = kv.second->kind == YNode::kScalar ? kv.second->scalar : "";
            int64_t m = 0;
            const ks_status r = quantity_milli(v.c_str(), &m);
            if (r == KS_EINVAL) {  // util.BuildResourceList: InvalidArgument
                set_err(err, err_len, "invalid %s value \"%s\"", kv.first.c_str(), v.c_str());
                return KS_EINVAL;
            }
            const int k = resource_index(kv.first);
            if (r != KS_OK || k < 0) {
                set_err(err, err_len, "%s value \"%s\" outside the engine's domain", kv.first.c_str(), v.c_str());
                return KS_ERANGE;
            }
            use[k] = m;
            mask |= (uint8_t)(1u << k);
        }
        if (n < max_phases) {
            seconds[n] = (int32_t)sec;
            for (int k = 0; k < 3; k++) usage[(int64_t)n * 3 + k] = use[k];
            usage_mask[n] = mask;
        }
        n++;
    }
    *n_phases = n;
    return KS_OK;
}

ks_status ks_cluster_parse_ex(const char* yaml, int32_t flags, ks_cluster** out, char* err, int32_t err_len) {
    if (!yaml || !out || (flags & ~KS_CLUSTER_DEFER_MASKS)) return KS_EINVAL;
    *out = nullptr;
    std::unique_ptr<YNode> doc;
    try {
        doc = yaml_parse(yaml);
    } catch (const YamlError& e) {
        set_err(err, err_len, "%s", e.msg.c_str());
        return KS_EINVAL;
    }
    if (doc->kind != YNode::kMap) {
        set_err(err, err_len, "config is not a YAML mapping");
        return KS_EINVAL;
    }
    auto c = std::make_unique<ks_cluster>();
    // viper matches keys case-insensitively (vendor/github.com/spf13/viper/util.go:69-89)
    if (const YNode* t = doc->get("tick", true)) {
        char* q = nullptr;
        const long long v = t->kind == YNode::kScalar ? std::strtoll(t->scalar.c_str(), &q, 10) : 0;
        if (t->kind != YNode::kScalar || *q != 0 || v < 1 || v > INT32_MAX) {
            set_err(err, err_len, "tick must be a positive integer");
            return KS_EINVAL;
        }
        c->tick = (int32_t)v;
    }
    if (const YNode* s = doc->get("startClock", true)) c->start_clock = s->kind == YNode::kScalar ? s->scalar : "";
    const YNode* cl = doc->get("cluster", true);
    const YNode* nodes = cl && cl->kind == YNode::kMap ? cl->get("nodes", true) : nullptr;
    if (nodes && nodes->kind != YNode::kSeq && nodes->kind != YNode::kNull) {
        set_err(err, err_len, "cluster.nodes is not a list");
        return KS_EINVAL;
    }
    struct NodeIn {
        int64_t alloc[4];
        std::vector<std::tuple<std::string, std::string, std::string>> taints;
        std::vector<std::pair<std::string, std::string>> labels;
        std::string ns, name;
    };
    std::vector<NodeIn> in;
    std::set<std::tuple<std::string, std::string, std::string>> tset;
    std::set<std::pair<std::string, std::string>> lset;
    if (nodes && nodes->kind == YNode::kSeq) {
        for (const auto& nd : nodes->seq) {
            if (nd->kind != YNode::kMap) {
                set_err(err, err_len, "node %zu is not a mapping", in.size());
                return KS_EINVAL;
            }
            NodeIn x{{-1, -1, -1, 0}, {}, {}, "", ""};
            const YNode* ns = nd->get("namespace", true);
            const YNode* nm = nd->get("name", true);
            x.ns = ns && ns->kind == YNode::kScalar ? ns->scalar : "";
            x.name = nm && nm->kind == YNode::kScalar ? nm->scalar : "";
            if (const YNode* cap = nd->get("capacity", true)) {
                for (const auto& kv : cap->map) {
                    const std::string v = kv.second->kind == YNode::kScalar ? kv.second->scalar : "";
                    int64_t m = 0;
                    ks_status r;
                    int k = resource_index(kv.first);
                    if (kv.first == "pods") {
                        k = 3;
                        r = quantity_value_ceil(v.c_str(), &m);  // Capacity.Pods().Value()
                    } else {
                        r = quantity_milli(v.c_str(), &m);
                    }
                    if (r == KS_EINVAL) {  // util.BuildResourceList (config.go:45-48)
                        set_err(err, err_len, "invalid %s value \"%s\"", kv.first.c_str(), v.c_str());
                        return KS_EINVAL;
                    }
                    if (r != KS_OK || m >= (1LL << 59)) {
                        set_err(err, err_len, "%s value \"%s\" outside the engine's domain", kv.first.c_str(), v.c_str());
                        return KS_ERANGE;
                    }
                    if (k >= 0) x.alloc[k] = m;  // other resource names never constrain a pod
                }
            }
            if (const YNode* tl = nd->get("taints", true)) {
                for (const auto& t : tl->seq) {
                    auto field = [&](const char* f) {
                        const YNode* v = t->kind == YNode::kMap ? t->get(f, true) : nullptr;
                        return v && v->kind == YNode::kScalar ? v->scalar : std::string();
                    };
                    const std::string eff = field("effect");
                    if (eff != "NoSchedule" && eff != "NoExecute" && eff != "PreferNoSchedule") {  // buildTaint
                        set_err(err, err_len, "taint effect \"%s\" is not supported", eff.c_str());
                        return KS_EINVAL;
                    }
                    x.taints.emplace_back(field("key"), field("value"), eff);
                }
            }
            if (const YNode* lb = nd->get("labels", true))
                for (const auto& kv : lb->map)
                    x.labels.emplace_back(kv.first, kv.second->kind == YNode::kScalar ? kv.second->scalar : "");
            // NewKubeSim keys nodes by name (kubesim/kubesim.go:37-47): a later node replaces an
            // earlier one of the same name
            in.erase(std::remove_if(in.begin(), in.end(), [&](const NodeIn& o) { return o.name == x.name; }), in.end());
            in.push_back(std::move(x));
        }
    }
    for (const auto& x : in) {
        c->names.push_back(x.ns + "/" + x.name);
        for (const auto& t : x.taints)
            if (std::get<2>(t) != "PreferNoSchedule") tset.insert(t);  // never filters
        for (const auto& l : x.labels) lset.insert(l);
    }
    c->all_taints.assign(tset.begin(), tset.end());
    c->all_pairs.assign(lset.begin(), lset.end());
    const size_t n = in.size();
    c->alloc.resize(4 * n);
    c->node_taints.resize(n);
    c->node_pairs.resize(n);
    for (size_t i = 0; i < n; i++) {
        for (int k = 0; k < 4; k++) c->alloc[4 * i + k] = in[i].alloc[k];
        for (const auto& t : in[i].taints) {
            const auto it = std::lower_bound(c->all_taints.begin(), c->all_taints.end(), t);
            if (it != c->all_taints.end() && *it == t) c->node_taints[i].push_back((int32_t)(it - c->all_taints.begin()));
        }
        for (const auto& l : in[i].labels)
            c->node_pairs[i].push_back((int32_t)(std::lower_bound(c->all_pairs.begin(), c->all_pairs.end(), l) -
                                                 c->all_pairs.begin()));
    }
    if (!(flags & KS_CLUSTER_DEFER_MASKS)) {
        const ks_status r = seal(c.get(), false, err, err_len);
        if (r != KS_OK) return r;
    }
    *out = c.release();
    return KS_OK;
}

ks_status ks_cluster_parse(const char* yaml, ks_cluster** out, char* err, int32_t err_len) {
    return ks_cluster_parse_ex(yaml, 0, out, err, err_len);
}

ks_status ks_cluster_note_pod(ks_cluster* c, int32_t n_tol, const char* const* key, const char* const* op,
                              const char* const* value, const char* const* effect, int32_t n_sel,
                              const char* const* sel_key, const char* const* sel_value) {
    if (!c || c->sealed || n_tol < 0 || n_sel < 0 || (n_tol > 0 && (!key || !op || !value || !effect)) ||
        (n_sel > 0 && (!sel_key || !sel_value)))
        return KS_EINVAL;
    std::vector<ks_cluster::Tol> tl;
    for (int32_t i = 0; i < n_tol; i++) tl.push_back({cstr(key[i]), cstr(op[i]), cstr(value[i]), cstr(effect[i])});
    std::sort(tl.begin(), tl.end());
    c->noted_tols.insert(std::move(tl));
    for (int32_t i = 0; i < n_sel; i++) c->noted_pairs.emplace(cstr(sel_key[i]), cstr(sel_value[i]));
    return KS_OK;
}

ks_status ks_cluster_seal(ks_cluster* c, char* err, int32_t err_len) {
    if (!c || c->sealed) return KS_EINVAL;
    return seal(c, true, err, err_len);
}

void ks_cluster_free(ks_cluster* c) { delete c; }
int64_t ks_cluster_nodes(const ks_cluster* c) { return c ? (int64_t)c->names.size() : -1; }
int32_t ks_cluster_tick(const ks_cluster* c) { return c ? c->tick : -1; }
const char* ks_cluster_start_clock(const ks_cluster* c) { return c ? c->start_clock.c_str() : ""; }
const char* ks_cluster_node_name(const ks_cluster* c, int64_t i) {
    return c && i >= 0 && i < (int64_t)c->names.size() ? c->names[i].c_str() : nullptr;
}

ks_status ks_cluster_arrays(const ks_cluster* c, int64_t* alloc, uint64_t* taint, uint64_t* label) {
    if (!c || !c->sealed) return KS_EINVAL;
    const size_t n = c->names.size();
    if (alloc) std::memcpy(alloc, c->alloc.data(), sizeof(int64_t) * 4 * n);
    if (taint) std::memcpy(taint, c->taint.data(), sizeof(uint64_t) * n);
    if (label) std::memcpy(label, c->label.data(), sizeof(uint64_t) * n);
    return KS_OK;
}

ks_status ks_cluster_tolerations(const ks_cluster* c, int32_t n, const char* const* key, const char* const* op,
                                 const char* const* value, const char* const* effect, uint64_t* tol_out) {
    if (!c || !c->sealed || !tol_out || n < 0 || (n > 0 && (!key || !op || !value || !effect))) return KS_EINVAL;
    std::vector<ks_cluster::Tol> tl;
    for (int32_t i = 0; i < n; i++) tl.push_back({cstr(key[i]), cstr(op[i]), cstr(value[i]), cstr(effect[i])});
    uint64_t m = 0, seen = 0;
    for (size_t t = 0; t < c->all_taints.size(); t++) {
        bool any = false;
        for (const auto& x : tl) any = any || tolerates(x, c->all_taints[t]);
        const uint64_t b = 1ull << c->taint_bit[t];
        // a class shares one bit only if this pod tolerates all of it or none of it: a pod the
        // seal never saw may split a class, and its mask would then be inexact
        if ((seen & b) && (bool)(m & b) != any) return KS_ERANGE;
        seen |= b;
        if (any) m |= b;
    }
    *tol_out = m;
    return KS_OK;
}

ks_status ks_cluster_selector(const ks_cluster* c, int32_t n, const char* const* key, const char* const* value,
                              uint64_t* sel_out) {
    if (!c || !c->sealed || !sel_out || n < 0 || (n > 0 && (!key || !value))) return KS_EINVAL;
    uint64_t m = 0;
    for (int32_t i = 0; i < n; i++) {
        const ks_cluster::Pair pr(cstr(key[i]), cstr(value[i]));
        const auto it = c->label_dict.find(pr);
        if (it != c->label_dict.end()) {
            m |= 1ull << it->second;
        } else if (std::binary_search(c->all_pairs.begin(), c->all_pairs.end(), pr)) {
            return KS_ERANGE;  // a pair some node carries that the seal did not see referenced
        } else {
            m |= 1ull << 63;   // no node carries it: infeasible everywhere
        }
    }
    *sel_out = m;
    return KS_OK;
}

}  // extern "C"
