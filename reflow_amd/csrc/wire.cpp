// wire.cpp -- host-only wire formats of the path (no HIP, no device):
//   * Fileset JSON: json.Marshal(Fileset), the assoc value CacheWrite stores
//     under every cache key (eval.go:1141, 1961-1967);
//   * the liveset bloom filter's binary and JSON forms (bloom.go:264-325,
//     bitset.go:623-721): parsed into host words for rf_bloom_load_*, and
//     formatted from host words for rf_bloom_marshal_*.
// These units build under g++ with -fsanitize=address,undefined alone
// (reflow_amd/csrc/Makefile `asan`, tests/cpp/asan_host.cpp).
#include <ctype.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "errors.h"
#include "wire.h"

using rf::fail;

// ---------------------------------------------------------------------------
// Fileset JSON: json.Marshal(Fileset) -> Repository.Put (eval.go:1961-1967),
// the assoc value CacheWrite stores under every cache key (eval.go:1141).
// Byte rules of Go 1.9/1.10 encoding/json (.travis.yml:3-5): struct fields
// in declaration order with their tags (executor.go:25-38: "List" and
// "Fileset", both omitempty, i.e. omitted when len == 0), map keys sorted
// bytewise, strings escaped by encodeState.string with escapeHTML.
static const char kHex[] = "0123456789abcdef";

// Length of the valid UTF-8 sequence at s[i] (s[i] >= 0x80), 0 if invalid:
// the acceptance ranges of unicode/utf8.DecodeRuneInString.
static size_t utf8_seq(const uint8_t* s, size_t n, size_t i) {
    const uint8_t b0 = s[i];
    auto in = [&](size_t j, uint8_t lo, uint8_t hi) { return j < n && s[j] >= lo && s[j] <= hi; };
    if (b0 >= 0xC2 && b0 <= 0xDF) return in(i + 1, 0x80, 0xBF) ? 2 : 0;
    if (b0 >= 0xE0 && b0 <= 0xEF) {
        const uint8_t lo = b0 == 0xE0 ? 0xA0 : 0x80, hi = b0 == 0xED ? 0x9F : 0xBF;
        return in(i + 1, lo, hi) && in(i + 2, 0x80, 0xBF) ? 3 : 0;
    }
    if (b0 >= 0xF0 && b0 <= 0xF4) {
        const uint8_t lo = b0 == 0xF0 ? 0x90 : 0x80, hi = b0 == 0xF4 ? 0x8F : 0xBF;
        return in(i + 1, lo, hi) && in(i + 2, 0x80, 0xBF) && in(i + 3, 0x80, 0xBF) ? 4 : 0;
    }
    return 0;
}

static void json_string(std::string& o, const uint8_t* s, size_t n) {
    o.push_back('"');
    size_t i = 0;
    while (i < n) {
        const uint8_t b = s[i];
        if (b < 0x80) {
            switch (b) {
                case '"': case '\\': o.push_back('\\'); o.push_back((char)b); break;
                case '\n': o += "\\n"; break;
                case '\r': o += "\\r"; break;
                case '\t': o += "\\t"; break;
                default:
                    if (b < 0x20 || b == '<' || b == '>' || b == '&') {
                        o += "\\u00";
                        o.push_back(kHex[b >> 4]);
                        o.push_back(kHex[b & 15]);
                    } else {
                        o.push_back((char)b);
                    }
            }
            ++i;
            continue;
        }
        const size_t len = utf8_seq(s, n, i);
        if (len == 0) {  // utf8.RuneError of size 1: one replacement per bad byte
            o += "\\ufffd";
            ++i;
        } else if (len == 3 && b == 0xE2 && s[i + 1] == 0x80 && (s[i + 2] == 0xA8 || s[i + 2] == 0xA9)) {
            o += "\\u202";  // U+2028 / U+2029
            o.push_back(kHex[s[i + 2] - 0xA0]);
            i += 3;
        } else {
            o.append(reinterpret_cast<const char*>(s + i), len);
            i += len;
        }
    }
    o.push_back('"');
}

static int marshal_fileset(const rf_fileset_tree* t, uint32_t node, int depth, std::string& o,
                           std::vector<uint64_t>& idx) {
    if (node >= t->n_nodes) return fail(RF_EINVAL, "fileset node %u >= n_nodes %llu", node,
                                        (unsigned long long)t->n_nodes);
    if (depth > 4096) return fail(RF_EINVAL, "fileset tree deeper than 4096 (cycle?)");
    const uint64_t lb = t->list_ptr[node], le = t->list_ptr[node + 1];
    const uint64_t eb = t->entry_ptr[node], ee = t->entry_ptr[node + 1];
    if (lb > le || eb > ee) return fail(RF_EINVAL, "fileset node %u: CSR not monotone", node);
    o.push_back('{');
    if (le > lb) {
        o += "\"List\":[";
        for (uint64_t c = lb; c < le; ++c) {
            if (c > lb) o.push_back(',');
            int rc = marshal_fileset(t, t->list_child[c], depth + 1, o, idx);
            if (rc) return rc;
        }
        o.push_back(']');
    }
    if (ee > eb) {
        if (le > lb) o.push_back(',');
        o += "\"Fileset\":{";
        const size_t base = idx.size();
        for (uint64_t e = eb; e < ee; ++e) idx.push_back(e);
        auto less = [&](uint64_t a, uint64_t b) {
            const size_t la = t->path_lens[a], lb2 = t->path_lens[b];
            const int c = memcmp(t->paths[a], t->paths[b], std::min(la, lb2));
            return c < 0 || (c == 0 && la < lb2);
        };
        std::sort(idx.begin() + base, idx.end(), less);
        for (size_t q = base; q < idx.size(); ++q) {
            const uint64_t e = idx[q];
            if (q > base && !less(idx[q - 1], e))
                return fail(RF_EINVAL, "fileset node %u: duplicate map key", node);
            const uint8_t* id = t->ids32 + 32 * e;
            bool zero = true;
            for (int k = 0; k < 32; ++k) zero &= id[k] == 0;
            if (zero)  // digest.Digest's zero text form is grailbio/base's (unvendored)
                return fail(RF_EINVAL, "fileset node %u: zero file ID has no pinned JSON form", node);
            if (q > base) o.push_back(',');
            json_string(o, reinterpret_cast<const uint8_t*>(t->paths[e]), t->path_lens[e]);
            o += ":{\"ID\":\"sha256:";
            for (int k = 0; k < 32; ++k) {
                o.push_back(kHex[id[k] >> 4]);
                o.push_back(kHex[id[k] & 15]);
            }
            o += "\",\"Size\":";
            o += std::to_string((long long)t->sizes[e]);
            o.push_back('}');
        }
        idx.resize(base);
        o.push_back('}');
    }
    o.push_back('}');
    return RF_OK;
}

static int check_tree(const rf_fileset_tree* t) {
    ARG(t && t->list_ptr && t->entry_ptr, "null fileset tree");
    const uint64_t nl = t->list_ptr[t->n_nodes], ne = t->entry_ptr[t->n_nodes];
    ARG(nl == 0 || t->list_child, "null list_child");
    ARG(ne == 0 || (t->paths && t->path_lens && t->ids32 && t->sizes), "null entry arrays");
    return RF_OK;
}

extern "C" int rf_fileset_marshal_json(const rf_fileset_tree* t, uint32_t root, uint8_t* out,
                                       uint64_t cap, uint64_t* out_len) {
    int rc = check_tree(t);
    if (rc) return rc;
    ARG(out_len, "null out_len");
    std::string o;
    std::vector<uint64_t> idx;
    if ((rc = marshal_fileset(t, root, 0, o, idx))) return rc;
    *out_len = o.size();
    if (o.size() > cap) return fail(RF_EINVAL, "output buffer too small: need %zu bytes", o.size());
    if (!o.empty() && out) memcpy(out, o.data(), o.size());
    return RF_OK;
}

int fileset_check_tree(const rf_fileset_tree* t) { return check_tree(t); }

int fileset_marshal_append(const rf_fileset_tree* t, uint32_t root, std::string& o) {
    std::vector<uint64_t> idx;
    return marshal_fileset(t, root, 0, o, idx);
}

// ---------------------------------------------------------------------------
// Liveset bloom filter wire forms
static uint64_t be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return v;
}

// wordsNeeded(length) without wrapping (bitset.go:89-94)
static uint64_t words_needed(uint64_t length) { return length / 64 + (length % 64 != 0); }

// bitset.ReadFrom: BE64 length, then wordsNeeded(length) BE64 words
static int parse_bitset(const uint8_t* p, size_t n, uint64_t* length, std::vector<uint64_t>& w) {
    ARG(n >= 8, "truncated bitset");
    *length = be64(p);
    const uint64_t nw = words_needed(*length);
    ARG((n - 8) / 8 >= nw, "truncated bitset words");
    w.resize(nw);
    for (uint64_t i = 0; i < nw; ++i) w[i] = be64(p + 8 + 8 * i);
    return RF_OK;
}

int bloom_parse_binary(const uint8_t* buf, size_t len, uint64_t* m, uint64_t* k, uint64_t* length,
                       std::vector<uint64_t>& words) {
    ARG(buf && len >= 16, "truncated bloom binary");  // BloomFilter.ReadFrom: BE64 m, BE64 k, bitset
    *m = be64(buf);
    *k = be64(buf + 8);
    return parse_bitset(buf + 16, len - 16, length, words);
}

static int b64url_val(char c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '-') return 62;
    if (c == '_') return 63;
    return -1;
}

static bool json_uint(const std::string& s, const char* key, uint64_t* v) {
    const std::string k = std::string("\"") + key + "\"";
    size_t p = s.find(k);
    if (p == std::string::npos) return false;
    p = s.find(':', p + k.size());
    if (p == std::string::npos) return false;
    ++p;
    while (p < s.size() && isspace((unsigned char)s[p])) ++p;
    if (p >= s.size() || !isdigit((unsigned char)s[p])) return false;
    uint64_t x = 0;
    while (p < s.size() && isdigit((unsigned char)s[p])) {
        const uint64_t d = (uint64_t)(s[p++] - '0');
        if (x > (UINT64_MAX - d) / 10) return false;  // not a uint64
        x = x * 10 + d;
    }
    *v = x;
    return true;
}

// BloomFilter.UnmarshalJSON: {"m":M,"k":K,"b":"<base64url(bitset binary)>"}
int bloom_parse_json(const char* json, size_t len, uint64_t* m, uint64_t* k, uint64_t* length,
                     std::vector<uint64_t>& words) {
    ARG(json, "null json");
    const std::string s(json, len);
    ARG(json_uint(s, "m", m) && json_uint(s, "k", k), "bloom json: missing m or k");
    size_t p = s.find("\"b\"");
    ARG(p != std::string::npos, "bloom json: missing b");
    const size_t colon = s.find(':', p + 3);
    ARG(colon != std::string::npos, "bloom json: b has no value");
    p = s.find('"', colon + 1);
    ARG(p != std::string::npos, "bloom json: b is not a string");
    const size_t q = s.find('"', p + 1);
    ARG(q != std::string::npos, "bloom json: unterminated b");
    std::vector<uint8_t> bytes;
    uint32_t acc = 0;
    int nbits = 0;
    for (size_t i = p + 1; i < q; ++i) {
        const char c = s[i];
        if (c == '=') break;
        const int v = b64url_val(c);
        ARG(v >= 0, "bloom json: bad base64url character");
        acc = (acc << 6) | (uint32_t)v;
        nbits += 6;
        if (nbits >= 8) {
            nbits -= 8;
            bytes.push_back((uint8_t)(acc >> nbits));
        }
    }
    return parse_bitset(bytes.data(), bytes.size(), length, words);
}

static int copy_out(const std::string& o, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    ARG(out_len, "null out_len");
    *out_len = o.size();
    if (o.size() > cap) return fail(RF_EINVAL, "output buffer too small: need %zu bytes", o.size());
    if (!o.empty() && out) memcpy(out, o.data(), o.size());
    return RF_OK;
}

static void put_be64(std::string& o, uint64_t v) {
    for (int i = 7; i >= 0; --i) o.push_back((char)(uint8_t)(v >> (8 * i)));
}

static int bitset_bytes(uint64_t length, const uint64_t* words, uint64_t nwords, std::string& o) {
    const uint64_t nw = words_needed(length);
    ARG(nwords >= nw && (nw == 0 || words), "fewer words than the bitset length needs");
    put_be64(o, length);  // bitset.WriteTo (bitset.go:628-640)
    for (uint64_t i = 0; i < nw; ++i) put_be64(o, words[i]);
    return RF_OK;
}

extern "C" int rf_bloom_parse_binary(const uint8_t* buf, size_t len, uint64_t* m, uint64_t* k, uint64_t* length,
                                     uint64_t* words, uint64_t cap_words, uint64_t* n_words) {
    ARG(m && k && length && n_words, "null argument");
    std::vector<uint64_t> w;
    int rc = bloom_parse_binary(buf, len, m, k, length, w);
    if (rc) return rc;
    *n_words = w.size();
    if (w.size() > cap_words) return fail(RF_EINVAL, "word buffer too small: need %zu words", w.size());
    if (!w.empty() && words) memcpy(words, w.data(), 8 * w.size());
    return RF_OK;
}

extern "C" int rf_bloom_parse_json(const char* json, size_t len, uint64_t* m, uint64_t* k, uint64_t* length,
                                   uint64_t* words, uint64_t cap_words, uint64_t* n_words) {
    ARG(m && k && length && n_words, "null argument");
    std::vector<uint64_t> w;
    int rc = bloom_parse_json(json, len, m, k, length, w);
    if (rc) return rc;
    *n_words = w.size();
    if (w.size() > cap_words) return fail(RF_EINVAL, "word buffer too small: need %zu words", w.size());
    if (!w.empty() && words) memcpy(words, w.data(), 8 * w.size());
    return RF_OK;
}

extern "C" int rf_bloom_format_binary(uint64_t m, uint64_t k, uint64_t length, const uint64_t* words,
                                      uint64_t n_words, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    std::string o;
    put_be64(o, m);  // BloomFilter.WriteTo: BE64 m, BE64 k, bitset
    put_be64(o, k);
    int rc = bitset_bytes(length, words, n_words, o);
    return rc ? rc : copy_out(o, out, cap, out_len);
}

extern "C" int rf_bloom_format_json(uint64_t m, uint64_t k, uint64_t length, const uint64_t* words,
                                    uint64_t n_words, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    std::string bits;
    int rc = bitset_bytes(length, words, n_words, bits);
    if (rc) return rc;
    // json.Marshal(bloomFilterJSON{m, k, b}) with b's MarshalJSON =
    // json.Marshal(base64.URLEncoding.EncodeToString(bits)) (padded; the
    // alphabet needs no JSON escaping)
    static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    std::string s = "{\"m\":" + std::to_string(m) + ",\"k\":" + std::to_string(k) + ",\"b\":\"";
    const uint8_t* b = reinterpret_cast<const uint8_t*>(bits.data());
    size_t i = 0;
    for (; i + 3 <= bits.size(); i += 3) {
        const uint32_t v = (uint32_t)b[i] << 16 | (uint32_t)b[i + 1] << 8 | b[i + 2];
        s += A[v >> 18];
        s += A[(v >> 12) & 63];
        s += A[(v >> 6) & 63];
        s += A[v & 63];
    }
    if (bits.size() - i == 1) {
        const uint32_t v = (uint32_t)b[i] << 16;
        s += A[v >> 18];
        s += A[(v >> 12) & 63];
        s += "==";
    } else if (bits.size() - i == 2) {
        const uint32_t v = (uint32_t)b[i] << 16 | (uint32_t)b[i + 1] << 8;
        s += A[v >> 18];
        s += A[(v >> 12) & 63];
        s += A[(v >> 6) & 63];
        s += '=';
    }
    s += "\"}";
    return copy_out(s, out, cap, out_len);
}
