// message.cpp -- the miner process's wire format and request handler.
//
// Reference: bitcoin/message.go:18-23 (Message{Type, Data, Lower, Upper,
// Hash, Nonce}), :7-13 (Join=0, Request=1, Result=2), :27-49 (NewRequest /
// NewResult / NewJoin) and the miner loop spec of bitcoin/miner/miner.go:33
// (Read Request -> scan [Lower, Upper] -> Write Result).  The payload is the
// Go encoding/json form of Message (the CMU convention; lsp/util.go:19-26
// marshals LSP frames the same way), so the codec here reproduces
// json.Marshal byte for byte for this struct and json.Unmarshal's decoding
// rules (case-insensitive keys, unknown keys ignored, invalid UTF-8 -> U+FFFD).
#include <string.h>

#include <string>

#include "../../include/minehip.h"
#include "msgcodec.hpp"

namespace {

const char kHex[] = "0123456789abcdef";

// Decode one UTF-8 sequence at s[i]; returns length (1 with cp = U+FFFD on error),
// following Go's utf8.DecodeRuneInString.
size_t utf8_decode(const uint8_t* s, size_t n, size_t i, uint32_t* cp) {
    const uint8_t c0 = s[i];
    if (c0 < 0x80) {
        *cp = c0;
        return 1;
    }
    auto cont = [&](size_t k) { return i + k < n && (s[i + k] & 0xC0) == 0x80; };
    if (c0 >= 0xC2 && c0 <= 0xDF && cont(1)) {
        *cp = ((uint32_t)(c0 & 0x1F) << 6) | (s[i + 1] & 0x3F);
        return 2;
    }
    if (c0 >= 0xE0 && c0 <= 0xEF && cont(1) && cont(2)) {
        const uint32_t v = ((uint32_t)(c0 & 0x0F) << 12) | ((uint32_t)(s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
        if (v >= 0x800 && !(v >= 0xD800 && v <= 0xDFFF)) {
            *cp = v;
            return 3;
        }
    }
    if (c0 >= 0xF0 && c0 <= 0xF4 && cont(1) && cont(2) && cont(3)) {
        const uint32_t v = ((uint32_t)(c0 & 0x07) << 18) | ((uint32_t)(s[i + 1] & 0x3F) << 12) |
                           ((uint32_t)(s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
        if (v >= 0x10000 && v <= 0x10FFFF) {
            *cp = v;
            return 4;
        }
    }
    *cp = 0xFFFD;
    return 1;
}

void utf8_encode(uint32_t cp, std::string* out) {
    if (cp < 0x80) {
        out->push_back((char)cp);
    } else if (cp < 0x800) {
        out->push_back((char)(0xC0 | (cp >> 6)));
        out->push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
        out->push_back((char)(0xE0 | (cp >> 12)));
        out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out->push_back((char)(0x80 | (cp & 0x3F)));
    } else {
        out->push_back((char)(0xF0 | (cp >> 18)));
        out->push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
        out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out->push_back((char)(0x80 | (cp & 0x3F)));
    }
}

// Go encoding/json string encoding with escapeHTML = true (json.Marshal).
void json_string(const uint8_t* s, size_t n, std::string* out) {
    out->push_back('"');
    size_t i = 0;
    while (i < n) {
        const uint8_t b = s[i];
        if (b < 0x80) {
            const bool safe = b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&';
            if (safe) {
                out->push_back((char)b);
            } else if (b == '"' || b == '\\') {
                out->push_back('\\');
                out->push_back((char)b);
            } else if (b == '\n') {
                out->append("\\n");
            } else if (b == '\r') {
                out->append("\\r");
            } else if (b == '\t') {
                out->append("\\t");
            } else {
                out->append("\\u00");
                out->push_back(kHex[b >> 4]);
                out->push_back(kHex[b & 0xF]);
            }
            ++i;
            continue;
        }
        uint32_t cp;
        const size_t k = utf8_decode(s, n, i, &cp);
        if (cp == 0xFFFD && k == 1) {
            out->append("\\ufffd");
        } else if (cp == 0x2028 || cp == 0x2029) {
            out->append("\\u202");
            out->push_back(kHex[cp & 0xF]);
        } else {
            out->append((const char*)s + i, k);
        }
        i += k;
    }
    out->push_back('"');
}

struct Parser {
    const char* s;
    size_t n, i = 0;
    void ws() {
        while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool lit(const char* w) {
        const size_t k = strlen(w);
        if (i + k > n || memcmp(s + i, w, k) != 0) return false;
        i += k;
        return true;
    }
    bool hex4(uint32_t* v) {
        if (i + 4 > n) return false;
        uint32_t r = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = s[i + k];
            r <<= 4;
            if (c >= '0' && c <= '9') r |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') r |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') r |= (uint32_t)(c - 'A' + 10);
            else return false;
        }
        i += 4;
        *v = r;
        return true;
    }
    // JSON string -> UTF-8 bytes; invalid UTF-8 / lone surrogates -> U+FFFD.
    bool str(std::string* out) {
        if (i >= n || s[i] != '"') return false;
        ++i;
        while (i < n) {
            const uint8_t c = (uint8_t)s[i];
            if (c == '"') {
                ++i;
                return true;
            }
            if (c < 0x20) return false;
            if (c == '\\') {
                if (++i >= n) return false;
                const char e = s[i++];
                switch (e) {
                    case '"': out->push_back('"'); break;
                    case '\\': out->push_back('\\'); break;
                    case '/': out->push_back('/'); break;
                    case 'b': out->push_back('\b'); break;
                    case 'f': out->push_back('\f'); break;
                    case 'n': out->push_back('\n'); break;
                    case 'r': out->push_back('\r'); break;
                    case 't': out->push_back('\t'); break;
                    case 'u': {
                        uint32_t v;
                        if (!hex4(&v)) return false;
                        if (v >= 0xD800 && v < 0xDC00) {
                            uint32_t lo;
                            const size_t save = i;
                            if (i + 1 < n && s[i] == '\\' && s[i + 1] == 'u') {
                                i += 2;
                                if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) {
                                    utf8_encode(0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00), out);
                                    break;
                                }
                            }
                            i = save;
                            v = 0xFFFD;
                        } else if (v >= 0xDC00 && v < 0xE000) {
                            v = 0xFFFD;
                        }
                        utf8_encode(v, out);
                        break;
                    }
                    default: return false;
                }
                continue;
            }
            uint32_t cp;
            const size_t k = utf8_decode((const uint8_t*)s, n, i, &cp);
            if (cp == 0xFFFD && k == 1) utf8_encode(0xFFFD, out);
            else out->append(s + i, k);
            i += k;
        }
        return false;
    }
    bool u64(uint64_t* v) {
        if (i >= n || s[i] < '0' || s[i] > '9') return false;
        if (s[i] == '0' && i + 1 < n && s[i + 1] >= '0' && s[i + 1] <= '9') return false;
        uint64_t r = 0;
        while (i < n && s[i] >= '0' && s[i] <= '9') {
            const uint64_t dgt = (uint64_t)(s[i] - '0');
            if (r > (~0ull - dgt) / 10u) return false;  // overflows uint64
            r = r * 10u + dgt;
            ++i;
        }
        if (i < n && (s[i] == '.' || s[i] == 'e' || s[i] == 'E')) return false;  // not an integer
        *v = r;
        return true;
    }
    bool skip_value(int depth = 0) {
        ws();
        if (i >= n || depth > 64) return false;
        const char c = s[i];
        if (c == '"') {
            std::string tmp;
            return str(&tmp);
        }
        if (c == '{' || c == '[') {
            const char close = (c == '{') ? '}' : ']';
            ++i;
            ws();
            if (i < n && s[i] == close) {
                ++i;
                return true;
            }
            for (;;) {
                if (c == '{') {
                    ws();
                    std::string k;
                    if (!str(&k)) return false;
                    ws();
                    if (i >= n || s[i] != ':') return false;
                    ++i;
                }
                if (!skip_value(depth + 1)) return false;
                ws();
                if (i < n && s[i] == ',') {
                    ++i;
                    continue;
                }
                if (i < n && s[i] == close) {
                    ++i;
                    return true;
                }
                return false;
            }
        }
        if (lit("true") || lit("false") || lit("null")) return true;
        if (c == '-' || (c >= '0' && c <= '9')) {
            ++i;
            while (i < n && (isdigitc(s[i]) || s[i] == '.' || s[i] == 'e' || s[i] == 'E' || s[i] == '+' || s[i] == '-'))
                ++i;
            return true;
        }
        return false;
    }
    static bool isdigitc(char c) { return c >= '0' && c <= '9'; }
};

bool key_is(const std::string& k, const char* name) {  // Go: case-insensitive field match
    const size_t m = strlen(name);
    if (k.size() != m) return false;
    for (size_t j = 0; j < m; ++j) {
        char a = k[j], b = name[j];
        if (a >= 'A' && a <= 'Z') a = (char)(a - 'A' + 'a');
        if (b >= 'A' && b <= 'Z') b = (char)(b - 'A' + 'a');
        if (a != b) return false;
    }
    return true;
}

}  // namespace

namespace mh {

bool decode(const char* js, size_t len, Msg* m) {
    Parser p{js, len};
    p.ws();
    if (p.i >= p.n || js[p.i] != '{') return false;
    ++p.i;
    p.ws();
    if (p.i < p.n && js[p.i] == '}') {
        ++p.i;
    } else {
        for (;;) {
            p.ws();
            std::string k;
            if (!p.str(&k)) return false;
            p.ws();
            if (p.i >= p.n || js[p.i] != ':') return false;
            ++p.i;
            p.ws();
            bool ok;
            if (p.lit("null")) {
                ok = true;  // Go leaves the field unchanged
            } else if (key_is(k, "Type")) {
                const bool neg = p.i < p.n && js[p.i] == '-';
                if (neg) ++p.i;
                uint64_t v;
                ok = p.u64(&v) && v <= (neg ? (1ull << 63) : ((1ull << 63) - 1u));
                if (ok) m->type = neg ? (int64_t)(0 - v) : (int64_t)v;
            } else if (key_is(k, "Data")) {
                m->data.clear();
                ok = p.str(&m->data);
            } else if (key_is(k, "Lower")) {
                ok = p.u64(&m->lower);
            } else if (key_is(k, "Upper")) {
                ok = p.u64(&m->upper);
            } else if (key_is(k, "Hash")) {
                ok = p.u64(&m->hash);
            } else if (key_is(k, "Nonce")) {
                ok = p.u64(&m->nonce);
            } else {
                ok = p.skip_value();
            }
            if (!ok) return false;
            p.ws();
            if (p.i < p.n && js[p.i] == ',') {
                ++p.i;
                continue;
            }
            if (p.i < p.n && js[p.i] == '}') {
                ++p.i;
                break;
            }
            return false;
        }
    }
    p.ws();
    return p.i == p.n;
}

std::string encode(int64_t type, const uint8_t* data, size_t dlen, uint64_t lower, uint64_t upper, uint64_t hash,
                   uint64_t nonce) {
    std::string o = "{\"Type\":" + std::to_string(type) + ",\"Data\":";
    json_string(data, dlen, &o);
    o += ",\"Lower\":" + std::to_string(lower) + ",\"Upper\":" + std::to_string(upper) +
         ",\"Hash\":" + std::to_string(hash) + ",\"Nonce\":" + std::to_string(nonce) + "}";
    return o;
}

}  // namespace mh

namespace {

using mh::decode;
using mh::encode;
using mh::Msg;

int copy_out(const std::string& s, char* out, size_t cap, size_t* out_len) {
    if (out_len) *out_len = s.size();
    if (!out || cap < s.size()) return mh::set_error(MH_EINVAL, "output buffer too small");
    memcpy(out, s.data(), s.size());
    return MH_OK;
}

}  // namespace

extern "C" {

int mh_msg_encode(int64_t type, const uint8_t* data, size_t dlen, uint64_t lower, uint64_t upper, uint64_t hash,
                  uint64_t nonce, char* out, size_t cap, size_t* out_len) {
    if (!data && dlen) return mh::set_error(MH_EINVAL, "data is NULL");
    return copy_out(encode(type, data, dlen, lower, upper, hash, nonce), out, cap, out_len);
}

int mh_msg_decode(const char* json, size_t len, mh_message* out, uint8_t* data, size_t data_cap) {
    if (!json || !out) return mh::set_error(MH_EINVAL, "NULL argument");
    Msg m;
    if (!decode(json, len, &m)) return mh::set_error(MH_EINVAL, "payload is not a JSON bitcoin.Message");
    out->type = m.type;
    out->lower = m.lower;
    out->upper = m.upper;
    out->hash = m.hash;
    out->nonce = m.nonce;
    out->data_len = m.data.size();
    if (m.data.size() > data_cap || (!data && !m.data.empty()))
        return mh::set_error(MH_ETOOLONG, "data buffer too small");
    if (!m.data.empty()) memcpy(data, m.data.data(), m.data.size());
    return MH_OK;
}

int mh_miner_handle(const int* devs, int ndev, const char* request, size_t len, char* out, size_t cap,
                    size_t* out_len) {
    if (!request || !devs || ndev <= 0) return mh::set_error(MH_EINVAL, "bad arguments");
    Msg m;
    if (!decode(request, len, &m)) return mh::set_error(MH_ENOTREQ, "payload is not a JSON bitcoin.Message");
    if (m.type != 1) return mh::set_error(MH_ENOTREQ, "not a Request");  // message.go:10
    if (m.lower > m.upper) return mh::set_error(MH_ERANGE, "lower > upper");
    uint64_t h = 0, n = 0;
    const int rc = (ndev == 1)
                       ? mh_search(devs[0], (const uint8_t*)m.data.data(), m.data.size(), m.lower, m.upper, &h, &n)
                       : mh_search_multi(devs, ndev, (const uint8_t*)m.data.data(), m.data.size(), m.lower, m.upper,
                                         0, &h, &n);
    if (rc) return rc;
    return copy_out(encode(2, nullptr, 0, 0, 0, h, n), out, cap, out_len);  // NewResult (message.go:38-44)
}

}  // extern "C"
