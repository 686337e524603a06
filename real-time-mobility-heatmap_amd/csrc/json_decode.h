// Kafka message values -> event columns: the producer's JSON records (mbta_to_kafka.py:66-74,
// json.dumps of {provider, vehicleId, lat, lon, speedKmh, bearing, accuracyM, ts}) parsed like the reference's
//   from_json(col("value").cast("string"), schema)   (heatmap_stream.py:51-61, 88-91; Spark 3.5 PERMISSIVE mode)
//   to_timestamp(col("ts"))                           (:92; session time zone UTC, :45)
// One device thread per record.  Host-callable too (HM_HD): the CPU tests run this same code against Python's json
// module and pandas.to_datetime (oracle/kafka_oracle.py).
//
// Record rules (from_json, PERMISSIVE, spark.sql.json.enablePartialResults = false in 3.5):
//  * the value must be a JSON object; anything else (invalid JSON, an array, a scalar, empty) -> every field null;
//  * a field of the wrong JSON type for its schema type makes the whole record null (a "malformed record");
//  * absent fields and JSON null -> null; unknown fields are skipped (still validated); a repeated field: last wins;
//  * DoubleType: JSON numbers (correctly rounded, Eisel-Lemire with the 128-bit product, which is always sufficient
//    for <= 19 significant digits -- Mushtak & Lemire, "Fast Number Parsing Without Fallback", 2023), the
//    non-numeric tokens NaN, Infinity, +Infinity, +INF, -Infinity, -INF, and the same words as JSON strings;
//  * IntegerType (bearing, accuracyM): integer tokens in int32 range only;
//  * StringType: JSON strings (escapes decoded; a lone surrogate escape becomes '?', as Java's UTF-8 encoder
//    writes it), integer tokens as their decimal text, true/false as text;
//  * content after the root object is ignored (Jackson parses the first value).
// Outside what the GPU decodes -- numbers of more than 19 significant digits that sit on a rounding boundary,
// floats/objects/arrays as values of string fields -- the record is counted as unsupported and the call fails
// (hm_decode_json), never silently differs.
// to_timestamp: YYYY-MM-DD, optionally followed by ('T' | ' ') HH:MM[:SS[.fraction]] [Z | +-HH[[:]MM]];
// no zone = UTC; the fraction is truncated to microseconds; out-of-range fields -> null.
#pragma once
#include <stdint.h>

#include "pow5_table.inc"

namespace hm {

#if defined(__HIPCC__)
__constant__ const unsigned long long c_pow5[] = {HM_POW5_ENTRIES};
#endif
static const unsigned long long h_pow5[] = {HM_POW5_ENTRIES};
HM_HD const unsigned long long *pow5_table() {
#if defined(__HIP_DEVICE_COMPILE__)
    return c_pow5;
#else
    return h_pow5;
#endif
}

HM_HD void mul64x64(uint64_t a, uint64_t b, uint64_t &hi, uint64_t &lo) {
#if defined(__HIP_DEVICE_COMPILE__)
    hi = __umul64hi(a, b);
    lo = a * b;
#else
    const unsigned __int128 p = (unsigned __int128)a * b;
    hi = (uint64_t)(p >> 64);
    lo = (uint64_t)p;
#endif
}
HM_HD int clz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __clzll((long long)x);
#else
    return __builtin_clzll(x);
#endif
}

// decimal w * 10^q -> binary64 bits (w != 0 handled inside; sign not included).  Eisel-Lemire (Lemire 2021, Alg. 1
// with the round-to-even and subnormal handling of the fast_float library's compute_float).
HM_HD uint64_t decimal_to_double_bits(int64_t q, uint64_t w) {
    if (w == 0 || q < HM_POW5_QMIN) return 0;
    if (q > HM_POW5_QMAX) return UINT64_C(0x7ff0000000000000);
    const int lz = clz64(w);
    w <<= lz;
    const unsigned long long *T = pow5_table();
    const int idx = 2 * (int)(q - HM_POW5_QMIN);
    uint64_t hi, lo;
    mul64x64(w, T[idx], hi, lo);
    const uint64_t mask = UINT64_C(0xFFFFFFFFFFFFFFFF) >> 55;   // mantissa bits + 3
    if ((hi & mask) == mask) {
        uint64_t h2, l2;
        mul64x64(w, T[idx + 1], h2, l2);
        lo += h2;
        if (h2 > lo) hi++;
    }
    const int upperbit = (int)(hi >> 63);
    const int shift = upperbit + 64 - 52 - 3;
    uint64_t mant = hi >> shift;
    int32_t p2 = (int32_t)((((152170 + 65536) * (int32_t)q) >> 16) + 63) + upperbit - lz + 1023;
    if (p2 <= 0) {   // subnormal
        if (-p2 + 1 >= 64) return 0;
        mant >>= -p2 + 1;
        mant += mant & 1;
        mant >>= 1;
        p2 = mant < (UINT64_C(1) << 52) ? 0 : 1;
        return ((uint64_t)p2 << 52) | (mant & ((UINT64_C(1) << 52) - 1));
    }
    if (lo <= 1 && q >= -4 && q <= 23 && (mant & 3) == 1 && (mant << shift) == hi) mant &= ~UINT64_C(1);
    mant += mant & 1;
    mant >>= 1;
    if (mant >= (UINT64_C(2) << 52)) {
        mant = UINT64_C(1) << 52;
        p2++;
    }
    mant &= ~(UINT64_C(1) << 52);
    if (p2 >= 0x7ff) return UINT64_C(0x7ff0000000000000);
    return ((uint64_t)p2 << 52) | mant;
}

// ---- a record's bytes, read through a 16-B window (one 16-B load per 16 bytes on the device) ----
// (windows are aligned on the absolute address, so a window never leaves the 16-B block -- nor the page -- of a
// byte the record owns)
struct ByteReader {
    const uint8_t *base;   // the batch's byte buffer
    int64_t end;           // one past the record's last byte (offset from base)
    uintptr_t wpos = 0;    // address of the current window (16-B aligned; 0 = none)
    uint32_t w[4];
    HM_HD int at(int64_t p) {   // the byte at offset p, -1 past the record's end
        if (p >= end) return -1;
        const uintptr_t addr = (uintptr_t)(base + p), a = addr & ~(uintptr_t)15;
        if (a != wpos) {
#if defined(__HIP_DEVICE_COMPILE__)
            const uint4 v = *(const uint4 *)a;
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
#else
            __builtin_memcpy(w, (const void *)a, 16);
#endif
            wpos = a;
        }
        const int k = (int)(addr - a);
        return (int)((w[k >> 2] >> ((k & 3) * 8)) & 0xffu);
    }
};

HM_HD bool json_ws(int c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
HM_HD int64_t skip_ws(ByteReader &R, int64_t p) {
    while (json_ws(R.at(p))) p++;
    return p;
}
HM_HD bool match_lit(ByteReader &R, int64_t p, const char *s) {
    for (int k = 0; s[k]; k++)
        if (R.at(p + k) != (uint8_t)s[k]) return false;
    return true;
}
HM_HD int hexval(int c) {
    return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
}

enum : int { JS_OK = 0, JS_BAD = 1, JS_UNSUP = 2 };

// a JSON string starting at the opening quote p: validates it (escapes, control characters, UTF-8 as Python's
// strict decoder) and, when out != nullptr, writes its decoded bytes to out + (start - base offset); returns the
// position after the closing quote (-1: invalid).  len = decoded length, esc = it had escapes.
struct StrSpan {
    int64_t start;   // first byte after the opening quote
    int32_t len;     // decoded length
    bool esc;
};
HM_HD int64_t parse_string(ByteReader &R, int64_t p, StrSpan &sp, uint8_t *out) {
    p++;   // opening quote
    sp.start = p;
    sp.esc = false;
    int32_t n = 0;
    auto put = [&](int b) { if (out) out[sp.start + n] = (uint8_t)b; n++; };
    for (;;) {
        int c = R.at(p);
        if (c < 0) return -1;
        if (c == '"') { sp.len = n; return p + 1; }
        if (c < 0x20) return -1;
        if (c == '\\') {
            sp.esc = true;
            const int e = R.at(p + 1);
            p += 2;
            switch (e) {
            case '"': put('"'); break;
            case '\\': put('\\'); break;
            case '/': put('/'); break;
            case 'b': put(8); break;
            case 'f': put(12); break;
            case 'n': put(10); break;
            case 'r': put(13); break;
            case 't': put(9); break;
            case 'u': {
                int u = 0;
                for (int k = 0; k < 4; k++) {
                    const int h = hexval(R.at(p + k));
                    if (h < 0) return -1;
                    u = u * 16 + h;
                }
                p += 4;
                uint32_t cp = (uint32_t)u;
                if (u >= 0xD800 && u <= 0xDBFF && R.at(p) == '\\' && R.at(p + 1) == 'u') {
                    int u2 = 0;
                    bool ok = true;
                    for (int k = 0; k < 4; k++) {
                        const int h = hexval(R.at(p + 2 + k));
                        if (h < 0) { ok = false; break; }
                        u2 = u2 * 16 + h;
                    }
                    if (!ok) return -1;
                    if (u2 >= 0xDC00 && u2 <= 0xDFFF) {
                        cp = 0x10000 + (((uint32_t)u - 0xD800) << 10) + ((uint32_t)u2 - 0xDC00);
                        p += 6;
                    }
                }
                if (cp >= 0xD800 && cp <= 0xDFFF) {
                    put('?');   // a lone surrogate (Java's UTF-8 encoder writes '?')
                } else if (cp < 0x80) {
                    put((int)cp);
                } else if (cp < 0x800) {
                    put(0xC0 | (int)(cp >> 6)); put(0x80 | (int)(cp & 63));
                } else if (cp < 0x10000) {
                    put(0xE0 | (int)(cp >> 12)); put(0x80 | (int)((cp >> 6) & 63)); put(0x80 | (int)(cp & 63));
                } else {
                    put(0xF0 | (int)(cp >> 18)); put(0x80 | (int)((cp >> 12) & 63)); put(0x80 | (int)((cp >> 6) & 63));
                    put(0x80 | (int)(cp & 63));
                }
                break;
            }
            default: return -1;
            }
            continue;
        }
        if (c < 0x80) { put(c); p++; continue; }
        // UTF-8 sequence (Python's strict decoder: no overlongs, no surrogates, <= U+10FFFF)
        int need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c == 0xE0) { need = 2; lo = 0xA0; }
        else if (c >= 0xE1 && c <= 0xEC) need = 2;
        else if (c == 0xED) { need = 2; hi = 0x9F; }
        else if (c >= 0xEE && c <= 0xEF) need = 2;
        else if (c == 0xF0) { need = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) need = 3;
        else if (c == 0xF4) { need = 3; hi = 0x8F; }
        else return -1;
        put(c);
        for (int k = 1; k <= need; k++) {
            const int b = R.at(p + k);
            if (b < (k == 1 ? lo : 0x80) || b > (k == 1 ? hi : 0xBF)) return -1;
            put(b);
        }
        p += need + 1;
    }
}

// a JSON number at p (grammar of RFC 8259); returns the position after it (-1: not a number)
struct NumTok {
    uint64_t bits;      // the binary64 value (sign included; integer tokens: -0 -> +0.0, as (double) of the integer)
    bool is_int;        // no fraction, no exponent
    bool int32_ok;      // an integer token within int32
    int32_t ival;
    int64_t text_start; // the token's text (integer tokens as string-field values)
    int64_t text_end;
    int status;         // JS_OK, or JS_UNSUP: > 19 significant digits on a rounding boundary
};
HM_HD int64_t parse_number(ByteReader &R, int64_t p, NumTok &t) {
    t.text_start = p;
    t.status = JS_OK;
    bool neg = false;
    if (R.at(p) == '-') { neg = true; p++; }
    int c = R.at(p);
    if (c < '0' || c > '9') return -1;
    uint64_t w = 0;
    int nd = 0;
    int64_t exp_adj = 0;
    bool trunc = false;
    int64_t ival = 0;
    bool ibig = false;
    if (c == '0') {
        p++;
        c = R.at(p);
        if (c >= '0' && c <= '9') return -1;   // no leading zeros
    } else {
        while (c >= '0' && c <= '9') {
            const int d = c - '0';
            if (nd < 19) { w = w * 10 + (uint64_t)d; nd++; }
            else { exp_adj++; if (d) trunc = true; }
            if (!ibig) { ival = ival * 10 + d; if (ival > INT64_C(2147483648)) ibig = true; }
            c = R.at(++p);
        }
    }
    t.is_int = true;
    if (c == '.') {
        t.is_int = false;
        c = R.at(++p);
        if (c < '0' || c > '9') return -1;
        while (c >= '0' && c <= '9') {
            const int d = c - '0';
            if (nd == 0 && d == 0) exp_adj--;
            else if (nd < 19) { w = w * 10 + (uint64_t)d; nd++; exp_adj--; }
            else if (d) trunc = true;
            c = R.at(++p);
        }
    }
    if (c == 'e' || c == 'E') {
        t.is_int = false;
        c = R.at(++p);
        bool eneg = false;
        if (c == '+' || c == '-') { eneg = c == '-'; c = R.at(++p); }
        if (c < '0' || c > '9') return -1;
        int64_t e = 0;
        while (c >= '0' && c <= '9') {
            if (e < 100000) e = e * 10 + (c - '0');
            c = R.at(++p);
        }
        exp_adj += eneg ? -e : e;
    }
    t.text_end = p;
    uint64_t bits = decimal_to_double_bits(exp_adj, w);
    if (trunc && w != 0 && decimal_to_double_bits(exp_adj, w + 1) != bits) t.status = JS_UNSUP;
    const bool neg_zero_int = t.is_int && w == 0;
    if (neg && !neg_zero_int) bits |= UINT64_C(1) << 63;
    t.bits = bits;
    t.int32_ok = t.is_int && !ibig && (neg ? ival <= INT64_C(2147483648) : ival <= INT64_C(2147483647));
    t.ival = (int32_t)(neg ? -ival : ival);
    return p;
}

// ---- the record's fields ----
enum : uint32_t {
    JF_LAT = 1, JF_LON = 2, JF_SPEED = 4, JF_TS = 8, JF_PROV = 16, JF_VEH = 32, JF_BEARING = 64, JF_ACC = 128,
    JF_PROV_ESC = 256, JF_VEH_ESC = 512,   // the string's decoded bytes are in the scratch buffer
    JF_MALFORMED = 1u << 16, JF_UNSUPPORTED = 1u << 17
};
enum : int { FLD_NONE = -1, FLD_PROVIDER, FLD_VEHICLE, FLD_LAT, FLD_LON, FLD_SPEED, FLD_BEARING, FLD_ACC, FLD_TS };

struct JsonRow {
    double lat, lon, speed;
    int64_t ts_us;
    int32_t bearing, accuracy;
    int64_t p_off, v_off;   // absolute offsets of the provider / vehicleId bytes (input, or scratch when *_ESC)
    int32_t p_len, v_len;
    uint32_t flags;
};

// the field a key names (decoded key bytes at key[0, n)), FLD_NONE if none
HM_HD int field_of(const uint8_t *key, int n) {
    auto eq = [&](const char *s) {
        int k = 0;
        for (; s[k]; k++)
            if (k >= n || key[k] != (uint8_t)s[k]) return false;
        return k == n;
    };
    if (n == 8 && eq("provider")) return FLD_PROVIDER;
    if (n == 9 && eq("vehicleId")) return FLD_VEHICLE;
    if (n == 3 && eq("lat")) return FLD_LAT;
    if (n == 3 && eq("lon")) return FLD_LON;
    if (n == 8 && eq("speedKmh")) return FLD_SPEED;
    if (n == 7 && eq("bearing")) return FLD_BEARING;
    if (n == 9 && eq("accuracyM")) return FLD_ACC;
    if (n == 2 && eq("ts")) return FLD_TS;
    return FLD_NONE;
}

// skip one JSON value at p (validated); returns the position after it, -1 if invalid
HM_HD int64_t skip_value(ByteReader &R, int64_t p, int depth) {
    const int c = R.at(p);
    if (c == '"') {
        StrSpan s;
        return parse_string(R, p, s, nullptr);
    }
    if (c == '{' || c == '[') {
        if (depth > 64) return -1;
        const int close = c == '{' ? '}' : ']';
        p = skip_ws(R, p + 1);
        if (R.at(p) == close) return p + 1;
        for (;;) {
            if (c == '{') {
                if (R.at(p) != '"') return -1;
                StrSpan s;
                p = parse_string(R, p, s, nullptr);
                if (p < 0) return -1;
                p = skip_ws(R, p);
                if (R.at(p) != ':') return -1;
                p = skip_ws(R, p + 1);
            }
            p = skip_value(R, p, depth + 1);
            if (p < 0) return -1;
            p = skip_ws(R, p);
            const int d = R.at(p);
            if (d == close) return p + 1;
            if (d != ',') return -1;
            p = skip_ws(R, p + 1);
        }
    }
    if (c == 't') return match_lit(R, p, "true") ? p + 4 : -1;
    if (c == 'f') return match_lit(R, p, "false") ? p + 5 : -1;
    if (c == 'n') return match_lit(R, p, "null") ? p + 4 : -1;
    if (c == 'N') return match_lit(R, p, "NaN") ? p + 3 : -1;
    if (c == 'I') return match_lit(R, p, "Infinity") ? p + 8 : -1;
    if (c == '+') return match_lit(R, p, "+Infinity") ? p + 9 : match_lit(R, p, "+INF") ? p + 4 : -1;
    if (c == '-' && R.at(p + 1) == 'I') return match_lit(R, p, "-Infinity") ? p + 9 : match_lit(R, p, "-INF") ? p + 4 : -1;
    NumTok t;
    return parse_number(R, p, t);
}

// non-numeric double tokens / strings: NaN, Infinity, +Infinity, +INF, -Infinity, -INF; 0 if none, else its length
HM_HD int special_double(ByteReader &R, int64_t p, uint64_t &bits) {
    if (match_lit(R, p, "NaN")) { bits = UINT64_C(0x7ff8000000000000); return 3; }
    if (match_lit(R, p, "Infinity")) { bits = UINT64_C(0x7ff0000000000000); return 8; }
    if (match_lit(R, p, "+Infinity")) { bits = UINT64_C(0x7ff0000000000000); return 9; }
    if (match_lit(R, p, "+INF")) { bits = UINT64_C(0x7ff0000000000000); return 4; }
    if (match_lit(R, p, "-Infinity")) { bits = UINT64_C(0xfff0000000000000); return 9; }
    if (match_lit(R, p, "-INF")) { bits = UINT64_C(0xfff0000000000000); return 4; }
    return 0;
}

HM_HD int64_t days_from_civil_d(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

// to_timestamp of a string's bytes s[0, n) (grammar above); false -> null
HM_HD bool parse_ts(const uint8_t *s, int n, int64_t &us) {
    int a = 0, b = n;
    while (a < b && s[a] <= ' ') a++;
    while (b > a && s[b - 1] <= ' ') b--;
    int p = a;
    auto dig = [&](int k, int &v) {
        v = 0;
        for (int q = 0; q < k; q++) {
            if (p >= b || s[p] < '0' || s[p] > '9') return false;
            v = v * 10 + (s[p++] - '0');
        }
        return true;
    };
    int Y, M, D, h = 0, mi = 0, sec = 0;
    int64_t frac = 0;
    if (!dig(4, Y) || p >= b || s[p++] != '-' || !dig(2, M) || p >= b || s[p++] != '-' || !dig(2, D)) return false;
    bool has_time = false;
    if (p < b && (s[p] == 'T' || s[p] == ' ')) {
        has_time = true;
        p++;
        if (!dig(2, h) || p >= b || s[p++] != ':' || !dig(2, mi)) return false;
        if (p < b && s[p] == ':') {
            p++;
            if (!dig(2, sec)) return false;
            if (p < b && s[p] == '.') {
                p++;
                int nf = 0;
                while (p < b && s[p] >= '0' && s[p] <= '9') {
                    if (nf < 6) frac = frac * 10 + (s[p] - '0');
                    nf++;
                    p++;
                }
                if (nf == 0 || nf > 9) return false;
                for (; nf < 6; nf++) frac *= 10;
            }
        }
    }
    int off = 0;
    if (p < b && has_time) {   // (a zone only after a time: "YYYY-MM-DDZ" is null in Spark and pandas alike)
        if (s[p] == 'Z') {
            p++;
        } else if (s[p] == '+' || s[p] == '-') {
            const int sg = s[p++] == '-' ? -1 : 1;
            int oh, om = 0;
            if (!dig(2, oh)) return false;
            if (p < b) {
                if (s[p] == ':') p++;
                if (!dig(2, om)) return false;
            }
            if (oh > 18 || om > 59) return false;
            off = sg * (oh * 3600 + om * 60);
        } else {
            return false;
        }
    }
    if (p != b) return false;
    if (M < 1 || M > 12 || D < 1 || h > 23 || mi > 59 || sec > 59) return false;
    const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
    const int dim[12] = {31, leap ? 29 : 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    if (D > dim[M - 1]) return false;
    const int64_t secs = days_from_civil_d(Y, M, D) * 86400 + h * 3600 + mi * 60 + sec - off;
    us = secs * 1000000 + frac;
    return true;
}

// one record bytes[start, end) -> row; scratch (may be nullptr: decoded strings not written) receives escaped
// strings' decoded bytes at their own offsets
HM_HD void parse_record(const uint8_t *bytes, int64_t start, int64_t end, uint8_t *scratch, JsonRow &r) {
    r.lat = r.lon = r.speed = __builtin_nan("");
    r.ts_us = 0;
    r.bearing = r.accuracy = 0;
    r.p_off = r.v_off = 0;
    r.p_len = r.v_len = 0;
    r.flags = 0;
    ByteReader R{bytes, end};
    uint32_t f = 0;
    int64_t p = skip_ws(R, start);
    bool bad = false, unsup = false;
    StrSpan ts_span{0, 0, false};
    if (R.at(p) != '{') {
        bad = true;
    } else {
        p = skip_ws(R, p + 1);
        if (R.at(p) == '}') {
            p++;
        } else {
            for (;;) {
                if (R.at(p) != '"') { bad = true; break; }
                StrSpan ks;
                // the key: decoded into a small local buffer when escaped (keys longer than 16 bytes match nothing)
                const int64_t kq = parse_string(R, p, ks, nullptr);
                if (kq < 0) { bad = true; break; }
                int fld = FLD_NONE;
                if (!ks.esc) {
                    uint8_t kb[16];
                    const int kn = ks.len <= 16 ? ks.len : 0;
                    for (int k = 0; k < kn; k++) kb[k] = (uint8_t)R.at(ks.start + k);
                    if (kn) fld = field_of(kb, kn);
                } else if (ks.len <= 16) {
                    uint8_t kb[16];   // the key decoded again into kb
                    int kn = 0;
                    int64_t q = ks.start;
                    while (kn < 16) {
                        const int c = R.at(q);
                        if (c == '"') break;
                        if (c == '\\') {
                            const int e = R.at(q + 1);
                            if (e == 'u') {
                                int u = 0;
                                for (int k = 0; k < 4; k++) u = u * 16 + hexval(R.at(q + 2 + k));
                                if (u >= 0x80) { kn = 0; break; }   // field names are ASCII
                                kb[kn++] = (uint8_t)u;
                                q += 6;
                            } else {
                                kb[kn++] = (uint8_t)(e == 'n' ? 10 : e == 't' ? 9 : e == 'r' ? 13 : e == 'b' ? 8 : e == 'f' ? 12 : e);
                                q += 2;
                            }
                        } else {
                            kb[kn++] = (uint8_t)c;
                            q++;
                        }
                    }
                    if (kn == ks.len) fld = field_of(kb, kn);
                }
                p = skip_ws(R, kq);
                if (R.at(p) != ':') { bad = true; break; }
                p = skip_ws(R, p + 1);
                const int c = R.at(p);
                if (c == 'n' && match_lit(R, p, "null")) {   // null: the field is null (a later repeat may set it)
                    p += 4;
                    if (fld == FLD_PROVIDER) f &= ~(uint32_t)(JF_PROV | JF_PROV_ESC);
                    else if (fld == FLD_VEHICLE) f &= ~(uint32_t)(JF_VEH | JF_VEH_ESC);
                    else if (fld == FLD_LAT) f &= ~(uint32_t)JF_LAT;
                    else if (fld == FLD_LON) f &= ~(uint32_t)JF_LON;
                    else if (fld == FLD_SPEED) f &= ~(uint32_t)JF_SPEED;
                    else if (fld == FLD_BEARING) f &= ~(uint32_t)JF_BEARING;
                    else if (fld == FLD_ACC) f &= ~(uint32_t)JF_ACC;
                    else if (fld == FLD_TS) f &= ~(uint32_t)JF_TS;
                } else if (fld == FLD_LAT || fld == FLD_LON || fld == FLD_SPEED) {
                    uint64_t bits = 0;
                    int sl;
                    if (c == '"') {   // a string: only the non-numeric words
                        StrSpan s;
                        const int64_t q = parse_string(R, p, s, nullptr);
                        if (q < 0) { bad = true; break; }
                        sl = s.esc ? 0 : special_double(R, s.start, bits);
                        if (sl == 0 || sl != s.len) { bad = true; break; }
                        p = q;
                    } else if ((sl = special_double(R, p, bits)) != 0) {
                        p += sl;
                    } else {
                        NumTok t;
                        const int64_t q = parse_number(R, p, t);
                        if (q < 0) { bad = true; break; }
                        if (t.status == JS_UNSUP) unsup = true;
                        bits = t.bits;
                        p = q;
                    }
                    const double v = __builtin_bit_cast(double, bits);
                    if (fld == FLD_LAT) { r.lat = v; f |= JF_LAT; }
                    else if (fld == FLD_LON) { r.lon = v; f |= JF_LON; }
                    else { r.speed = v; f |= JF_SPEED; }
                } else if (fld == FLD_BEARING || fld == FLD_ACC) {
                    NumTok t;
                    const int64_t q = (c == '-' || (c >= '0' && c <= '9')) ? parse_number(R, p, t) : -1;
                    if (q < 0 || !t.int32_ok) { bad = true; break; }
                    if (fld == FLD_BEARING) { r.bearing = t.ival; f |= JF_BEARING; }
                    else { r.accuracy = t.ival; f |= JF_ACC; }
                    p = q;
                } else if (fld == FLD_PROVIDER || fld == FLD_VEHICLE || fld == FLD_TS) {
                    int64_t off = 0;
                    int32_t len = 0;
                    bool esc = false;
                    if (c == '"') {
                        StrSpan s;
                        const int64_t q = parse_string(R, p, s, fld == FLD_TS ? nullptr : scratch);
                        if (q < 0) { bad = true; break; }
                        off = s.start;
                        len = s.len;
                        esc = s.esc;
                        if (fld == FLD_TS) ts_span = s;
                        p = q;
                    } else if (c == 't' && match_lit(R, p, "true")) {
                        off = p; len = 4; p += 4;
                    } else if (c == 'f' && match_lit(R, p, "false")) {
                        off = p; len = 5; p += 5;
                    } else if (c == '-' || (c >= '0' && c <= '9')) {
                        NumTok t;
                        const int64_t q = parse_number(R, p, t);
                        if (q < 0) { bad = true; break; }
                        if (!t.is_int) unsup = true;   // a float as a string field: Jackson's re-serialisation
                        off = t.text_start;
                        len = (int32_t)(t.text_end - t.text_start);
                        if (len == 2 && R.at(off) == '-' && R.at(off + 1) == '0') { off++; len = 1; }   // "-0" -> "0"
                        p = q;
                    } else {
                        const int64_t q = skip_value(R, p, 0);   // an object or array as a string field
                        if (q < 0) { bad = true; break; }
                        unsup = true;
                        p = q;
                    }
                    if (fld == FLD_PROVIDER) {
                        r.p_off = off; r.p_len = len;
                        f = (f & ~(uint32_t)JF_PROV_ESC) | JF_PROV | (esc ? JF_PROV_ESC : 0u);
                    } else if (fld == FLD_VEHICLE) {
                        r.v_off = off; r.v_len = len;
                        f = (f & ~(uint32_t)JF_VEH_ESC) | JF_VEH | (esc ? JF_VEH_ESC : 0u);
                    } else {
                        f |= JF_TS;
                        if (c != '"') ts_span = StrSpan{off, len, false};
                    }
                } else {
                    const int64_t q = skip_value(R, p, 0);
                    if (q < 0) { bad = true; break; }
                    p = q;
                }
                p = skip_ws(R, p);
                const int d = R.at(p);
                if (d == '}') { p++; break; }
                if (d != ',') { bad = true; break; }
                p = skip_ws(R, p + 1);
            }
        }
    }
    if (bad) {
        r.flags = JF_MALFORMED;
        r.lat = r.lon = r.speed = __builtin_nan("");
        return;
    }
    if (f & JF_TS) {   // to_timestamp: the decoded ts string (<= 64 bytes; longer strings are never valid)
        uint8_t tb[64];
        int n = 0;
        bool ok = ts_span.len <= 64;
        if (ok) {
            if (!ts_span.esc) {
                for (int k = 0; k < ts_span.len; k++) tb[n++] = (uint8_t)R.at(ts_span.start + k);
            } else {
                // re-decode the escaped string into tb (escapes in a timestamp: rare)
                ByteReader R2{bytes, end};
                int64_t q = ts_span.start;
                while (n < 64) {
                    const int c = R2.at(q);
                    if (c == '"' || c < 0) break;
                    if (c == '\\') {
                        const int e = R2.at(q + 1);
                        if (e == 'u') {
                            int u = 0;
                            for (int k = 0; k < 4; k++) u = u * 16 + hexval(R2.at(q + 2 + k));
                            if (u >= 0x80) { ok = false; break; }   // non-ASCII: not a timestamp
                            tb[n++] = (uint8_t)u;
                            q += 6;
                        } else {
                            tb[n++] = (uint8_t)(e == 'n' ? 10 : e == 't' ? 9 : e == 'r' ? 13 : e == 'b' ? 8 : e == 'f' ? 12 : e);
                            q += 2;
                        }
                    } else {
                        tb[n++] = (uint8_t)c;
                        q++;
                    }
                }
            }
        }
        if (!ok || !parse_ts(tb, n, r.ts_us)) f &= ~(uint32_t)JF_TS;
    }
    if (unsup) f |= JF_UNSUPPORTED;
    r.flags = f;
}

}  // namespace hm
