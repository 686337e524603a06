// latLngToCell for CDNA4 (gfx950): one lane per event, fp64 VALU.
//
// Restates upstream H3 v4 latLngToCell (h3Index.c) -> _geoToFaceIjk -> _geoToHex2d (faceijk.c) ->
// _hex2dToCoordIJK (coordijk.c) -> _faceIjkToH3 (faceijk.c), i.e. what the reference's UDF calls per row
// (reference heatmap_stream.py:65-75 -> h3.latlng_to_cell, h3-py 4.x).
//
// Bit-exactness notes:
//  * upstream declares several constants as `long double` (M_PI_180, M_2PI, M_AP7_ROT_RADS, M_SQRT7,
//    M_RSIN60, EPSILON); compiled on x86-64 those expressions run in x87 80-bit (64-bit mantissa, round to
//    nearest even) and are rounded again to double on assignment.  hm::xld_* reproduce that double rounding
//    exactly with 128-bit integer arithmetic (selftest: hm_selftest_ld_ops vs the x87 oracle).
//  * every fp64 expression keeps upstream's operation order and is compiled with -ffp-contract=off
//    (no v_fma_f64 contraction: x86-64 h3 builds have none).
//  * sin/cos of the face-centre latitudes are precomputed on the host with the same libm the reference
//    uses (glibc) and uploaded; the exact path's per-event sincos/acos/atan2/tan are glibc 2.35's own routines
//    restated for the device (glibc_libm.h), so even knife-edge inputs get the glibc-linked reference's bits.
//
// Functions are __host__ __device__ so the same code can be executed on the CPU by the self-test entry
// points (where the transcendental calls resolve to the host libm).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>

#include "glibc_libm.h"

#define HM_HD __host__ __device__ __forceinline__

namespace hm {

typedef unsigned __int128 u128;

// ---- x87 long double constants of upstream constants.h (exact 64-bit mantissa, value = M * 2^E) ----
#define HM_LD_PI_180_M UINT64_C(0x8efa351294e9c8ae)
#define HM_LD_PI_180_E (-69)
#define HM_LD_2PI_M UINT64_C(0xc90fdaa22168c235)
#define HM_LD_2PI_E (-61)
#define HM_LD_AP7_ROT_M UINT64_C(0xaabcfee1d47a0aea)
#define HM_LD_AP7_ROT_E (-65)
#define HM_LD_SQRT7_M UINT64_C(0xa953fd4e97c74dbc)
#define HM_LD_SQRT7_E (-62)
#define HM_LD_RSIN60_M UINT64_C(0x93cd3a2c8198e269)
#define HM_LD_RSIN60_E (-63)
#define HM_LD_EPSILON_M UINT64_C(0xe69594bec44de15b)
#define HM_LD_EPSILON_E (-117)
// exact split of each constant: C = HI + LO, HI = RN53(C), LO exactly representable (<= 11 bits)
#define HM_LD_PI_180_HI 0x1.1df46a2529d39p-6
#define HM_LD_PI_180_LO 0x1.5c00000000000p-62
#define HM_LD_2PI_HI 0x1.921fb54442d18p+2
#define HM_LD_2PI_LO 0x1.1a80000000000p-52
#define HM_LD_AP7_ROT_HI 0x1.5579fdc3a8f41p-2
#define HM_LD_AP7_ROT_LO 0x1.7500000000000p-56
#define HM_LD_SQRT7_HI 0x1.52a7fa9d2f8eap+1
#define HM_LD_SQRT7_LO -0x1.2200000000000p-53
#define HM_LD_RSIN60_HI 0x1.279a74590331cp+0
#define HM_LD_RSIN60_LO 0x1.3480000000000p-54
// double constants (no L suffix upstream)
#define HM_INV_RES0_U_GNOMONIC 2.61803398874989588842

HM_HD int clz128(u128 x) {
    uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
    return hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
}

// Round P * 2^E (P != 0; `sticky` = nonzero bits below P's LSB) first to a 64-bit mantissa (x87 extended,
// round-to-nearest-even), then to double (round-to-nearest-even), as x87 arithmetic + store does.
HM_HD double round_x87_then_double(u128 P, int E, bool sticky, bool neg) {
    int L = 127 - clz128(P);
    uint64_t keep;
    if (L >= 64) {
        int sh = L - 63;
        keep = (uint64_t)(P >> sh);
        u128 rem = P & ((((u128)1) << sh) - 1);
        u128 half = ((u128)1) << (sh - 1);
        bool up = rem > half || (rem == half && (sticky || (keep & 1)));
        E += sh;
        if (up) {
            keep += 1;
            if (keep == 0) { keep = UINT64_C(1) << 63; E += 1; }
        }
    } else {
        keep = (uint64_t)P << (63 - L);
        E -= (63 - L);
    }
    // keep in [2^63, 2^64): value = keep * 2^E; now round to double
    int lead = 63 + E;
    int lsb = lead - 52;
    if (lsb < -1074) lsb = -1074;
    int drop = lsb - E;  // >= 11
    uint64_t m;
    if (drop >= 65) {
        m = 0;
    } else if (drop == 64) {
        m = (keep > (UINT64_C(1) << 63)) ? 1 : 0;  // tie (== 2^63) rounds to even 0
    } else {
        m = keep >> drop;
        uint64_t rem = keep & ((UINT64_C(1) << drop) - 1);
        uint64_t half = UINT64_C(1) << (drop - 1);
        if (rem > half || (rem == half && (m & 1))) m += 1;
    }
    double r = ldexp((double)m, lsb);
    return neg ? -r : r;
}

HM_HD void split_double(double a, uint64_t &m, int &e, bool &neg) {
    uint64_t b = __builtin_bit_cast(uint64_t, a);
    neg = (b >> 63) != 0;
    int ex = (int)((b >> 52) & 0x7ff);
    uint64_t fr = b & ((UINT64_C(1) << 52) - 1);
    if (ex == 0) { m = fr; e = -1074; }
    else { m = fr | (UINT64_C(1) << 52); e = ex - 1075; }
}

// (double)((long double)a * C)
HM_HD double xld_mul(double a, uint64_t cm, int ce) {
    if (a == 0.0 || !__builtin_isfinite(a)) return a * ldexp((double)cm, ce);
    uint64_t ma; int ea; bool neg;
    split_double(a, ma, ea, neg);
    u128 P = (u128)ma * (u128)cm;
    return round_x87_then_double(P, ea + ce, false, neg);
}

// (double)((long double)a + (negc ? -C : C))
HM_HD double xld_add(double a, bool negc, uint64_t cm, int ce) {
    if (!__builtin_isfinite(a)) return a;
    uint64_t ma = 0; int ea = 0; bool na = false;
    if (a != 0.0) split_double(a, ma, ea, na);
    int lc = ce + 63;
    int la = ma ? ea + (63 - __builtin_clzll(ma)) : -100000;
    int top = la > lc ? la : lc;
    int B = top - 125;
    bool sticky = false;
    u128 xa = 0, xc = 0;
    if (ma) {
        int s = ea - B;
        if (s >= 0) xa = ((u128)ma) << s;
        else if (s > -128) { xa = ((u128)ma) >> (-s); sticky = ((((u128)ma) << (128 + s)) != 0); }
        else { xa = 0; sticky = true; }
    }
    {
        int s = ce - B;
        if (s >= 0) xc = ((u128)cm) << s;
        else if (s > -128) { xc = ((u128)cm) >> (-s); sticky = ((((u128)cm) << (128 + s)) != 0); }
        else { xc = 0; sticky = true; }
    }
    u128 R;
    bool neg;
    if (na == negc) {
        R = xa + xc;
        neg = na;
    } else {
        // magnitudes: the operand that lost bits (if any) is the smaller one
        if (xa >= xc) { R = xa - xc; neg = na; if (sticky && la < lc) { /* a was the smaller: impossible */ } }
        else { R = xc - xa; neg = negc; }
        if (sticky) { R -= 1; }   // true value lies strictly between R-1 and R (smaller operand truncated)
    }
    if (R == 0 && !sticky) return 0.0;
    return round_x87_then_double(R, B, sticky, neg);
}

// ---- fast paths: fp64 error-free transformations, exact integer path only near a rounding midpoint ----
// E = exact result.  With p (or s) the fp64 head and t the fp64 tail, E = p + t + d, |d| <= 2^-53 ulp(p).
// Rounding E to 64 bits and then to 53 bits can differ from RN53(E) = RN53(p + t) only when E lies within
// 2^-12 ulp(p) of a 53-bit midpoint; lanes within 2^-10 ulp (and binade edges, zeros, non-finite values)
// take the exact path.
// Fast exact path for the x87 ops: with head + tail == a op C up to ~2^-52 ulp(head) (tail from an FMA
// product or TwoSum), x87 first rounds the exact value to a 64-bit mantissa -- a grid of 2^-11 ulp(head)
// while the result stays in head's binade -- and the store rounds that to double (RNE).  So round the tail
// to the 2^-11 grid (exact unless it sits within ~2^-38 of a grid midpoint, where the 128-bit path takes
// over) and let one double add do the second rounding.  Returns false when the slow path is needed.
HM_HD bool xld_fast_round(double head, double tail, double &out) {
    uint64_t b = __builtin_bit_cast(uint64_t, head);
    int ex = (int)((b >> 52) & 0x7ff);
    uint64_t fr = b & ((UINT64_C(1) << 52) - 1);
    if (ex == 0 || ex >= 0x7fe || fr < 4 || fr > (UINT64_C(1) << 52) - 4) return false;
    double g = ldexp(tail, 1075 + 11 - ex);    // tail in units of 2^-11 ulp(head), exact scaling
    if (!(__builtin_fabs(g) <= 4096.0)) return false;
    double fl = floor(g);
    if (__builtin_fabs((g - fl) - 0.5) < 0x1p-38) return false;
    double gr = (g - fl) < 0.5 ? fl : fl + 1.0;
    out = head + ldexp(gr, ex - 1075 - 11);    // exact 64-bit-mantissa value, rounded to double (RNE)
    return true;
}
HM_HD double xmul(double a, uint64_t cm, int ce, double chi, double clo) {
    double p = a * chi;
    double e = fma(a, chi, -p);
    double t = fma(a, clo, e);
    double r;
    if (xld_fast_round(p, t, r)) return r;
    return xld_mul(a, cm, ce);
}
HM_HD double xadd(double a, bool negc, uint64_t cm, int ce, double chi, double clo) {
    double ch = negc ? -chi : chi, cl = negc ? -clo : clo;
    double s = a + ch;
    double bb = s - a;
    double e = (a - (s - bb)) + (ch - bb);      // TwoSum: a + ch == s + e exactly
    double t = e + cl;
    double r;
    if (xld_fast_round(s, t, r)) return r;
    return xld_add(a, negc, cm, ce);
}
#define XMUL(a, K) xmul((a), HM_LD_##K##_M, HM_LD_##K##_E, HM_LD_##K##_HI, HM_LD_##K##_LO)
#define XADD(a, neg, K) xadd((a), (neg), HM_LD_##K##_M, HM_LD_##K##_E, HM_LD_##K##_HI, HM_LD_##K##_LO)

// a >= C (C > 0, long double), exactly
HM_HD bool xld_ge(double a, uint64_t cm, int ce) {
    if (!(a > 0.0)) return false;
    if (!__builtin_isfinite(a)) return true;
    uint64_t ma; int ea; bool neg;
    split_double(a, ma, ea, neg);
    int la = ea + (63 - __builtin_clzll(ma));
    int lc = ce + 63;
    if (la != lc) return la > lc;
    uint64_t an = ma << (__builtin_clzll(ma));  // normalise to 64-bit with top bit set
    return an >= cm;
}
HM_HD bool xld_lt(double a, uint64_t cm, int ce) { return !xld_ge(a, cm, ce); }

// ---- upstream helpers ----
HM_HD double posAngleRads(double rads) {
    // double tmp = ((rads < 0.0L) ? rads + M_2PI : rads); if (rads >= M_2PI) tmp -= M_2PI;
    double tmp = (rads < 0.0) ? XADD(rads, false, 2PI) : rads;
    if (xld_ge(rads, HM_LD_2PI_M, HM_LD_2PI_E)) tmp = XADD(tmp, true, 2PI);
    return tmp;
}

struct IJK { int i, j, k; };

HM_HD void ijkNormalize(IJK &c) {
    if (c.i < 0) { c.j -= c.i; c.k -= c.i; c.i = 0; }
    if (c.j < 0) { c.i -= c.j; c.k -= c.j; c.j = 0; }
    if (c.k < 0) { c.i -= c.k; c.j -= c.k; c.k = 0; }
    int mn = c.i;
    if (c.j < mn) mn = c.j;
    if (c.k < mn) mn = c.k;
    if (mn > 0) { c.i -= mn; c.j -= mn; c.k -= mn; }
}

// lround(n * M_ONESEVENTH): n/7 is never within 1/14 of a half-integer, so round-half-away-from-zero of
// the exact quotient, in integers.
// Equivalently floor((n + 3) / 7), done as one unsigned division by the constant (|n| < 2^28 here: the
// coordinates of a res-15 point on its face stay below 2^24).
HM_HD int round_div7(int n) { return (int)((unsigned)(n + 3 + 7 * (1 << 27)) / 7u) - (1 << 27); }

// One aperture-7 step up in axial coordinates (x, y) = (i - k, j - k) (_upAp7r / _upAp7 of the normalised IJK: they
// read only these; _downAp7r / _downAp7 are linear and keep the (1,1,1) direction, so the parent and its centre child
// need no normalisation): (x, y) becomes the parent, the result is the child's digit -- the normalised unit IJK of
// (child - centre child), a lookup on (dx, dy) in {-1,0,1}^2, 7 when that is not a unit vector (cf. _unitIjkToDigit).
// Class II: _upAp7r, centre child by _downAp7r (i -> (3,1,0), j -> (0,3,1)); Class III: _upAp7, by _downAp7
// (i -> (3,0,1), j -> (1,3,0)).
template <bool kClass3>
HM_HD unsigned ap7Up(int &x, int &y) {
    int px, py, cx, cy;
    if (kClass3) {
        px = round_div7(3 * x - y);
        py = round_div7(x + 2 * y);
        cx = 2 * px + py;
        cy = 3 * py - px;
    } else {
        px = round_div7(2 * x + y);
        py = round_div7(3 * y - x);
        cx = 3 * px - py;
        cy = px + 2 * py;
    }
    const int dx = x - cx, dy = y - cy;
    unsigned digit = 7;
    if ((unsigned)(dx + 1) <= 2u && (unsigned)(dy + 1) <= 2u) digit = (0x69d0bd9u >> (3 * ((dx + 1) * 3 + (dy + 1)))) & 7u;
    x = px;
    y = py;
    return digit;
}
// Steps in pairs and quads.  A Class II step's centre-child map times the next Class III step's is 7 I in axial
// coordinates ([[3,-1],[1,2]] [[2,1],[-1,3]]), so (x, y) -> (x, y) + 7 e moves that step pair's grandparent by e and
// leaves both digits alone: two steps' digits and the grandparent's offset from floor((x, y) / 7) depend only on
// (x mod 7, y mod 7), and four steps' on (x mod 49, y mod 49).  ap7Pair[7 a + b] / ap7Quad[49 a + b] hold them for
// (x, y) = (a, b): the digits of the steps in order from bit 0 (3 bits each: 6 / 12 bits), then the ancestor's x + 2
// and y + 2 in 3 bits each -- computed by running the single steps (hm_make_tables), so equal to them for every
// input, digit 7 included.
constexpr int AP7_PAIR = 49, AP7_QUAD = 2401;
HM_HD int floor_div7(int n) { return (int)((unsigned)(n + 7 * (1 << 27)) / 7u) - (1 << 27); }
HM_HD int floor_div49(int n) { return (int)((unsigned)(n + 49 * (1 << 24)) / 49u) - (1 << 24); }
inline unsigned ap7TableEntry(int a, int b, int nsteps) {
    int x = a, y = b;
    unsigned e = 0;
    for (int q = 0; q < nsteps; q++) e |= ((q & 1) ? ap7Up<true>(x, y) : ap7Up<false>(x, y)) << (3 * q);
    if (x < -2 || x > 5 || y < -2 || y > 5) abort();   // (cannot happen: |ancestor| <= (a, b) / 7^(steps/2) + 1)
    return e | (unsigned)(x + 2) << (3 * nsteps) | (unsigned)(y + 2) << (3 * nsteps + 3);
}

// _hex2dToCoordIJK (coordijk.c)
HM_HD IJK hex2dToCoordIJK(double vx, double vy) {
    IJK h;
    h.k = 0;
    double a1 = __builtin_fabs(vx);
    double a2 = __builtin_fabs(vy);
    double x2 = XMUL(a2, RSIN60);
    double x1 = a1 + x2 / 2.0;
    int m1 = (int)x1;
    int m2 = (int)x2;
    double r1 = x1 - m1;
    double r2 = x2 - m2;
    if (r1 < 0.5) {
        if (r1 < 1.0 / 3.0) {
            if (r2 < (1.0 + r1) / 2.0) { h.i = m1; h.j = m2; }
            else { h.i = m1; h.j = m2 + 1; }
        } else {
            h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
            h.i = ((1.0 - r1) <= r2 && r2 < (2.0 * r1)) ? m1 + 1 : m1;
        }
    } else {
        if (r1 < 2.0 / 3.0) {
            h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
            h.i = ((2.0 * r1 - 1.0) < r2 && r2 < (1.0 - r1)) ? m1 : m1 + 1;
        } else {
            if (r2 < (r1 / 2.0)) { h.i = m1 + 1; h.j = m2; }
            else { h.i = m1 + 1; h.j = m2 + 1; }
        }
    }
    if (vx < 0.0) {
        // upstream: h->i = h->i - 2.0 * diff (exact small integers)
        if ((h.j % 2) == 0) {
            long long axisi = h.j / 2;
            long long diff = h.i - axisi;
            h.i = (int)(h.i - 2 * diff);
        } else {
            long long axisi = (h.j + 1) / 2;
            long long diff = h.i - axisi;
            h.i = (int)(h.i - (2 * diff + 1));
        }
    }
    if (vy < 0.0) {
        h.i = h.i - (2 * h.j + 1) / 2;
        h.j = -1 * h.j;
    }
    ijkNormalize(h);
    return h;
}

// digit rotation tables (Direction enum: 0 center, 1 K, 2 J, 3 JK, 4 I, 5 IK, 6 IJ)
HM_HD int getDigit(uint64_t h, int r) { return (int)((h >> ((15 - r) * 3)) & 7); }
HM_HD void setDigit(uint64_t &h, int r, int d) {
    int s = (15 - r) * 3;
    h = (h & ~(UINT64_C(7) << s)) | ((uint64_t)d << s);
}

// Digit rotations, bit-parallel over all 15 digits. A digit is a unit IJK vector (i, j, k bits); 60 deg ccw
// maps 1->5->4->6->2->3->1 (0 and 7 fixed): i' = ~j&(i|k) | ijk, j' = ~k&(i|j) | ijk, k' = ~i&(j|k) | ijk,
// and cw assigns the same three terms to the planes shifted by one.  Digits past the resolution are 7, which
// is fixed, so rotating all 15 equals upstream's loop over digits 1..res (_h3Rotate60ccw/_h3Rotate60cw).
constexpr uint64_t HM_DIG_LO = UINT64_C(0x49249249249);          // bit 0 of each digit
constexpr uint64_t HM_DIG_MASK = (UINT64_C(1) << 45) - 1;
HM_HD uint64_t rotate60(uint64_t h, bool cw) {
    const uint64_t k = h & HM_DIG_LO, j = (h >> 1) & HM_DIG_LO, i = (h >> 2) & HM_DIG_LO;
    const uint64_t all = i & j & k;
    const uint64_t a = (~j & (i | k)) | all, b = (~k & (i | j)) | all, c = (~i & (j | k)) | all;
    const uint64_t ni = cw ? b : a, nj = cw ? c : b, nk = cw ? a : c;
    return (h & ~HM_DIG_MASK) | (ni << 2) | (nj << 1) | nk;
}
// first non-zero digit among 1..res, 0 if none (_h3LeadingNonZeroDigit)
HM_HD int leadingNonZeroDigit(uint64_t h, int res) {
    uint64_t nz = (h | (h >> 1) | (h >> 2)) & HM_DIG_LO;
    nz &= ~((UINT64_C(1) << (3 * (15 - res))) - 1);   // digit r's low bit is bit 3 * (15 - r)
    if (!nz) return 0;
    return (int)((h >> (63 - __builtin_clzll(nz))) & 7);
}
// _h3RotatePent60ccw: rotate; when the new leading digit is K (the deleted K-axes subsequence of a pentagon),
// rotate once more (upstream does it as soon as the loop meets the first non-zero digit, which is the same)
HM_HD uint64_t rotatePent60ccw(uint64_t h, int res) {
    h = rotate60(h, false);
    if (leadingNonZeroDigit(h, res) == 1) h = rotate60(h, false);
    return h;
}
// m (0..5) ccw 60-degree rotations of every digit in one step.  In digit bits (i = 4, j = 2, k = 1), two rotations
// (1->4, 2->1, 4->2, ...) move the planes: i' = k, j' = i, k' = j; three (1->6, 5->2, ...) complement every digit
// other than 0 and 7; so m rotations = the planes moved (2m mod 3) times, complemented when m is odd.  Branch-free
// (m varies by lane): replaces up to five data-dependent applications of rotate60.
HM_HD uint64_t rotate60k(uint64_t h, int m) {
    const uint64_t K = h & HM_DIG_LO, J = (h >> 1) & HM_DIG_LO, I = (h >> 2) & HM_DIG_LO;
    const int pr = (2 * m) % 3;
    const uint64_t ni = pr == 0 ? I : pr == 1 ? K : J;
    const uint64_t nj = pr == 0 ? J : pr == 1 ? I : K;
    const uint64_t nk = pr == 0 ? K : pr == 1 ? J : I;
    uint64_t d = (ni << 2) | (nj << 1) | nk;
    const uint64_t nf = (m & 1) ? (I | J | K) & ~(I & J & K) : 0;   // digits 1..6
    d ^= nf | (nf << 1) | (nf << 2);
    return (h & ~HM_DIG_MASK) | d;
}
// position of a leading digit in the cycle a pentagon's rotations visit (5 -> 4 -> 6 -> 2 -> 3 -> 5: the deleted K
// digit is skipped), 3 bits per digit value; 0 for the digits 0, 1 and 7
constexpr uint32_t HM_PENT_CYCLE_POS = (3u << 6) | (4u << 9) | (1u << 12) | (0u << 15) | (2u << 18);

// Tables the kernels read (device: __constant__ copies; host self-test: static copies).
struct H3Tables {
    double faceCenterGeo[20][2];
    double faceCenterPoint[20][3];
    double faceAxesAz0[20];
    double faceCosLat[20];   // cos(faceCenterGeo[f].lat), host libm
    double faceSinLat[20];   // sin(faceCenterGeo[f].lat), host libm
    float faceCenterPointF[20][3];   // (float)faceCenterPoint: the closest-face prefilter
    // fast path (latLngToCellFast): per face the gnomonic axes u = (ux, uy) with hex2d = S_res (p.u) / (p.c),
    // [0] Class II, [1] Class III (rotated by -M_AP7_ROT_RADS); S_res = (1/RES0_U_GNOMONIC) sqrt(7)^res
    double fastU[2][20][2][3];
    double fastScale[16];
    double fastTauS[16];   // the margin bound's S term: 8 x 32 eps S_res (a table constant: a uniform scalar load)
    int faceIjkBaseCells[20][3][3][3][2];
    int baseCellData[122][7];
    // cellToBoundary (h3_boundary.h): faceNeighbors[f][dir] = {face, translate i, j, k, ccwRot60} (dir 0 centre,
    // 1 IJ, 2 KI, 3 JK), adjacentFaceDir[from][to] (0 same face, -1 not adjacent), and the icosahedron-face edge
    // ordinate (double)(3.0L * M_SQRT3_2 * maxDimByCIIres[r]) of each substrate resolution r
    int faceNeighbors[20][4][5];
    signed char adjacentFaceDir[20][20];
    double edgeY[17];
    unsigned ap7Quad[AP7_QUAD];    // _faceIjkToH3's digits four steps at a time (ap7TableEntry)
    unsigned short ap7Pair[AP7_PAIR];
    // _faceIjkToH3's reads of faceIjkBaseCells and baseCellData, packed (one LDS read each in k_ingest):
    // fijkPacked[((face * 3 + i) * 3 + j) * 3 + k] = base cell | numRots << 8;
    // bcdPacked[base cell] = pentagon | (cw offset face 0 + 1) << 8 | (cw offset face 1 + 1) << 16
    unsigned short fijkPacked[20 * 27];
    unsigned bcdPacked[122];
    // glibc's sincos/acos/atan2/tan tables (glibc_libm.h): the device copy for c_tab, the host copy for self-tests
    const glm::Tables *glm;
};

// the tables _faceIjkToH3 reads (k_ingest keeps a copy in LDS)
struct H3BaseTables {
    unsigned ap7Quad[AP7_QUAD];
    unsigned bcdPacked[122];
    unsigned short fijkPacked[20 * 27];
    unsigned short ap7Pair[AP7_PAIR];
};

// _faceIjkToH3 (faceijk.c), res >= 1.  TT: any table holding the packed base-cell tables (H3Tables, or the
// LDS copy k_ingest keeps: lane-indexed reads there do not wait behind the vector loads in flight)
template <typename TT>
HM_HD uint64_t faceIjkToH3(int face, IJK ijk, int res, const TT &T) {
    uint64_t h = UINT64_C(0x00001fffffffffff) | (UINT64_C(1) << 59) | ((uint64_t)res << 52);
    if (res == 0) {
        if (ijk.i > 2 || ijk.j > 2 || ijk.k > 2) return 0;
        return h | ((uint64_t)(T.fijkPacked[((face * 3 + ijk.i) * 3 + ijk.j) * 3 + ijk.k] & 0x7fu) << 45);
    }
    // Digits from the finest resolution up, in axial coordinates (ap7Up): step r (r = res - 1 .. 0) writes the
    // digit of resolution r + 1 and is Class III when r is even.  After a first single step when res - 1 is even,
    // the steps run in Class II / Class III pairs: one pair from ap7Pair when their count is odd, then quads from
    // ap7Quad (res 8: two quad lookups instead of eight steps).
    int x = ijk.i - ijk.k, y = ijk.j - ijk.k;
    uint64_t digits = 0;
    int r = res - 1;
    if (!(r & 1)) {
        digits = (uint64_t)ap7Up<true>(x, y) << ((14 - r) * 3);
        r--;
    }
    if ((r + 1) & 2) {
        const int qx = floor_div7(x), qy = floor_div7(y);
        const unsigned e = T.ap7Pair[(x - 7 * qx) * 7 + (y - 7 * qy)];
        digits |= (uint64_t)(e & 63u) << ((14 - r) * 3);
        x = qx + (int)((e >> 6) & 7u) - 2;
        y = qy + (int)((e >> 9) & 7u) - 2;
        r -= 2;
    }
    for (; r >= 3; r -= 4) {
        const int qx = floor_div49(x), qy = floor_div49(y);
        const unsigned e = T.ap7Quad[(x - 49 * qx) * 49 + (y - 49 * qy)];
        digits |= (uint64_t)(e & 4095u) << ((14 - r) * 3);
        x = qx + (int)((e >> 12) & 7u) - 2;
        y = qy + (int)((e >> 15) & 7u) - 2;
    }
    h = (h & ~(HM_DIG_MASK & ~((UINT64_C(1) << (3 * (15 - res))) - 1))) | digits;
    ijk.i = x;
    ijk.j = y;
    ijk.k = 0;
    ijkNormalize(ijk);
    if (ijk.i > 2 || ijk.j > 2 || ijk.k > 2) return 0;
    const unsigned fe = T.fijkPacked[((face * 3 + ijk.i) * 3 + ijk.j) * 3 + ijk.k];
    const int baseCell = (int)(fe & 0x7fu);
    const int numRots = (int)(fe >> 8);
    h |= (uint64_t)baseCell << 45;
    // the rotations as one count m of 60-degree ccw steps, applied once (rotate60k).  Hexagon: numRots.  Pentagon
    // (upstream: a leading K digit is first rotated out, cw on the base cell's cw-offset faces, then numRots
    // _h3RotatePent60ccw, each of which takes one extra step when it lands on a leading K): from the leading digit's
    // position q in the cycle 5 -> 4 -> 6 -> 2 -> 3, numRots steps pass the deleted K (q + numRots) / 5 times
    // (numRots <= 5, q <= 4).  Equal to rotatePent60ccw applied numRots times (test_device_numerics_host).
    int m = numRots;
    const unsigned bd = T.bcdPacked[baseCell];
    if (bd & 1u) {
        int lead = leadingNonZeroDigit(h, res);
        int m0 = 0;
        if (lead == 1) {
            const bool cw = ((bd >> 8) & 0xffu) == (unsigned)face + 1u || ((bd >> 16) & 0xffu) == (unsigned)face + 1u;
            m0 = cw ? 5 : 1;
            lead = cw ? 3 : 5;
        }
        const int q = (int)((HM_PENT_CYCLE_POS >> (3 * lead)) & 7u);
        m = m0 + numRots + (q + numRots) / 5;
        m = m >= 6 ? m - 6 : m;
    }
    return rotate60k(h, m);
}

// squared distance from face f's centre, upstream's operation order (_geoToClosestFace)
HM_HD double faceSqDist(const H3Tables &T, int f, double vx, double vy, double vz) {
    double dx = T.faceCenterPoint[f][0] - vx;
    double dy = T.faceCenterPoint[f][1] - vy;
    double dz = T.faceCenterPoint[f][2] - vz;
    double s = dx * dx + dy * dy;
    return s + dz * dz;
}
// upstream's loop: first face with the smallest squared distance
// (out of line: the near-tie path is rare, and inlined its 60 constants would occupy registers)
__host__ __device__ __attribute__((noinline)) inline void closestFaceExact(const H3Tables &T, double vx, double vy, double vz, int &face, double &sqd) {
    face = 0;
    sqd = 5.0;
    for (int f = 0; f < 20; ++f) {
        double s = faceSqDist(T, f, vx, vy, vz);
        if (s < sqd) { face = f; sqd = s; }
    }
}

// latLngToCell with h3-py's deg2coord: degrees in; returns 0 where the reference UDF returns None
// (the range guard of heatmap_stream.py:66-69; NaN fails it).
HM_HD uint64_t latLngToCellDeg(double lat_deg, double lng_deg, int res, const H3Tables &T) {
    if (!(lat_deg >= -90.0 && lat_deg <= 90.0 && lng_deg >= -180.0 && lng_deg <= 180.0)) return 0;
    double glat = XMUL(lat_deg, PI_180);
    double glng = XMUL(lng_deg, PI_180);
    // _geoToVec3d
    // glibc's sincos (gcc fuses upstream's sin/cos pairs; glibc_libm.h)
    const glm::Tables &G = *T.glm;
    double clat, slat, clng, slng;
    glm::sincos(glat, slat, clat, G);
    glm::sincos(glng, slng, clng, G);
    double vz = slat;
    double vx = clng * clat;
    double vy = slng * clat;
    // _geoToClosestFace.  Prefilter in fp32: sqd = 2 - 2 (c . v) for unit vectors, and the fp32 dot products
    // are within ~1e-6 of the exact ones, so when the best face leads the runner-up by more than 1e-5 it is
    // upstream's fp64 argmin (no tie possible) and only its fp64 distance is computed; otherwise the full
    // upstream loop runs.
    int face;
    double sqd;
    {
        const float fx = (float)vx, fy = (float)vy, fz = (float)vz;
        float best = -4.0f, second = -4.0f;
        int bf = 0;
        for (int f = 0; f < 20; ++f) {
            const float d = T.faceCenterPointF[f][0] * fx + T.faceCenterPointF[f][1] * fy + T.faceCenterPointF[f][2] * fz;
            if (d > best) { second = best; best = d; bf = f; }
            else if (d > second) second = d;
        }
        if (best - second > 1e-5f) {
            face = bf;
            sqd = faceSqDist(T, bf, vx, vy, vz);
        } else {
            closestFaceExact(T, vx, vy, vz, face, sqd);
        }
    }
    // _geoToHex2d
    double r = glm::acos(1 - sqd / 2, G);
    double hx, hy;
    if (xld_lt(r, HM_LD_EPSILON_M, HM_LD_EPSILON_E)) {
        hx = hy = 0.0;
    } else {
        double dlng = glng - T.faceCenterGeo[face][1];
        double sd, cd;
        glm::sincos(dlng, sd, cd, G);
        double num = clat * sd;
        double t1 = T.faceCosLat[face] * slat;
        double t2 = T.faceSinLat[face] * clat;
        t2 = t2 * cd;
        double az = glm::atan2(num, t1 - t2, G);
        double theta = posAngleRads(T.faceAxesAz0[face] - posAngleRads(az));
        if (res & 1) theta = posAngleRads(XADD(theta, true, AP7_ROT));
        r = glm::tan(r, G);
        r *= HM_INV_RES0_U_GNOMONIC;
        for (int i = 0; i < res; i++) r = XMUL(r, SQRT7);
        double st, ct;
        glm::sincos(theta, st, ct, G);
        hx = r * ct;
        hy = r * st;
    }
    IJK ijk = hex2dToCoordIJK(hx, hy);
    return faceIjkToH3(face, ijk, res, T);
}


// =====================================================================================================
// Fast path with exact fallback.
// latLngToCellDeg above follows upstream's operation sequence bit for bit, which costs ~2.7k VALU
// instructions and ~170 VGPRs per event (five device-library transcendentals, x87 emulation).  The cell is a
// discrete function of the hex2d coordinates, so any evaluation accurate to within tau gives upstream's cell
// whenever every decision upstream takes (closest face, the lattice truncations, the comparisons of
// _hex2dToCoordIJK, the two sign folds) has a margin above tau in our evaluation.  The fast path evaluates
// the gnomonic projection directly as a ratio of dot products -- no acos/atan2/tan/sincos(theta) -- and
// returns false (caller runs latLngToCellDeg, out of line) when a margin is below tau:
//   tan(r) (cos az, sin az) = (p.n, p.e) / (p.c)   (n, e = north/east at the face centre, upstream's azimuth)
//   hex2d = S_res tan(r) (cos(az0 - az), sin(az0 - az)) = S_res (p.ux, p.uy) / (p.c)
//   ux = cos(az0) n + sin(az0) e,  uy = sin(az0) n - cos(az0) e   (Class III: rotated by -M_AP7_ROT_RADS)
// tau bounds |our hex2d - upstream's hex2d| from both sides' rounding: upstream's acos(1 - sqd/2) loses
// ~2^-53/sqd relative near a face centre, the rest is O(res) ulps of |hex2d| plus O(1) ulps of S_res.
// =====================================================================================================
// sin and cos of |x| <= pi + 1e-9 (absolute error < 4e-16): Cody-Waite reduction by pi/2 and fdlibm's
// kernel polynomials; no large-argument path, so a few registers.
HM_HD void sincos_small(double x, double &s, double &c) {
    const double q = rint(x * 0.63661977236758134308);   // 2/pi; |q| <= 2
    double y = fma(-q, 1.57079632673412561417e+00, x);   // pi/2 head (33 bits): q * head exact
    y = fma(-q, 6.07710050650619224932e-11, y);          // pi/2 tail
    const double z = y * y;
    double ps = fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
    ps = fma(z, ps, 2.75573137070700676789e-06);
    ps = fma(z, ps, -1.98412698298579493134e-04);
    ps = fma(z, ps, 8.33333333332248946124e-03);
    ps = fma(z, ps, -1.66666666666666324348e-01);
    const double sy = fma(y * z, ps, y);
    double pc = fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
    pc = fma(z, pc, -2.75573143513906633035e-07);
    pc = fma(z, pc, 2.48015872894767294178e-05);
    pc = fma(z, pc, -1.38888888888741095749e-03);
    pc = fma(z, pc, 4.16666666666666019037e-02);
    const double cy = fma(z * z, pc, fma(-0.5, z, 1.0));
    const int k = (int)q & 3;
    const double a = (k & 1) ? cy : sy, b = (k & 1) ? sy : cy;
    s = (k & 2) ? -a : a;
    c = ((k + 1) & 2) ? -b : b;
}

// (v_min_f64: one instruction instead of a compare and two selects; the margins it takes are never NaN)
HM_HD double dmin(double a, double b) { return __builtin_fmin(a, b); }

#include "face_dodeca.inc"
// Closest face from the dodecahedron's symmetry (tools/gen_face_dodeca.py): R takes H3's face centres onto the
// canonical dodecahedron -- (+-1, +-1, +-1) and the cyclic permutations of (0, +-1/phi, +-phi), over sqrt(3) -- so
// with q = R p and a, b, c = |q.x|, |q.y|, |q.z| the best vertex of each family is the one whose signs match q's
// (a + b + c; b/phi + c phi; a/phi + b phi; a phi + c/phi) and a family's runner-up flips the sign of its smaller term.
// The closest face and its lead over the runner-up follow from these eight values (values in units of sqrt(3) times
// the dot product).  Equal, up to fp32 rounding, to the argmax and lead over the 20 fp32 dot products; the lead test
// (> 1e-5 in dot-product units, else the exact path) absorbs the difference.  ~45 VALU instead of ~160 for the 20
// products, no memory access.
HM_HD bool closestFaceDodeca(float px, float py, float pz, int &face) {
    constexpr float R[3][3] = {{H3T_DODECA_R0}, {H3T_DODECA_R1}, {H3T_DODECA_R2}};
    constexpr float P = 1.6180339887498949f, IP = 0.61803398874989490f;
    const float qx = R[0][0] * px + R[0][1] * py + R[0][2] * pz;
    const float qy = R[1][0] * px + R[1][1] * py + R[1][2] * pz;
    const float qz = R[2][0] * px + R[2][1] * py + R[2][2] * pz;
    const float a = __builtin_fabsf(qx), b = __builtin_fabsf(qy), c = __builtin_fabsf(qz);
    const unsigned nx = qx < 0.0f, ny = qy < 0.0f, nz = qz < 0.0f;
    const float ba = b * IP, cb = c * P, aa = a * IP, bb = b * P, ac = a * P, cc = c * IP;
    const float f0 = (a + b) + c, f1 = ba + cb, f2 = aa + bb, f3 = ac + cc;
    const float m0 = a < b ? a : b;
    const float s0 = f0 - 2.0f * (m0 < c ? m0 : c), s1 = f1 - 2.0f * (ba < cb ? ba : cb);
    const float s2 = f2 - 2.0f * (aa < bb ? aa : bb), s3 = f3 - 2.0f * (ac < cc ? ac : cc);
    // the winner (first family on ties) and the best of the others' firsts and its own runner-up
    float best = f0, second = s0;
    unsigned idx = 4 * nx + 2 * ny + nz;
    auto take = [&](float f, float s, unsigned i) __attribute__((always_inline)) {
        const bool w = f > best;
        second = w ? (best > s ? best : s) : (second > f ? second : f);
        idx = w ? i : idx;
        best = w ? f : best;
    };
    take(f1, s1, 8 + 3 * (2 * ny + nz));
    take(f2, s2, 9 + 3 * (2 * nx + ny));
    take(f3, s3, 10 + 3 * (2 * nx + nz));
    face = (int)((idx < 12 ? H3T_DODECA_FACE_LO >> (5 * idx) : H3T_DODECA_FACE_HI >> (5 * (idx - 12))) & 31u);
    return best - second > 1e-5f * 1.7320508f;
}

// The fast path.  Returns false when the caller must use latLngToCellDeg; otherwise `out` is upstream's cell
// (0 where the reference's UDF returns None).  fc = T.faceCenterPoint, fu = T.fastU[res & 1], or copies of them
// (k_ingest keeps them in LDS: lane-indexed reads there do not queue behind its outstanding global loads).
template <typename TT = H3Tables>
HM_HD bool latLngToCellFastP(double lat_deg, double lng_deg, int res, const H3Tables &T, const double (*fc)[3],
                             const double (*fu)[2][3], uint64_t &out, const TT &bt) {
    out = 0;
    if (!(lat_deg >= -90.0 && lat_deg <= 90.0 && lng_deg >= -180.0 && lng_deg <= 180.0)) return true;
    double sl, cl, sg, cg;
    sincos_small(lat_deg * 0.017453292519943295, sl, cl);
    sincos_small(lng_deg * 0.017453292519943295, sg, cg);
    const double px = cg * cl, py = sg * cl, pz = sl;
    // closest face: fp32 dot products (within ~1e-6 of upstream's fp64 argmin); a lead below 1e-5 -> exact path
    int face = 0;
    if (!closestFaceDodeca((float)px, (float)py, (float)pz, face)) return false;
    const double *c = fc[face];
    const double pc = fma(px, c[0], fma(py, c[1], pz * c[2]));
    const double sqd = 2.0 - 2.0 * pc;
    if (!(sqd > 1e-12)) return false;                     // within ~6 m of a face centre: exact path
    const double(*u)[3] = fu[face];
    const double S = T.fastScale[res];
    const double inv = S / pc;
    const double vx = fma(px, u[0][0], fma(py, u[0][1], pz * u[0][2])) * inv;
    const double vy = fma(px, u[1][0], fma(py, u[1][1], pz * u[1][2])) * inv;
    const double a1 = __builtin_fabs(vx), a2 = __builtin_fabs(vy);
    const double M = a1 + a2;
    const double eps = 0x1p-52;
    // an upper bound of M ((4 / sqd + 2) + res + 128) eps + S 32 eps: 4 / sqd from an fp32 reciprocal (relative
    // error < 3e-7, inflated by 2^-20) instead of an fp64 division, and res bounded by 15 (a loop-invariant
    // (double)res was the register the cell computation's peak spilled to scratch, reloaded with a full wait)
#ifdef __HIP_DEVICE_COMPILE__
    const double rq = (double)__builtin_amdgcn_rcpf((float)sqd) * (1.0 + 0x1p-20);
#else
    const double rq = (double)(1.0f / (float)sqd) * (1.0 + 0x1p-20);
#endif
    // tau = 8 x that bound (the S term from the table: a loop-invariant fp64 value computed here was the register the
    // resolution-specialised kernels spilled to scratch, reloaded with a full wait every round)
    const double tau = (M * (4.0 * rq + 145.0)) * (8.0 * eps) + T.fastTauS[res];
    // _hex2dToCoordIJK with the margin of every comparison it makes
    const double x2 = a2 * 1.15470053837925152902;        // M_RSIN60
    const double x1 = a1 + x2 / 2.0;
    const int m1 = (int)x1, m2 = (int)x2;
    const double r1 = x1 - m1, r2 = x2 - m2;
    double d = dmin(a1, a2);
    d = dmin(d, dmin(r1, 1.0 - r1));
    d = dmin(d, dmin(r2, 1.0 - r2));
    d = dmin(d, __builtin_fabs(r1 - 1.0 / 3.0));
    d = dmin(d, __builtin_fabs(r1 - 0.5));
    d = dmin(d, __builtin_fabs(r1 - 2.0 / 3.0));
    d = dmin(d, __builtin_fabs(r2 - (1.0 + r1) / 2.0));
    d = dmin(d, __builtin_fabs(r2 - (1.0 - r1)));
    d = dmin(d, __builtin_fabs(r2 - 2.0 * r1));
    d = dmin(d, __builtin_fabs(r2 - (2.0 * r1 - 1.0)));
    d = dmin(d, __builtin_fabs(r2 - r1 / 2.0));
    if (!(d > tau) || !(x1 < 1e9)) return false;
    IJK h;
    h.k = 0;
    if (r1 < 0.5) {
        if (r1 < 1.0 / 3.0) {
            h.i = m1;
            h.j = (r2 < (1.0 + r1) / 2.0) ? m2 : m2 + 1;
        } else {
            h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
            h.i = ((1.0 - r1) <= r2 && r2 < (2.0 * r1)) ? m1 + 1 : m1;
        }
    } else {
        if (r1 < 2.0 / 3.0) {
            h.j = (r2 < (1.0 - r1)) ? m2 : m2 + 1;
            h.i = ((2.0 * r1 - 1.0) < r2 && r2 < (1.0 - r1)) ? m1 : m1 + 1;
        } else {
            h.i = m1 + 1;
            h.j = (r2 < (r1 / 2.0)) ? m2 : m2 + 1;
        }
    }
    if (vx < 0.0) {
        if ((h.j % 2) == 0) h.i = h.i - 2 * (h.i - h.j / 2);
        else h.i = h.i - (2 * (h.i - (h.j + 1) / 2) + 1);
    }
    if (vy < 0.0) {
        h.i = h.i - (2 * h.j + 1) / 2;
        h.j = -1 * h.j;
    }
    ijkNormalize(h);
    out = faceIjkToH3(face, h, res, bt);   // (bt: a reference -- as a pointer tested for null, both variants were
                                           // compiled, since an LDS variable's generic address may be 0)
    return true;
}
HM_HD bool latLngToCellFast(double lat_deg, double lng_deg, int res, const H3Tables &T, uint64_t &out) {
    return latLngToCellFastP(lat_deg, lng_deg, res, T, T.faceCenterPoint, T.fastU[res & 1], out, T);
}

}  // namespace hm
