// The glibc double routines upstream H3's latLngToCell and cellToBoundary call, restated for host and device (CDNA4
// fp64 VALU).
//
// Why: the reference's cell ids come from h3 linked against the host's glibc (reference heatmap_stream.py:65-75 ->
// h3.latlng_to_cell -> H3 C latLngToCell: sincos (gcc fuses upstream's sin/cos pairs), acos, atan2, tan), and so do
// its cell boundaries (reference app.py:19-41 -> h3.cell_to_boundary: sincos, asin, atan2, atan).  On a knife-edge
// input the last bit of one of those results decides the cell, so the exact path (h3_device.h latLngToCellDeg, run
// for the ~0.01% of events whose fast-path margins are too small) and the boundary kernel (h3_boundary.h) compute
// them exactly as glibc 2.35 does on the reference's x86-64 hosts:
//   * sincos -- generic dbl-64 s_sincos.c + s_sin.c (do_sin, do_cos, TAYLOR_SIN, reduce_sincos): 2.35 has no
//     multiarch sincos, so this is plain IEEE double arithmetic in source order, no FMA;
//   * acos, asin, atan2, atan, tan -- the variants glibc's IFUNC resolvers pick on an FMA+AVX2 CPU
//     (__ieee754_acos_fma, __ieee754_asin_fma, __ieee754_atan2_fma, __atan_fma, __tan_fma: e_asin.c, e_atan2.c,
//     s_atan.c, s_tan.c built with -mfma -mavx2), whose fused multiply-adds are part of the result; every fma()
//     below is one vfmadd/vfnmadd/vfmsub of that machine code.
// Constants and tables: glibc_libm.inc (tools/gen_glibc_libm.py reads them from the image's libm.so.6).  The same
// code runs on the host (hm_selftest_glibc_libm_host) and on the GPU (hm_selftest_glibc_libm_device); tests/
// test_glibc_libm.py compares both with the running glibc on >= 1e7 arguments per function.
// Domain: everything latLngToCell and cellToBoundary pass (|x| < 105414350 for sincos -- glibc's __branred range is
// not restated --, |x| <= 0.787 for tan -- r = acos(1 - sqd/2) <= 0.66 --, all of acos, asin, atan and atan2);
// outside it the functions return NaN, which no caller produces.
// The whole file must be compiled with -ffp-contract=off (the Makefile does): the non-fma expressions are separate
// roundings, as in glibc's code.
//
// License: the routines below are a restatement (a derived work) of the GNU C Library's dbl-64 sources (s_sin.c,
// s_sincos.c, e_asin.c, e_atan2.c, s_tan.c, s_atan.c and their tables: IBM Accurate Mathematical Library, Copyright
// (C) 2001-2022 Free Software Foundation, Inc.), which are licensed under the GNU Lesser General Public License 2.1 or
// later.  This file and glibc_libm.inc are distributed under the same license; see NOTICE at the repository root.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_libm.inc"

namespace hm {
namespace glm {

struct Tables {
    double sincostab[440];
    double tan_tab[186 * 4];
    double atan_cij[241 * 7];
    double asncs[2566];
    double inroot[128];
    double powtwo[28];
    double atan1_cij[241 * 7];
};

#define GLM_HD __host__ __device__ __forceinline__

GLM_HD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
GLM_HD double dbl(uint64_t b) { return __builtin_bit_cast(double, b); }
GLM_HD int32_t hi32(double x) { return (int32_t)(bits(x) >> 32); }
GLM_HD uint32_t lo32(double x) { return (uint32_t)bits(x); }
GLM_HD double fabs_(double x) { return dbl(bits(x) & 0x7fffffffffffffffull); }                            // andpd
GLM_HD double copysign_(double x, double s) { return dbl((bits(x) & 0x7fffffffffffffffull) | (bits(s) & (1ull << 63))); }
GLM_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
GLM_HD double qnan() { return dbl(0x7ff8000000000000ull); }

// ---------------------------------------------------------------- sincos (s_sin.c / s_sincos.c, dbl-64)
// TAYLOR_SIN(xx, a, da): a + ((POLYNOMIAL(xx) * a - 0.5 * da) * xx + da)
GLM_HD double taylor_sin(double xx, double a, double da) {
    double p = GLM_S5 * xx + GLM_S4;
    p = p * xx - GLM_S3N;
    p = p * xx + GLM_S2;
    p = p * xx - GLM_S1N;
    const double t = (p * a - GLM_HALF * da) * xx + da;
    return a + t;
}

GLM_HD double do_sin(double x, double dx, const Tables &G) {
    const double xold = x;
    if (fabs_(x) < GLM_SMALL) return taylor_sin(x * x, x, dx);
    if (x <= 0) dx = -dx;
    const double u = GLM_BIG + fabs_(x);
    x = fabs_(x) - (u - GLM_BIG);
    const double xx = x * x;
    const double s = x + (dx + (x * xx) * (xx * GLM_SN5 - GLM_SN3N));
    const double c = x * dx + xx * (xx * (xx * GLM_CS6 - GLM_CS4N) + GLM_HALF);
    const double *t = &G.sincostab[lo32(u) << 2];   // SINCOS_TABLE_LOOKUP: sn, ssn, cs, ccs
    const double cor = (t[1] + s * t[3] - t[0] * c) + t[2] * s;
    return copysign_(t[0] + cor, xold);
}

GLM_HD double do_cos(double x, double dx, const Tables &G) {
    if (x < 0) dx = -dx;
    const double u = GLM_BIG + fabs_(x);
    x = fabs_(x) - (u - GLM_BIG) + dx;
    const double xx = x * x;
    const double s = x + (x * xx) * (xx * GLM_SN5 - GLM_SN3N);
    const double c = xx * (xx * (xx * GLM_CS6 - GLM_CS4N) + GLM_HALF);
    const double *t = &G.sincostab[lo32(u) << 2];
    const double cor = (t[3] - s * t[1] - t[2] * c) - t[0] * s;
    return t[2] + cor;
}

// reduce_sincos: x = n pi/2 + (a + da), |x| < 105414350
GLM_HD int reduce_sincos(double x, double &a, double &da) {
    const double t = x * GLM_HPINV + GLM_TOINT;
    const double xn = t - GLM_TOINT;
    const int n = (int)(lo32(t) & 3);
    const double y = (x - xn * GLM_MP1) - xn * GLM_MP2;
    double t1 = xn * GLM_PP3;
    const double t2 = y - t1;
    double db = (y - t2) - t1;
    t1 = xn * GLM_PP4;
    const double b = t2 - t1;
    db += (t2 - b) - t1;
    a = b;
    da = db;
    return n;
}

GLM_HD void sincos(double x, double &sinx, double &cosx, const Tables &G) {
    const int32_t k = hi32(x) & 0x7fffffff;
    if (k < 0x400368fd) {
        if (k < 0x3e400000) {   // |x| < 2^-27
            sinx = x;
            cosx = 1.0;
            return;
        }
        if (k < 0x3feb6000) {   // |x| < 0.855469
            sinx = do_sin(x, 0, G);
            cosx = do_cos(x, 0, G);
            return;
        }
        const double y = GLM_HP0 - fabs_(x);   // |x| < 2.426265
        const double a = y + GLM_HP1;
        const double da = (y - a) + GLM_HP1;
        sinx = copysign_(do_cos(a, da, G), x);
        cosx = do_sin(a, da, G);
        return;
    }
    if (k < 0x419921FB) {
        double a, da;
        const int n = reduce_sincos(x, a, da);
        if (n == 1 || n == 2) {
            a = -a;
            da = -da;
        }
        const double s = do_sin(a, da, G);
        double c = do_cos(a, da, G);
        if (n & 2) c = -c;
        if (n & 1) {
            sinx = c;
            cosx = s;
        } else {
            sinx = s;
            cosx = c;
        }
        return;
    }
    sinx = cosx = qnan();   // __branred's range and inf/NaN: not restated (see the header)
}

// ---------------------------------------------------------------- tan (s_tan.c, __tan_fma), |x| <= 0.787
GLM_HD double tan(double x, const Tables &G) {
    const double w = x < 0 ? -x : x;
    if (GLM_TN_TINY >= w) return x;
    if (GLM_TN_SMALL >= w) {
        const double x2 = x * x;
        double p = fma_(x2, GLM_TN_A9, GLM_TN_A7);
        p = fma_(x2, p, GLM_TN_A5);
        p = fma_(x2, p, GLM_TN_A3);
        p = fma_(x2, p, GLM_TN_A1);
        return fma_(x * x2, p, x);
    }
    if (GLM_TN_MID >= w) {
        const int i = (int)fma_(w, GLM_TWO8, GLM_TN_OFF);   // cvttsd2si(256 w - 15.5)
        const double sgn = (x < 0) ? GLM_MONE : GLM_ONE;
        const double *e = &G.tan_tab[4 * i];                 // x_i, tan(x_i), 1/tan(x_i)
        const double z = w - e[0];
        const double z2 = z * z;
        const double z3 = z * z2;
        const double p = fma_(z2, GLM_TN_B3, GLM_TN_B1);
        const double pz = fma_(z3, p, z);
        const double num = (e[1] + e[2]) * pz;
        const double den = e[2] - pz;
        return (num / den + e[1]) * sgn;
    }
    return qnan();   // |x| > 0.787: not restated (see the header)
}

// ---------------------------------------------------------------- acos (e_asin.c, __ieee754_acos_fma)
// one interval polynomial of the asncs table: T[0] the interval point, z = |x| - T[0],
// res1 = z T[1] + (z^2 (z-Horner of T[top..2]) + T[top+1]), then acos = (hp1 - res1) + (hp0 - T[top+2]) for x > 0
GLM_HD double asncs_res1(double ax, const double *T, int top) {
    const double z = ax - T[0];
    double p = fma_(z, T[top], T[top - 1]);
    const double z2 = z * z;
    for (int j = top - 2; j >= 2; j--) p = fma_(z, p, T[j]);
    p = fma_(z2, p, T[top + 1]);
    return fma_(z, T[1], p);
}
GLM_HD double acos_interval(double ax, int32_t hx, const double *T, int top) {
    const double res1 = asncs_res1(ax, T, top);
    const double c = T[top + 2];
    if (hx > 0) return (GLM_HP1 - res1) + (GLM_HP0 - c);
    return (res1 + GLM_HP1) + (c + GLM_HP0);
}

GLM_HD double acos(double x, const Tables &G) {
    const int32_t hx = hi32(x);
    const int32_t k = hx & 0x7fffffff;
    const double ax = hx > 0 ? x : -x;
    if (k < 0x3c880000) return GLM_HP0;
    if (k < 0x3fc00000) {   // |x| < 0.125
        const double x2 = x * x;
        double p = fma_(x2, GLM_AC_F6, GLM_AC_F5);
        p = fma_(x2, p, GLM_AC_F4);
        const double r = GLM_HP0 - x;
        p = fma_(x2, p, GLM_AC_F3);
        p = fma_(x2, p, GLM_AC_F2);
        p = fma_(x2, p, GLM_AC_F1);
        const double t = ((GLM_HP0 - r) - x) + GLM_HP1;
        return r + fma_(-p, x * x2, t);
    }
    if (k < 0x3fd00000) return acos_interval(ax, hx, &G.asncs[11 * ((k >> 15) & 0x1f)], 6);
    if (k < 0x3fe00000) return acos_interval(ax, hx, &G.asncs[11 * ((k >> 14) & 0x3f) + 0x160], 6);
    if (k < 0x3fe80000) return acos_interval(ax, hx, &G.asncs[3 * ((k >> 11) & 0x1fc) + 0x420], 7);
    if (k < 0x3fed8000) return acos_interval(ax, hx, &G.asncs[13 * ((k >> 13) & 0x7f) + 0x3e0], 8);
    if (k < 0x3fee8000) return acos_interval(ax, hx, &G.asncs[14 * ((k >> 13) & 0x7f) + 0x374], 9);
    if (k < 0x3fef0000) return acos_interval(ax, hx, &G.asncs[15 * ((k >> 13) & 0x7f) + 0x300], 10);
    if (k < 0x3ff00000) {   // 0.96875 <= |x| < 1: 2 asin(sqrt((1 - |x|) / 2)) via root.tbl's inverse square root
        double w = hx > 0 ? GLM_ONE - x : x + GLM_ONE;
        w = w * GLM_HALF;
        const uint64_t b = bits(w);
        const int e = 0x1ff - (int)(b >> 53);
        const int m = (int)(b >> 46) & 0x7f;
        const double y0 = G.inroot[m] * G.powtwo[e];
        const double t = fma_(-(y0 * y0), w, GLM_ONE);
        double q = fma_(t, GLM_RT3, GLM_RT2);
        q = fma_(t, q, GLM_RT1);
        q = fma_(t, q, GLM_RT0);
        const double y = q * y0;
        const double s = w * y;
        const double d = fma_(-s, y * GLM_HALF, GLM_THREE_HALVES);
        const double hs = fma_(-GLM_SPLIT27, s, fma_(s, GLM_SPLIT27, s));   // s rounded to 26 bits
        const double den = fma_(d, s, hs);
        const double cc = fma_(-hs, hs, w) / den;
        double p = fma_(w, GLM_AC_F6, GLM_AC_F5);
        p = fma_(w, p, GLM_AC_F4);
        p = fma_(w, p, GLM_AC_F3);
        p = fma_(w, p, GLM_AC_F2);
        p = fma_(w, p, GLM_AC_F1);
        const double pw = (p * w) * (hs + cc);
        if (hx < 0) {
            const double r = ((GLM_HP1 - cc) - pw) + (GLM_HP0 - hs);
            return r + r;
        }
        const double r = (cc + pw) + hs;
        return r + r;
    }
    if (k == 0x3ff00000 && lo32(x) == 0) return hx > 0 ? 0.0 : GLM_PI;
    if (k > 0x7ff00000 || (k == 0x7ff00000 && lo32(x) != 0)) return x + x;
    return qnan();   // |x| > 1
}

// ---------------------------------------------------------------- atan2 (e_atan2.c, __ieee754_atan2_fma)
// atan of the reduced argument u (+ du) from the cij table row nearest u: zz, t1 = cij[i][1] as the caller combines
GLM_HD const double *atan_row(double u, const double *cij) {
    const int i = (int)(fma_(u, GLM_TWO8, GLM_TWO52) - GLM_TWO52) - 16;
    return &cij[7 * i];
}
GLM_HD double atan_poly5(double v, const double *c) {   // c2 + v (c3 + v (c4 + v (c5 + v c6)))
    double p = fma_(v, c[6], c[5]);
    p = fma_(v, p, c[4]);
    p = fma_(v, p, c[3]);
    return fma_(v, p, c[2]);
}
GLM_HD double atan_small(double v) {   // d3 + v (d5 + v (d7 + v (d9 + v (d11 + v d13))))
    double p = fma_(v, GLM_D13, GLM_D11);
    p = fma_(v, p, GLM_D9);
    p = fma_(v, p, GLM_D7);
    p = fma_(v, p, GLM_D5);
    return fma_(v, p, GLM_D3);
}

GLM_HD double atan2(double y, double x, const Tables &G) {
    const int32_t hx = hi32(x), hy = hi32(y);
    const uint32_t lx = lo32(x), ly = lo32(y);
    if ((hx & 0x7ff00000) == 0x7ff00000 && ((hx & 0xfffff) | lx) != 0) return x + y;
    if ((hy & 0x7ff00000) == 0x7ff00000 && ((hy & 0xfffff) | ly) != 0) return y + y;
    if (hy == 0 && ly == 0) return hx < 0 ? GLM_PI : 0.0;                           // y = +0
    if ((uint32_t)hy == 0x80000000u && ly == 0) return hx < 0 ? GLM_MPI : -0.0;     // y = -0
    if (x == 0.0) return hy < 0 ? GLM_MHP0 : GLM_HP0;
    if (hx == 0x7ff00000 && lx == 0) {                                               // x = +inf
        if (hy == 0x7ff00000) return GLM_QPI;
        if ((uint32_t)hy == 0xfff00000u) return GLM_MQPI;
        return hy < 0 ? -0.0 : 0.0;
    }
    if ((uint32_t)hx == 0xfff00000u && lx == 0) {                                    // x = -inf
        if (hy == 0x7ff00000) return GLM_TQPI;
        if ((uint32_t)hy == 0xfff00000u) return GLM_MTQPI;
        return hy < 0 ? GLM_MPI : GLM_PI;
    }
    if (hy == 0x7ff00000 && ly == 0) return GLM_HP0;
    if ((uint32_t)hy == 0xfff00000u && ly == 0) return GLM_MHP0;

    double ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
    const int32_t de = (hy & 0x7ff00000) - (hx & 0x7ff00000);
    if (de > 0x38fffff) return (0 < y) ? GLM_HP0 : GLM_MHP0;
    if (de < -0x38fffff) {
        if (x > 0) return copysign_(ay / ax, y);
        return (0 < y) ? GLM_PI : GLM_MPI;
    }
    if (ax < GLM_TWOM500 || ay < GLM_TWOM500) {
        ax *= GLM_TWO500;
        ay *= GLM_TWO500;
    }
    if (ax > GLM_TWO500 || ay > GLM_TWO500) {
        ax *= GLM_TWOM500;
        ay *= GLM_TWOM500;
    }
    double u, du;
    if (ay < ax) {
        u = ay / ax;
        const double v = ax * u, vv = fma_(ax, u, -v);   // EMULV
        du = ((ay - v) - vv) / ax;
    } else {
        u = ax / ay;
        const double v = ay * u, vv = fma_(ay, u, -v);
        du = ((ax - v) - vv) / ay;
    }
    if (x > 0) {
        if (ay < ax) {   // (i) atan(ay/ax)
            if (u < GLM_INV16) {
                const double v = u * u;
                const double p = atan_small(v);
                return copysign_(u + fma_(u * v, p, du), y);
            }
            const double *c = atan_row(u, G.atan_cij);
            const double t3 = u - c[0];
            const double v = du + t3;   // EADD(t3, du, v, dv)
            const double dv = fabs_(t3) > fabs_(du) ? (t3 - v) + du : (du - v) + t3;
            double p = fma_(v, c[6], c[5]);
            p = fma_(v, p, c[4]);
            p = fma_(v, p, c[3]);
            p = (v * v) * p;
            p = fma_(dv, c[2], p);
            return copysign_(fma_(v, c[2], p) + c[1], y);
        }
        // (ii) pi/2 - atan(ax/ay)
        if (u < GLM_INV16) {
            const double v = u * u;
            const double p = atan_small(v);
            const double t2 = GLM_HP0 - u;   // ESUB(hpi, u, t2, cor)
            const double zz = (u * v) * p;
            const double cor = GLM_HP0 > fabs_(u) ? (GLM_HP0 - t2) - u : GLM_HP0 - (u + t2);
            return copysign_((((cor + GLM_HP1) - du) - zz) + t2, y);
        }
        const double *c = atan_row(u, G.atan_cij);
        const double v = (u - c[0]) + du;
        const double zz = fma_(-v, atan_poly5(v, c), GLM_HP1);
        return copysign_((GLM_HP0 - c[1]) + zz, y);
    }
    if (ax < ay) {   // (iii) pi/2 + atan(ax/ay)
        if (u < GLM_INV16) {
            const double v = u * u;
            const double p = atan_small(v);
            const double t2 = u + GLM_HP0;   // EADD(hpi, u, t2, cor)
            const double zz = (v * u) * p;
            const double cor = GLM_HP0 > fabs_(u) ? (GLM_HP0 - t2) + u : (u - t2) + GLM_HP0;
            return copysign_((((cor + GLM_HP1) + du) + zz) + t2, y);
        }
        const double *c = atan_row(u, G.atan_cij);
        const double v = (u - c[0]) + du;
        const double zz = fma_(v, atan_poly5(v, c), GLM_HP1);
        return copysign_((GLM_HP0 + c[1]) + zz, y);
    }
    // (iv) pi - atan(ay/ax)
    if (u < GLM_INV16) {
        const double v = u * u;
        const double p = atan_small(v);
        const double t2 = GLM_PI - u;   // ESUB(opi, u, t2, cor)
        const double zz = (v * u) * p;
        const double cor = GLM_PI > fabs_(u) ? (GLM_PI - t2) - u : GLM_PI - (t2 + u);
        return copysign_((((cor + GLM_PI1) - du) - zz) + t2, y);
    }
    const double *c = atan_row(u, G.atan_cij);
    const double v = (u - c[0]) + du;
    const double zz = fma_(-v, atan_poly5(v, c), GLM_PI1);
    return copysign_((GLM_PI - c[1]) + zz, y);
}

// ---------------------------------------------------------------- asin (e_asin.c, __ieee754_asin_fma)
// the interval polynomials are acos's (asncs_res1): asin(|x|) = res1 + T[top + 2]
GLM_HD double asin(double x, const Tables &G) {
    const int32_t hx = hi32(x);
    const int32_t k = hx & 0x7fffffff;
    if (k < 0x3e500000) return x;   // |x| < 2^-26
    if (k < 0x3fc00000) {            // |x| < 0.125: Taylor
        const double x2 = x * x;
        double p = fma_(x2, GLM_AC_F6, GLM_AC_F5);
        p = fma_(x2, p, GLM_AC_F4);
        p = fma_(x2, p, GLM_AC_F3);
        p = fma_(x2, p, GLM_AC_F2);
        p = fma_(x2, p, GLM_AC_F1);
        return fma_(p, x * x2, x);
    }
    const double ax = hx > 0 ? x : -x;
    double r;
    if (k < 0x3fd00000) r = asncs_res1(ax, &G.asncs[11 * ((k >> 15) & 0x1f)], 6) + G.asncs[11 * ((k >> 15) & 0x1f) + 8];
    else if (k < 0x3fe00000) {
        const double *T = &G.asncs[11 * ((k >> 14) & 0x3f) + 0x160];
        r = asncs_res1(ax, T, 6) + T[8];
    } else if (k < 0x3fe80000) {
        const double *T = &G.asncs[3 * ((k >> 11) & 0x1fc) + 0x420];
        r = asncs_res1(ax, T, 7) + T[9];
    } else if (k < 0x3fed8000) {
        const double *T = &G.asncs[13 * ((k >> 13) & 0x7f) + 0x3e0];
        r = asncs_res1(ax, T, 8) + T[10];
    } else if (k < 0x3fee8000) {
        const double *T = &G.asncs[14 * ((k >> 13) & 0x7f) + 0x374];
        r = asncs_res1(ax, T, 9) + T[11];
    } else if (k < 0x3fef0000) {
        const double *T = &G.asncs[15 * ((k >> 13) & 0x7f) + 0x300];
        r = asncs_res1(ax, T, 10) + T[12];
    } else if (k < 0x3ff00000) {   // 0.96875 <= |x| < 1: pi/2 - 2 asin(sqrt((1 - |x|) / 2)), root.tbl's 1/sqrt
        double z = hx > 0 ? GLM_ONE - x : x + GLM_ONE;
        z = z * GLM_HALF;
        const uint64_t b = bits(z);
        const double y0 = G.inroot[(int)(b >> 46) & 0x7f] * G.powtwo[0x1ff - (int)(b >> 53)];
        const double rr = fma_(-(y0 * y0), z, GLM_ONE);
        double q = fma_(rr, GLM_RT3, GLM_RT2);
        q = fma_(rr, q, GLM_RT1);
        q = fma_(rr, q, GLM_RT0);
        const double t = q * y0;
        const double c = z * t;
        const double d = fma_(-c, t * GLM_HALF, GLM_THREE_HALVES);
        const double y = (c + GLM_T24) - GLM_T24;
        const double cc = fma_(-y, y, z) / fma_(d, c, y);
        double p = fma_(z, GLM_AC_F6, GLM_AC_F5);
        p = fma_(z, p, GLM_AC_F4);
        p = fma_(z, p, GLM_AC_F3);
        p = fma_(z, p, GLM_AC_F2);
        p = fma_(z, p, GLM_AC_F1);
        p = p * z;
        const double yc = y + cc;
        const double cor = fma_(-(yc + yc), p, fma_(-GLM_TWO, cc, GLM_HP1));
        r = cor + fma_(-GLM_TWO, y, GLM_HP0);
    } else {
        if (k == 0x3ff00000 && lo32(x) == 0) return hx > 0 ? GLM_HP0 : GLM_MHP0;
        if (k > 0x7ff00000 || (k == 0x7ff00000 && lo32(x) != 0)) return x + x;
        return qnan();   // |x| > 1
    }
    return hx > 0 ? r : -r;
}

// ---------------------------------------------------------------- atan (s_atan.c, __atan_fma)
// thresholds A (~1.29e-8), B = 1/16, C = 1, D = 16, E (~5.8e15); the cij rows are s_atan.c's own table
GLM_HD double atan(double x, const Tables &G) {
    const int32_t hx = hi32(x);
    if ((hx & 0x7ff00000) == 0x7ff00000 && ((hx & 0xfffff) | lo32(x)) != 0) return x + x;
    const double u = x < 0 ? -x : x;
    if (u < GLM_ONE) {
        if (u < GLM_INV16) {
            if (u < GLM_AT_A) return x;
            const double v = x * x;
            return fma_(x * v, atan_small(v), x);
        }
        const double *c = atan_row(u, G.atan1_cij);
        const double z = u - c[0];
        return copysign_(fma_(atan_poly5(z, c), z, c[1]), x);
    }
    if (u < GLM_AT_D) {   // 1 <= u < 16: pi/2 - atan(1/u)
        const double w = GLM_ONE / u;
        const double t1 = u * w, t2 = fma_(u, w, -t1);   // EMULV
        const double *c = atan_row(w, G.atan1_cij);
        const double z = fma_((GLM_ONE - t1) - t2, w, w - c[0]);
        const double yy = fma_(-z, atan_poly5(z, c), GLM_HP1);
        return copysign_((GLM_HP0 - c[1]) + yy, x);
    }
    if (u < GLM_AT_E) {   // 16 <= u < E
        const double w = GLM_ONE / u;
        const double v = w * w;
        const double t1 = u * w, t2 = fma_(u, w, -t1);
        const double yy = (w * v) * atan_small(v);
        const double ww = ((GLM_ONE - t1) - t2) * w;
        const double t3 = GLM_HP0 - w;   // ESUB(hpi, w, t3, cor)
        const double cor = GLM_HP0 > fabs_(w) ? (GLM_HP0 - t3) - w : GLM_HP0 - (w + t3);
        return copysign_((((cor + GLM_HP1) - ww) - yy) + t3, x);
    }
    return 0 < x ? GLM_HP0 : GLM_MHP0;
}

}  // namespace glm
}  // namespace hm
