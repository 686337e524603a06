#!/usr/bin/env python3
"""Generate csrc/glibc_libm.inc: the constants and tables of the glibc double routines that upstream H3's
latLngToCell and cellToBoundary call (sincos, acos, atan2, tan, asin, atan), read from this image's libm.so.6.

Why: the reference's cell ids come from h3 linked against the host libm (reference heatmap_stream.py:65-75 ->
h3.latlng_to_cell -> H3 C latLngToCell -> glibc).  Bit-exactness on knife-edge inputs needs the same double
results, so csrc/glibc_libm.h restates those glibc 2.35 routines (IBM Accurate Mathematical Library, dbl-64) for
host and device; the numbers they use are read here from the library itself, so that they are exactly glibc's.

Which variants: on an x86-64 host with FMA and AVX2 (this image and the GPU box) glibc's IFUNC resolvers pick
__ieee754_acos_fma, __ieee754_asin_fma, __ieee754_atan2_fma, __atan_fma and __tan_fma (sysdeps/x86_64/fpu/multiarch, built with -mfma -mavx2,
so their FMA contractions are part of the result); sincos has no multiarch variant in 2.35 and is the generic
non-FMA dbl-64 code.  csrc/glibc_libm.h follows the machine code of exactly those variants.

The virtual addresses below are of glibc 2.35-0ubuntu3.12's libm.so.6 (build-id pinned below); each table is
sanity-checked against its defining property before it is written.  With another libm the generator refuses to
regenerate and keeps the committed file (tests/test_glibc_libm.py then reports whether the restatement still equals
the running libm).
"""
import hashlib
import math
import os
import struct
import sys

LIBM = "/lib/x86_64-linux-gnu/libm.so.6"
BUILD_ID = "df46fc5774ae8aaaf6efcb97dc7b91532056b898"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "glibc_libm.inc")

# (name, vaddr, count, row): read-only data of libm.so.6 (vaddr == file offset in its R segment at 0x8a000)
TABLES = [
    ("sincostab", 0xAEB80, 440, 4),   # s_sin.c __sincostab: sin hi/lo, cos hi/lo of k/128, k = 0..109
    ("tan_tab", 0xC15C0, 186 * 4, 4),  # __tan_fma: x_i, tan(x_i), 1/tan(x_i), (unused) for 256 x - 15.5 in [0, 185]
    ("atan_cij", 0xBE0E0, 241 * 7, 7),  # e_atan2.c cij[241][7]: x_i, atan(x_i), Taylor coefficients
    ("asncs", 0xB90A0, 2566, 1),       # e_asin.c asncs table (acos's interval polynomials)
    ("inroot", 0xB8CA0, 128, 1),       # root.tbl inroot: 1/sqrt of the mantissa buckets
    ("powtwo", 0xB8BC0, 28, 1),        # root.tbl powtwo: 2^-(e/2) scale, indexed 0x1ff - (bits >> 53)
    ("atan1_cij", 0xB56E0, 241 * 7, 7),  # s_atan.c (uatan.tbl) cij[241][7], __atan_fma's own copy
]
# scalar constants referenced by the machine code (name, vaddr)
SCALARS = [
    ("HP0", 0x93048), ("HP1", 0x930B8), ("MHP0", 0x93040), ("PI", 0x930C0), ("MPI", 0x96598),
    ("PI1", 0x96618), ("QPI", 0x965A0), ("MQPI", 0x965A8), ("TQPI", 0x965B0), ("MTQPI", 0x965B8),
    ("TINY", 0x93050), ("ONE", 0x8A2D0), ("HALF", 0x8AAB0), ("TWO52", 0x8A2F0), ("TWO8", 0x96610),
    # sincos (usncs.h)
    ("BIG", 0x9A8A8), ("SN5", 0x9A8B0), ("SN3N", 0x9A8B8), ("CS6", 0x9A8C0), ("CS4N", 0x9A8C8),
    ("S5", 0x9A880), ("S4", 0x9A888), ("S3N", 0x9A890), ("S2", 0x9A898), ("S1N", 0x9A8A0), ("SMALL", 0x9A878),
    ("HPINV", 0x969B8), ("TOINT", 0x97010), ("MP1", 0x9A8D0), ("MP2", 0x9A8D8), ("PP3", 0x9A8E0), ("PP4", 0x9A8E8),
    ("MONE", 0x969B0),
    # acos (e_asin.c, __ieee754_acos_fma)
    ("AC_F6", 0x93058), ("AC_F5", 0x93060), ("AC_F4", 0x93068), ("AC_F3", 0x93070), ("AC_F2", 0x93078),
    ("AC_F1", 0x93080), ("RT3", 0x93088), ("RT2", 0x93090), ("RT1", 0x93098), ("RT0", 0x930A0),
    ("THREE_HALVES", 0x930A8), ("SPLIT27", 0x930C8),
    # asin (e_asin.c, __ieee754_asin_fma; the F and RT constants are acos's)
    ("T24", 0x930B0), ("TWO", 0x96D90),
    # atan (s_atan.c, __atan_fma; B = INV16, C = ONE, d3..d13 are atan2's)
    ("AT_A", 0x9A558), ("AT_D", 0x9A560), ("AT_E", 0x9A568),
    # atan2 (e_atan2.c, __ieee754_atan2_fma)
    ("TWOM500", 0x965C0), ("TWO500", 0x965C8), ("INV16", 0x965D8), ("D13", 0x965E0), ("D11", 0xB8B98),
    ("D9", 0x965F0), ("D7", 0xB8BA0), ("D5", 0x96600), ("D3", 0xB8BA8),
    # tan (s_tan.c, __tan_fma)
    ("TN_TINY", 0x9C040), ("TN_SMALL", 0x9C048), ("TN_A9", 0x9C050), ("TN_A7", 0x9C058), ("TN_A5", 0x9C060),
    ("TN_A3", 0x9C068), ("TN_A1", 0x96608), ("TN_MID", 0x9C070), ("TN_B3", 0x9C080), ("TN_B1", 0x9C088),
    ("TN_OFF", 0xC2D00),
]


def build_id(b):
    i = b.find(b"GNU\x00")
    while i >= 0:
        # note header: namesz (4) descsz (4) type (4) "GNU\0" desc
        namesz, descsz, typ = struct.unpack_from("<III", b, i - 12)
        if namesz == 4 and typ == 3 and descsz == 20:
            return b[i + 4:i + 24].hex()
        i = b.find(b"GNU\x00", i + 1)
    return None


def dbl(b, a):
    return struct.unpack_from("<d", b, a)[0]


def check(b):
    rd = lambda name: [dbl(b, a + 8 * k) for n, a, c, _ in TABLES if n == name for k in range(c)]
    st = rd("sincostab")
    for k in range(110):
        x = k / 128.0
        assert abs(st[4 * k] - math.sin(x)) < 1e-15 and abs(st[4 * k] + st[4 * k + 1] - math.sin(x)) < 1e-16
        assert abs(st[4 * k + 2] - math.cos(x)) < 1e-15
    tt = rd("tan_tab")
    for i in range(186):
        x, t, r = tt[4 * i:4 * i + 3]
        assert abs(x - (i + 16) / 256.0) < 1e-2 and abs(t - math.tan(x)) < 1e-15 and abs(r * t - 1) < 1e-14, i
    at = rd("atan_cij")
    for i in range(241):
        x, t = at[7 * i:7 * i + 2]
        assert abs(x - (i + 16) / 256.0) < 2e-3 and abs(t - math.atan(x)) < 1e-15, i
        assert abs(at[7 * i + 2] - 1 / (1 + x * x)) < 1e-14, i
    a1 = rd("atan1_cij")
    for i in range(241):
        x, t = a1[7 * i:7 * i + 2]
        assert abs(x - (i + 16) / 256.0) < 2e-3 and abs(t - math.atan(x)) < 1e-15, i
    inr = rd("inroot")
    assert all(0.7 < v < 1.5 for v in inr), inr[:4]
    sc = dict((n, dbl(b, a)) for n, a in SCALARS)
    assert sc["HP0"] == math.pi / 2 and sc["PI"] == math.pi and sc["BIG"] == 1.5 * 2 ** 45 and sc["TOINT"] == 1.5 * 2 ** 52
    assert sc["T24"] == 2.0 ** 24 and sc["TWO"] == 2.0 and sc["THREE_HALVES"] == 1.5
    assert sc["AT_D"] == 16.0 and 1e-9 < sc["AT_A"] < 1e-7 and 1e15 < sc["AT_E"] < 1e16
    assert sc["TWO8"] == 256.0 and sc["TWO52"] == 2.0 ** 52 and sc["TN_OFF"] == -15.5


def main():
    b = open(LIBM, "rb").read()
    bid = build_id(b)
    if bid != BUILD_ID:
        print(f"gen_glibc_libm: {LIBM} build-id {bid} is not the pinned glibc 2.35-0ubuntu3.12 ({BUILD_ID}); "
              f"keeping the committed {os.path.basename(OUT)}", file=sys.stderr)
        return
    check(b)
    lines = ["/* GENERATED by real-time-mobility-heatmap_amd/tools/gen_glibc_libm.py -- do not edit.",
             f" * Read from {LIBM}: glibc 2.35-0ubuntu3.12, build-id {BUILD_ID},",
             f" * sha256 {hashlib.sha256(b).hexdigest()}.",
             " * Constants and tables of sincos (generic dbl-64), __ieee754_acos_fma, __ieee754_asin_fma,",
             " * __ieee754_atan2_fma, __atan_fma and __tan_fma; csrc/glibc_libm.h restates the routines.  Names follow",
             " * glibc's sources (usncs.h, e_asin.c, e_atan2.c, s_atan.c, s_tan.c, root.tbl); a trailing N marks a constant the machine code subtracts (its negation).",
             " * The values are data of the GNU C Library (sysdeps/ieee754/dbl-64, IBM Accurate Mathematical Library),",
             " * Copyright (C) 2001-2022 Free Software Foundation, Inc., licensed under the GNU Lesser General Public",
             " * License 2.1 or later; see NOTICE at the repository root. */"]
    for n, a in SCALARS:
        lines.append(f"#define GLM_{n} {dbl(b, a).hex()}  /* libm+0x{a:x} */")
    lines.append("#define GLM_TABLE_INIT \\")
    for ti, (n, a, c, row) in enumerate(TABLES):
        vals = [dbl(b, a + 8 * k).hex() for k in range(c)]
        lines.append(f"    /* {n}: libm+0x{a:x}, {c} doubles */ {{ \\")
        for k in range(0, c, row if row > 1 else 4):
            w = row if row > 1 else 4
            lines.append("        " + ", ".join(vals[k:k + w]) + ", \\")
        lines.append("    }" + (", \\" if ti + 1 < len(TABLES) else ""))
    text = "\n".join(lines) + "\n"
    old = open(OUT).read() if os.path.exists(OUT) else None
    if old == text:
        print(f"unchanged {os.path.abspath(OUT)}")
        return
    open(OUT, "w").write(text)
    print(f"wrote {os.path.abspath(OUT)}")


if __name__ == "__main__":
    main()
