/*
 * ORACLE -- test infrastructure only. Never linked into, loaded by or called from the product path
 * (real-time-mobility-heatmap_amd/). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * CPU restatement of the H3 v4 cell-indexing path the reference runs per row:
 *   reference heatmap_stream.py:65-75  to_h3(lat, lon) -> h3.latlng_to_cell(lat, lon, H3_RES)   (h3-py 4.x)
 *   h3-py _cy/latlng.pyx latlng_to_cell -> deg2coord (degsToRads) -> H3 C latLngToCell
 * Upstream H3 C v4 (third-party, unpinned by the reference: README.md:95; absent from this image) is
 * restated function by function below, names kept: degsToRads, _geoToVec3d, _pointSquareDist,
 * _geoToClosestFace, _geoAzimuthRads, _posAngleRads, _geoToHex2d, _hex2dToCoordIJK, _ijkNormalize,
 * _upAp7/_upAp7r, _downAp7/_downAp7r, _unitIjkToDigit, _faceIjkToH3, _h3Rotate60ccw/cw,
 * _h3RotatePent60ccw.  Upstream's `long double` constants (…L literals) are kept as long double so gcc on
 * x86-64 evaluates them in x87 extended precision exactly like the compiled h3 library does.
 * Compile with -O2 -ffp-contract=off (no FMA contraction; x86-64 SSE2 doubles), link glibc libm.
 *
 * Also restates the inverse (cellToLatLng: _h3ToFaceIjk, _adjustOverageClassII, _faceIjkToGeo) used to
 * validate the tables by round trip (latLngToCell(cellToLatLng(c)) == c), and the read side's cellToBoundary
 * (reference app.py:19-41 h3_boundary_geojson -> h3.cell_to_boundary; upstream h3Index.c cellToBoundary ->
 * faceijk.c _faceIjkToCellBoundary / _faceIjkPentToCellBoundary, _faceIjkToVerts, _faceIjkPentToVerts,
 * _adjustPentVertOverage, _hex2dToGeo with substrate grids; vec2d.c _v2dIntersect (upstream's `float t`),
 * _v2dAlmostEquals; coordijk.c _ijkToHex2d, _downAp3, _downAp3r), the checker of SURVEY §8f row f4.
 *
 * Parity status: UNPINNED against h3-py (not importable here; the reference ships no fixtures).  Anchors:
 * three public known-answer vectors from upstream READMEs, round-trip and table self-consistency checks.
 */
#define _GNU_SOURCE   /* sincos */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <stdio.h>

/* upstream constants.h / coordijk.h (v4) */
#define M_PI_180 0.0174532925199432957692369076848861271111L
#define M_180_PI 57.29577951308232087679815481410517033240547L
#define M_2PI 6.28318530717958647692528676655900576839433L
#define EPSILON 0.0000000000000001L
#define M_SQRT3_2 0.8660254037844386467637231707529361834714L
#define M_AP7_ROT_RADS 0.333473172251832115336090755351601070065900389L
#define RES0_U_GNOMONIC 0.38196601125010500003
#define INV_RES0_U_GNOMONIC 2.61803398874989588842
#define M_SQRT7 2.6457513110645905905016157536392604257102L
#define M_RSQRT7 0.37796447300922722721451653623418006081576L
#define M_RSIN60 1.1547005383792515290182975610039149112953L
#define M_ONESEVENTH 0.14285714285714285714285714285714285L
#define M_ONETHIRD 0.333333333333333333333333333333333333333L
#define MAX_H3_RES 15
#define MAX_FACE_COORD 2
#define H3_INIT UINT64_C(0x00001fffffffffff)

typedef struct { double lat, lng; } LatLng;
typedef struct { double x, y, z; } Vec3d;
typedef struct { double x, y; } Vec2d;
typedef struct { int i, j, k; } CoordIJK;
typedef struct { int face; CoordIJK coord; } FaceIJK;

/* the oracle's own tables: primary constants + derived discrete tables (not the product's h3_tables.inc) */
#include "h3_tables_oracle.h"

enum { CENTER_DIGIT = 0, K_AXES_DIGIT = 1, J_AXES_DIGIT = 2, JK_AXES_DIGIT = 3, I_AXES_DIGIT = 4,
       IK_AXES_DIGIT = 5, IJ_AXES_DIGIT = 6, INVALID_DIGIT = 7 };

#define GET_RES(h) ((int)(((h) >> 52) & 0xf))
#define GET_BC(h) ((int)(((h) >> 45) & 0x7f))
#define GET_DIGIT(h, r) ((int)(((h) >> ((MAX_H3_RES - (r)) * 3)) & 7))
#define SET_DIGIT(h, r, d) \
    (h) = (((h) & ~(UINT64_C(7) << ((MAX_H3_RES - (r)) * 3))) | ((uint64_t)(d) << ((MAX_H3_RES - (r)) * 3)))

static double degsToRads(double degrees) { return degrees * M_PI_180; }
static double radsToDegs(double radians) { return radians * M_180_PI; }

static double _posAngleRads(double rads) {
    double tmp = ((rads < 0.0L) ? rads + M_2PI : rads);
    if (rads >= M_2PI) tmp -= M_2PI;
    return tmp;
}

/* libm-sensitivity probe (tests only, oracle_latlng_to_cell_perturbed): the result of transcendental call site
 * `pt_site` of latLngToCell's forward path is moved by `pt_ulps` ulps; -1 = off.  Sites: 0 cos(lat), 1 sin(lat),
 * 2 cos(lng), 3 sin(lng), 4 acos, 5 sin(dlng), 6 cos(dlng), 7 atan2, 8 tan, 9 cos(theta), 10 sin(theta)
 * (cos/sin of the point's latitude are the same values wherever upstream recomputes them). */
static __thread int pt_site = -1, pt_ulps = 0;
/* argument capture (tests only, oracle_latlng_to_cell_args_batch): the arguments of the forward path's glibc calls --
 * 0 sincos(lat), 1 sincos(lng), 2 acos, 3 sincos(dlng), 4/5 atan2 (y, x), 6 tan, 7 sincos(theta) */
static __thread double *arg_cap = 0;
#define CAP(site, x) (arg_cap ? (arg_cap[site] = (x)) : (x))
static double PT(int site, double x) {
    if (site != pt_site) return x;
    for (int u = 0; u < pt_ulps; u++) x = nextafter(x, INFINITY);
    for (int u = 0; u > pt_ulps; u--) x = nextafter(x, -INFINITY);
    return x;
}

/* sin and cos of one argument as one sincos() call: gcc merges upstream's separate calls so (-O1 and up, no fast-math),
 * and glibc's sincos can differ from its sin/cos in the last bit (their FMA variants) */
static void _geoToVec3d(const LatLng *geo, Vec3d *v) {
    double s, c, sg, cg;
    sincos(CAP(0, geo->lat), &s, &c);
    sincos(CAP(1, geo->lng), &sg, &cg);
    double r = PT(0, c);
    v->z = PT(1, s);
    v->x = PT(2, cg) * r;
    v->y = PT(3, sg) * r;
}

static double _square(double x) { return x * x; }

static double _pointSquareDist(const Vec3d *v1, const Vec3d *v2) {
    return _square(v1->x - v2->x) + _square(v1->y - v2->y) + _square(v1->z - v2->z);
}

static void _geoToClosestFace(const LatLng *g, int *face, double *sqd) {
    Vec3d v3d;
    _geoToVec3d(g, &v3d);
    *face = 0;
    *sqd = 5.0;
    for (int f = 0; f < H3T_NUM_FACES; ++f) {
        Vec3d c = {H3T_faceCenterPoint[f][0], H3T_faceCenterPoint[f][1], H3T_faceCenterPoint[f][2]};
        double sqdT = _pointSquareDist(&c, &v3d);
        if (sqdT < *sqd) {
            *face = f;
            *sqd = sqdT;
        }
    }
}

static double _geoAzimuthRads(const LatLng *p1, const LatLng *p2) {
    double s2, c2, s1, c1, sd, cd;
    sincos(p2->lat, &s2, &c2);
    sincos(CAP(3, p2->lng - p1->lng), &sd, &cd);
    sincos(p1->lat, &s1, &c1);
    c2 = PT(0, c2);
    return PT(7, atan2(CAP(4, c2 * PT(5, sd)), CAP(5, c1 * PT(1, s2) - s1 * c2 * PT(6, cd))));
}

static int isResolutionClassIII(int r) { return r % 2; }

static void _geoToHex2d(const LatLng *g, int res, int *face, Vec2d *v) {
    double sqd;
    _geoToClosestFace(g, face, &sqd);
    double r = PT(4, acos(CAP(2, 1 - sqd / 2)));
    if (r < EPSILON) {
        v->x = v->y = 0.0;
        return;
    }
    LatLng fc = {H3T_faceCenterGeo[*face][0], H3T_faceCenterGeo[*face][1]};
    double theta = _posAngleRads(H3T_faceAxesAzRadsCII[*face][0] - _posAngleRads(_geoAzimuthRads(&fc, g)));
    if (isResolutionClassIII(res)) theta = _posAngleRads(theta - M_AP7_ROT_RADS);
    r = PT(8, tan(CAP(6, r)));
    r *= INV_RES0_U_GNOMONIC;
    for (int i = 0; i < res; i++) r *= M_SQRT7;
    double st, ct;
    sincos(CAP(7, theta), &st, &ct);
    v->x = r * PT(9, ct);
    v->y = r * PT(10, st);
}

static void _ijkNormalize(CoordIJK *c) {
    if (c->i < 0) { c->j -= c->i; c->k -= c->i; c->i = 0; }
    if (c->j < 0) { c->i -= c->j; c->k -= c->j; c->j = 0; }
    if (c->k < 0) { c->i -= c->k; c->j -= c->k; c->k = 0; }
    int min = c->i;
    if (c->j < min) min = c->j;
    if (c->k < min) min = c->k;
    if (min > 0) { c->i -= min; c->j -= min; c->k -= min; }
}

static void _hex2dToCoordIJK(const Vec2d *v, CoordIJK *h) {
    double a1, a2, x1, x2, r1, r2;
    int m1, m2;
    h->k = 0;
    a1 = fabsl(v->x);
    a2 = fabsl(v->y);
    x2 = a2 * M_RSIN60;
    x1 = a1 + x2 / 2.0;
    m1 = x1;
    m2 = x2;
    r1 = x1 - m1;
    r2 = x2 - m2;
    if (r1 < 0.5) {
        if (r1 < 1.0 / 3.0) {
            if (r2 < (1.0 + r1) / 2.0) { h->i = m1; h->j = m2; }
            else { h->i = m1; h->j = m2 + 1; }
        } else {
            if (r2 < (1.0 - r1)) h->j = m2; else h->j = m2 + 1;
            if ((1.0 - r1) <= r2 && r2 < (2.0 * r1)) h->i = m1 + 1; else h->i = m1;
        }
    } else {
        if (r1 < 2.0 / 3.0) {
            if (r2 < (1.0 - r1)) h->j = m2; else h->j = m2 + 1;
            if ((2.0 * r1 - 1.0) < r2 && r2 < (1.0 - r1)) h->i = m1; else h->i = m1 + 1;
        } else {
            if (r2 < (r1 / 2.0)) { h->i = m1 + 1; h->j = m2; }
            else { h->i = m1 + 1; h->j = m2 + 1; }
        }
    }
    if (v->x < 0.0) {
        if ((h->j % 2) == 0) {
            long long int axisi = h->j / 2;
            long long int diff = h->i - axisi;
            h->i = h->i - 2.0 * diff;
        } else {
            long long int axisi = (h->j + 1) / 2;
            long long int diff = h->i - axisi;
            h->i = h->i - (2.0 * diff + 1);
        }
    }
    if (v->y < 0.0) {
        h->i = h->i - (2 * h->j + 1) / 2;
        h->j = -1 * h->j;
    }
    _ijkNormalize(h);
}

static void _upAp7(CoordIJK *ijk) {
    int i = ijk->i - ijk->k, j = ijk->j - ijk->k;
    ijk->i = (int)lround((3 * i - j) * M_ONESEVENTH);
    ijk->j = (int)lround((i + 2 * j) * M_ONESEVENTH);
    ijk->k = 0;
    _ijkNormalize(ijk);
}
static void _upAp7r(CoordIJK *ijk) {
    int i = ijk->i - ijk->k, j = ijk->j - ijk->k;
    ijk->i = (int)lround((2 * i + j) * M_ONESEVENTH);
    ijk->j = (int)lround((3 * j - i) * M_ONESEVENTH);
    ijk->k = 0;
    _ijkNormalize(ijk);
}
static void _ijkScaleAdd(CoordIJK *acc, const int v[3], int s) {
    acc->i += v[0] * s; acc->j += v[1] * s; acc->k += v[2] * s;
}
static void _downAp7(CoordIJK *ijk) {
    static const int iv[3] = {3, 0, 1}, jv[3] = {1, 3, 0}, kv[3] = {0, 1, 3};
    CoordIJK r = {0, 0, 0};
    _ijkScaleAdd(&r, iv, ijk->i); _ijkScaleAdd(&r, jv, ijk->j); _ijkScaleAdd(&r, kv, ijk->k);
    *ijk = r;
    _ijkNormalize(ijk);
}
static void _downAp7r(CoordIJK *ijk) {
    static const int iv[3] = {3, 1, 0}, jv[3] = {0, 3, 1}, kv[3] = {1, 0, 3};
    CoordIJK r = {0, 0, 0};
    _ijkScaleAdd(&r, iv, ijk->i); _ijkScaleAdd(&r, jv, ijk->j); _ijkScaleAdd(&r, kv, ijk->k);
    *ijk = r;
    _ijkNormalize(ijk);
}
static const int UNIT_VECS[7][3] = {{0, 0, 0}, {0, 0, 1}, {0, 1, 0}, {0, 1, 1}, {1, 0, 0}, {1, 0, 1}, {1, 1, 0}};
static int _unitIjkToDigit(const CoordIJK *ijk) {
    CoordIJK c = *ijk;
    _ijkNormalize(&c);
    for (int d = CENTER_DIGIT; d < 7; d++)
        if (c.i == UNIT_VECS[d][0] && c.j == UNIT_VECS[d][1] && c.k == UNIT_VECS[d][2]) return d;
    return INVALID_DIGIT;
}
static int _rotate60ccw(int d) {
    static const int t[8] = {0, 5, 3, 1, 6, 4, 2, 7};
    return t[d];
}
static int _rotate60cw(int d) {
    static const int t[8] = {0, 3, 6, 2, 5, 1, 4, 7};
    return t[d];
}
static int _h3LeadingNonZeroDigit(uint64_t h) {
    for (int r = 1; r <= GET_RES(h); r++)
        if (GET_DIGIT(h, r)) return GET_DIGIT(h, r);
    return CENTER_DIGIT;
}
static uint64_t _h3Rotate60ccw(uint64_t h) {
    for (int r = 1, res = GET_RES(h); r <= res; r++) SET_DIGIT(h, r, _rotate60ccw(GET_DIGIT(h, r)));
    return h;
}
static uint64_t _h3Rotate60cw(uint64_t h) {
    for (int r = 1, res = GET_RES(h); r <= res; r++) SET_DIGIT(h, r, _rotate60cw(GET_DIGIT(h, r)));
    return h;
}
static uint64_t _h3RotatePent60ccw(uint64_t h) {
    int foundFirstNonZeroDigit = 0;
    for (int r = 1, res = GET_RES(h); r <= res; r++) {
        SET_DIGIT(h, r, _rotate60ccw(GET_DIGIT(h, r)));
        if (!foundFirstNonZeroDigit && GET_DIGIT(h, r) != 0) {
            foundFirstNonZeroDigit = 1;
            if (_h3LeadingNonZeroDigit(h) == K_AXES_DIGIT) h = _h3Rotate60ccw(h);
        }
    }
    return h;
}
static uint64_t _h3RotatePent60cw(uint64_t h) {
    int foundFirstNonZeroDigit = 0;
    for (int r = 1, res = GET_RES(h); r <= res; r++) {
        SET_DIGIT(h, r, _rotate60cw(GET_DIGIT(h, r)));
        if (!foundFirstNonZeroDigit && GET_DIGIT(h, r) != 0) {
            foundFirstNonZeroDigit = 1;
            if (_h3LeadingNonZeroDigit(h) == K_AXES_DIGIT) h = _h3Rotate60cw(h);
        }
    }
    return h;
}

static uint64_t _faceIjkToH3(const FaceIJK *fijk, int res) {
    uint64_t h = H3_INIT;
    h |= UINT64_C(1) << 59;           /* mode = cell */
    h |= (uint64_t)res << 52;
    if (res == 0) {
        if (fijk->coord.i > MAX_FACE_COORD || fijk->coord.j > MAX_FACE_COORD || fijk->coord.k > MAX_FACE_COORD)
            return 0;
        h |= (uint64_t)H3T_faceIjkBaseCells[fijk->face][fijk->coord.i][fijk->coord.j][fijk->coord.k][0] << 45;
        return h;
    }
    FaceIJK fijkBC = *fijk;
    CoordIJK *ijk = &fijkBC.coord;
    for (int r = res - 1; r >= 0; r--) {
        CoordIJK lastIJK = *ijk, lastCenter;
        if (isResolutionClassIII(r + 1)) {
            _upAp7(ijk);
            lastCenter = *ijk;
            _downAp7(&lastCenter);
        } else {
            _upAp7r(ijk);
            lastCenter = *ijk;
            _downAp7r(&lastCenter);
        }
        CoordIJK diff = {lastIJK.i - lastCenter.i, lastIJK.j - lastCenter.j, lastIJK.k - lastCenter.k};
        _ijkNormalize(&diff);
        SET_DIGIT(h, r + 1, _unitIjkToDigit(&diff));
    }
    if (fijkBC.coord.i > MAX_FACE_COORD || fijkBC.coord.j > MAX_FACE_COORD || fijkBC.coord.k > MAX_FACE_COORD)
        return 0;
    const int *bcr = H3T_faceIjkBaseCells[fijkBC.face][fijkBC.coord.i][fijkBC.coord.j][fijkBC.coord.k];
    int baseCell = bcr[0];
    h |= (uint64_t)baseCell << 45;
    int numRots = bcr[1];
    if (H3T_baseCellData[baseCell][4]) {
        if (_h3LeadingNonZeroDigit(h) == K_AXES_DIGIT) {
            if (H3T_baseCellData[baseCell][5] == fijkBC.face || H3T_baseCellData[baseCell][6] == fijkBC.face)
                h = _h3Rotate60cw(h);
            else
                h = _h3Rotate60ccw(h);
        }
        for (int i = 0; i < numRots; i++) h = _h3RotatePent60ccw(h);
    } else {
        for (int i = 0; i < numRots; i++) h = _h3Rotate60ccw(h);
    }
    return h;
}

/* upstream latLngToCell (h3Index.c) with h3-py's deg2coord in front: degrees in, 0 (H3_NULL) on error. */
uint64_t oracle_latlng_to_cell(double lat_deg, double lng_deg, int res) {
    if (res < 0 || res > MAX_H3_RES) return 0;
    LatLng g = {degsToRads(lat_deg), degsToRads(lng_deg)};
    if (!isfinite(g.lat) || !isfinite(g.lng)) return 0;
    FaceIJK fijk;
    Vec2d v;
    _geoToHex2d(&g, res, &fijk.face, &v);
    _hex2dToCoordIJK(&v, &fijk.coord);
    return _faceIjkToH3(&fijk, res);
}

void oracle_latlng_to_cell_batch(const double *lat, const double *lng, int64_t n, int res, uint64_t *out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) out[i] = oracle_latlng_to_cell(lat[i], lng[i], res);
}

/* the arguments latLngToCell hands glibc for each point (8 per point, NaN where a call is not reached; see CAP) */
void oracle_latlng_to_cell_args_batch(const double *lat, const double *lng, int64_t n, int res, double *args) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        for (int k = 0; k < 8; k++) args[8 * i + k] = NAN;
        arg_cap = args + 8 * i;
        oracle_latlng_to_cell(lat[i], lng[i], res);
        arg_cap = 0;
    }
}

/* latLngToCell with the result of one transcendental call site moved by `ulps` ulps (see PT): the answers a libm
 * differing from this one in the last bits of that function could give.  An input whose cell changes under such a
 * perturbation is libm-sensitive: h3 itself returns different cells for it on different platforms (glibc's FMA and
 * non-FMA variants, other libms). */
void oracle_latlng_to_cell_perturbed_batch(const double *lat, const double *lng, int64_t n, int res, int site, int ulps,
                                           uint64_t *out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        pt_site = site;
        pt_ulps = ulps;
        out[i] = oracle_latlng_to_cell(lat[i], lng[i], res);
        pt_site = -1;
    }
}

/* glibc's own sincos / acos / atan2 / tan, called through this process's libm (the reference's h3 calls them so):
 * the checker of the product's restatement of those routines (csrc/glibc_libm.h).  fn as hm_selftest_glibc_libm_host. */
void oracle_libm_batch(int fn, const double *a, const double *b, int64_t n, double *out, double *out2) {
    /* through a pointer: gcc would otherwise fold this sincos() into separate sin() and cos() calls here, and
     * glibc's (FMA) sin/cos differ from its sincos in the last bit for ~0.1% of arguments */
    void (*volatile libm_sincos)(double, double *, double *) = sincos;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        switch (fn) {
            case 0: libm_sincos(a[i], &out[i], &out2[i]); break;
            case 1: out[i] = acos(a[i]); break;
            case 2: out[i] = atan2(a[i], b[i]); break;
            case 3: out[i] = tan(a[i]); break;
            case 4: out[i] = asin(a[i]); break;
            default: out[i] = atan(a[i]); break;
        }
    }
}

/* ---------------- inverse, validation only: cellToLatLng ---------------- */
static const int maxDimByCIIres[] = {2, -1, 14, -1, 98, -1, 686, -1, 4802, -1, 33614, -1, 235298, -1, 1647086, -1, 11529602};
static const int unitScaleByCIIres[] = {1, -1, 7, -1, 49, -1, 343, -1, 2401, -1, 16807, -1, 117649, -1, 823543, -1, 5764801};

static void _neighbor(CoordIJK *ijk, int digit) {
    if (digit > CENTER_DIGIT && digit < 7) {
        ijk->i += UNIT_VECS[digit][0]; ijk->j += UNIT_VECS[digit][1]; ijk->k += UNIT_VECS[digit][2];
        _ijkNormalize(ijk);
    }
}
static void _ijkRotate60ccw(CoordIJK *ijk) {
    CoordIJK r = {0, 0, 0};
    static const int iv[3] = {1, 1, 0}, jv[3] = {0, 1, 1}, kv[3] = {1, 0, 1};
    _ijkScaleAdd(&r, iv, ijk->i); _ijkScaleAdd(&r, jv, ijk->j); _ijkScaleAdd(&r, kv, ijk->k);
    *ijk = r;
    _ijkNormalize(ijk);
}
static void _ijkRotate60cw(CoordIJK *ijk) {
    CoordIJK r = {0, 0, 0};
    static const int iv[3] = {1, 0, 1}, jv[3] = {1, 1, 0}, kv[3] = {0, 1, 1};
    _ijkScaleAdd(&r, iv, ijk->i); _ijkScaleAdd(&r, jv, ijk->j); _ijkScaleAdd(&r, kv, ijk->k);
    *ijk = r;
    _ijkNormalize(ijk);
}
enum { NO_OVERAGE = 0, FACE_EDGE = 1, NEW_FACE = 2 };
static int _adjustOverageClassII(FaceIJK *fijk, int res, int pentLeading4, int substrate) {
    int overage = NO_OVERAGE;
    CoordIJK *ijk = &fijk->coord;
    int maxDim = maxDimByCIIres[res];
    if (substrate) maxDim *= 3;
    if (substrate && ijk->i + ijk->j + ijk->k == maxDim) {
        overage = FACE_EDGE;
    } else if (ijk->i + ijk->j + ijk->k > maxDim) {
        overage = NEW_FACE;
        const int *o;
        if (ijk->k > 0) {
            if (ijk->j > 0) {
                o = H3T_faceNeighbors[fijk->face][3];
            } else {
                o = H3T_faceNeighbors[fijk->face][2];
                if (pentLeading4) {
                    CoordIJK tmp = {ijk->i - maxDim, ijk->j, ijk->k};
                    _ijkRotate60cw(&tmp);
                    ijk->i = tmp.i + maxDim; ijk->j = tmp.j; ijk->k = tmp.k;
                }
            }
        } else {
            o = H3T_faceNeighbors[fijk->face][1];
        }
        fijk->face = o[0];
        for (int i = 0; i < o[4]; i++) _ijkRotate60ccw(ijk);
        int unitScale = unitScaleByCIIres[res];
        if (substrate) unitScale *= 3;
        ijk->i += o[1] * unitScale; ijk->j += o[2] * unitScale; ijk->k += o[3] * unitScale;
        _ijkNormalize(ijk);
        if (substrate && ijk->i + ijk->j + ijk->k == maxDim) overage = FACE_EDGE;
    }
    return overage;
}
static int _h3ToFaceIjkWithInitializedFijk(uint64_t h, FaceIJK *fijk) {
    CoordIJK *ijk = &fijk->coord;
    int res = GET_RES(h);
    int possibleOverage = 1;
    if (!H3T_baseCellData[GET_BC(h)][4] && (res == 0 || (ijk->i == 0 && ijk->j == 0 && ijk->k == 0)))
        possibleOverage = 0;
    for (int r = 1; r <= res; r++) {
        if (isResolutionClassIII(r)) _downAp7(ijk); else _downAp7r(ijk);
        _neighbor(ijk, GET_DIGIT(h, r));
    }
    return possibleOverage;
}
static void _h3ToFaceIjk(uint64_t h, FaceIJK *fijk) {
    int baseCell = GET_BC(h);
    if (H3T_baseCellData[baseCell][4] && _h3LeadingNonZeroDigit(h) == IK_AXES_DIGIT) h = _h3Rotate60cw(h);
    fijk->face = H3T_baseCellData[baseCell][0];
    fijk->coord.i = H3T_baseCellData[baseCell][1];
    fijk->coord.j = H3T_baseCellData[baseCell][2];
    fijk->coord.k = H3T_baseCellData[baseCell][3];
    if (!_h3ToFaceIjkWithInitializedFijk(h, fijk)) return;
    CoordIJK origIJK = fijk->coord;
    int res = GET_RES(h);
    if (isResolutionClassIII(res)) {
        _downAp7r(&fijk->coord);
        res++;
    }
    int pentLeading4 = (H3T_baseCellData[baseCell][4] && _h3LeadingNonZeroDigit(h) == I_AXES_DIGIT);
    if (_adjustOverageClassII(fijk, res, pentLeading4, 0) != NO_OVERAGE) {
        if (H3T_baseCellData[baseCell][4])
            while (_adjustOverageClassII(fijk, res, 0, 0) != NO_OVERAGE) continue;
        if (res != GET_RES(h)) _upAp7r(&fijk->coord);
    } else if (res != GET_RES(h)) {
        fijk->coord = origIJK;
    }
}
static void _geoAzDistanceRads(const LatLng *p1, double az, double distance, LatLng *p2) {
    if (distance < EPSILON) { *p2 = *p1; return; }
    double sinlat, sinlng, coslng;
    az = _posAngleRads(az);
    if (az < EPSILON || fabs(az - M_PI) < EPSILON) {
        p2->lat = (az < EPSILON) ? p1->lat + distance : p1->lat - distance;
        if (fabs(p2->lat - M_PI_2) < EPSILON) { p2->lat = M_PI_2; p2->lng = 0.0; }
        else if (fabs(p2->lat + M_PI_2) < EPSILON) { p2->lat = -M_PI_2; p2->lng = 0.0; }
        else p2->lng = p1->lng;
    } else {
        sinlat = sin(p1->lat) * cos(distance) + cos(p1->lat) * sin(distance) * cos(az);
        if (sinlat > 1.0) sinlat = 1.0;
        if (sinlat < -1.0) sinlat = -1.0;
        p2->lat = asin(sinlat);
        if (fabs(p2->lat - M_PI_2) < EPSILON) { p2->lat = M_PI_2; p2->lng = 0.0; }
        else if (fabs(p2->lat + M_PI_2) < EPSILON) { p2->lat = -M_PI_2; p2->lng = 0.0; }
        else {
            double invcosp2lat = 1.0 / cos(p2->lat);
            sinlng = sin(az) * sin(distance) * invcosp2lat;
            coslng = (cos(distance) - sin(p1->lat) * sin(p2->lat)) / cos(p1->lat) * invcosp2lat;
            if (sinlng > 1.0) sinlng = 1.0;
            if (sinlng < -1.0) sinlng = -1.0;
            if (coslng > 1.0) coslng = 1.0;
            if (coslng < -1.0) coslng = -1.0;
            p2->lng = p1->lng + atan2(sinlng, coslng);
        }
    }
    /* constrainLng */
    while (p2->lng > M_PI) p2->lng = p2->lng - (2 * M_PI);
    while (p2->lng < -M_PI) p2->lng = p2->lng + (2 * M_PI);
}
int oracle_cell_to_latlng(uint64_t h, double *lat_deg, double *lng_deg) {
    if (((h >> 59) & 0xf) != 1 || GET_RES(h) > MAX_H3_RES || GET_BC(h) >= H3T_NUM_BASE_CELLS) return -1;
    FaceIJK fijk;
    _h3ToFaceIjk(h, &fijk);
    int res = GET_RES(h);
    /* _ijkToHex2d + _hex2dToGeo (substrate = 0) */
    int i = fijk.coord.i - fijk.coord.k, j = fijk.coord.j - fijk.coord.k;
    Vec2d v = {i - 0.5 * j, j * M_SQRT3_2};
    LatLng g;
    LatLng fc = {H3T_faceCenterGeo[fijk.face][0], H3T_faceCenterGeo[fijk.face][1]};
    double r = sqrt(v.x * v.x + v.y * v.y);
    if (r < EPSILON) {
        g = fc;
    } else {
        double theta = atan2(v.y, v.x);
        for (int q = 0; q < res; q++) r *= M_RSQRT7;
        r *= RES0_U_GNOMONIC;
        r = atan(r);
        if (isResolutionClassIII(res)) theta = _posAngleRads(theta + M_AP7_ROT_RADS);
        theta = _posAngleRads(H3T_faceAxesAzRadsCII[fijk.face][0] - theta);
        _geoAzDistanceRads(&fc, theta, r, &g);
    }
    *lat_deg = radsToDegs(g.lat);
    *lng_deg = radsToDegs(g.lng);
    return 0;
}

void oracle_cell_to_latlng_batch(const uint64_t *cells, int64_t n, double *lat, double *lng) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        if (oracle_cell_to_latlng(cells[i], &lat[i], &lng[i])) lat[i] = lng[i] = NAN;
    }
}

/* Host x87 reference for the device code's extended-precision emulation (see csrc/h3_device.h):
 * op 0: (double)(a * M_PI_180); 1: (double)(a * M_SQRT7); 2: (double)(a * M_RSIN60);
 * 3: (double)(a + M_2PI); 4: (double)(a - M_2PI); 5: (double)(a - M_AP7_ROT_RADS); 6: (double)(a + M_AP7_ROT_RADS) */
void oracle_ld_ops(const double *a, int64_t n, int op, double *out) {
    for (int64_t i = 0; i < n; i++) {
        long double x = a[i];
        switch (op) {
            case 0: out[i] = (double)(x * M_PI_180); break;
            case 1: out[i] = (double)(x * M_SQRT7); break;
            case 2: out[i] = (double)(x * M_RSIN60); break;
            case 3: out[i] = (double)(x + M_2PI); break;
            case 4: out[i] = (double)(x - M_2PI); break;
            case 5: out[i] = (double)(x - M_AP7_ROT_RADS); break;
            case 6: out[i] = (double)(x + M_AP7_ROT_RADS); break;
            case 7: out[i] = (double)(x * M_SQRT3_2); break;
            case 8: out[i] = (double)(x * M_RSQRT7); break;
            case 9: out[i] = (double)(x * M_ONETHIRD); break;
            case 17: out[i] = (double)(x * M_180_PI); break;
            default: out[i] = NAN;
        }
    }
}

/* ---------------- read side (row f4): cellToBoundary ---------------- */
enum { IJ_DIR = 1, KI_DIR = 2, JK_DIR = 3 };
static int adjacentFaceDir(int from, int to) {   /* upstream's adjacentFaceDir table, from faceNeighbors */
    if (from == to) return 0;
    for (int d = 1; d <= 3; d++)
        if (H3T_faceNeighbors[from][d][0] == to) return d;
    return -1;
}
static void _ijkToHex2d(const CoordIJK *h, Vec2d *v) {
    int i = h->i - h->k;
    int j = h->j - h->k;
    v->x = i - 0.5 * j;
    v->y = j * M_SQRT3_2;
}
static void _downAp3(CoordIJK *ijk) {
    static const int iv[3] = {2, 0, 1}, jv[3] = {1, 2, 0}, kv[3] = {0, 1, 2};
    CoordIJK r = {0, 0, 0};
    _ijkScaleAdd(&r, iv, ijk->i); _ijkScaleAdd(&r, jv, ijk->j); _ijkScaleAdd(&r, kv, ijk->k);
    *ijk = r;
    _ijkNormalize(ijk);
}
static void _downAp3r(CoordIJK *ijk) {
    static const int iv[3] = {2, 1, 0}, jv[3] = {0, 2, 1}, kv[3] = {1, 0, 2};
    CoordIJK r = {0, 0, 0};
    _ijkScaleAdd(&r, iv, ijk->i); _ijkScaleAdd(&r, jv, ijk->j); _ijkScaleAdd(&r, kv, ijk->k);
    *ijk = r;
    _ijkNormalize(ijk);
}
static void _hex2dToGeo(const Vec2d *v, int face, int res, int substrate, LatLng *g) {
    double r = sqrt(v->x * v->x + v->y * v->y);
    LatLng fc = {H3T_faceCenterGeo[face][0], H3T_faceCenterGeo[face][1]};
    if (r < EPSILON) { *g = fc; return; }
    double theta = atan2(v->y, v->x);
    for (int i = 0; i < res; i++) r *= M_RSQRT7;
    if (substrate) {
        r *= M_ONETHIRD;
        if (isResolutionClassIII(res)) r *= M_RSQRT7;
    }
    r *= RES0_U_GNOMONIC;
    r = atan(r);
    if (!substrate && isResolutionClassIII(res)) theta = _posAngleRads(theta + M_AP7_ROT_RADS);
    theta = _posAngleRads(H3T_faceAxesAzRadsCII[face][0] - theta);
    _geoAzDistanceRads(&fc, theta, r, g);
}
static void _v2dIntersect(const Vec2d *p0, const Vec2d *p1, const Vec2d *p2, const Vec2d *p3, Vec2d *inter) {
    Vec2d s1, s2;
    s1.x = p1->x - p0->x;
    s1.y = p1->y - p0->y;
    s2.x = p3->x - p2->x;
    s2.y = p3->y - p2->y;
    float t;
    t = (s2.x * (p0->y - p2->y) - s2.y * (p0->x - p2->x)) / (-s2.x * s1.y + s1.x * s2.y);
    inter->x = p0->x + (t * s1.x);
    inter->y = p0->y + (t * s1.y);
}
static int _v2dAlmostEquals(const Vec2d *a, const Vec2d *b) {
    return fabsf(a->x - b->x) < 1.1920929e-07F && fabsf(a->y - b->y) < 1.1920929e-07F;   /* FLT_EPSILON */
}
static void _faceIjkVerts(FaceIJK *fijk, int *res, FaceIJK *verts, int nverts) {
    static const int vertsCII[6][3] = {{2, 1, 0}, {1, 2, 0}, {0, 2, 1}, {0, 1, 2}, {1, 0, 2}, {2, 0, 1}};
    static const int vertsCIII[6][3] = {{5, 4, 0}, {1, 5, 0}, {0, 5, 4}, {0, 1, 5}, {4, 0, 5}, {5, 0, 1}};
    const int (*vs)[3] = isResolutionClassIII(*res) ? vertsCIII : vertsCII;
    _downAp3(&fijk->coord);
    _downAp3r(&fijk->coord);
    if (isResolutionClassIII(*res)) {
        _downAp7r(&fijk->coord);
        *res += 1;
    }
    for (int v = 0; v < nverts; v++) {
        verts[v].face = fijk->face;
        verts[v].coord.i = fijk->coord.i + vs[v][0];
        verts[v].coord.j = fijk->coord.j + vs[v][1];
        verts[v].coord.k = fijk->coord.k + vs[v][2];
        _ijkNormalize(&verts[v].coord);
    }
}
/* the two icosahedron-face edge endpoints of direction dir in a substrate grid of resolution adjRes */
static void _faceEdge(int adjRes, int dir, Vec2d *e0, Vec2d *e1) {
    int maxDim = maxDimByCIIres[adjRes];
    Vec2d v0 = {3.0 * maxDim, 0.0};
    Vec2d v1 = {-1.5 * maxDim, 3.0 * M_SQRT3_2 * maxDim};
    Vec2d v2 = {-1.5 * maxDim, -3.0 * M_SQRT3_2 * maxDim};
    if (dir == IJ_DIR) { *e0 = v0; *e1 = v1; }
    else if (dir == JK_DIR) { *e0 = v1; *e1 = v2; }
    else { *e0 = v2; *e1 = v0; }
}
static int _faceIjkToCellBoundary(const FaceIJK *h, int res, double *lat, double *lng) {
    int adjRes = res, n = 0;
    FaceIJK centerIJK = *h;
    FaceIJK fijkVerts[6];
    _faceIjkVerts(&centerIJK, &adjRes, fijkVerts, 6);
    int lastFace = -1, lastOverage = NO_OVERAGE;
    for (int vert = 0; vert < 6 + 1; vert++) {
        int v = vert % 6;
        FaceIJK fijk = fijkVerts[v];
        int overage = _adjustOverageClassII(&fijk, adjRes, 0, 1);
        if (isResolutionClassIII(res) && vert > 0 && fijk.face != lastFace && lastOverage != FACE_EDGE) {
            int lastV = (v + 5) % 6;
            Vec2d orig2d0, orig2d1, e0, e1, inter;
            _ijkToHex2d(&fijkVerts[lastV].coord, &orig2d0);
            _ijkToHex2d(&fijkVerts[v].coord, &orig2d1);
            int face2 = (lastFace == centerIJK.face) ? fijk.face : lastFace;
            _faceEdge(adjRes, adjacentFaceDir(centerIJK.face, face2), &e0, &e1);
            _v2dIntersect(&orig2d0, &orig2d1, &e0, &e1, &inter);
            if (!(_v2dAlmostEquals(&orig2d0, &inter) || _v2dAlmostEquals(&orig2d1, &inter))) {
                LatLng g;
                _hex2dToGeo(&inter, centerIJK.face, adjRes, 1, &g);
                lat[n] = radsToDegs(g.lat); lng[n] = radsToDegs(g.lng); n++;
            }
        }
        if (vert < 6) {
            Vec2d vec;
            LatLng g;
            _ijkToHex2d(&fijk.coord, &vec);
            _hex2dToGeo(&vec, fijk.face, adjRes, 1, &g);
            lat[n] = radsToDegs(g.lat); lng[n] = radsToDegs(g.lng); n++;
        }
        lastFace = fijk.face;
        lastOverage = overage;
    }
    return n;
}
static int _faceIjkPentToCellBoundary(const FaceIJK *h, int res, double *lat, double *lng) {
    int adjRes = res, n = 0;
    FaceIJK centerIJK = *h;
    FaceIJK fijkVerts[5];
    _faceIjkVerts(&centerIJK, &adjRes, fijkVerts, 5);
    FaceIJK lastFijk = fijkVerts[0];
    for (int vert = 0; vert < 5 + 1; vert++) {
        int v = vert % 5;
        FaceIJK fijk = fijkVerts[v];
        while (_adjustOverageClassII(&fijk, adjRes, 0, 1) == NEW_FACE) continue;   /* _adjustPentVertOverage */
        if (isResolutionClassIII(res) && vert > 0) {
            FaceIJK tmpFijk = fijk;
            Vec2d orig2d0, orig2d1, e0, e1, inter;
            _ijkToHex2d(&lastFijk.coord, &orig2d0);
            int currentToLastDir = adjacentFaceDir(tmpFijk.face, lastFijk.face);
            const int *o = H3T_faceNeighbors[tmpFijk.face][currentToLastDir];
            tmpFijk.face = o[0];
            CoordIJK *ijk = &tmpFijk.coord;
            for (int i = 0; i < o[4]; i++) _ijkRotate60ccw(ijk);
            int unitScale = unitScaleByCIIres[adjRes] * 3;
            ijk->i += o[1] * unitScale; ijk->j += o[2] * unitScale; ijk->k += o[3] * unitScale;
            _ijkNormalize(ijk);
            _ijkToHex2d(ijk, &orig2d1);
            _faceEdge(adjRes, adjacentFaceDir(tmpFijk.face, fijk.face), &e0, &e1);
            _v2dIntersect(&orig2d0, &orig2d1, &e0, &e1, &inter);
            LatLng g;
            _hex2dToGeo(&inter, tmpFijk.face, adjRes, 1, &g);
            lat[n] = radsToDegs(g.lat); lng[n] = radsToDegs(g.lng); n++;
        }
        if (vert < 5) {
            Vec2d vec;
            LatLng g;
            _ijkToHex2d(&fijk.coord, &vec);
            _hex2dToGeo(&vec, fijk.face, adjRes, 1, &g);
            lat[n] = radsToDegs(g.lat); lng[n] = radsToDegs(g.lng); n++;
        }
        lastFijk = fijk;
    }
    return n;
}
/* cellToBoundary in degrees (h3-py cell_to_boundary: radsToDegs of each vertex); returns the vertex count, -1 if
 * h is not a valid cell index */
int oracle_cell_to_boundary(uint64_t h, double *lat, double *lng) {
    if (((h >> 59) & 0xf) != 1 || GET_RES(h) > MAX_H3_RES || GET_BC(h) >= H3T_NUM_BASE_CELLS) return -1;
    FaceIJK fijk;
    _h3ToFaceIjk(h, &fijk);
    int res = GET_RES(h);
    if (H3T_baseCellData[GET_BC(h)][4] && _h3LeadingNonZeroDigit(h) == 0)
        return _faceIjkPentToCellBoundary(&fijk, res, lat, lng);
    return _faceIjkToCellBoundary(&fijk, res, lat, lng);
}
void oracle_cell_to_boundary_batch(const uint64_t *cells, int64_t n, double *lat, double *lng, int32_t *nverts) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) nverts[i] = oracle_cell_to_boundary(cells[i], lat + 10 * i, lng + 10 * i);
}

/* derivation of the discrete tables at load (needs the projections above) */
#include "h3_tables_derive.c"
