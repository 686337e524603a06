// cellToBoundary for CDNA4 (the read side: reference app.py:19-41 h3_boundary_geojson ->
// h3.cell_to_boundary, h3-py 4.x).  One lane per cell.
//
// Restates upstream H3 v4 cellToBoundary (h3Index.c) -> _h3ToFaceIjk -> _faceIjkToCellBoundary /
// _faceIjkPentToCellBoundary (faceijk.c) with their substrate-grid helpers, in the operation order of the CPU
// oracle (oracle/h3_oracle.c, the checker).  upstream's long double constants (M_SQRT3_2, M_RSQRT7, M_ONETHIRD,
// M_180_PI, M_AP7_ROT_RADS, M_2PI, EPSILON) are applied with the exact x87 emulation of h3_device.h; the
// face-centre sin/cos come from the host libm (H3Tables); sincos/asin/atan2/atan of per-vertex values are glibc's own
// (glibc_libm.h: the FMA variants the reference host's libm runs), so the vertices are bit-identical to the
// glibc-linked oracle's (tests/test_gpu_boundary.py).
#pragma once
#include "h3_device.h"

namespace hm {

#define HM_LD_SQRT3_2_M UINT64_C(0xddb3d742c265539e)
#define HM_LD_SQRT3_2_E (-64)
#define HM_LD_SQRT3_2_HI 0x1.bb67ae8584caap-1
#define HM_LD_SQRT3_2_LO 0x1.cfp-55
#define HM_LD_RSQRT7_M UINT64_C(0xc1848f353fbf3445)
#define HM_LD_RSQRT7_E (-65)
#define HM_LD_RSQRT7_HI 0x1.83091e6a7f7e7p-2
#define HM_LD_RSQRT7_LO -0x1.dd8p-56
#define HM_LD_ONETHIRD_M UINT64_C(0xaaaaaaaaaaaaaaab)
#define HM_LD_ONETHIRD_E (-65)
#define HM_LD_ONETHIRD_HI 0x1.5555555555555p-2
#define HM_LD_ONETHIRD_LO 0x1.558p-56
#define HM_LD_180_PI_M UINT64_C(0xe52ee0d31e0fbdc3)
#define HM_LD_180_PI_E (-58)
#define HM_LD_180_PI_HI 0x1.ca5dc1a63c1f8p+5
#define HM_LD_180_PI_LO -0x1.1e8p-49
#define HM_RES0_U_GNOMONIC 0.38196601125010500003

HM_HD int maxDimByCIIres(int r) {   // upstream maxDimByCIIres / unitScaleByCIIres (Class II resolutions)
    int m = 2;
    for (int q = 0; q < r; q += 2) m *= 7;
    return m;
}
HM_HD int unitScaleByCIIres(int r) {
    int u = 1;
    for (int q = 0; q < r; q += 2) u *= 7;
    return u;
}

HM_HD void ijkAddScaled(IJK &r, int a, int b, int c, int s) { r.i += a * s; r.j += b * s; r.k += c * s; }
// r = i * I + j * J + k * K (unit-vector images of an aperture step or rotation), normalised
HM_HD void ijkMap(IJK &c, const int I[3], const int J[3], const int K[3]) {
    IJK r{0, 0, 0};
    ijkAddScaled(r, I[0], I[1], I[2], c.i);
    ijkAddScaled(r, J[0], J[1], J[2], c.j);
    ijkAddScaled(r, K[0], K[1], K[2], c.k);
    c = r;
    ijkNormalize(c);
}
HM_HD void downAp7(IJK &c) { const int I[3] = {3, 0, 1}, J[3] = {1, 3, 0}, K[3] = {0, 1, 3}; ijkMap(c, I, J, K); }
HM_HD void downAp7r(IJK &c) { const int I[3] = {3, 1, 0}, J[3] = {0, 3, 1}, K[3] = {1, 0, 3}; ijkMap(c, I, J, K); }
HM_HD void downAp3(IJK &c) { const int I[3] = {2, 0, 1}, J[3] = {1, 2, 0}, K[3] = {0, 1, 2}; ijkMap(c, I, J, K); }
HM_HD void downAp3r(IJK &c) { const int I[3] = {2, 1, 0}, J[3] = {0, 2, 1}, K[3] = {1, 0, 2}; ijkMap(c, I, J, K); }
HM_HD void ijkRotate60ccw(IJK &c) { const int I[3] = {1, 1, 0}, J[3] = {0, 1, 1}, K[3] = {1, 0, 1}; ijkMap(c, I, J, K); }
HM_HD void ijkRotate60cw(IJK &c) { const int I[3] = {1, 0, 1}, J[3] = {1, 1, 0}, K[3] = {0, 1, 1}; ijkMap(c, I, J, K); }
HM_HD void upAp7r(IJK &c) {   // lround((2i + j) / 7), lround((3j - i) / 7) on IJ coordinates
    const int i = c.i - c.k, j = c.j - c.k;
    c.i = round_div7(2 * i + j);
    c.j = round_div7(3 * j - i);
    c.k = 0;
    ijkNormalize(c);
}
HM_HD void ijkNeighbor(IJK &c, int digit) {   // UNIT_VECS[digit] = (digit >> 2 & 1, digit >> 1 & 1, digit & 1)
    if (digit > 0 && digit < 7) {
        c.i += (digit >> 2) & 1;
        c.j += (digit >> 1) & 1;
        c.k += digit & 1;
        ijkNormalize(c);
    }
}

enum : int { HM_NO_OVERAGE = 0, HM_FACE_EDGE = 1, HM_NEW_FACE = 2 };

// _adjustOverageClassII (faceijk.c)
HM_HD int adjustOverageClassII(int &face, IJK &ijk, int res, bool pentLeading4, bool substrate, const H3Tables &T) {
    int overage = HM_NO_OVERAGE;
    int maxDim = maxDimByCIIres(res);
    if (substrate) maxDim *= 3;
    const int sum = ijk.i + ijk.j + ijk.k;
    if (substrate && sum == maxDim) {
        overage = HM_FACE_EDGE;
    } else if (sum > maxDim) {
        overage = HM_NEW_FACE;
        int dir;
        if (ijk.k > 0) {
            if (ijk.j > 0) {
                dir = 3;   // JK
            } else {
                dir = 2;   // KI
                if (pentLeading4) {
                    IJK tmp{ijk.i - maxDim, ijk.j, ijk.k};
                    ijkRotate60cw(tmp);
                    ijk = IJK{tmp.i + maxDim, tmp.j, tmp.k};
                }
            }
        } else {
            dir = 1;       // IJ
        }
        const int *o = T.faceNeighbors[face][dir];
        face = o[0];
        for (int q = 0; q < o[4]; q++) ijkRotate60ccw(ijk);
        int unitScale = unitScaleByCIIres(res);
        if (substrate) unitScale *= 3;
        ijkAddScaled(ijk, o[1], o[2], o[3], unitScale);
        ijkNormalize(ijk);
        if (substrate && ijk.i + ijk.j + ijk.k == maxDim) overage = HM_FACE_EDGE;
    }
    return overage;
}

// _h3ToFaceIjk (h3Index.c): the cell's centre as face + IJK at its resolution
HM_HD void h3ToFaceIjk(uint64_t h, int &face, IJK &ijk, const H3Tables &T) {
    const int bc = (int)((h >> 45) & 0x7f), res = (int)((h >> 52) & 0xf);
    const int *bd = T.baseCellData[bc];
    if (bd[4] && leadingNonZeroDigit(h, res) == 5) h = rotate60(h, true);   // IK_AXES_DIGIT: rotate cw
    face = bd[0];
    ijk = IJK{bd[1], bd[2], bd[3]};
    bool possibleOverage = !(!bd[4] && (res == 0 || (ijk.i == 0 && ijk.j == 0 && ijk.k == 0)));
    for (int r = 1; r <= res; r++) {
        if (r & 1) downAp7(ijk);
        else downAp7r(ijk);
        ijkNeighbor(ijk, getDigit(h, r));
    }
    if (!possibleOverage) return;
    const IJK orig = ijk;
    int ares = res;
    if (res & 1) {
        downAp7r(ijk);
        ares++;
    }
    const bool pentLeading4 = bd[4] && leadingNonZeroDigit(h, res) == 4;
    if (adjustOverageClassII(face, ijk, ares, pentLeading4, false, T) != HM_NO_OVERAGE) {
        if (bd[4])
            while (adjustOverageClassII(face, ijk, ares, false, false, T) != HM_NO_OVERAGE) {
            }
        if (ares != res) upAp7r(ijk);
    } else if (ares != res) {
        ijk = orig;
    }
}

struct V2 { double x, y; };
HM_HD V2 ijkToHex2d(const IJK &h) {
    const int i = h.i - h.k, j = h.j - h.k;
    return V2{i - 0.5 * j, XMUL((double)j, SQRT3_2)};
}
HM_HD bool ld_eps_lt(double a) { return xld_lt(a, HM_LD_EPSILON_M, HM_LD_EPSILON_E); }   // a < EPSILON (long double)

// _geoAzDistanceRads (latLng.c) from face centre f
HM_HD void geoAzDistanceFromFace(const H3Tables &T, int f, double az, double distance, double &lat, double &lng) {
    const double p1lat = T.faceCenterGeo[f][0], p1lng = T.faceCenterGeo[f][1];
    if (ld_eps_lt(distance)) { lat = p1lat; lng = p1lng; return; }
    az = posAngleRads(az);
    if (ld_eps_lt(az) || ld_eps_lt(__builtin_fabs(az - M_PI))) {
        lat = ld_eps_lt(az) ? p1lat + distance : p1lat - distance;
        if (ld_eps_lt(__builtin_fabs(lat - M_PI_2))) { lat = M_PI_2; lng = 0.0; }
        else if (ld_eps_lt(__builtin_fabs(lat + M_PI_2))) { lat = -M_PI_2; lng = 0.0; }
        else lng = p1lng;
    } else {
        // sin and cos of one argument as one sincos, as the gcc-built library computes them (gcc fuses the pair;
        // glibc's sincos and sin differ in the last bit for ~0.1% of arguments)
        const double s1 = T.faceSinLat[f], c1 = T.faceCosLat[f];
        double sd, cd, saz, caz;
        const glm::Tables &G = *T.glm;
        glm::sincos(distance, sd, cd, G);
        glm::sincos(az, saz, caz, G);
        double sinlat = s1 * cd + c1 * sd * caz;
        if (sinlat > 1.0) sinlat = 1.0;
        if (sinlat < -1.0) sinlat = -1.0;
        lat = glm::asin(sinlat, G);
        if (ld_eps_lt(__builtin_fabs(lat - M_PI_2))) { lat = M_PI_2; lng = 0.0; }
        else if (ld_eps_lt(__builtin_fabs(lat + M_PI_2))) { lat = -M_PI_2; lng = 0.0; }
        else {
            double s2, c2;
            glm::sincos(lat, s2, c2, G);
            const double invcosp2lat = 1.0 / c2;
            double sinlng = saz * sd * invcosp2lat;
            double coslng = (cd - s1 * s2) / c1 * invcosp2lat;
            if (sinlng > 1.0) sinlng = 1.0;
            if (sinlng < -1.0) sinlng = -1.0;
            if (coslng > 1.0) coslng = 1.0;
            if (coslng < -1.0) coslng = -1.0;
            lng = p1lng + glm::atan2(sinlng, coslng, G);
        }
    }
    while (lng > M_PI) lng = lng - (2 * M_PI);   // constrainLng
    while (lng < -M_PI) lng = lng + (2 * M_PI);
}

// _hex2dToGeo on a substrate grid (substrate = 1: every caller of the boundary), result in degrees (radsToDegs)
HM_HD void hex2dToGeoDeg(const H3Tables &T, V2 v, int face, int res, double &lat_deg, double &lng_deg) {
    double r = sqrt(v.x * v.x + v.y * v.y);
    double lat, lng;
    if (ld_eps_lt(r)) {
        lat = T.faceCenterGeo[face][0];
        lng = T.faceCenterGeo[face][1];
    } else {
        double theta = glm::atan2(v.y, v.x, *T.glm);
        for (int i = 0; i < res; i++) r = XMUL(r, RSQRT7);
        r = XMUL(r, ONETHIRD);
        if (res & 1) r = XMUL(r, RSQRT7);
        r *= HM_RES0_U_GNOMONIC;
        r = glm::atan(r, *T.glm);
        theta = posAngleRads(T.faceAxesAz0[face] - theta);
        geoAzDistanceFromFace(T, face, theta, r, lat, lng);
    }
    lat_deg = XMUL(lat, 180_PI);
    lng_deg = XMUL(lng, 180_PI);
}

// _v2dIntersect (vec2d.c; upstream keeps the parameter t in a float)
HM_HD V2 v2dIntersect(V2 p0, V2 p1, V2 p2, V2 p3) {
    const V2 s1{p1.x - p0.x, p1.y - p0.y}, s2{p3.x - p2.x, p3.y - p2.y};
    const float t = (float)((s2.x * (p0.y - p2.y) - s2.y * (p0.x - p2.x)) / (-s2.x * s1.y + s1.x * s2.y));
    return V2{p0.x + (t * s1.x), p0.y + (t * s1.y)};
}
HM_HD bool v2dAlmostEquals(V2 a, V2 b) {
    return __builtin_fabsf((float)(a.x - b.x)) < 1.1920929e-07F && __builtin_fabsf((float)(a.y - b.y)) < 1.1920929e-07F;
}
// the icosahedron-face edge of direction dir (1 IJ, 2 KI, 3 JK) on a substrate grid of Class II resolution adjRes
HM_HD void faceEdge(const H3Tables &T, int adjRes, int dir, V2 &e0, V2 &e1) {
    const int maxDim = maxDimByCIIres(adjRes);
    const double ey = T.edgeY[adjRes];   // (double)(3.0L * M_SQRT3_2 * maxDim), from the host
    const V2 v0{3.0 * maxDim, 0.0}, v1{-1.5 * maxDim, ey}, v2{-1.5 * maxDim, -ey};
    if (dir == 1) { e0 = v0; e1 = v1; }
    else if (dir == 3) { e0 = v1; e1 = v2; }
    else { e0 = v2; e1 = v0; }
}

// cellToBoundary: up to 10 vertices (degrees) into lat/lng; returns the count (0: not a valid cell index)
HM_HD int cellToBoundaryDeg(uint64_t h, const H3Tables &T, double *lat, double *lng) {
    if (((h >> 59) & 0xf) != 1 || ((h >> 45) & 0x7f) >= 122) return 0;
    const int res = (int)((h >> 52) & 0xf);
    int cface;
    IJK c;
    h3ToFaceIjk(h, cface, c, T);
    const bool pent = T.baseCellData[(h >> 45) & 0x7f][4] && leadingNonZeroDigit(h, res) == 0;
    const int nv = pent ? 5 : 6;
    // _faceIjkToVerts / _faceIjkPentToVerts: the centre on the 33r(7r) substrate grid + the origin cell's vertices
    const int vCII[6][3] = {{2, 1, 0}, {1, 2, 0}, {0, 2, 1}, {0, 1, 2}, {1, 0, 2}, {2, 0, 1}};
    const int vCIII[6][3] = {{5, 4, 0}, {1, 5, 0}, {0, 5, 4}, {0, 1, 5}, {4, 0, 5}, {5, 0, 1}};
    int adjRes = res;
    downAp3(c);
    downAp3r(c);
    if (res & 1) {
        downAp7r(c);
        adjRes++;
    }
    IJK verts[6];
    for (int v = 0; v < nv; v++) {
        const int *d = (res & 1) ? vCIII[v] : vCII[v];
        verts[v] = IJK{c.i + d[0], c.j + d[1], c.k + d[2]};
        ijkNormalize(verts[v]);
    }
    int n = 0;
    if (!pent) {   // _faceIjkToCellBoundary
        int lastFace = -1, lastOverage = HM_NO_OVERAGE;
        for (int vert = 0; vert < 6 + 1; vert++) {
            const int v = vert % 6;
            int face = cface;
            IJK ijk = verts[v];
            const int overage = adjustOverageClassII(face, ijk, adjRes, false, true, T);
            if ((res & 1) && vert > 0 && face != lastFace && lastOverage != HM_FACE_EDGE) {
                const V2 o0 = ijkToHex2d(verts[(v + 5) % 6]), o1 = ijkToHex2d(verts[v]);
                const int face2 = lastFace == cface ? face : lastFace;
                V2 e0, e1;
                faceEdge(T, adjRes, T.adjacentFaceDir[cface][face2], e0, e1);
                const V2 inter = v2dIntersect(o0, o1, e0, e1);
                if (!(v2dAlmostEquals(o0, inter) || v2dAlmostEquals(o1, inter))) {
                    hex2dToGeoDeg(T, inter, cface, adjRes, lat[n], lng[n]);
                    n++;
                }
            }
            if (vert < 6) {
                hex2dToGeoDeg(T, ijkToHex2d(ijk), face, adjRes, lat[n], lng[n]);
                n++;
            }
            lastFace = face;
            lastOverage = overage;
        }
    } else {       // _faceIjkPentToCellBoundary
        int lastFace = cface;
        IJK lastIjk = verts[0];
        for (int vert = 0; vert < 5 + 1; vert++) {
            const int v = vert % 5;
            int face = cface;
            IJK ijk = verts[v];
            while (adjustOverageClassII(face, ijk, adjRes, false, true, T) == HM_NEW_FACE) {   // _adjustPentVertOverage
            }
            if ((res & 1) && vert > 0) {
                const V2 o0 = ijkToHex2d(lastIjk);
                const int dir = T.adjacentFaceDir[face][lastFace];
                const int *o = T.faceNeighbors[face][dir];
                const int tface = o[0];
                IJK t = ijk;
                for (int q = 0; q < o[4]; q++) ijkRotate60ccw(t);
                ijkAddScaled(t, o[1], o[2], o[3], unitScaleByCIIres(adjRes) * 3);
                ijkNormalize(t);
                const V2 o1 = ijkToHex2d(t);
                V2 e0, e1;
                faceEdge(T, adjRes, T.adjacentFaceDir[tface][face], e0, e1);
                hex2dToGeoDeg(T, v2dIntersect(o0, o1, e0, e1), tface, adjRes, lat[n], lng[n]);
                n++;
            }
            if (vert < 5) {
                hex2dToGeoDeg(T, ijkToHex2d(ijk), face, adjRes, lat[n], lng[n]);
                n++;
            }
            lastFace = face;
            lastIjk = ijk;
        }
    }
    return n;
}

}  // namespace hm
