/*
 * ORACLE -- test infrastructure only (included at the end of oracle/h3_oracle.c).
 *
 * Derives the discrete H3 v4 res-0 tables (upstream baseCells.c baseCellData / faceIjkBaseCells, faceijk.c
 * faceNeighbors) from the primary constants in h3_tables_oracle.h, with the oracle's own restated projections:
 *   dv_hex2d_to_geo  = upstream _hex2dToGeo at res 0 (gnomonic inverse: atan + _geoAzDistanceRads)
 *   dv_geo_to_hex2d  = upstream _geoToHex2d at res 0 on a GIVEN face (acos + _geoAzimuthRads + tan)
 * Independently of tools/gen_h3_tables.py (numpy vector geometry) -- the two are compared by
 * tests/test_h3_oracle.py.  Methods:
 *   base cells     the Class II res-0 lattice points of each face inside its triangle (centre, 3 unit vectors,
 *                  3 edge midpoints, 3 vertices) projected to the sphere and merged: 122 cells, numbered by the
 *                  latitude of the centre, north to south (upstream's numbering)
 *   home faces     single view: that face; pentagon: the lowest face that sees it at (2,0,0); edge cells: the
 *                  recalled northern entries and the antipodal symmetry for the southern half
 *   rotations      for a base cell seen from face f, f's +x hex2d axis is stepped where f and the home face meet
 *                  and re-projected onto the home face: its angle there is ccwRot60 x 60 degrees
 *   pentagons      the faces around the vertex ordered clockwise in the home face's frame take the home frame's
 *                  sectors JK, J, IJ, I, IK (K deleted); ccwRot60 = steps along the pentagon's 5-cycle
 *   faceNeighbors  the neighbour across each quadrant is the face centred at (2,2,0)/(2,0,2)/(0,2,2); its
 *                  rotation is measured at the shared edge's midpoint; every entry is then checked DISCRETELY:
 *                  res-2 lattice points of the neighbour near the edge, located on f by projection, must land on
 *                  their own coordinates after upstream's overage transform (rotate, translate x 7, normalise)
 * Every check failure sets ORC_derive_error; oracle_tables() reports it.
 */
#include <stdio.h>

static const char *ORC_derive_error = NULL;
static char ORC_err_buf[256];
#define DV_FAIL(...)                                                         \
    do {                                                                     \
        snprintf(ORC_err_buf, sizeof ORC_err_buf, __VA_ARGS__);              \
        if (!ORC_derive_error) ORC_derive_error = ORC_err_buf;               \
        return;                                                              \
    } while (0)

static void dv_hex2d_to_geo(int face, double x, double y, LatLng *g) {
    LatLng fc = {H3T_faceCenterGeo[face][0], H3T_faceCenterGeo[face][1]};
    double r = sqrt(x * x + y * y);
    if (r < EPSILON) { *g = fc; return; }
    double theta = atan2(y, x);
    r *= RES0_U_GNOMONIC;
    r = atan(r);
    theta = _posAngleRads(H3T_faceAxesAzRadsCII[face][0] - theta);
    _geoAzDistanceRads(&fc, theta, r, g);
}
static void dv_geo_to_hex2d(int face, const LatLng *g, double *x, double *y) {
    Vec3d v, c = {H3T_faceCenterPoint[face][0], H3T_faceCenterPoint[face][1], H3T_faceCenterPoint[face][2]};
    _geoToVec3d(g, &v);
    double r = acos(1 - _pointSquareDist(&c, &v) / 2);
    if (r < EPSILON) { *x = *y = 0.0; return; }
    LatLng fc = {H3T_faceCenterGeo[face][0], H3T_faceCenterGeo[face][1]};
    double theta = _posAngleRads(H3T_faceAxesAzRadsCII[face][0] - _posAngleRads(_geoAzimuthRads(&fc, g)));
    r = tan(r) * INV_RES0_U_GNOMONIC;
    *x = r * cos(theta);
    *y = r * sin(theta);
}
static void dv_ijk_hex2d(int i, int j, int k, double *x, double *y) {
    *x = (i - k) - 0.5 * (j - k);
    *y = (j - k) * M_SQRT3_2;
}
static double dv_dist(const LatLng *a, const LatLng *b) {
    Vec3d u, v;
    _geoToVec3d(a, &u);
    _geoToVec3d(b, &v);
    return sqrt(_pointSquareDist(&u, &v));
}

typedef struct { int face, i, j, k; } DvView;
static LatLng dv_center[122];
static DvView dv_views[122][5];
static int dv_nviews[122];
static int dv_anti[20];
static int dv_pent_rot[20][122];   /* ccwRot60 of face f's view of pentagon b (-1: not a view) */

/* base cell nearest to g; *d0 / *d1 = distances to the nearest and the runner-up */
static int dv_nearest(const LatLng *g, double *d0, double *d1) {
    int best = -1;
    double b0 = 1e9, b1 = 1e9;
    for (int b = 0; b < 122; b++) {
        const double d = dv_dist(g, &dv_center[b]);
        if (d < b0) { b1 = b0; b0 = d; best = b; }
        else if (d < b1) b1 = d;
    }
    *d0 = b0;
    *d1 = b1;
    return best;
}

/* ccw 60-degree steps from face `from`'s frame to face `to`'s frame at point p: the angle, in `to`'s hex2d frame,
 * of a short step along `from`'s +x axis */
static int dv_rot(int to, int from, const LatLng *p, int *ok) {
    double fx, fy, tx, ty, qx, qy;
    LatLng q;
    dv_geo_to_hex2d(from, p, &fx, &fy);
    dv_hex2d_to_geo(from, fx + 0.01, fy, &q);
    dv_geo_to_hex2d(to, p, &tx, &ty);
    dv_geo_to_hex2d(to, &q, &qx, &qy);
    const double a = atan2(qy - ty, qx - tx) * (180.0 / M_PI) / 60.0;
    const double n = floor(a + 0.5);
    *ok = fabs(a - n) < 0.1;
    return (((int)n % 6) + 6) % 6;
}

static void dv_normalize(int *i, int *j, int *k) {
    CoordIJK c = {*i, *j, *k};
    _ijkNormalize(&c);
    *i = c.i; *j = c.j; *k = c.k;
}

static void oracle_derive_tables(void) {
    static const int IN_FACE[10][3] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {1, 1, 0},
                                       {1, 0, 1}, {0, 1, 1}, {2, 0, 0}, {0, 2, 0}, {0, 0, 2}};
    /* 1. res-0 lattice points of every face, merged into base cells */
    LatLng cen[200];
    DvView vw[200][5];
    int nv[200], nc = 0;
    for (int f = 0; f < 20; f++)
        for (int q = 0; q < 10; q++) {
            double x, y;
            LatLng g;
            dv_ijk_hex2d(IN_FACE[q][0], IN_FACE[q][1], IN_FACE[q][2], &x, &y);
            dv_hex2d_to_geo(f, x, y, &g);
            int c = 0;
            while (c < nc && dv_dist(&g, &cen[c]) > 1e-9) c++;
            if (c == nc) {
                if (nc == 200) DV_FAIL("too many res-0 points");
                cen[nc] = g;
                nv[nc++] = 0;
            }
            if (nv[c] == 5) DV_FAIL("a res-0 point seen by more than 5 faces");
            vw[c][nv[c]++] = (DvView){f, IN_FACE[q][0], IN_FACE[q][1], IN_FACE[q][2]};
        }
    if (nc != 122) DV_FAIL("expected 122 res-0 cells, got %d", nc);
    /* 2. numbered by latitude, north to south (selection sort; no two centres share a latitude) */
    int used[122] = {0};
    for (int b = 0; b < 122; b++) {
        int best = -1;
        for (int c = 0; c < 122; c++)
            if (!used[c] && (best < 0 || cen[c].lat > cen[best].lat)) best = c;
        used[best] = 1;
        dv_center[b] = cen[best];
        dv_nviews[b] = nv[best];
        for (int q = 0; q < nv[best]; q++) dv_views[b][q] = vw[best][q];
        if (b > 0 && !(dv_center[b - 1].lat - dv_center[b].lat > 1e-12)) DV_FAIL("latitude tie at base cell %d", b);
    }
    int npent = 0;
    for (int b = 0; b < 122; b++) {
        if (dv_nviews[b] == 5) npent++;
        else if (dv_nviews[b] != 1 && dv_nviews[b] != 2) DV_FAIL("base cell %d seen by %d faces", b, dv_nviews[b]);
    }
    if (npent != 12) DV_FAIL("expected 12 pentagons, got %d", npent);
    for (int f = 0; f < 20; f++) {
        dv_anti[f] = -1;
        for (int g = 0; g < 20; g++) {
            const double s = fabs(H3T_faceCenterPoint[f][0] + H3T_faceCenterPoint[g][0]) +
                             fabs(H3T_faceCenterPoint[f][1] + H3T_faceCenterPoint[g][1]) +
                             fabs(H3T_faceCenterPoint[f][2] + H3T_faceCenterPoint[g][2]);
            if (s < 1e-12) dv_anti[f] = g;
        }
        if (dv_anti[f] < 0) DV_FAIL("face %d has no antipodal face", f);
    }
    /* 3. home faces */
    int home[122][4];
    for (int b = 0; b < 61; b++) {
        const DvView *v = dv_views[b];
        if (dv_nviews[b] == 1) {
            home[b][0] = v[0].face; home[b][1] = v[0].i; home[b][2] = v[0].j; home[b][3] = v[0].k;
        } else if (dv_nviews[b] == 5) {
            int h = -1;
            for (int q = 0; q < 5; q++)
                if (v[q].i == 2 && (h < 0 || v[q].face < v[h].face)) h = q;
            if (h < 0) DV_FAIL("pentagon %d is nowhere at (2,0,0)", b);
            home[b][0] = v[h].face; home[b][1] = 2; home[b][2] = 0; home[b][3] = 0;
        } else {
            if (b > 58) DV_FAIL("no recalled home face for edge base cell %d", b);
            for (int q = 0; q < 4; q++) home[b][q] = ORC_recalled_home[b][q];
        }
        int seen = 0;
        for (int q = 0; q < dv_nviews[b]; q++)
            seen |= v[q].face == home[b][0] && v[q].i == home[b][1] && v[q].j == home[b][2] && v[q].k == home[b][3];
        if (!seen) DV_FAIL("home view of base cell %d is not one of its views", b);
        if (b <= 58)
            for (int q = 0; q < 4; q++)
                if (home[b][q] != ORC_recalled_home[b][q]) DV_FAIL("base cell %d: derived home differs from recalled", b);
    }
    for (int b = 61; b < 122; b++) {
        const int *m = home[121 - b];
        home[b][0] = dv_anti[m[0]]; home[b][1] = m[1]; home[b][2] = m[3]; home[b][3] = m[2];
        int seen = 0;
        for (int q = 0; q < dv_nviews[b]; q++) {
            const DvView *v = &dv_views[b][q];
            seen |= v->face == home[b][0] && v->i == home[b][1] && v->j == home[b][2] && v->k == home[b][3];
        }
        if (!seen) DV_FAIL("antipodal home of base cell %d is not one of its views", b);
    }
    for (int b = 0; b < 122; b++) {
        int *d = H3T_baseCellData[b];
        for (int q = 0; q < 4; q++) d[q] = home[b][q];
        d[4] = dv_nviews[b] == 5;
        d[5] = d[6] = 0;
        if (d[4]) {   /* cwOffsetPent: the faces that see the vertex at (0,2,0), ascending; none -> -1, -1 */
            int c[2] = {-1, -1}, m = 0;
            for (int q = 0; q < 5; q++)
                if (dv_views[b][q].j == 2) {
                    if (m == 2) DV_FAIL("pentagon %d: more than two cw-offset faces", b);
                    c[m++] = dv_views[b][q].face;
                }
            if (m == 2 && c[0] > c[1]) { int t = c[0]; c[0] = c[1]; c[1] = t; }
            d[5] = c[0];
            d[6] = c[1];
        }
    }
    for (int q = 0; q < 6; q++) {
        const int *r = ORC_recalled_cw[q];
        if (H3T_baseCellData[r[0]][5] != r[1] || H3T_baseCellData[r[0]][6] != r[2])
            DV_FAIL("cwOffsetPent[%d] differs from recalled", r[0]);
    }
    /* 4. pentagon rotations: clockwise order of the faces around the vertex in the home frame */
    static const int CYC_POS[7] = {-1, -1, 2, 3, 0, 4, 1};   /* digit -> position on the ccw 5-cycle I IJ J JK IK */
    static const int TARGET[5] = {3, 2, 6, 4, 5};            /* home frame sectors, clockwise from the home face's */
    for (int f = 0; f < 20; f++)
        for (int b = 0; b < 122; b++) dv_pent_rot[f][b] = -1;
    for (int b = 0; b < 122; b++) {
        if (dv_nviews[b] != 5) continue;
        const int hf = home[b][0];
        double px, py;
        dv_geo_to_hex2d(hf, &dv_center[b], &px, &py);
        double ang[5];
        for (int q = 0; q < 5; q++) {   /* clockwise angle from the home face's centre, seen from the vertex */
            const int f = dv_views[b][q].face;
            LatLng c = {H3T_faceCenterGeo[f][0], H3T_faceCenterGeo[f][1]};
            double cx, cy, hx, hy;
            dv_geo_to_hex2d(hf, &c, &cx, &cy);
            dv_hex2d_to_geo(hf, 0.0, 0.0, &c);
            dv_geo_to_hex2d(hf, &c, &hx, &hy);
            const double a0 = atan2(hy - py, hx - px), a = atan2(cy - py, cx - px);
            ang[q] = fmod(a0 - a + 4 * M_PI, 2 * M_PI);
            if (f == hf) ang[q] = 0.0;
        }
        for (int q = 0; q < 5; q++) {
            int rank = 0;
            for (int p = 0; p < 5; p++) rank += ang[p] < ang[q];
            const DvView *v = &dv_views[b][q];
            const int sector = v->i == 2 ? 3 : v->j == 2 ? 5 : 6;   /* digit from the vertex towards the face centre */
            dv_pent_rot[v->face][b] = ((CYC_POS[TARGET[rank]] - CYC_POS[sector]) % 5 + 5) % 5;
        }
    }
    /* 5. faceIjkBaseCells */
    for (int f = 0; f < 20; f++)
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                for (int k = 0; k < 3; k++) {
                    int a = i, c = j, e = k;
                    dv_normalize(&a, &c, &e);
                    double x, y, d0, d1;
                    LatLng g;
                    dv_ijk_hex2d(a, c, e, &x, &y);
                    dv_hex2d_to_geo(f, x, y, &g);
                    const int b = dv_nearest(&g, &d0, &d1);
                    if (d0 > 0.1 || d1 < 2 * d0) DV_FAIL("face %d (%d,%d,%d) is not near one base cell", f, a, c, e);
                    int rot, ok = 1;
                    if (dv_nviews[b] == 5) {
                        rot = dv_pent_rot[f][b];
                        if (rot < 0) DV_FAIL("face %d is not a view of pentagon %d", f, b);
                    } else if (home[b][0] == f) {
                        rot = 0;
                    } else {
                        /* measured where the two faces meet: the midpoint of their centres (the shared edge's
                         * midpoint for adjacent faces; far from both planes' centres the gnomonic distortion
                         * bends the axes off the lattice) */
                        const int hf = home[b][0];
                        Vec3d m = {H3T_faceCenterPoint[f][0] + H3T_faceCenterPoint[hf][0],
                                   H3T_faceCenterPoint[f][1] + H3T_faceCenterPoint[hf][1],
                                   H3T_faceCenterPoint[f][2] + H3T_faceCenterPoint[hf][2]};
                        const double nm = sqrt(m.x * m.x + m.y * m.y + m.z * m.z);
                        if (nm < 1.0) DV_FAIL("base cell %d: home face %d is not adjacent to face %d", b, hf, f);
                        LatLng mp = {asin(m.z / nm), atan2(m.y, m.x)};
                        rot = dv_rot(hf, f, &mp, &ok);
                        if (!ok) DV_FAIL("non-lattice rotation face %d -> %d at base cell %d", f, hf, b);
                    }
                    H3T_faceIjkBaseCells[f][i][j][k][0] = b;
                    H3T_faceIjkBaseCells[f][i][j][k][1] = rot;
                }
    for (int b = 0; b < 122; b++) {
        const int *h = home[b];
        const int *e = H3T_faceIjkBaseCells[h[0]][h[1]][h[2]][h[3]];
        if (e[0] != b || e[1] != 0) DV_FAIL("home entry of base cell %d is not (b, 0)", b);
    }
    /* 6. faceNeighbors: central, IJ, KI, JK */
    static const int QUAD[4][3] = {{0, 0, 0}, {2, 2, 0}, {2, 0, 2}, {0, 2, 2}};
    int nbr[20][4];
    for (int f = 0; f < 20; f++)
        for (int q = 1; q < 4; q++) {
            double x, y, d0, d1;
            LatLng g;
            dv_ijk_hex2d(QUAD[q][0], QUAD[q][1], QUAD[q][2], &x, &y);
            dv_hex2d_to_geo(f, x, y, &g);
            const int b = dv_nearest(&g, &d0, &d1);
            if (dv_nviews[b] != 1 || home[b][1] || home[b][2] || home[b][3])
                DV_FAIL("quadrant %d of face %d is not centred on a face", q, f);
            nbr[f][q] = home[b][0];
        }
    for (int f = 0; f < 20; f++) {
        int *o = H3T_faceNeighbors[f][0];
        o[0] = f; o[1] = o[2] = o[3] = o[4] = 0;
        for (int q = 1; q < 4; q++) {
            const int g = nbr[f][q];
            int back = -1;
            for (int p = 1; p < 4; p++)
                if (nbr[g][p] == f) {
                    if (back >= 0) DV_FAIL("faces %d and %d share two edges", f, g);
                    back = p;
                }
            if (back < 0) DV_FAIL("face adjacency %d -> %d is not symmetric", f, g);
            double x, y;
            LatLng mid;   /* the shared edge's midpoint: half way to the neighbour's centre lattice point */
            dv_ijk_hex2d(QUAD[q][0] / 2, QUAD[q][1] / 2, QUAD[q][2] / 2, &x, &y);
            dv_hex2d_to_geo(f, x, y, &mid);
            int ok;
            const int rot = dv_rot(g, f, &mid, &ok);
            if (!ok) DV_FAIL("non-lattice rotation face %d -> %d", f, g);
            o = H3T_faceNeighbors[f][q];
            o[0] = g; o[1] = QUAD[back][0]; o[2] = QUAD[back][1]; o[3] = QUAD[back][2]; o[4] = rot;
        }
    }
    /* discrete check of every neighbour entry: res-2 lattice points of g near the shared edge, located on f (overage
     * coordinates), map to their own coordinates under upstream's transform (_adjustOverageClassII at res 2) */
    for (int f = 0; f < 20; f++)
        for (int q = 1; q < 4; q++) {
            const int *o = H3T_faceNeighbors[f][q];
            const int g = o[0];
            int checked = 0;
            for (int i = 0; i <= 14; i++)
                for (int j = 0; j <= 14; j++)
                for (int s = 0; s < 3; s++) {
                    CoordIJK c = {s == 2 ? 0 : i, s == 1 ? 0 : (s == 2 ? i : j), s == 0 ? 0 : j};
                    _ijkNormalize(&c);
                    if (c.i + c.j + c.k > 14) continue;   /* inside g's triangle */
                    double x, y;
                    LatLng p;
                    dv_ijk_hex2d(c.i, c.j, c.k, &x, &y);
                    dv_hex2d_to_geo(g, x / 7.0, y / 7.0, &p);   /* res 2 (Class II): hex2d scaled by 7 */
                    double fx, fy;
                    dv_geo_to_hex2d(f, &p, &fx, &fy);
                    Vec2d v = {fx * 7.0, fy * 7.0};
                    CoordIJK h;
                    _hex2dToCoordIJK(&v, &h);
                    const int sum = h.i + h.j + h.k;
                    if (sum <= 14 || sum > 16) continue;   /* only points just over f's edge */
                    int quad = h.k > 0 ? (h.j > 0 ? 3 : 2) : 1;   /* the quadrant _adjustOverageClassII picks */
                    if (quad != q) continue;
                    for (int r = 0; r < o[4]; r++) _ijkRotate60ccw(&h);
                    h.i += o[1] * 7; h.j += o[2] * 7; h.k += o[3] * 7;
                    _ijkNormalize(&h);
                    if (h.i != c.i || h.j != c.j || h.k != c.k)
                        DV_FAIL("faceNeighbors[%d][%d]: res-2 point (%d,%d,%d) of face %d maps to (%d,%d,%d)", f, q, c.i,
                                c.j, c.k, g, h.i, h.j, h.k);
                    checked++;
                }
            if (checked < 3) DV_FAIL("faceNeighbors[%d][%d]: only %d points checked", f, q, checked);
        }
}

__attribute__((constructor)) static void oracle_tables_init(void) { oracle_derive_tables(); }

/* The oracle's derived tables, for the comparison with the product's generated ones (tests/test_h3_oracle.py).
 * Returns 0, or -1 with *err set when a derivation check failed. */
int oracle_tables(int *base_cell_data, int *face_ijk_base_cells, int *face_neighbors, const char **err) {
    memcpy(base_cell_data, H3T_baseCellData, sizeof H3T_baseCellData);
    memcpy(face_ijk_base_cells, H3T_faceIjkBaseCells, sizeof H3T_faceIjkBaseCells);
    memcpy(face_neighbors, H3T_faceNeighbors, sizeof H3T_faceNeighbors);
    *err = ORC_derive_error;
    return ORC_derive_error ? -1 : 0;
}
