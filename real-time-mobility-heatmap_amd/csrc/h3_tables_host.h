// Host construction of hm::H3Tables from the generated tables (h3_tables.inc must be included first).
#pragma once
#include <cmath>
#include <cstring>

#include "h3_device.h"

// glibc's sincos/acos/atan2/tan tables (glibc_libm.inc), host copy (the device copy is mobheat.hip's g_glm)
static const hm::glm::Tables hm_glm_host = {GLM_TABLE_INIT};

static hm::H3Tables hm_make_tables() {
    hm::H3Tables T;
    T.glm = &hm_glm_host;
    const long double ap7 = 0.333473172251832115336090755351601070065900389L;   // M_AP7_ROT_RADS
    for (int f = 0; f < 20; f++) {
        T.faceCenterGeo[f][0] = H3T_faceCenterGeo[f][0];
        T.faceCenterGeo[f][1] = H3T_faceCenterGeo[f][1];
        for (int c = 0; c < 3; c++) {
            T.faceCenterPoint[f][c] = H3T_faceCenterPoint[f][c];
            T.faceCenterPointF[f][c] = (float)H3T_faceCenterPoint[f][c];
        }
        T.faceAxesAz0[f] = H3T_faceAxesAzRadsCII[f][0];
        // upstream evaluates cos/sin(p1->lat) per call with the host libm; identical values
        volatile double lat = H3T_faceCenterGeo[f][0];
        sincos(lat, &T.faceSinLat[f], &T.faceCosLat[f]);   // (the pair gcc fuses; equal to sin/cos for all 20 here)
        // fast-path gnomonic axes (h3_device.h, latLngToCellFast), in x87 extended precision
        const long double phi = H3T_faceCenterGeo[f][0], lam = H3T_faceCenterGeo[f][1], az0 = H3T_faceAxesAzRadsCII[f][0];
        const long double n[3] = {-sinl(phi) * cosl(lam), -sinl(phi) * sinl(lam), cosl(phi)};
        const long double e[3] = {-sinl(lam), cosl(lam), 0.0L};
        long double ux[3], uy[3];
        for (int k = 0; k < 3; k++) {
            ux[k] = cosl(az0) * n[k] + sinl(az0) * e[k];
            uy[k] = sinl(az0) * n[k] - cosl(az0) * e[k];
        }
        for (int k = 0; k < 3; k++) {
            T.fastU[0][f][0][k] = (double)ux[k];
            T.fastU[0][f][1][k] = (double)uy[k];
            T.fastU[1][f][0][k] = (double)(cosl(ap7) * ux[k] + sinl(ap7) * uy[k]);
            T.fastU[1][f][1][k] = (double)(cosl(ap7) * uy[k] - sinl(ap7) * ux[k]);
        }
    }
    for (int r = 0; r < 16; r++) {
        T.fastScale[r] = (double)((long double)HM_INV_RES0_U_GNOMONIC * powl(sqrtl(7.0L), r));
        T.fastTauS[r] = T.fastScale[r] * 32.0 * 0x1p-52 * 8.0;
    }
    memcpy(T.faceIjkBaseCells, H3T_faceIjkBaseCells, sizeof(T.faceIjkBaseCells));
    memcpy(T.baseCellData, H3T_baseCellData, sizeof(T.baseCellData));
    for (int f = 0; f < 20; f++)
        for (int q = 0; q < 27; q++) {
            const int bc = H3T_faceIjkBaseCells[f][q / 9][(q / 3) % 3][q % 3][0], rots = H3T_faceIjkBaseCells[f][q / 9][(q / 3) % 3][q % 3][1];
            if (bc < 0 || bc >= 122 || rots < 0 || rots > 5) abort();
            T.fijkPacked[f * 27 + q] = (unsigned short)(bc | rots << 8);
        }
    for (int b = 0; b < 122; b++) {
        const int *d = H3T_baseCellData[b];
        if (d[5] < -1 || d[5] > 19 || d[6] < -1 || d[6] > 19) abort();
        T.bcdPacked[b] = (d[4] ? 1u : 0u) | (unsigned)(d[5] + 1) << 8 | (unsigned)(d[6] + 1) << 16;
    }
    memcpy(T.faceNeighbors, H3T_faceNeighbors, sizeof(T.faceNeighbors));
    for (int a = 0; a < 49; a++)
        for (int b = 0; b < 49; b++) {
            T.ap7Quad[a * 49 + b] = hm::ap7TableEntry(a, b, 4);
            if (a < 7 && b < 7) T.ap7Pair[a * 7 + b] = (unsigned short)hm::ap7TableEntry(a, b, 2);
        }
    for (int a = 0; a < 20; a++)
        for (int b = 0; b < 20; b++) {
            signed char d = a == b ? 0 : -1;
            for (int dir = 1; dir <= 3; dir++)
                if (H3T_faceNeighbors[a][dir][0] == b) d = (signed char)dir;
            T.adjacentFaceDir[a][b] = d;
        }
    const long double sqrt3_2 = 0.8660254037844386467637231707529361834714L;   // M_SQRT3_2
    for (int r = 0; r < 17; r++) {
        int m = 2;
        for (int q = 0; q < r; q += 2) m *= 7;
        volatile long double three = 3.0L;   // (3.0 * M_SQRT3_2) * maxDim, both in long double, as upstream
        T.edgeY[r] = (double)((three * sqrt3_2) * (long double)m);
    }
    return T;
}
