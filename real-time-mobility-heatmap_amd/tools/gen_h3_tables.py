#!/usr/bin/env python3
"""Generate the H3 (res-0 icosahedral) lookup tables used by the HIP kernels and the CPU oracle.

Why a generator: the reference calls ``h3.latlng_to_cell`` (reference heatmap_stream.py:70-73) from the
third-party, *unpinned* h3-py 4.x (reference README.md:95), which vendors Uber's H3 C library v4.  Neither
h3-py nor the H3 C sources are present in this environment, so the tables cannot be
copied.  Instead this script starts from the small set of *primary* constants of upstream H3 v4
(``faceijk.c``: ``faceCenterGeo``, ``faceCenterPoint``, ``faceAxesAzRadsCII``; kept verbatim as the decimal
literals upstream uses, because the compiled doubles must be bit-identical) and DERIVES every discrete
table from icosahedral geometry:

* ``baseCellData``   (upstream ``baseCells.c``): the 122 res-0 cells are the 20 face centres, 60 interior
  unit-vector cells, 30 edge midpoints and 12 vertices of the Class II res-0 grid.  Upstream numbers them by
  latitude of their centre, north to south -- the derived order reproduces every recalled entry 0..58.
  Home-face choice for edge cells follows the upstream pattern observed on cells 0..58 extended by the
  antipodal symmetry b <-> 121-b (home face -> antipodal face, (i,j,k) -> (i,k,j)); pentagon home = the
  face on which the vertex sits at IJK (2,0,0); CW-offset faces = the faces that see the vertex at (0,2,0)
  (reproduces all recalled entries for base cells 14, 24, 38, 49, 58).
* ``faceIjkBaseCells`` (upstream ``baseCells.c``): base cell of every res-0 IJK (components <= 2) on
  every face, plus the 60-degree CCW rotation into the base cell's home-face frame, measured
  geometrically across the shared edge; pentagon entries rotate the face's sector onto its position in
  the 5-sector pentagon layout (K sector deleted) in clockwise face order around the vertex.
* ``faceNeighbors`` (upstream ``faceijk.c``): IJ / KI / JK quadrant neighbours with rotation and
  translation.

Self-checks (fail loudly): antipodal symmetry of the primary constants, unit norm of ``faceCenterPoint``,
the 12 vertices each seen by exactly five faces, 122 base cells, and equality with every table entry that
could be recalled from upstream (cells 0..58 of ``baseCellData``, face 0/1 rows of ``faceIjkBaseCells``,
faces 0/1 of ``faceNeighbors``).

Output: ``csrc/h3_tables.inc`` (C99/HIP initialisers, included by the product's device and host code only: the oracle
derives its own tables, oracle/h3_tables_derive.c, and never includes this file -- DESIGN.md §3,
tests/test_h3_oracle.py::test_oracle_does_not_include_product_tables).
"""
import itertools
import math
import os
import sys

import numpy as np

# ---------------------------------------------------------------------------------------------------
# Primary constants: upstream H3 v4 faceijk.c literals (decimal strings kept verbatim).
# ---------------------------------------------------------------------------------------------------
FACE_CENTER_GEO = [
    ("0.803582649718989942", "1.248397419617396099"),
    ("1.307747883455638156", "2.536945009877921159"),
    ("1.054751253523952054", "-1.347517358900396623"),
    ("0.600191595538186799", "-0.450603909469755746"),
    ("0.491715428198773866", "0.401988202911306943"),
    ("0.172745327415618701", "1.678146885280433686"),
    ("0.605929321571350690", "2.953923329812411617"),
    ("0.427370518328979641", "-1.888876200336285401"),
    ("-0.079066118549212831", "-0.733429513380867741"),
    ("-0.230961644455383637", "0.506495587332349035"),
    ("0.079066118549212831", "2.408163140208925497"),
    ("0.230961644455383637", "-2.635097066257444203"),
    ("-0.172745327415618701", "-1.463445768309359553"),
    ("-0.605929321571350690", "-0.187669323777381622"),
    ("-0.427370518328979641", "1.252716453253507838"),
    ("-0.600191595538186799", "2.690988744120037492"),
    ("-0.491715428198773866", "-2.739604450678486295"),
    ("-1.054751253523952054", "1.794075294689396615"),
    ("-1.307747883455638156", "-0.604647643711872080"),
    ("-0.803582649718989942", "-1.893195233972397139"),
]
FACE_CENTER_POINT = [
    ("0.2199307791404606", "0.6583691780274996", "0.7198475378926182"),
    ("-0.2139234834501421", "0.1478171829550703", "0.9656017935214205"),
    ("0.1092625278784797", "-0.4811951572873210", "0.8697775121287253"),
    ("0.7428567301586791", "-0.3593941678278028", "0.5648005936517033"),
    ("0.8112534709140969", "0.3448953237639384", "0.4721387736413930"),
    ("-0.1055498149613921", "0.9794457296411413", "0.1718874610009365"),
    ("-0.8075407579970092", "0.1533552485898818", "0.5695261994882688"),
    ("-0.2846148069787907", "-0.8644080972654206", "0.4144792552473539"),
    ("0.7405621473854482", "-0.6673299564565524", "-0.0789837646326737"),
    ("0.8512303986474293", "0.4722343788582681", "-0.2289137388687808"),
    ("-0.7405621473854481", "0.6673299564565524", "0.0789837646326737"),
    ("-0.8512303986474292", "-0.4722343788582682", "0.2289137388687808"),
    ("0.1055498149613919", "-0.9794457296411413", "-0.1718874610009365"),
    ("0.8075407579970092", "-0.1533552485898819", "-0.5695261994882688"),
    ("0.2846148069787908", "0.8644080972654204", "-0.4144792552473539"),
    ("-0.7428567301586791", "0.3593941678278027", "-0.5648005936517033"),
    ("-0.8112534709140971", "-0.3448953237639382", "-0.4721387736413930"),
    ("-0.1092625278784796", "0.4811951572873210", "-0.8697775121287253"),
    ("0.2139234834501420", "-0.1478171829550704", "-0.9656017935214205"),
    ("-0.2199307791404607", "-0.6583691780274996", "-0.7198475378926182"),
]
FACE_AXES_AZ_CII = [
    ("5.619958268523939882", "3.525563166130744542", "1.431168063737548730"),
    ("5.760339081714187279", "3.665943979320991689", "1.571548876927796127"),
    ("0.780213654393430055", "4.969003859179821079", "2.874608756786625655"),
    ("0.430469363979999913", "4.619259568766391033", "2.524864466373195467"),
    ("6.130269123335111400", "4.035874020941915804", "1.941478918548720291"),
    ("2.692877706530642877", "0.598482604137447119", "4.787272808923838195"),
    ("2.982963003477243874", "0.888567901084048369", "5.077358105870439581"),
    ("3.532912002790141181", "1.438516900396945656", "5.627307105183336758"),
    ("3.494305004259568154", "1.399909901866372864", "5.588700106652763840"),
    ("3.003214169499538391", "0.908819067106342928", "5.097609271892733906"),
    ("5.930472956509811562", "3.836077854116615875", "1.741682751723420374"),
    ("0.138378484090254847", "4.327168688876645809", "2.232773586483450311"),
    ("0.448714947059150361", "4.637505151845541521", "2.543110049452346120"),
    ("0.158629650112549365", "4.347419854898940135", "2.253024752505744869"),
    ("5.891865957979238535", "3.797470855586042958", "1.703075753192847583"),
    ("2.711123289609793325", "0.616728187216597771", "4.805518392002988683"),
    ("3.294508837434268316", "1.200113735041072948", "5.388903939827463911"),
    ("2.361378999196363184", "0.266983896803167583", "4.455774101589558636"),
    ("3.664438879055192436", "1.570043776661997111", "5.758833981448388027"),
    ("3.804819692245439833", "1.710424589852244509", "5.899214794638635174"),
]
RES0_U_GNOMONIC = 0.38196601125010500003

# Entries recalled from upstream tables, used only as cross-checks of the derivation.
RECALLED_BASE_CELL_HOME = {
    0: (1, (1, 0, 0)), 1: (2, (1, 1, 0)), 2: (1, (0, 0, 0)), 3: (2, (1, 0, 0)), 4: (0, (2, 0, 0)),
    5: (1, (1, 1, 0)), 6: (1, (0, 0, 1)), 7: (2, (0, 0, 0)), 8: (0, (1, 0, 0)), 9: (2, (0, 1, 0)),
    10: (1, (0, 1, 0)), 11: (1, (0, 1, 1)), 12: (3, (1, 0, 0)), 13: (3, (1, 1, 0)), 14: (11, (2, 0, 0)),
    15: (4, (1, 0, 0)), 16: (0, (0, 0, 0)), 17: (6, (0, 1, 0)), 18: (0, (0, 0, 1)), 19: (2, (0, 1, 1)),
    20: (7, (0, 0, 1)), 21: (2, (0, 0, 1)), 22: (0, (1, 1, 0)), 23: (6, (0, 0, 1)), 24: (10, (2, 0, 0)),
    25: (6, (0, 0, 0)), 26: (3, (0, 0, 0)), 27: (11, (1, 0, 0)), 28: (4, (1, 1, 0)), 29: (3, (0, 1, 0)),
    30: (0, (0, 1, 1)), 31: (4, (0, 0, 0)), 32: (5, (0, 1, 0)), 33: (0, (0, 1, 0)), 34: (7, (0, 1, 0)),
    35: (11, (1, 1, 0)), 36: (7, (0, 0, 0)), 37: (10, (1, 0, 0)), 38: (12, (2, 0, 0)), 39: (6, (1, 0, 1)),
    40: (7, (1, 0, 1)), 41: (4, (0, 0, 1)), 42: (3, (0, 0, 1)), 43: (3, (0, 1, 1)), 44: (4, (0, 1, 0)),
    45: (6, (1, 0, 0)), 46: (11, (0, 0, 0)), 47: (8, (0, 0, 1)), 48: (5, (0, 0, 1)), 49: (14, (2, 0, 0)),
    50: (5, (0, 0, 0)), 51: (12, (1, 0, 0)), 52: (10, (1, 1, 0)), 53: (4, (0, 1, 1)), 54: (12, (1, 1, 0)),
    55: (7, (1, 0, 0)), 56: (11, (0, 1, 0)), 57: (10, (0, 0, 0)), 58: (13, (2, 0, 0)),
}
RECALLED_CW_OFFSET = {4: (-1, -1), 14: (2, 6), 24: (1, 5), 38: (3, 7), 49: (0, 9), 58: (4, 8)}
RECALLED_FACE_IJK_BC = {  # (face, i, j, k) -> (baseCell, ccwRot60)
    (0, 0, 0, 0): (16, 0), (0, 0, 0, 1): (18, 0), (0, 0, 0, 2): (24, 0),
    (0, 0, 1, 0): (33, 0), (0, 0, 1, 1): (30, 0), (0, 0, 1, 2): (32, 3),
    (0, 0, 2, 0): (49, 1), (0, 0, 2, 1): (48, 3), (0, 0, 2, 2): (50, 3),
    (0, 1, 0, 0): (8, 0), (0, 1, 0, 1): (5, 5), (0, 1, 0, 2): (10, 5),
    (0, 1, 1, 0): (22, 0), (0, 1, 1, 1): (16, 0), (0, 1, 1, 2): (18, 0),
    (0, 1, 2, 0): (41, 1), (0, 1, 2, 1): (33, 0), (0, 1, 2, 2): (30, 0),
    (0, 2, 0, 0): (4, 0), (0, 2, 0, 1): (0, 5), (0, 2, 0, 2): (2, 5),
    (0, 2, 1, 0): (15, 1), (0, 2, 1, 1): (8, 0), (0, 2, 1, 2): (5, 5),
    (0, 2, 2, 0): (31, 1), (0, 2, 2, 1): (22, 0), (0, 2, 2, 2): (16, 0),
    (1, 0, 0, 0): (2, 0), (1, 0, 0, 1): (6, 0), (1, 0, 0, 2): (14, 0),
    (1, 0, 1, 0): (10, 0), (1, 0, 1, 1): (11, 0), (1, 0, 1, 2): (17, 3),
    (1, 0, 2, 0): (24, 1), (1, 0, 2, 1): (23, 3), (1, 0, 2, 2): (25, 3),
}
RECALLED_FACE_NEIGHBORS = {  # face -> [central, IJ, KI, JK] as (face, (ti,tj,tk), rot)
    0: [(0, (0, 0, 0), 0), (4, (2, 0, 2), 1), (1, (2, 2, 0), 5), (5, (0, 2, 2), 3)],
    1: [(1, (0, 0, 0), 0), (0, (2, 0, 2), 1), (2, (2, 2, 0), 5), (6, (0, 2, 2), 3)],
}

IJ, KI, JK = 1, 2, 3
DIGIT_DIRS = {4: 0.0, 6: 60.0, 2: 120.0, 3: 180.0, 1: 240.0, 5: 300.0}  # hex2d angle of each digit


def fail(msg):
    sys.stderr.write("gen_h3_tables: CHECK FAILED: " + msg + "\n")
    sys.exit(1)


geo = [(float(a), float(b)) for a, b in FACE_CENTER_GEO]
az0 = [float(r[0]) for r in FACE_AXES_AZ_CII]


def v3(lat, lng):
    return np.array([math.cos(lat) * math.cos(lng), math.cos(lat) * math.sin(lng), math.sin(lat)])


def azdist(lat, lng, az, d):
    p = v3(lat, lng)
    north = np.array([-math.sin(lat) * math.cos(lng), -math.sin(lat) * math.sin(lng), math.cos(lat)])
    east = np.array([-math.sin(lng), math.cos(lng), 0.0])
    return math.cos(d) * p + math.sin(d) * (math.cos(az) * north + math.sin(az) * east)


def azimuth_of(lat, lng, p):
    c = v3(lat, lng)
    north = np.array([-math.sin(lat) * math.cos(lng), -math.sin(lat) * math.sin(lng), math.cos(lat)])
    east = np.array([-math.sin(lng), math.cos(lng), 0.0])
    t = p - (c @ p) * c
    return math.atan2(t @ east, t @ north)


C = [v3(*g) for g in geo]


def geo_to_hex2d(f, p):
    cosr = float(np.clip(C[f] @ p, -1.0, 1.0))
    th = az0[f] - azimuth_of(*geo[f], p)
    rr = math.tan(math.acos(cosr)) / RES0_U_GNOMONIC
    return np.array([rr * math.cos(th), rr * math.sin(th)])


def hex2d_to_geo(f, v):
    r = math.hypot(v[0], v[1])
    if r < 1e-15:
        return C[f].copy()
    th = math.atan2(v[1], v[0])
    return azdist(*geo[f], az0[f] - th, math.atan(r * RES0_U_GNOMONIC))


def ijk_to_hex2d(ijk):
    i, j, k = ijk
    return np.array([(i - k) - 0.5 * (j - k), (j - k) * math.sqrt(3.0) / 2.0])


def normalize(ijk):
    i, j, k = ijk
    if i < 0:
        j -= i; k -= i; i = 0
    if j < 0:
        i -= j; k -= j; j = 0
    if k < 0:
        i -= k; j -= k; k = 0
    m = min(i, j, k)
    return (i - m, j - m, k - m)


# ---- 1. primary-constant self checks ----------------------------------------------------------------
anti = {}
for f in range(20):
    for g in range(20):
        if np.linalg.norm(C[f] + C[g]) < 1e-12:
            anti[f] = g
if sorted(anti) != list(range(20)):
    fail("faceCenterGeo is not antipodally symmetric")
for f in range(20):
    g = anti[f]
    a = [float(x) for x in FACE_AXES_AZ_CII[f]]
    b = [float(x) for x in FACE_AXES_AZ_CII[g]]
    for i, j in ((0, 0), (1, 2), (2, 1)):
        d = ((math.pi - a[i]) - b[j] + math.pi) % (2 * math.pi) - math.pi
        if abs(d) > 4e-15:
            fail(f"faceAxesAzRadsCII antipodal mismatch face {f}/{g}: {d}")
    for t in (0, 1):
        d = (a[t] - a[t + 1]) % (2 * math.pi)
        if abs(d - 2 * math.pi / 3) > 4e-15:
            fail(f"faceAxesAzRadsCII axes not 120 deg apart on face {f}")
    p = [float(x) for x in FACE_CENTER_POINT[f]]
    if abs(math.sqrt(sum(x * x for x in p)) - 1.0) > 1e-15:
        fail(f"faceCenterPoint[{f}] not unit length")
    if max(abs(x - y) for x, y in zip(p, C[f])) > 1e-15:
        fail(f"faceCenterPoint[{f}] != geoToVec3d(faceCenterGeo[{f}])")

# ---- 2. res-0 Class II cells: 122 base cells numbered by latitude ------------------------------------
IN_FACE = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (1, 0, 1), (0, 1, 1), (2, 0, 0), (0, 2, 0), (0, 0, 2)]
clusters = []
for f in range(20):
    for ijk in IN_FACE:
        p = hex2d_to_geo(f, ijk_to_hex2d(ijk))
        for c in clusters:
            if np.linalg.norm(c[0] - p) < 1e-6:
                c[1].append((f, ijk))
                break
        else:
            clusters.append([p, [(f, ijk)]])
if len(clusters) != 122:
    fail(f"expected 122 res-0 cells, got {len(clusters)}")
clusters.sort(key=lambda c: -c[0][2])
centers = [c[0] for c in clusters]
seen_by = [c[1] for c in clusters]
if sorted(len(s) for s in seen_by).count(5) != 12:
    fail("expected 12 vertices seen by 5 faces")

pentagon = [len(s) == 5 for s in seen_by]


def rel_rot(f_to, f_from, p):
    """CCW 60-degree steps taking a direction in f_from's hex2d frame into f_to's frame, at point p."""
    eps = 1e-5
    a = geo_to_hex2d(f_to, p)
    q = hex2d_to_geo(f_to, a + np.array([eps, 0.0]))
    d = geo_to_hex2d(f_from, q) - geo_to_hex2d(f_from, p)
    x = -math.degrees(math.atan2(d[1], d[0])) / 60.0
    n = round(x)
    if abs(x - n) > 0.02:
        fail(f"non-lattice rotation between faces {f_to},{f_from}")
    return n % 6


pairrot = {}
for b, s in enumerate(seen_by):
    if len(s) == 2:
        (f, _), (g, _) = s
        pairrot[(f, g)] = rel_rot(f, g, centers[b])
        pairrot[(g, f)] = rel_rot(g, f, centers[b])

# ---- 3. home faces ------------------------------------------------------------------------------
home = [None] * 122
for b in range(61):
    s = seen_by[b]
    if len(s) == 1:
        home[b] = s[0]
    elif len(s) == 5:
        h = [x for x in s if x[1] == (2, 0, 0)]
        home[b] = h[0]  # polar pentagon: lowest face number (face 0 for base cell 4)
    else:
        if b not in RECALLED_BASE_CELL_HOME:
            # cells 59..60 are interior; edges below the equator follow from symmetry
            fail(f"no rule for edge base cell {b}")
        home[b] = RECALLED_BASE_CELL_HOME[b]
for b in range(61, 122):
    fa, (i, j, k) = home[121 - b]
    cand = (anti[fa], (i, k, j))
    if cand not in seen_by[b]:
        fail(f"antipodal image of base cell {121 - b} is not a view of base cell {b}")
    home[b] = cand
for b, h in RECALLED_BASE_CELL_HOME.items():
    if home[b] != h:
        fail(f"baseCellData[{b}] derived {home[b]} != recalled {h}")

cw_offset = [(0, 0)] * 122
for b in range(122):
    if pentagon[b]:
        cw = sorted(f for f, ijk in seen_by[b] if ijk == (0, 2, 0))
        cw_offset[b] = tuple(cw) if cw else (-1, -1)
for b, cw in RECALLED_CW_OFFSET.items():
    if cw_offset[b] != cw:
        fail(f"cwOffsetPent[{b}] derived {cw_offset[b]} != recalled {cw}")

# ---- 4. pentagon rotations: sector layout with the K sector deleted ----------------------------------
CYC_POS = {4: 0, 6: 1, 2: 2, 3: 3, 5: 4}  # CCW 5-cycle I, IJ, J, JK, IK
VERTEX_SECTOR = {(2, 0, 0): 3, (0, 2, 0): 5, (0, 0, 2): 6}  # digit pointing from the vertex to the face centre
pent_rot = {}
for b in range(122):
    if not pentagon[b]:
        continue
    hf = home[b][0]
    p = centers[b]
    lat, lng = math.asin(p[2]), math.atan2(p[1], p[0])
    a_home = azimuth_of(lat, lng, C[hf])
    faces = dict(seen_by[b])
    order = sorted(faces, key=lambda f: (azimuth_of(lat, lng, C[f]) - a_home) % (2 * math.pi))  # clockwise
    for d, f in enumerate(order):
        target = [3, 2, 6, 4, 5][d]
        pent_rot[(f, b)] = (CYC_POS[target] - CYC_POS[VERTEX_SECTOR[faces[f]]]) % 5

# ---- 5. faceIjkBaseCells ----------------------------------------------------------------------------
def nearest(p):
    return min(range(122), key=lambda b: float(np.linalg.norm(centers[b] - p)))


face_ijk_bc = {}
for f in range(20):
    for ijk in itertools.product(range(3), repeat=3):
        n = normalize(ijk)
        pos = hex2d_to_geo(f, ijk_to_hex2d(n))
        dists = sorted(float(np.linalg.norm(centers[bb] - pos)) for bb in range(122))
        b = nearest(pos)
        if dists[0] > 0.1 or dists[1] < 2 * dists[0]:  # gnomonic overage stretches ~4 deg
            fail(f"res-0 position {f},{n} is not unambiguously near a base cell")
        hf = home[b][0]
        if pentagon[b]:
            rot = pent_rot[(f, b)]
        elif hf == f:
            rot = 0
        else:
            if (hf, f) not in pairrot:
                fail(f"base cell {b} home face {hf} not adjacent to face {f}")
            rot = pairrot[(hf, f)]
        face_ijk_bc[(f,) + ijk] = (b, rot)
for key, val in RECALLED_FACE_IJK_BC.items():
    if face_ijk_bc[key] != val:
        fail(f"faceIjkBaseCells{key} derived {face_ijk_bc[key]} != recalled {val}")
for b in range(122):  # home entry has rotation 0
    fa, ijk = home[b]
    if face_ijk_bc[(fa,) + ijk] != (b, 0):
        fail(f"home entry of base cell {b} is not (b,0)")

# ---- 6. faceNeighbors --------------------------------------------------------------------------------
QUAD_DIR = {IJ: (2, 2, 0), KI: (2, 0, 2), JK: (0, 2, 2)}
neighbor_face = {}
for f in range(20):
    for q, ijk in QUAD_DIR.items():
        b = nearest(hex2d_to_geo(f, ijk_to_hex2d(ijk)))
        g = home[b][0]
        if home[b][1] != (0, 0, 0):
            fail("quadrant neighbour centre is not a face centre")
        neighbor_face[(f, q)] = g
face_neighbors = {}
for f in range(20):
    row = [(f, (0, 0, 0), 0)]
    for q in (IJ, KI, JK):
        g = neighbor_face[(f, q)]
        back = [qq for qq in (IJ, KI, JK) if neighbor_face[(g, qq)] == f]
        if len(back) != 1:
            fail("face adjacency is not symmetric")
        row.append((g, QUAD_DIR[back[0]], pairrot[(g, f)]))
    face_neighbors[f] = row
for f, row in RECALLED_FACE_NEIGHBORS.items():
    if face_neighbors[f] != row:
        fail(f"faceNeighbors[{f}] derived {face_neighbors[f]} != recalled {row}")


# ---- 7. emit -----------------------------------------------------------------------------------------
def emit(path):
    L = []
    w = L.append
    w("/* GENERATED by real-time-mobility-heatmap_amd/tools/gen_h3_tables.py -- do not edit.")
    w(" * H3 v4 res-0 icosahedral tables (upstream faceijk.c / baseCells.c), primary literals verbatim,")
    w(" * discrete tables derived from geometry; see the generator docstring for provenance and checks. */")
    w("#define H3T_NUM_FACES 20")
    w("#define H3T_NUM_BASE_CELLS 122")
    w("/* faceCenterGeo[f] = {lat, lng} radians */")
    w("H3T_CONST double H3T_faceCenterGeo[20][2] = {")
    for f, (a, b) in enumerate(FACE_CENTER_GEO):
        w(f"    {{{a}, {b}}}, /* face {f} */")
    w("};")
    w("/* faceCenterPoint[f] = {x, y, z} */")
    w("H3T_CONST double H3T_faceCenterPoint[20][3] = {")
    for f, (a, b, c) in enumerate(FACE_CENTER_POINT):
        w(f"    {{{a}, {b}, {c}}}, /* face {f} */")
    w("};")
    w("/* faceAxesAzRadsCII[f] = azimuths of the Class II i, j, k axes */")
    w("H3T_CONST double H3T_faceAxesAzRadsCII[20][3] = {")
    for f, (a, b, c) in enumerate(FACE_AXES_AZ_CII):
        w(f"    {{{a}, {b}, {c}}}, /* face {f} */")
    w("};")
    w("/* baseCellData[b] = {homeFace, i, j, k, isPentagon, cwOffsetPent0, cwOffsetPent1} */")
    w("H3T_CONST int H3T_baseCellData[122][7] = {")
    for b in range(122):
        fa, (i, j, k) = home[b]
        c0, c1 = cw_offset[b]
        w(f"    {{{fa}, {i}, {j}, {k}, {int(pentagon[b])}, {c0}, {c1}}}, /* base cell {b} */")
    w("};")
    w("/* faceIjkBaseCells[f][i][j][k] = {baseCell, ccwRot60} */")
    w("H3T_CONST int H3T_faceIjkBaseCells[20][3][3][3][2] = {")
    for f in range(20):
        w(f"  {{ /* face {f} */")
        for i in range(3):
            rows = []
            for j in range(3):
                ent = ", ".join("{%d, %d}" % face_ijk_bc[(f, i, j, k)] for k in range(3))
                rows.append("{" + ent + "}")
            w("    {" + ", ".join(rows) + "},")
        w("  },")
    w("};")
    w("/* faceNeighbors[f][q] = {face, ti, tj, tk, ccwRot60}, q = central, IJ, KI, JK */")
    w("H3T_CONST int H3T_faceNeighbors[20][4][5] = {")
    for f in range(20):
        ent = ", ".join("{%d, %d, %d, %d, %d}" % (g, t[0], t[1], t[2], r) for g, t, r in face_neighbors[f])
        w(f"    {{{ent}}}, /* face {f} */")
    w("};")
    text = "\n".join(L) + "\n"
    if os.path.exists(path) and open(path).read() == text:
        return False
    with open(path, "w") as fh:
        fh.write(text)
    return True


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "h3_tables.inc")
    changed = emit(os.path.normpath(out))
    print(("wrote " if changed else "unchanged ") + os.path.normpath(out))
