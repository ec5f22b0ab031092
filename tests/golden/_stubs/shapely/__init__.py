"""Exact-rational model of the three shapely/GEOS calls on ap_gym's LIDAR path.

TEST INFRASTRUCTURE (build container only). shapely/GEOS is not installed and cannot be, so the
golden LIDAR fixtures are produced by running the reference's own lidar_localization2d.py with
this module standing in for shapely.  It is a MODEL of GEOS (OverlayNG, non-strict mode), not
GEOS: the fixtures pin the reference's Python control flow (RNG draw order, move/slide, obs,
loss, TimeLimit, SyncVectorEnv autoreset) and the repo's restatements against one another, while
the GEOS semantics themselves stay "parity unpinned" (DESIGN.md §Oracle).

Call sites modelled (ap_gym/envs/lidar_localization2d.py):
  :288-290  shapely.union_all([shapely.box(x, y, x+1, y+1) ...])   -> closed union U of cells
  :500-501  shapely.LineString([pos, target]).intersection(U)       -> typed result
Semantics assumed (GEOS >= 3.9 OverlayNG, floating precision model):
  (1) union_all keeps every lattice point on the boundary of U as a ring vertex, so boundary edges
      are unit segments;
  (2) the line is noded at every intersection with a boundary edge (crossings, lattice vertices on
      the line, endpoints of collinear overlaps); every noded piece inside closed U is emitted as
      its own LineString, in the input line's direction (LineBuilder.addResultLines / toLine);
  (3) a node on the boundary with no adjacent result piece is emitted as a Point
      (IntersectionPointBuilder, non-strict mode);
  (4) results are assembled by GeometryFactory.buildGeometry: one type -> single or Multi*, mixed
      points and lines -> GeometryCollection; nothing -> LINESTRING EMPTY;
  (5) a proper crossing's coordinate is computed by algorithm::Intersection::intersection (the
      midpoint-conditioned homogeneous formula) in IEEE double without FMA; endpoints and
      lattice vertices are exact.
This module deliberately uses a different algorithm (brute force over all boundary edges, exact
fractions) from the C oracle (sorted breakpoints) and the HIP kernel (DDA walk with filtered
predicates), so agreement between the three is evidence, not tautology.
"""

from __future__ import annotations

from fractions import Fraction as Fr
from math import floor

__all__ = [
    "box",
    "union_all",
    "LineString",
    "Point",
    "MultiPoint",
    "MultiLineString",
    "GeometryCollection",
]


class _Geom:
    is_empty = False


class Point(_Geom):
    def __init__(self, xy):
        self._xy = (float(xy[0]), float(xy[1]))

    @property
    def xy(self):
        return ([self._xy[0]], [self._xy[1]])


class MultiPoint(_Geom):
    def __init__(self, pts):
        self.geoms = list(pts)


class MultiLineString(_Geom):
    def __init__(self, lines):
        self.geoms = list(lines)


class GeometryCollection(_Geom):
    def __init__(self, geoms):
        self.geoms = list(geoms)
        self.is_empty = len(self.geoms) == 0


class _Box(_Geom):
    def __init__(self, x0, y0, x1, y1):
        assert x1 - x0 == 1 and y1 - y0 == 1, "only unit boxes are modelled"
        self.cell = (int(x0), int(y0))


class _CellUnion(_Geom):
    def __init__(self, cells):
        self.cells = frozenset(cells)
        self._edges = None

    def occ(self, cx, cy):
        return (cx, cy) in self.cells

    def boundary_edges(self):
        """Unit boundary edges keyed by their first vertex: {(x0, y0): [((x0, y0), (x1, y1)), ...]}."""
        if self._edges is None:
            edges: dict = {}
            for (cx, cy) in self.cells:
                if not self.occ(cx - 1, cy):
                    edges.setdefault((cx, cy), []).append(((cx, cy), (cx, cy + 1)))
                if not self.occ(cx + 1, cy):
                    edges.setdefault((cx + 1, cy), []).append(((cx + 1, cy), (cx + 1, cy + 1)))
                if not self.occ(cx, cy - 1):
                    edges.setdefault((cx, cy), []).append(((cx, cy), (cx + 1, cy)))
                if not self.occ(cx, cy + 1):
                    edges.setdefault((cx, cy + 1), []).append(((cx, cy + 1), (cx + 1, cy + 1)))
            self._edges = edges
        return self._edges

    def edges_near(self, lo_x, hi_x, lo_y, hi_y):
        e = self.boundary_edges()
        for vx in range(floor(lo_x), floor(hi_x) + 1):
            for vy in range(floor(lo_y), floor(hi_y) + 1):
                yield from e.get((vx, vy), ())

    def contains_closed(self, x: Fr, y: Fr) -> bool:
        xs = [floor(x)] + ([int(x) - 1] if x.denominator == 1 else [])
        ys = [floor(y)] + ([int(y) - 1] if y.denominator == 1 else [])
        return any(self.occ(cx, cy) for cx in xs for cy in ys)


def box(x0, y0, x1, y1):
    return _Box(x0, y0, x1, y1)


def union_all(geoms):
    return _CellUnion(g.cell for g in geoms)


def _geos_intersection(p1, p2, q1, q2):
    """algorithm::Intersection::intersection (GEOS >= 3.8), evaluated in IEEE double."""
    minX0 = p1[0] if p1[0] < p2[0] else p2[0]
    minY0 = p1[1] if p1[1] < p2[1] else p2[1]
    maxX0 = p1[0] if p1[0] > p2[0] else p2[0]
    maxY0 = p1[1] if p1[1] > p2[1] else p2[1]
    minX1 = q1[0] if q1[0] < q2[0] else q2[0]
    minY1 = q1[1] if q1[1] < q2[1] else q2[1]
    maxX1 = q1[0] if q1[0] > q2[0] else q2[0]
    maxY1 = q1[1] if q1[1] > q2[1] else q2[1]
    intMinX = minX0 if minX0 > minX1 else minX1
    intMaxX = maxX0 if maxX0 < maxX1 else maxX1
    intMinY = minY0 if minY0 > minY1 else minY1
    intMaxY = maxY0 if maxY0 < maxY1 else maxY1
    midx = (intMinX + intMaxX) / 2.0
    midy = (intMinY + intMaxY) / 2.0
    p1x = p1[0] - midx
    p1y = p1[1] - midy
    p2x = p2[0] - midx
    p2y = p2[1] - midy
    q1x = q1[0] - midx
    q1y = q1[1] - midy
    q2x = q2[0] - midx
    q2y = q2[1] - midy
    px = p1y - p2y
    py = p2x - p1x
    pw = p1x * p2y - p2x * p1y
    qx = q1y - q2y
    qy = q2x - q1x
    qw = q1x * q2y - q2x * q1y
    x = py * qw - qy * pw
    y = qx * pw - px * qw
    w = px * qy - qx * py
    return (x / w + midx, y / w + midy)


def _cross(ax, ay, bx, by):
    return ax * by - ay * bx


class LineString(_Geom):
    def __init__(self, coords=None):
        coords = [] if coords is None else [(float(c[0]), float(c[1])) for c in coords]
        self._coords = coords
        self.is_empty = len(coords) == 0

    @property
    def xy(self):
        return ([c[0] for c in self._coords], [c[1] for c in self._coords])

    def intersection(self, other: _CellUnion):
        (fpx, fpy), (fqx, fqy) = self._coords
        px, py, qx, qy = Fr(fpx), Fr(fpy), Fr(fqx), Fr(fqy)
        dx, dy = qx - px, qy - py
        dd = dx * dx + dy * dy
        lo_x, hi_x = min(px, qx) - 1, max(px, qx) + 1
        lo_y, hi_y = min(py, qy) - 1, max(py, qy) + 1
        # node parameter -> (on_boundary, coordinate in double)
        nodes: dict[Fr, list] = {Fr(0): [False, (fpx, fpy)], Fr(1): [False, (fqx, fqy)]}

        def add(t, coord_fn):
            if t in nodes:
                nodes[t][0] = True
            else:
                nodes[t] = [True, coord_fn()]

        for (v0, v1) in other.edges_near(lo_x, hi_x, lo_y, hi_y):
            ex, ey = v1[0] - v0[0], v1[1] - v0[1]
            wx, wy = v0[0] - px, v0[1] - py
            den = _cross(dx, dy, ex, ey)
            if den != 0:
                t = _cross(wx, wy, ex, ey) / den
                u = _cross(wx, wy, dx, dy) / den
                if 0 <= t <= 1 and 0 <= u <= 1:
                    if t == 0 or t == 1:
                        add(t, lambda: None)
                    elif u == 0:
                        add(t, lambda v=v0: (float(v[0]), float(v[1])))
                    elif u == 1:
                        add(t, lambda v=v1: (float(v[0]), float(v[1])))
                    else:
                        add(
                            t,
                            lambda v0=v0, v1=v1: _geos_intersection(
                                (fpx, fpy), (fqx, fqy), (float(v0[0]), float(v0[1])), (float(v1[0]), float(v1[1]))
                            ),
                        )
            elif _cross(wx, wy, dx, dy) == 0 and dd != 0:
                ta = (wx * dx + wy * dy) / dd
                tb = ((v1[0] - px) * dx + (v1[1] - py) * dy) / dd
                lo, hi = max(Fr(0), min(ta, tb)), min(Fr(1), max(ta, tb))
                if lo <= hi:
                    for t, v in ((ta, v0), (tb, v1)):
                        if 0 < t < 1:
                            add(t, lambda v=v: (float(v[0]), float(v[1])))
                    for t in (lo, hi):
                        if t == 0 or t == 1:
                            add(t, lambda: None)
        ts = sorted(nodes)
        piece_in = []
        for a, b in zip(ts[:-1], ts[1:]):
            m = (a + b) / 2
            piece_in.append(other.contains_closed(px + m * dx, py + m * dy))
        lines, points = [], []
        for i, (a, b) in enumerate(zip(ts[:-1], ts[1:])):
            if piece_in[i]:
                lines.append(LineString([nodes[a][1], nodes[b][1]]))
        for i, t in enumerate(ts):
            if not nodes[t][0]:
                continue
            left = piece_in[i - 1] if i > 0 else False
            right = piece_in[i] if i < len(piece_in) else False
            if not left and not right:
                points.append(Point(nodes[t][1]))
        if lines and points:
            return GeometryCollection(points + lines)
        if len(lines) == 1:
            return lines[0]
        if len(lines) > 1:
            return MultiLineString(lines)
        if len(points) == 1:
            return points[0]
        if len(points) > 1:
            return MultiPoint(points)
        return LineString()
