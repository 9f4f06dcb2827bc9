import math


class _Geom(object):
    is_empty = False


class _Empty(_Geom):
    is_empty = True


class _NonEmpty(_Geom):
    is_empty = False


class Polygon(_Geom):
    """Convex polygon given by its exterior ring (no closing vertex stored)."""

    def __init__(self, pts):
        pts = [(float(x), float(y)) for x, y in pts]
        if len(pts) > 1 and pts[0] == pts[-1]:
            pts = pts[:-1]
        self.coords = pts

    def intersects(self, other):
        return _convex_intersects(self.coords, other.coords)

    def simplify(self, tol):
        return self


class Point(_Geom):
    def __init__(self, x, y):
        self.x, self.y = float(x), float(y)

    def buffer(self, distance, quad_segs=16):
        # OffsetSegmentGenerator::createCircle: start (x+d, y), then clockwise fillet over 2*pi
        pts = [(self.x + distance, self.y)]
        total = abs(0.0 - 2.0 * math.pi)
        quantum = math.pi / 2.0 / quad_segs
        nsegs = int(total / quantum + 0.5)
        inc = total / nsegs
        for i in range(nsegs):
            ang = 0.0 + (-1 * i) * inc
            p = (self.x + distance * math.cos(ang), self.y + distance * math.sin(ang))
            if p != pts[-1]:
                pts.append(p)
        return Polygon(pts)


class LineString(_Geom):
    def __init__(self, pts):
        self.coords = [(float(x), float(y)) for x, y in pts]

    def intersection(self, poly):
        a, b = self.coords[0], self.coords[-1]
        return _NonEmpty() if _segment_hits_convex(a, b, poly.coords) else _Empty()


def box(minx, miny, maxx, maxy, ccw=True):
    return Polygon([(maxx, miny), (maxx, maxy), (minx, maxy), (minx, miny)])


def _orient(a, b, c):
    return (b[0] - a[0]) * (c[1] - a[1]) - (b[1] - a[1]) * (c[0] - a[0])


def _on_seg(a, b, p):
    return min(a[0], b[0]) <= p[0] <= max(a[0], b[0]) and min(a[1], b[1]) <= p[1] <= max(a[1], b[1])


def _segs_intersect(p1, p2, q1, q2):
    d1, d2 = _orient(q1, q2, p1), _orient(q1, q2, p2)
    d3, d4 = _orient(p1, p2, q1), _orient(p1, p2, q2)
    if ((d1 > 0 and d2 < 0) or (d1 < 0 and d2 > 0)) and ((d3 > 0 and d4 < 0) or (d3 < 0 and d4 > 0)):
        return True
    if d1 == 0 and _on_seg(q1, q2, p1):
        return True
    if d2 == 0 and _on_seg(q1, q2, p2):
        return True
    if d3 == 0 and _on_seg(p1, p2, q1):
        return True
    if d4 == 0 and _on_seg(p1, p2, q2):
        return True
    return False


def _inside_convex(p, ring):
    s = 0
    n = len(ring)
    for k in range(n):
        o = _orient(ring[k], ring[(k + 1) % n], p)
        if o > 0:
            if s < 0:
                return False
            s = 1
        elif o < 0:
            if s > 0:
                return False
            s = -1
    return True


def _segment_hits_convex(a, b, ring):
    if _inside_convex(a, ring) or _inside_convex(b, ring):
        return True
    n = len(ring)
    return any(_segs_intersect(a, b, ring[k], ring[(k + 1) % n]) for k in range(n))


def _convex_intersects(A, B):
    """Separating-axis test over edge normals and edge directions of both rings (closed sets)."""
    for ring in (A, B):
        n = len(ring)
        for k in range(n):
            ex = ring[(k + 1) % n][0] - ring[k][0]
            ey = ring[(k + 1) % n][1] - ring[k][1]
            if ex == 0.0 and ey == 0.0:
                continue
            for nx, ny in ((-ey, ex), (ex, ey)):
                pa = [x * nx + y * ny for x, y in A]
                pb = [x * nx + y * ny for x, y in B]
                if max(pa) < min(pb) or max(pb) < min(pa):
                    return False
    return True
