"""shapely stand-in for fixture generation (oracle only; see ../README.md).

Restates, analytically in float64, exactly the shapely 2.x / GEOS operations the reference calls:
  Point(x, y).buffer(r)                      GEOS OffsetSegmentGenerator::createCircle, quadSegs = 16
  LineString(pts).intersection(g).is_empty   closed-set segment vs convex polygon
  box(minx, miny, maxx, maxy)                ccw ring [(maxx,miny),(maxx,maxy),(minx,maxy),(minx,miny)]
  affinity.translate / affinity.rotate       shapely.affinity formulas (rotate snaps |cos|,|sin| < 2.5e-16)
  Polygon.intersects(Polygon)                closed-set intersection of convex (possibly degenerate) rings
GEOS is not available here, so these semantics are PARITY UNPINNED.
"""
from . import geometry  # noqa: F401
from . import affinity  # noqa: F401
