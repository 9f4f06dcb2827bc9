import math

from .geometry import Polygon


def translate(geom, xoff=0.0, yoff=0.0, zoff=0.0):
    return Polygon([(x + xoff, y + yoff) for x, y in geom.coords])


def rotate(geom, angle, origin="center", use_radians=False):
    if not use_radians:
        angle = angle * math.pi / 180.0
    cosp, sinp = math.cos(angle), math.sin(angle)
    if abs(cosp) < 2.5e-16:
        cosp = 0.0
    if abs(sinp) < 2.5e-16:
        sinp = 0.0
    if origin == "center" or origin == "centroid":
        xs = [p[0] for p in geom.coords]
        ys = [p[1] for p in geom.coords]
        x0, y0 = (min(xs) + max(xs)) / 2.0, (min(ys) + max(ys)) / 2.0
    else:
        x0, y0 = float(origin[0]), float(origin[1])
    xoff = x0 - x0 * cosp + y0 * sinp
    yoff = y0 - x0 * sinp - y0 * cosp
    return Polygon([(cosp * x + (-sinp) * y + xoff, sinp * x + cosp * y + yoff) for x, y in geom.coords])
