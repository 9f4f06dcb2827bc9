"""CPU restatement of the ConvGRU observation with its LiDAR scan — TEST INFRASTRUCTURE ONLY (imported by
tests/ as the checker; never by the product path, which is cn_lidar_obs in crowdnav_dsrnn_amd/csrc).

Follows the reference as shipped (pinned by tests/golden/lidar_*.npz, recorded from the reference itself):
  crowd_sim_dict.py:96-101    obs = [clip(robot full state (no v) / max_range, 0, 1), lidar_rel_dist]
  crowd_sim_dict.py:166-191   the scan runs in reset() only, AFTER reset()'s observation was built (which
                              so carries the previous scan, zeros before the first), robot heading
                              atan2(0, 0) = 0, against the LAST human only (the append sits after the
                              loop) and the world walls; step() observations carry the scan of the reset
  lidarv2.py:17-52            get_valid_angles;   :55-75 get_valid_angle_idx (mutates its input in place,
                              the same arrays serve every beam);   :112-161 beam sample points
                              (np.linspace(0, max_range, 500), rotated, translated);   :164-198 first sample
                              strictly inside the closest valid obstacle;   :201-292 walls via
                              get_intersect.py, range check, robot-radius clamp;   :398-427 distances
numpy float64 throughout, like the reference; numpy arrays per env (all beams x all samples at once).
"""
import numpy as np


def _rescale(t):
    return (t + 2 * np.pi) % (2 * np.pi)


def _orient(p, q, r):
    v = (float(q[1] - p[1]) * (r[0] - q[0])) - (float(q[0] - p[0]) * (r[1] - q[1]))
    return 1 if v > 0 else (2 if v < 0 else 0)


def _on_seg(p, q, r):
    return max(p[0], r[0]) >= q[0] >= min(p[0], r[0]) and max(p[1], r[1]) >= q[1] >= min(p[1], r[1])


def _segments_cross(p1, q1, p2, q2):
    o1, o2, o3, o4 = _orient(p1, q1, p2), _orient(p1, q1, q2), _orient(p2, q2, p1), _orient(p2, q2, q1)
    if o1 != o2 and o3 != o4:
        return True
    return ((o1 == 0 and _on_seg(p1, p2, q1)) or (o2 == 0 and _on_seg(p1, q2, q1)) or
            (o3 == 0 and _on_seg(p2, p1, q2)) or (o4 == 0 and _on_seg(p2, q1, q2)))


def _line_intersection(p1, q1, p2, q2):
    xd = (p1[0] - q1[0], p2[0] - q2[0])
    yd = (p1[1] - q1[1], p2[1] - q2[1])
    det = lambda a, b: a[0] * b[1] - a[1] * b[0]  # noqa: E731
    div = det(xd, yd)
    if div == 0:
        return None
    d = (det(p1, q1), det(p2, q2))
    return (det(d, xd) / div, det(d, yd) / div)


def scan(sensor, human_xyr, beams=180, max_range=5.0, robot_radius=0.3, half_world=10.0):
    """LidarSensor.sensor_spin(normalize=True) at heading 0 against one disc obstacle -> |1 - rel_dist|."""
    sx, sy = float(sensor[0]), float(sensor[1])
    n_pts = 500
    s = np.linspace(0, max_range, n_pts)
    ang = _rescale(np.linspace(0, 2 * np.pi, beams) + 0.0)
    c, sn = np.cos(ang), np.sin(ang)
    bx = c[:, None] * s[None, :] + sx
    by = sn[:, None] * s[None, :] + sy
    hx, hy, hr = (float(v) for v in human_xyr)
    rel_x, rel_y = hx - sx, hy - sy
    head = _rescale(np.arctan2(rel_y, rel_x))
    dx, dy = hr * np.sin(head), hr * np.cos(head)
    mm = np.sort([_rescale(np.arctan2(rel_y - dy, rel_x + dx)), _rescale(np.arctan2(rel_y + dy, rel_x - dx))])
    lo, up = float(mm[0]), float(mm[1])
    walls = [(-half_world, -half_world), (half_world, -half_world), (half_world, half_world),
             (-half_world, half_world), (-half_world, -half_world)]
    out = np.zeros(beams)
    for b in range(beams):
        tt = ang[b]
        if up - lo >= np.pi:          # the in-place mutation of get_valid_angle_idx, carried to later beams
            lo, up = up - 2 * np.pi, lo
            tt = tt - 2 * np.pi
        valid = (tt - lo) % (2 * np.pi) < (up - lo) % (2 * np.pi)
        end = (bx[b, -1], by[b, -1])
        hit = False
        if valid:
            res = np.sqrt((hx - bx[b]) ** 2 + (hy - by[b]) ** 2)
            idx = np.where(res < hr)[0]
            if len(idx):
                end = (bx[b, idx.min()], by[b, idx.min()])
                hit = True
        if not hit:
            p1, q1 = (bx[b, 0], by[b, 0]), (bx[b, -1], by[b, -1])
            for j in range(4):
                if _segments_cross(p1, q1, walls[j], walls[j + 1]):
                    ip = _line_intersection(p1, q1, walls[j], walls[j + 1])
                    if ip is not None and np.linalg.norm([ip[0] - sx, ip[1] - sy]) <= max_range:
                        end = ip
                    break
        if np.linalg.norm([end[0] - sx, end[1] - sy]) < robot_radius:
            end = (sx + robot_radius * np.cos(ang[b]), sy + robot_radius * np.sin(ang[b]))
        out[b] = np.sqrt((end[0] - sx) ** 2 + (end[1] - sy) ** 2)
    return np.abs(1 - np.clip(out / max_range, 0, 1))


def robot_part(sv):
    """(E, 7) float32: clip(robot full state without velocity / max_range, 0, 1)."""
    rs = np.stack([sv.r_px, sv.r_py, sv.r_radius, sv.r_gx, sv.r_gy, sv.r_vpref, sv.r_theta], 1).astype(np.float64)
    return rs


def convgru_scans(sv, beams=180, max_range=5.0, robot_radius=0.3, half_world=10.0):
    """(E, beams) float32: the scan reset() takes from this (post-reset) state."""
    N = sv.N
    return np.stack([scan((sv.r_px[e], sv.r_py[e]), (sv.h_px[e, N - 1], sv.h_py[e, N - 1], sv.h_r[e, N - 1]),
                          beams, max_range, robot_radius, half_world) for e in range(sv.E)]).astype(np.float32)


def convgru_obs(sv, held_scan, max_range=5.0):
    """(E, 1, 7 + beams) float32 observation for state sv carrying the held scan (E, beams)."""
    out = np.zeros((sv.E, 1, 7 + held_scan.shape[1]), np.float32)
    out[:, 0, :7] = np.clip(robot_part(sv) / max_range, 0, 1)
    out[:, 0, 7:] = held_scan
    return out
