"""Step event classes (crowd_sim/envs/utils/info.py). When the reference package is importable its own
classes are used, so callers' `isinstance(info['info']['event'], ReachGoal)` checks (train.py:270-278,
evaluation.py) keep working unchanged."""
from . import abi

try:  # the user's checkout of the reference, if on sys.path
    from crowd_sim.envs.utils.info import Collision, Danger, Nothing, ReachGoal, Timeout  # noqa: F401
except Exception:  # noqa: BLE001

    class Timeout:
        def __str__(self):
            return "Timeout"

    class ReachGoal:
        def __str__(self):
            return "Reaching goal"

    class Danger:
        def __init__(self, min_dist):
            self.min_dist = min_dist

        def __str__(self):
            return "Too close"

    class Collision:
        def __str__(self):
            return "Collision"

    class Nothing:
        def __str__(self):
            return ""


def make_event(code, min_dist):
    """Event code (include/crowdnav.h CN_EV_*) -> info.py instance; Danger carries dmin."""
    if code == abi.EV_NOTHING:
        return Nothing()
    if code == abi.EV_DANGER:
        return Danger(float(min_dist))
    if code == abi.EV_COLLISION:
        return Collision()
    if code == abi.EV_REACHGOAL:
        return ReachGoal()
    if code == abi.EV_TIMEOUT:
        return Timeout()
    raise ValueError("unknown event code %r" % (code,))
