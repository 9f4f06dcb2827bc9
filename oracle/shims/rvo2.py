"""Python-RVO2 stand-in (oracle fixture generation only; see README.md).

Restates the RVO2 v2.0 library (third-party C++, not vendored in the reference, not installed here)
with numpy float32 scalars — every operation is an IEEE single-precision op like the C++ `float`
code (x86-64 SSE, no FMA contraction). Only agent 0's new velocity is computed in doStep: orca.py
reads only getAgentVelocity(0) and overwrites every agent's position and velocity before the next
doStep (orca.py:110-136), so the other agents' updates are unobservable. The KdTree's agent order
(KdTree::agents_) persists across doStep calls exactly as in RVO2.
PARITY vs the real RVO2 UNPINNED (no RVO2 binary exists here); pinned by the analytic known answers of
SURVEY Appendix A.4 in tests/test_orca_known_answers.py (which also checks it equals oracle/cpu_ref.c).
"""
import numpy as np

f32 = np.float32
RVO_EPSILON = f32(0.00001)
MAX_LEAF_SIZE = 10
ZERO = f32(0.0)
HALF = f32(0.5)
ONE = f32(1.0)


def _v(x, y):
    return (f32(x), f32(y))


def _add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def _mul(s, a):
    return (s * a[0], s * a[1])


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1]


def _div(a, s):  # Vector2::operator/ : multiply by 1/s
    inv = ONE / s
    return (a[0] * inv, a[1] * inv)


def _det(a, b):
    return a[0] * b[1] - a[1] * b[0]


def _abs(a):
    return np.sqrt(_dot(a, a))


def _normalize(a):
    return _div(a, _abs(a))


def _min(a, b):  # std::min
    return b if b < a else a


def _max(a, b):  # std::max
    return b if a < b else a


class _Agent(object):
    def __init__(self, pos, neighborDist, maxNeighbors, timeHorizon, timeHorizonObst, radius, maxSpeed, velocity):
        self.position = _v(*pos)
        self.velocity = _v(*velocity)
        self.prefVelocity = _v(0.0, 0.0)
        self.neighborDist = f32(neighborDist)
        self.maxNeighbors = int(maxNeighbors)
        self.timeHorizon = f32(timeHorizon)
        self.timeHorizonObst = f32(timeHorizonObst)
        self.radius = f32(radius)
        self.maxSpeed = f32(maxSpeed)


class _Node(object):
    __slots__ = ("begin", "end", "left", "right", "minX", "maxX", "minY", "maxY")


class PyRVOSimulator(object):
    def __init__(self, timeStep, neighborDist, maxNeighbors, timeHorizon, timeHorizonObst, radius, maxSpeed,
                 velocity=(0, 0)):
        self.timeStep = f32(timeStep)
        self.defaults = (neighborDist, maxNeighbors, timeHorizon, timeHorizonObst, radius, maxSpeed, velocity)
        self.agents = []
        self.kd_agents = []  # KdTree::agents_ (indices), persists across doStep
        self.tree = []

    # --- API used by orca.py ---
    def addAgent(self, pos, neighborDist=None, maxNeighbors=None, timeHorizon=None, timeHorizonObst=None,
                 radius=None, maxSpeed=None, velocity=None):
        d = self.defaults
        args = [neighborDist, maxNeighbors, timeHorizon, timeHorizonObst, radius, maxSpeed, velocity]
        args = [d[k] if a is None else a for k, a in enumerate(args)]
        self.agents.append(_Agent(pos, *args))
        return len(self.agents) - 1

    def getNumAgents(self):
        return len(self.agents)

    def setAgentPosition(self, i, pos):
        self.agents[i].position = _v(*pos)

    def setAgentVelocity(self, i, vel):
        self.agents[i].velocity = _v(*vel)

    def setAgentPrefVelocity(self, i, vel):
        self.agents[i].prefVelocity = _v(*vel)

    def getAgentVelocity(self, i):
        v = self.agents[i].velocity
        return (float(v[0]), float(v[1]))

    def getAgentRadius(self, i):
        return float(self.agents[i].radius)

    def getAgentMaxSpeed(self, i):
        return float(self.agents[i].maxSpeed)

    def doStep(self):
        # KdTree::buildAgentTree
        while len(self.kd_agents) < len(self.agents):
            self.kd_agents.append(len(self.kd_agents))
        n = len(self.kd_agents)
        self.tree = [_Node() for _ in range(2 * n - 1)]
        if n:
            self._build(0, n, 0)
        a = self.agents[0]
        nbrs = self._compute_neighbors(0)
        a.velocity = self._compute_new_velocity(a, nbrs)
        # (Agent::update's position integration of agent 0 is unobservable: orca.py resets it)

    # --- KdTree ---
    def _pos(self, k):
        return self.agents[self.kd_agents[k]].position

    def _build(self, begin, end, node):
        T = self.tree[node]
        T.begin, T.end = begin, end
        T.minX = T.maxX = self._pos(begin)[0]
        T.minY = T.maxY = self._pos(begin)[1]
        for i in range(begin + 1, end):
            x, y = self._pos(i)
            T.maxX = _max(T.maxX, x)
            T.minX = _min(T.minX, x)
            T.maxY = _max(T.maxY, y)
            T.minY = _min(T.minY, y)
        if end - begin > MAX_LEAF_SIZE:
            vertical = (T.maxX - T.minX) > (T.maxY - T.minY)
            split = HALF * (T.maxX + T.minX) if vertical else HALF * (T.maxY + T.minY)
            c = 0 if vertical else 1
            left, right = begin, end
            while left < right:
                while left < right and self._pos(left)[c] < split:
                    left += 1
                while right > left and self._pos(right - 1)[c] >= split:
                    right -= 1
                if left < right:
                    ka = self.kd_agents
                    ka[left], ka[right - 1] = ka[right - 1], ka[left]
                    left += 1
                    right -= 1
            if left == begin:
                left += 1
                right += 1
            T.left = node + 1
            T.right = node + 2 * (left - begin)
            self._build(begin, left, T.left)
            self._build(left, end, T.right)

    def _compute_neighbors(self, idx):
        agent = self.agents[idx]
        nbrs = []
        state = {"rangeSq": agent.neighborDist * agent.neighborDist}
        if agent.maxNeighbors > 0:
            self._query(idx, agent, state, 0, nbrs)
        return nbrs

    def _insert(self, idx, agent, other_idx, state, nbrs):
        if other_idx == idx:
            return
        d = _sub(agent.position, self.agents[other_idx].position)
        distSq = _dot(d, d)
        if distSq < state["rangeSq"]:
            if len(nbrs) < agent.maxNeighbors:
                nbrs.append((distSq, other_idx))
            i = len(nbrs) - 1
            while i != 0 and distSq < nbrs[i - 1][0]:
                nbrs[i] = nbrs[i - 1]
                i -= 1
            nbrs[i] = (distSq, other_idx)
            if len(nbrs) == agent.maxNeighbors:
                state["rangeSq"] = nbrs[-1][0]

    def _query(self, idx, agent, state, node, nbrs):
        T = self.tree[node]
        if T.end - T.begin <= MAX_LEAF_SIZE:
            for i in range(T.begin, T.end):
                self._insert(idx, agent, self.kd_agents[i], state, nbrs)
            return
        x, y = agent.position
        L, R = self.tree[T.left], self.tree[T.right]

        def bd(N):
            return (_max(ZERO, N.minX - x) ** 2 + _max(ZERO, x - N.maxX) ** 2 +
                    _max(ZERO, N.minY - y) ** 2 + _max(ZERO, y - N.maxY) ** 2)

        def sq(v):
            return v * v

        dl = sq(_max(ZERO, L.minX - x)) + sq(_max(ZERO, x - L.maxX)) + sq(_max(ZERO, L.minY - y)) + sq(_max(ZERO, y - L.maxY))
        dr = sq(_max(ZERO, R.minX - x)) + sq(_max(ZERO, x - R.maxX)) + sq(_max(ZERO, R.minY - y)) + sq(_max(ZERO, y - R.maxY))
        if dl < dr:
            if dl < state["rangeSq"]:
                self._query(idx, agent, state, T.left, nbrs)
                if dr < state["rangeSq"]:
                    self._query(idx, agent, state, T.right, nbrs)
        else:
            if dr < state["rangeSq"]:
                self._query(idx, agent, state, T.right, nbrs)
                if dl < state["rangeSq"]:
                    self._query(idx, agent, state, T.left, nbrs)

    # --- Agent::computeNewVelocity (agents only; no obstacles) ---
    def _compute_new_velocity(self, a, nbrs):
        lines = []
        invTimeHorizon = ONE / a.timeHorizon
        for _, oi in nbrs:
            other = self.agents[oi]
            relativePosition = _sub(other.position, a.position)
            relativeVelocity = _sub(a.velocity, other.velocity)
            distSq = _dot(relativePosition, relativePosition)
            combinedRadius = a.radius + other.radius
            combinedRadiusSq = combinedRadius * combinedRadius
            if distSq > combinedRadiusSq:
                w = _sub(relativeVelocity, _mul(invTimeHorizon, relativePosition))
                wLengthSq = _dot(w, w)
                dotProduct1 = _dot(w, relativePosition)
                if dotProduct1 < ZERO and dotProduct1 * dotProduct1 > combinedRadiusSq * wLengthSq:
                    wLength = np.sqrt(wLengthSq)
                    unitW = _div(w, wLength)
                    direction = (unitW[1], -unitW[0])
                    u = _mul(combinedRadius * invTimeHorizon - wLength, unitW)
                else:
                    leg = np.sqrt(distSq - combinedRadiusSq)
                    rx, ry = relativePosition
                    if _det(relativePosition, w) > ZERO:
                        direction = _div((rx * leg - ry * combinedRadius, rx * combinedRadius + ry * leg), distSq)
                    else:
                        direction = _div((-(rx * leg + ry * combinedRadius), -(-rx * combinedRadius + ry * leg)), distSq)
                    dotProduct2 = _dot(relativeVelocity, direction)
                    u = _sub(_mul(dotProduct2, direction), relativeVelocity)
            else:
                invTimeStep = ONE / self.timeStep
                w = _sub(relativeVelocity, _mul(invTimeStep, relativePosition))
                wLength = _abs(w)
                unitW = _div(w, wLength)
                direction = (unitW[1], -unitW[0])
                u = _mul(combinedRadius * invTimeStep - wLength, unitW)
            point = _add(a.velocity, _mul(HALF, u))
            lines.append((point, direction))
        lineFail, result = _lp2(lines, a.maxSpeed, a.prefVelocity, False, (ZERO, ZERO))
        if lineFail < len(lines):
            result = _lp3(lines, 0, lineFail, a.maxSpeed, result)
        return result


def _lp1(lines, lineNo, radius, optVelocity, directionOpt, result):
    point, direction = lines[lineNo]
    dotProduct = _dot(point, direction)
    discriminant = dotProduct * dotProduct + radius * radius - _dot(point, point)
    if discriminant < ZERO:
        return False, result
    sqrtDiscriminant = np.sqrt(discriminant)
    tLeft = -dotProduct - sqrtDiscriminant
    tRight = -dotProduct + sqrtDiscriminant
    for i in range(lineNo):
        pi, di = lines[i]
        denominator = _det(direction, di)
        numerator = _det(di, _sub(point, pi))
        if abs(denominator) <= RVO_EPSILON:
            if numerator < ZERO:
                return False, result
            continue
        t = numerator / denominator
        if denominator >= ZERO:
            tRight = _min(tRight, t)
        else:
            tLeft = _max(tLeft, t)
        if tLeft > tRight:
            return False, result
    if directionOpt:
        if _dot(optVelocity, direction) > ZERO:
            result = _add(point, _mul(tRight, direction))
        else:
            result = _add(point, _mul(tLeft, direction))
    else:
        t = _dot(direction, _sub(optVelocity, point))
        if t < tLeft:
            result = _add(point, _mul(tLeft, direction))
        elif t > tRight:
            result = _add(point, _mul(tRight, direction))
        else:
            result = _add(point, _mul(t, direction))
    return True, result


def _lp2(lines, radius, optVelocity, directionOpt, result):
    if directionOpt:
        result = (optVelocity[0] * radius, optVelocity[1] * radius)
    elif _dot(optVelocity, optVelocity) > radius * radius:
        n = _normalize(optVelocity)
        result = (n[0] * radius, n[1] * radius)
    else:
        result = optVelocity
    for i in range(len(lines)):
        point, direction = lines[i]
        if _det(direction, _sub(point, result)) > ZERO:
            temp = result
            ok, result = _lp1(lines, i, radius, optVelocity, directionOpt, result)
            if not ok:
                return i, temp
    return len(lines), result


def _lp3(lines, numObstLines, beginLine, radius, result):
    distance = ZERO
    for i in range(beginLine, len(lines)):
        pi, di = lines[i]
        if _det(di, _sub(pi, result)) > distance:
            projLines = list(lines[:numObstLines])
            for j in range(numObstLines, i):
                pj, dj = lines[j]
                determinant = _det(di, dj)
                if abs(determinant) <= RVO_EPSILON:
                    if _dot(di, dj) > ZERO:
                        continue
                    point = _mul(HALF, _add(pi, pj))
                else:
                    point = _add(pi, _mul(_det(dj, _sub(pi, pj)) / determinant, di))
                direction = _normalize(_sub(dj, di))
                projLines.append((point, direction))
            temp = result
            fail, result = _lp2(projLines, radius, (-di[1], di[0]), True, result)
            if fail < len(projLines):
                result = temp
            distance = _det(di, _sub(pi, result))
    return result
