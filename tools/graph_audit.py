"""HIP-graph audit of the captured rollout.

Round 4 saw the captured rollout return the f64 episode-return sum's bits as the int64 episode count on
one replay of five (profiles/r04/ge.log). This tool finds out why, from the captured graph itself:

  python tools/graph_audit.py iso      [R]   the two reductions alone in a graph, replayed R times
  python tools/graph_audit.py rollout  [E U] C4's rollout with the round-4 in-graph reductions (U updates)
  python tools/graph_audit.py current  [E U] C4's rollout as the trainer captures it now (U updates)

For each captured graph it walks the node list through the HIP graph API (node types, the dependency
structure, every memset node's destination / size / value, every memcpy node) and writes the runtime's
own DOT dump (hipGraphDebugDotPrint, verbose) to gpurun_out/. After each replay it reads back the words
every memset node initialises, which tells a memset that ran where the capture put it (the reduction that
follows leaves its semaphore at its own block count) from one that was skipped or ran late.
"""
import ctypes
import json
import os
import re
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "gpurun_out", "graph_audit")

NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
              7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait", 10: "mem_alloc", 11: "mem_free",
              12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


class MemsetParams(ctypes.Structure):   # hip_runtime_api.h hipMemsetParams
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint), ("height", ctypes.c_size_t),
                ("pitch", ctypes.c_size_t), ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


class Dim3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint), ("y", ctypes.c_uint), ("z", ctypes.c_uint)]


class KernelParams(ctypes.Structure):   # hip_runtime_api.h hipKernelNodeParams
    _fields_ = [("blockDim", Dim3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p), ("gridDim", Dim3),
                ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]


_HIP = None


def hip():
    """The HIP runtime torch loaded (same file, so dlopen returns the same instance: no second runtime)."""
    global _HIP
    if _HIP is None:
        path = None
        for line in open("/proc/self/maps"):
            if "libamdhip64" in line:
                path = line.split()[-1]
                break
        if path is None:
            raise RuntimeError("torch has not loaded libamdhip64")
        L = ctypes.CDLL(path)
        vp, szp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)
        L.hipGraphGetNodes.argtypes = [vp, ctypes.POINTER(vp), szp]
        L.hipGraphNodeGetType.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
        L.hipGraphNodeGetDependencies.argtypes = [vp, ctypes.POINTER(vp), szp]
        L.hipGraphMemsetNodeGetParams.argtypes = [vp, ctypes.POINTER(MemsetParams)]
        L.hipGraphKernelNodeGetParams.argtypes = [vp, ctypes.POINTER(KernelParams)]
        L.hipGraphDebugDotPrint.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint]
        L.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
        _HIP = L
    return _HIP


def _ck(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: hipError %d" % (what, rc))


def walk(graph):
    """Nodes of a hipGraph_t in the runtime's order: type, dependencies (as node indices), and the
    parameters of memset and kernel nodes."""
    L = hip()
    n = ctypes.c_size_t(0)
    _ck(L.hipGraphGetNodes(graph, None, ctypes.byref(n)), "hipGraphGetNodes")
    arr = (ctypes.c_void_p * n.value)()
    _ck(L.hipGraphGetNodes(graph, arr, ctypes.byref(n)), "hipGraphGetNodes")
    idx = {arr[i]: i for i in range(n.value)}
    nodes = []
    for i in range(n.value):
        t = ctypes.c_int(-1)
        _ck(L.hipGraphNodeGetType(arr[i], ctypes.byref(t)), "hipGraphNodeGetType")
        nd = ctypes.c_size_t(0)
        _ck(L.hipGraphNodeGetDependencies(arr[i], None, ctypes.byref(nd)), "hipGraphNodeGetDependencies")
        deps = []
        if nd.value:
            da = (ctypes.c_void_p * nd.value)()
            _ck(L.hipGraphNodeGetDependencies(arr[i], da, ctypes.byref(nd)), "hipGraphNodeGetDependencies")
            deps = [idx.get(da[j], -1) for j in range(nd.value)]
        rec = {"i": i, "type": NODE_TYPES.get(t.value, str(t.value)), "deps": deps}
        if t.value == 2:
            p = MemsetParams()
            _ck(L.hipGraphMemsetNodeGetParams(arr[i], ctypes.byref(p)), "hipGraphMemsetNodeGetParams")
            rec["memset"] = {"dst": p.dst, "elementSize": p.elementSize, "width": p.width, "height": p.height,
                             "value": p.value, "bytes": p.elementSize * p.width * max(p.height, 1)}
        elif t.value == 0:
            p = KernelParams()
            _ck(L.hipGraphKernelNodeGetParams(arr[i], ctypes.byref(p)), "hipGraphKernelNodeGetParams")
            rec["grid"] = [p.gridDim.x, p.gridDim.y, p.gridDim.z]
            rec["block"] = [p.blockDim.x, p.blockDim.y, p.blockDim.z]
            rec["lds"] = p.sharedMemBytes
        nodes.append(rec)
    return nodes


def dot(graph, path):
    """hipGraphDebugDotPrint(verbose) -> path; returns the kernel names in the order the dump lists them."""
    _ck(hip().hipGraphDebugDotPrint(graph, path.encode(), 1 << 0 | 1 << 2 | 1 << 3 | 1 << 4), "hipGraphDebugDotPrint")
    txt = open(path).read()
    return re.findall(r'label="[^"]*?(?:\\n)?([A-Za-z_][A-Za-z0-9_:<>,\s\*\(\)&]*?)\\n', txt), txt


def summarize(nodes):
    """Type histogram, whether the graph is one chain (every node after the first depends on exactly its
    predecessor), fan-in / fan-out points, memset and memcpy nodes with what precedes them."""
    hist = {}
    for nd in nodes:
        hist[nd["type"]] = hist.get(nd["type"], 0) + 1
    users = {}
    for nd in nodes:
        for d in nd["deps"]:
            users.setdefault(d, []).append(nd["i"])
    roots = [nd["i"] for nd in nodes if not nd["deps"]]
    fan_in = [nd["i"] for nd in nodes if len(nd["deps"]) > 1]
    fan_out = [i for i, u in users.items() if len(u) > 1]
    chain = len(roots) == 1 and not fan_in and not fan_out
    memsets = [dict(nd["memset"], i=nd["i"], deps=nd["deps"],
                    prev_type=[nodes[d]["type"] for d in nd["deps"]]) for nd in nodes if nd["type"] == "memset"]
    dsts = {}
    for m in memsets:
        dsts.setdefault(m["dst"], []).append(m["i"])
    return {"nodes": len(nodes), "types": hist, "single_chain": chain, "roots": roots[:8], "fan_in": fan_in[:16],
            "fan_out": fan_out[:16], "memsets": memsets, "memset_dsts_shared": {hex(k): v for k, v in dsts.items()
                                                                               if len(v) > 1}}


def read_words(addr, n=1):
    buf = (ctypes.c_uint32 * n)()
    torch.cuda.synchronize()
    _ck(hip().hipMemcpy(ctypes.cast(buf, ctypes.c_void_p), ctypes.c_void_p(addr), 4 * n, 2), "hipMemcpy")
    return list(buf)


def report(tag, graph):
    os.makedirs(OUT, exist_ok=True)
    nodes = walk(graph)
    s = summarize(nodes)
    dpath = os.path.join(OUT, "%s.dot" % tag)
    try:
        _, txt = dot(graph, dpath)
        s["dot"] = os.path.relpath(dpath, REPO)
        s["dot_kernel_labels"] = sorted(set(re.findall(r'\\n([A-Za-z_][\w:<>, ]{3,120})\\n', txt)))[:80]
    except Exception as e:   # the walk above is the evidence; the dump is a convenience
        s["dot_error"] = str(e)
    json.dump({"summary": s, "nodes": nodes}, open(os.path.join(OUT, "%s.json" % tag), "w"), indent=1, default=str)
    brief = {k: v for k, v in s.items() if k not in ("memsets", "dot_kernel_labels")}
    print("[%s] %s" % (tag, json.dumps(brief, default=str)), flush=True)
    for m in s["memsets"]:
        print("[%s]   memset node %d: dst 0x%x, %d B, value %d, after %s" % (tag, m["i"], m["dst"], m["bytes"],
                                                                       m["value"], m["prev_type"]), flush=True)
    return s


# ---------------------------------------------------------------------------------------------------------------
def iso(R=2000):
    """The two round-4 reductions alone: ep_sum += x.sum() (f64, T x E), ep_cnt += (m == 0).sum() (int64),
    captured once, replayed R times with the accumulators zeroed eagerly before each replay."""
    dev = torch.device("cuda:0")
    T, E = 128, 4096
    g0 = torch.Generator(device=dev)
    g0.manual_seed(3)
    x = torch.randn((T, E), generator=g0, device=dev, dtype=torch.float64)
    m = (torch.rand((T, E, 1), generator=g0, device=dev) > 0.02).float()
    want_s, want_c = float(x.sum()), int((m == 0).sum())
    ep_s = torch.zeros((), dtype=torch.float64, device=dev)
    ep_c = torch.zeros((), dtype=torch.int64, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside capture
        ep_s += x.sum()
        ep_c += (m == 0).sum()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        ep_s += x.sum()
        ep_c += (m == 0).sum()
    summ = report("iso", g.raw_cuda_graph())
    sems = [ms["dst"] for ms in summ["memsets"]]
    bad = []
    hist = {}
    for r in range(R):
        ep_s.zero_()
        ep_c.zero_()
        g.replay()
        torch.cuda.synchronize()
        words = tuple(read_words(a)[0] for a in sems)
        hist[words] = hist.get(words, 0) + 1
        cs, cc = float(ep_s), int(ep_c)
        if cs != want_s or cc != want_c:
            bad.append((r, cs, cc, words))
    print("[iso] %d replays, %d wrong; semaphore words after replay: %s" % (R, len(bad), {str(k): v for k, v in hist.items()}),
          flush=True)
    for b in bad[:10]:
        print("[iso]   replay %d: sum %r count %d (want %r, %d); words %s" % (b[0], b[1], b[2], want_s, want_c, b[3]),
              flush=True)


def _trainer(E, old):
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.learner import PPO
    from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer
    from crowdnav_dsrnn_amd.policy import Policy

    c = clone_config(Config())
    c.sim.human_num = 10
    c.humans.policy = "orca"
    c.action_space.kinematics = "holonomic"
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    c.training.num_processes = E
    c.ppo.num_steps = 128
    c.ppo.epoch = 5
    c.ppo.num_mini_batch = 2
    torch.manual_seed(11)
    envs = CrowdNavVecEnv(c, E, c.env.seed, "cuda:0", nenv=E, phase="train")
    pol = Policy(envs.observation_space.spaces, envs.action_space, base="srnn", base_kwargs=c).to("cuda:0")
    agent = PPO(pol, c.ppo.clip_param, c.ppo.epoch, 2, c.ppo.value_loss_coef, c.ppo.entropy_coef, lr=4e-5, eps=1e-5,
                max_grad_norm=0.5)

    class Audited(RolloutTrainer):
        """RolloutTrainer whose capture keeps its hipGraph_t for the walk; old=True also restores round 4's
        in-graph reductions (ep_sum += _ep_ret.sum(); ep_cnt += (masks[1:] == 0).sum(), zeroed eagerly)."""

        def _rollout(self):
            super()._rollout()
            if old:
                self._ep[0].add_(self._ep_ret.sum())
                self._ep[1].add_((self.rollouts.masks[1:] == 0).sum())

        def collect(self):
            if old:
                if getattr(self, "_ep", None) is None:
                    self._ep = (torch.zeros((), dtype=torch.float64, device=self.device),
                                torch.zeros((), dtype=torch.int64, device=self.device))
                self._ep[0].zero_()
                self._ep[1].zero_()
            r = self.rollouts
            if self._warm and self._graph is None:
                g = torch.cuda.CUDAGraph(keep_graph=True)
                step0 = r.step
                self.envs.engine.set_graph_mode(True)
                with torch.cuda.graph(g):
                    self._rollout()
                r.step = step0
                self._graph = g
                self.audit = report("rollout_old" if old else "rollout_current", g.raw_cuda_graph())
            if self._graph is not None:
                self._graph.replay()
            else:
                self._rollout()
                self._warm = True
            self.env_steps += r.num_steps * self.envs.num_envs
            if old:
                return self._ep[0].clone(), self._ep[1].clone()
            return self._ep_ret.sum(), (r.masks[1:] == 0).sum()

    return Audited(c, envs, pol, agent, deterministic=True, graphs=True), envs


def rollout(E=4096, U=8, old=True):
    tr, envs = _trainer(E, old)
    bad = 0
    for u in range(U):
        st = tr.update()
        r = tr.rollouts
        dones = int((r.masks[1:] == 0).sum())
        ssum = float(tr._ep_ret.sum())
        words = None
        if getattr(tr, "audit", None):
            words = [read_words(ms["dst"])[0] for ms in tr.audit["memsets"]]
        ok = st["episodes"] == dones and abs(st["mean_episode_return"] * max(st["episodes"], 1) - ssum) <= 1e-6 * abs(ssum) + 1e-9
        bad += not ok
        print("[%s] update %d graph=%s episodes %d (storage %d) sum %.3f (storage %.3f) %s memset words after: %s"
              % ("old" if old else "current", u, tr._graph is not None, st["episodes"], dones,
                 st["mean_episode_return"] * max(st["episodes"], 1), ssum, "OK" if ok else "WRONG", words), flush=True)
    print("[%s] %d of %d updates wrong" % ("old" if old else "current", bad, U), flush=True)
    envs.close()


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "iso"
    if mode == "iso":
        iso(int(sys.argv[2]) if len(sys.argv) > 2 else 2000)
    else:
        E = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
        U = int(sys.argv[3]) if len(sys.argv) > 3 else 8
        rollout(E, U, old=(mode == "rollout"))
