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
        L.hipMemsetAsync.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, vp]
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


def dot_names(txt):
    """{node index: label} of a hipGraphDebugDotPrint dump (kernel nodes: the mangled kernel name)."""
    out = {}
    for i, lab in re.findall(r'"graph_0_node_(\d+)"\[[^\]]*?label="\d+\n(.*?)"\];', txt, re.S):
        out[int(i)] = lab.strip().split("\n")[0]
    return out


def report(tag, graph):
    os.makedirs(OUT, exist_ok=True)
    nodes = walk(graph)
    s = summarize(nodes)
    dpath = os.path.join(OUT, "%s.dot" % tag)
    names = {}
    try:
        _, txt = dot(graph, dpath)
        s["dot"] = os.path.relpath(dpath, REPO)
        names = dot_names(txt)
    except Exception as e:   # the walk above is the evidence; the dump is a convenience
        s["dot_error"] = str(e)
    for nd in nodes:
        nd["name"] = names.get(nd["i"], "")
    kh = {}
    for nd in nodes:
        if nd["type"] == "kernel":
            kh[nd["name"][:110]] = kh.get(nd["name"][:110], 0) + 1
    s["kernel_histogram"] = dict(sorted(kh.items(), key=lambda kv: -kv[1]))
    json.dump({"summary": s, "nodes": nodes}, open(os.path.join(OUT, "%s.json" % tag), "w"), indent=1, default=str)
    brief = {k: v for k, v in s.items() if k not in ("memsets", "kernel_histogram")}
    print("[%s] %s" % (tag, json.dumps(brief, default=str)), flush=True)
    for k, v in s["kernel_histogram"].items():
        print("[%s]   %5d x %s" % (tag, v, k), flush=True)
    for m in s["memsets"]:
        i = m["i"]
        nxt = nodes[i + 1]["name"][:90] if i + 1 < len(nodes) else ""
        prv = nodes[i - 1]["name"][:90] if i > 0 else ""
        print("[%s]   memset node %d: dst 0x%x, %d B, value %d, after [%s] before [%s]"
              % (tag, i, m["dst"], m["bytes"], m["value"], prv, nxt), flush=True)
    return s


# ---------------------------------------------------------------------------------------------------------------
def _alloc_trace():
    """Allocator events recorded since _record_memory_history was switched on: (action, addr, size)."""
    snap = torch.cuda.memory._snapshot()
    out = []
    for dev_trace in snap.get("device_traces", []):
        for ev in dev_trace:
            out.append((ev["action"], ev["addr"], ev["size"]))
    return out


def iso(R=2000):
    """The two round-4 reductions alone: ep_sum += x.sum() (f64, T x E), ep_cnt += (m == 0).sum() (int64),
    captured once and replayed R times. Before each replay the inputs are redrawn in place (so an output a
    reduction failed to write is stale and shows) and the accumulators zeroed; after it the results are
    compared with the same reductions run eagerly, and 8 words at each memset destination are read back."""
    dev = torch.device("cuda:0")
    T, E = 128, 4096
    g0 = torch.Generator(device=dev)
    g0.manual_seed(3)
    x = torch.randn((T, E), generator=g0, device=dev, dtype=torch.float64)
    m = (torch.rand((T, E, 1), generator=g0, device=dev) > 0.02).float()
    ep_s = torch.zeros((), dtype=torch.float64, device=dev)
    ep_c = torch.zeros((), dtype=torch.int64, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside capture
        ep_s += x.sum()
        ep_c += (m == 0).sum()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    torch.cuda.memory._record_memory_history(max_entries=100000)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        ep_s += x.sum()
        ep_c += (m == 0).sum()
    trace = _alloc_trace()
    torch.cuda.memory._record_memory_history(enabled=None)
    summ = report("iso", g.raw_cuda_graph())
    for a in trace:
        print("[iso] allocator during capture: %-14s addr 0x%x size %d" % a, flush=True)
    sems = [ms["dst"] for ms in summ["memsets"]]
    bad_s = bad_c = 0
    hist = {}
    first = []
    for r in range(R):
        x.normal_(generator=g0)
        m.copy_((torch.rand((T, E, 1), generator=g0, device=dev) > 0.02).float())
        ep_s.zero_()
        ep_c.zero_()
        g.replay()
        torch.cuda.synchronize()
        words = tuple(tuple(read_words(a, 8)) for a in sems)
        key = tuple(w[0] for w in words)
        hist[key] = hist.get(key, 0) + 1
        want_s, want_c = float(x.sum()), int((m == 0).sum())
        cs, cc = float(ep_s), int(ep_c)
        ws, wc = cs != want_s, cc != want_c
        bad_s += ws
        bad_c += wc
        if (ws or wc or r < 3) and len(first) < 12:
            first.append((r, cs, want_s, cc, want_c, ["%08x" % v for w in words for v in w]))
    print("[iso] %d replays with fresh inputs: %d wrong sums, %d wrong counts" % (R, bad_s, bad_c), flush=True)
    print("[iso] first word at each memset destination after the replay: %s" % {str(k): v for k, v in hist.items()},
          flush=True)
    for f in first:
        print("[iso]   replay %d: sum %r (eager %r) count %d (eager %d); words at memset dsts %s" % f, flush=True)


def iso_const(R=2000, sentinel=False):
    """The round-4 reductions with CONSTANT inputs and only the accumulators' zero fills between replays (the
    first probe's condition, under which the second memset's destination read 0x01010141 after every replay
    but the first). sentinel=True: the two sums go to preallocated outputs that are filled with a sentinel
    (NaN / -7) before each replay, so a reduction that does not write its output shows."""
    dev = torch.device("cuda:0")
    T, E = 128, 4096
    g0 = torch.Generator(device=dev)
    g0.manual_seed(3)
    x = torch.randn((T, E), generator=g0, device=dev, dtype=torch.float64)
    m = (torch.rand((T, E, 1), generator=g0, device=dev) > 0.02).float()
    want_s, want_c = float(x.sum()), int((m == 0).sum())
    ep_s = torch.zeros((), dtype=torch.float64, device=dev)
    ep_c = torch.zeros((), dtype=torch.int64, device=dev)
    s_out = torch.zeros((), dtype=torch.float64, device=dev)
    c_out = torch.zeros((), dtype=torch.int64, device=dev)

    def body():
        if sentinel:
            torch.sum(x, dim=(0, 1), out=s_out)
            torch.sum(m == 0, dim=(0, 1, 2), out=c_out)
            ep_s.add_(s_out)
            ep_c.add_(c_out)
        else:
            ep_s.add_(x.sum())
            ep_c.add_((m == 0).sum())

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        body()
    tag = "iso_sentinel" if sentinel else "iso_const"
    summ = report(tag, g.raw_cuda_graph())
    sems = [ms["dst"] for ms in summ["memsets"]]
    hist, bad, unwritten, first = {}, 0, [0, 0], []
    for r in range(R):
        ep_s.zero_()
        ep_c.zero_()
        if sentinel:
            s_out.fill_(float("nan"))
            c_out.fill_(-7)
        g.replay()
        torch.cuda.synchronize()
        words = tuple(tuple(read_words(a, 4)) for a in sems)
        key = tuple(w[0] for w in words)
        hist[key] = hist.get(key, 0) + 1
        cs, cc = float(ep_s), int(ep_c)
        wrong = cs != want_s or cc != want_c
        bad += wrong
        if sentinel:
            unwritten[0] += s_out.isnan().item()
            unwritten[1] += int(c_out.item()) == -7
        if (wrong or r < 3 or (r > 0 and key != first[-1][-1] if first else False)) and len(first) < 12:
            first.append((r, cs, cc, key))
    print("[%s] %d replays (constant inputs, want sum %r count %d): %d wrong; outputs left unwritten: %s"
          % (tag, R, want_s, want_c, bad, unwritten if sentinel else "n/a"), flush=True)
    print("[%s] first word at each memset destination after the replay: %s"
          % (tag, {"(" + ", ".join("0x%08x" % v for v in k) + ")": n for k, n in hist.items()}), flush=True)
    for f in first:
        print("[%s]   replay %d: sum %r count %d; memset words %s" % ((tag,) + f[:3] + (["0x%08x" % v for v in f[3]],)),
              flush=True)


def memset_probe(R=2000):
    """Memset nodes alone: a graph of hipMemsetAsync(value 0) nodes (4 and 16 bytes) around one small
    kernel, replayed R times; before each replay the destinations are filled with 0x7f7f7f7f eagerly. In the
    second half an eager hipMemsetAsync(value 1, 4 bytes) to another buffer also precedes each replay (the
    engine's graph-mode cn_reset / cn_set_state issue exactly that: CN_CTL_ALL = 1). After each replay
    every destination must read 0."""
    dev = torch.device("cuda:0")
    L = hip()
    A = torch.zeros(4096, dtype=torch.int32, device=dev)
    Bz = torch.zeros(1024, dtype=torch.int32, device=dev)
    base = A.data_ptr()

    def ms(off_words, nbytes, value, stream):
        _ck(L.hipMemsetAsync(ctypes.c_void_p(base + 4 * off_words), value, nbytes,
                             ctypes.c_void_p(stream.cuda_stream)), "hipMemsetAsync")

    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        cs = torch.cuda.current_stream()
        ms(0, 4, 0, cs)
        A[512:1024].add_(1)
        ms(1024, 4, 0, cs)
        ms(2048, 16, 0, cs)
    report("memset_probe", g.raw_cuda_graph())
    bad = [0, 0]
    seen = {}
    for r in range(R):
        A[0:1].fill_(0x7f7f7f7f)
        A[1024:1025].fill_(0x7f7f7f7f)
        A[2048:2052].fill_(0x7f7f7f7f)
        half = r >= R // 2
        if half:
            _ck(L.hipMemsetAsync(ctypes.c_void_p(Bz.data_ptr()), 1, 4,
                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "hipMemsetAsync")
        g.replay()
        torch.cuda.synchronize()
        vals = (int(A[0]), int(A[1024])) + tuple(int(v) for v in A[2048:2052].tolist())
        if any(vals):
            bad[half] += 1
            key = tuple("0x%08x" % (v & 0xffffffff) for v in vals)
            seen[key] = seen.get(key, 0) + 1
    print("[memset_probe] %d replays: %d with a nonzero destination without an eager value-1 memset before them, "
          "%d with one; values seen: %s" % (R, bad[0], bad[1], seen), flush=True)


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

        @torch.no_grad()
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
    elif mode == "memset":
        memset_probe(int(sys.argv[2]) if len(sys.argv) > 2 else 2000)
    elif mode in ("iso_const", "iso_sentinel"):
        iso_const(int(sys.argv[2]) if len(sys.argv) > 2 else 2000, sentinel=mode == "iso_sentinel")
    else:
        E = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
        U = int(sys.argv[3]) if len(sys.argv) > 3 else 8
        rollout(E, U, old=(mode == "rollout"))
