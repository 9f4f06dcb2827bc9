"""Batched test-time evaluation and social metrics.

Same entry points as the reference:
    evaluate(actor_critic, ob_rms, eval_envs, num_processes, device, config, logging, visualize=False,
             recurrent_type="GRU")                         pytorchBaselines/evaluation.py:14-334
    Metrics(logging).add_metric(name, sample) / log_metrics()  pytorchBaselines/metrics.py:5-44

The reference runs test_size episodes one after the other in a single env. Env i of a VecEnv with
num_envs = E envs (phase 'test', nenv = E) draws its k-th episode from seed offset + i + k*E
(crowd_sim_dict.py:147-164), so the E envs together run exactly the reference's episodes 0..test_size-1
(global episode index g = i + k*E), concurrently. Per-env running sums live on the device
(EpisodeRecorder) and are written, at each episode end, into per-episode records at index g; episodes
with g >= test_size are run but not counted. After the loop the records are copied to the host once and
the reference's bookkeeping (outcome bins, scenario breakdown, side-preference counters, Metrics) is
replayed in episode order, so the logged numbers are the ones the sequential loop produces.

Reference quirks kept on purpose:
  * the "time in danger" log line is always 0 / nan (see _report);
  * path length and heading change are accumulated in float32 from the float32 observation (NEP 50:
    `0.0 + np.float32` stays float32) and the step that ends an episode measures the jump to the NEXT
    episode's first observation (auto-reset returns it; evaluation.py:158-178). In the sequential loop
    that is episode k+1's spawn; here the env's next episode is k+E, so the device sums stop before that
    last jump and the host adds ||last_pos_k - first_pos_{k+1}|| (episode test_size re-uses seed 0's
    spawn because the test case counter wraps, crowd_sim_dict.py:162-164). The heading change of that
    jump needs no fix-up: every reset observation has zero velocity, so its heading is atan2(0, 0) = 0;
  * the recorded time of an episode is the env time before its last step (evaluation.py:148-149);
  * the side-preference counters are never reset between episodes, only divided by the episode length
    (evaluation.py:85-86,237-239).
Multi-GPU: with torch.distributed initialised each rank evaluates its env shard (global env index
rank*E + i, nenv = world*E) with no communication in the loop; the records are summed once at the end.
"""
import numpy as np
import torch

from . import abi

_SUCCESS, _COLLISION, _TIMEOUT = "success", "collision", "timeout"


class Metrics:
    """metrics.py:5-44: mean, population std and a 90% Student-t confidence interval per metric."""

    def __init__(self, logging_obj):
        self._metrics_dict = dict()
        self.logging = logging_obj

    def add_metric(self, name, sample):
        self._metrics_dict[name] = self._calculate_metrics(sample)

    @staticmethod
    def _calculate_metrics(sample, confidence_level=0.9):
        import scipy.stats

        a = np.array(sample)
        mean = np.mean(a)
        ci = scipy.stats.t.interval(confidence_level, a.size - 1, mean, scipy.stats.sem(a))
        return [mean, np.std(a), list(ci)]

    def __getitem__(self, name):
        return self._metrics_dict[name]

    def keys(self):
        return self._metrics_dict.keys()

    def log_metrics(self, name="all"):
        def one(key):
            m = self._metrics_dict[key]
            self.logging.info("")
            self.logging.info(f"{key} ======")
            self.logging.info(f"MEAN: {m[0]:.4f}")
            self.logging.info(f"STD DEV: {m[1]:.4f}")
            self.logging.info(f"CI: [{m[2][0]:.4f},{m[2][1]:.4f}]")

        if "all" in name:
            for key in self._metrics_dict:
                one(key)
        elif name in self._metrics_dict:
            one(name)
        else:
            raise KeyError(f"{name} not in metrics_dict")


def create_events_dict(config):
    """helper.py:58-78: outcome x scenario counters."""
    scenarios = set(config.sim.train_val_sim).union(set(config.sim.test_sim))
    return {k: dict([("total", 0)] + [(s, 0) for s in scenarios]) for k in (_SUCCESS, _COLLISION, _TIMEOUT)}


def log_events_dict(events_dict, logger):
    """helper.py:88-102."""
    for k in events_dict:
        logger.info("")
        logger.info(f"{k.upper()} CASES: ")
        for scenario, count in events_dict[k].items():
            logger.info(f"{scenario}: {count}")


class EpisodeRecorder:
    """Per-env episode sums on the device and per-episode records indexed by the global episode index.

    step(obs, reward, done, event, info) consumes one VecEnv step (the tensors of CrowdNavVecEnv.step_device)
    without any host synchronisation."""

    F64 = ("gt", "raw", "disc", "pv", "pathv", "agg", "jerk", "sv", "dsum")
    F32 = ("path", "chc", "lastx", "lasty")
    I32 = ("steps", "left", "right", "dcnt")

    def __init__(self, num_envs, test_size, env_offset, nenv, device, time_step, gamma, v_pref,
                 side_preference=False, side_scenario=None, scenario_names=(), keep_traces=True):
        E = int(num_envs)
        self.E, self.test_size, self.nenv = E, int(test_size), int(nenv)
        self.dev = torch.device(device)
        self.dt, self.gamma, self.v_pref = float(time_step), float(gamma), float(v_pref)
        self.side = bool(side_preference)
        self.side_id = list(scenario_names).index(side_scenario) if self.side else -1
        self.keep_traces = keep_traces
        z = lambda dt: torch.zeros(E, dtype=dt, device=self.dev)  # noqa: E731
        self.run = {k: z(torch.float64) for k in self.F64}
        self.run.update({k: z(torch.float32) for k in self.F32})
        self.run.update({k: z(torch.int32) for k in self.I32})
        self.ep = torch.arange(E, dtype=torch.int64, device=self.dev) + int(env_offset)
        # one spare slot (index test_size) absorbs the writes of uncounted episodes
        n = self.test_size + 1
        self.rec = {k: torch.zeros(n, dtype=v.dtype, device=self.dev) for k, v in self.run.items()}
        self.rec["event"] = torch.zeros(n, dtype=torch.int32, device=self.dev)
        self.rec["scenario"] = torch.zeros(n, dtype=torch.int32, device=self.dev)
        self.rec["done"] = torch.zeros(n, dtype=torch.int32, device=self.dev)
        self.rec["firstx"] = torch.zeros(n, dtype=torch.float32, device=self.dev)
        self.rec["firsty"] = torch.zeros(n, dtype=torch.float32, device=self.dev)
        self.recorded = torch.zeros((), dtype=torch.int64, device=self.dev)
        g0 = int(env_offset)
        self.target = sum(max(0, -(-(self.test_size - (g0 + i)) // self.nenv)) for i in range(E))
        self.last_pos = None
        self.last_angle = None
        self.traces = []

    def start(self, obs):
        self.last_pos = obs["robot_node"][:, 0, 0:2].float().clone()
        te = obs["temporal_edges"][:, 0, :].float()
        self.last_angle = torch.atan2(te[:, 1], te[:, 0])
        self._write_first(torch.ones(self.E, dtype=torch.bool, device=self.dev), self.ep, self.last_pos)

    def _write_first(self, mask, ep, pos):
        idx = torch.where(mask & (ep < self.test_size), ep, torch.full_like(ep, self.test_size))
        self.rec["firstx"].scatter_(0, idx, pos[:, 0].contiguous())
        self.rec["firsty"].scatter_(0, idx, pos[:, 1].contiguous())

    def step(self, obs, reward, done, event, info):
        r, run, dt = self.run, self.run, self.dt
        rew = reward.reshape(-1).double()
        ev = event.reshape(-1).to(torch.int32)
        done_b = done.reshape(-1).bool()
        f = info.float()
        t = r["steps"].double()
        # evaluation.py:254-257 discount pow(gamma, t * time_step * v_pref); sums in episode order
        run["raw"] += rew
        run["disc"] += torch.pow(torch.tensor(self.gamma, dtype=torch.float64, device=self.dev),
                                 t * dt * self.v_pref) * rew
        pos = obs["robot_node"][:, 0, 0:2].float()
        d = self.last_pos - pos
        run["lastx"] = self.last_pos[:, 0].clone()
        run["lasty"] = self.last_pos[:, 1].clone()
        jump = torch.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
        run["path"] += torch.where(done_b, torch.zeros_like(jump), jump)   # the terminal jump: see module doc
        te = obs["temporal_edges"][:, 0, :].float()
        ang = torch.atan2(te[:, 1], te[:, 0])
        run["chc"] += (ang - self.last_angle).abs()
        self.last_pos = pos.clone()
        self.last_angle = ang
        # evaluation.py:188-230 (info fields are integers except jerk / min_dist)
        pv = f[:, abi.INFO_PERSONAL_VIOLATION].to(torch.int32)
        pathv = f[:, abi.INFO_PATH_VIOLATION].to(torch.int32)
        agg = f[:, abi.INFO_AGG_NAV_TIME].to(torch.int32)
        sv = f[:, abi.INFO_SPEED_VIOLATION].to(torch.int32)
        zero = torch.zeros_like(rew)
        run["pv"] += torch.where(pv == 1, zero + dt, zero)
        run["pathv"] += torch.where(pathv != 0, dt * pathv.double(), zero)
        run["agg"] += torch.where(agg != 0, dt * agg.double(), zero)
        run["jerk"] += f[:, abi.INFO_JERK_COST].double()
        run["sv"] += torch.where(sv == 1, zero + dt, zero)
        danger = ev == abi.EV_DANGER
        run["dsum"] += torch.where(danger, f[:, abi.INFO_MIN_DIST].double(), zero)
        run["dcnt"] += danger.to(torch.int32)
        if self.side:
            here = f[:, abi.INFO_SCENARIO].to(torch.int32) == self.side_id
            left = here & (f[:, abi.INFO_SIDE_LEFT].to(torch.int32) == 1)
            right = here & ~left & (f[:, abi.INFO_SIDE_RIGHT].to(torch.int32) == 1)
            run["left"] += left.to(torch.int32)
            run["right"] += right.to(torch.int32)
        run["steps"] += 1
        if self.keep_traces:
            self.traces.append((reward.reshape(-1).float().clone(), f[:, abi.INFO_DIST_TO_GOAL].clone(),
                                done_b.clone(), self.ep.clone()))
        counted = done_b & (self.ep < self.test_size)
        idx = torch.where(counted, self.ep, torch.full_like(self.ep, self.test_size))
        for k, v in run.items():
            self.rec[k].scatter_(0, idx, v)
        self.rec["event"].scatter_(0, idx, ev)
        self.rec["scenario"].scatter_(0, idx, f[:, abi.INFO_SCENARIO].to(torch.int32))
        self.rec["done"].scatter_(0, idx, counted.to(torch.int32))
        self.recorded += counted.sum()
        # global_time advances by dt per step (crowd_sim_dict.py:253) and restarts at the auto-reset
        run["gt"] += dt
        for k, v in run.items():
            v.masked_fill_(done_b, 0)
        self.ep += torch.where(done_b, self.nenv, 0)
        self._write_first(done_b, self.ep, pos)

    def finished(self):
        return int(self.recorded.item()) >= self.target

    def host_records(self, dist=None):
        rec = {k: v[:self.test_size].clone() for k, v in self.rec.items()}
        if dist is not None:
            for v in rec.values():
                dist.all_reduce(v)
        return {k: v.cpu().numpy() for k, v in rec.items()}

    def episode_traces(self):
        """Per counted episode g: (per-step rewards, per-step non-zero dist_to_goal) as Python lists."""
        out = {}
        if not self.traces:
            return out
        rew = torch.stack([x[0] for x in self.traces]).cpu().numpy()
        d2g = torch.stack([x[1] for x in self.traces]).cpu().numpy()
        dn = torch.stack([x[2] for x in self.traces]).cpu().numpy()
        ep = torch.stack([x[3] for x in self.traces]).cpu().numpy()
        for e in range(rew.shape[1]):
            r_l, d_l = [], []
            for s in range(rew.shape[0]):
                r_l.append(float(rew[s, e]))
                if float(d2g[s, e]):
                    d_l.append(float(d2g[s, e]))
                if dn[s, e]:
                    if ep[s, e] < self.test_size:
                        out[int(ep[s, e])] = (r_l, d_l)
                    r_l, d_l = [], []
        return out


def _dist():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def evaluate(actor_critic, ob_rms, eval_envs, num_processes, device, config, logging, visualize=False,
             recurrent_type="GRU", keep_traces=True, verbose=True, check_every=8):
    """evaluation.py:14-334 over a batched CrowdNavVecEnv (see the module docstring). Returns
    (raw_rewards, discounted_rewards, dist_to_goal) binned by outcome like the reference (per-episode
    per-step lists; empty lists when keep_traces=False)."""
    if ob_rms:
        raise NotImplementedError("observation normalisation (VecNormalize) is not part of the build")
    E = eval_envs.num_envs
    if num_processes != E:
        raise ValueError("num_processes=%d but the VecEnv holds %d envs" % (num_processes, E))
    dist = _dist()
    cn = eval_envs.cn_cfg
    rnn_factor = 2 if recurrent_type == "LSTM" else 1
    hxs = {"human_node_rnn": torch.zeros(E, 1, config.SRNN.human_node_rnn_size * rnn_factor, device=device),
           "human_human_edge_rnn": torch.zeros(E, actor_critic.base.human_num + 1,
                                               config.SRNN.human_human_edge_rnn_size * rnn_factor, device=device)}
    masks = torch.zeros(E, 1, device=device)
    test_size = int(config.env.test_size)
    side = bool(config.test.side_preference)
    scenario = None
    if side:
        assert len(config.sim.test_sim) == 1
        scenario = config.sim.test_sim[0]
    gamma = 0.99
    dt = float(config.env.time_step)
    rec = EpisodeRecorder(E, test_size, int(cn.env_offset), int(cn.nenv), eval_envs.engine.device, dt, gamma,
                          float(config.robot.v_pref), side, scenario, eval_envs.scenario_names, keep_traces)
    obs = eval_envs.reset()
    rec.start(obs)
    n = 0
    while True:
        with torch.no_grad():
            _, action, _, hxs = actor_critic.act(obs, hxs, masks, deterministic=True)
        if visualize:
            eval_envs.render()
        obs, reward, done, event, info, _, _ = eval_envs.step_device(action)
        rec.step(obs, reward, done, event, info)
        masks = (1.0 - done.float()).unsqueeze(1).to(device)
        n += 1
        if n % check_every == 0 and rec.finished():
            break
    r = rec.host_records(dist)
    traces = rec.episode_traces() if keep_traces else {}
    if dist is not None and keep_traces:
        gathered = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, traces)
        traces = {k: v for d in gathered for k, v in d.items()}
    return _report(r, traces, config, logging, test_size, dt, gamma, side, scenario, eval_envs, verbose)


def _report(r, traces, config, logging, test_size, dt, gamma, side, scenario, eval_envs, verbose):
    """The reference's per-episode bookkeeping and logging (evaluation.py:233-332), replayed in episode
    order from the records."""
    if not np.all(r["done"] == 1):
        raise RuntimeError("evaluation ended with %d of %d episodes unrecorded" % (int((r["done"] != 1).sum()),
                                                                                  test_size))
    names = eval_envs.scenario_names
    time_limit = float(config.env.time_limit)
    v_pref = float(config.robot.v_pref)
    metrics = Metrics(logging)
    success_times, success_cases, collision_times, collision_cases, timeout_times, timeout_cases = ([] for _ in
                                                                                                   range(6))
    bins = {_SUCCESS: [], _COLLISION: [], _TIMEOUT: []}
    raw_rewards = {k: [] for k in bins}
    discounted_rewards = {k: [] for k in bins}
    dist_to_goal = {k: [] for k in bins}
    raw_sums = {k: [] for k in bins}
    disc_sums = {k: [] for k in bins}
    path_lengths, chc_total = [], []
    pv_t, pathv_t, agg_t, jerk_t, sv_t = [], [], [], [], []
    side_pref = {s: {"left": 0, "right": 0} for s in ("side_pref_passing", "side_pref_overtaking",
                                                      "side_pref_crossing")}
    side_counter = {"left": 0, "right": 0}
    num_events = create_events_dict(config)
    path = []
    for k in range(test_size):
        nk = (k + 1) % test_size
        jump = np.linalg.norm(np.array([r["lastx"][k] - r["firstx"][nk], r["lasty"][k] - r["firsty"][nk]]))
        path.append(r["path"][k] + jump)
    n_danger = 0
    danger_sum = 0.0
    for k in range(test_size):
        steps = int(r["steps"][k])
        ev = int(r["event"][k])
        gt = float(r["gt"][k])
        n_danger += int(r["dcnt"][k])
        danger_sum += float(r["dsum"][k])
        if side:
            for _ in range(int(r["left"][k])):
                side_counter["left"] += 1
            for _ in range(int(r["right"][k])):
                side_counter["right"] += 1
            for s in side_counter:
                side_counter[s] /= steps
        if traces:
            ep_rew, ep_d2g = traces[k]
            ep_disc = [pow(gamma, t * dt * v_pref) * x for t, x in enumerate(ep_rew)]
        else:
            ep_rew, ep_d2g, ep_disc = [], [], []
        raw = float(r["raw"][k])
        disc = float(r["disc"][k])
        if verbose:
            print("")
            print("Episode", k, "ends in", steps, "steps")
        scen = names[int(r["scenario"][k])]
        if ev == abi.EV_REACHGOAL:
            key = _SUCCESS
            success_times.append(gt)
            success_cases.append(k)
            chc_total.append(float(r["chc"][k]))
            path_lengths.append(path[k])
            pv_t.append(float(r["pv"][k]))
            pathv_t.append(float(r["pathv"][k]))
            agg_t.append(float(r["agg"][k]))
            jerk_t.append(float(r["jerk"][k]))
            sv_t.append(float(r["sv"][k]))
            if side:
                if side_counter["left"] > side_counter["right"]:
                    side_pref[scenario]["left"] += 1
                elif side_counter["left"] < side_counter["right"]:
                    side_pref[scenario]["right"] += 1
            msg = "Success"
        elif ev == abi.EV_COLLISION:
            key = _COLLISION
            collision_cases.append(k)
            collision_times.append(gt)
            msg = "Collision"
        elif ev == abi.EV_TIMEOUT:
            key = _TIMEOUT
            timeout_cases.append(k)
            timeout_times.append(time_limit)
            msg = "Time out"
        else:
            raise ValueError("Invalid end signal from environment")
        raw_rewards[key].append(ep_rew)
        discounted_rewards[key].append(ep_disc)
        dist_to_goal[key].append(ep_d2g)
        raw_sums[key].append(raw)
        disc_sums[key].append(disc)
        num_events[key]["total"] += 1
        num_events[key][scen] += 1
        if verbose:
            print(msg)
            print(f"Reward={raw}")
            print(f"Path Length: {path[k]:.2f}")
            print(f"Time Taken: {gt:.2f}")

    success_rate = len(success_times) / test_size
    collision_rate = len(collision_times) / test_size
    timeout_rate = len(timeout_times) / test_size
    assert len(success_times) + len(collision_times) + len(timeout_times) == test_size
    logging.info("TEST")
    total_time = sum(success_times + collision_times + timeout_times)
    # evaluation.py:147-148 tests isinstance(info["info"], Danger), but info["info"] is the step_info dict,
    # so the reference's min_dist list stays empty and it always logs 0 / nan here. The log keeps that;
    # the real danger statistics are in evaluate.last["danger_steps"] / ["avg_min_dist"].
    ref_n_danger = 0
    logging.info(f"Total time in danger: {(ref_n_danger * dt / total_time):.4f}, "
                 f"average min distance in danger: {float('nan'):.4f}")
    avg_min_dist = danger_sum / n_danger if n_danger > 0 else float("nan")
    logging.info(f"success rate: {success_rate:.3f}")
    logging.info(f"collision rate: {collision_rate:.3f}")
    logging.info(f"timeout rate: {timeout_rate:.3f}")
    logging.info("Success cases: " + " ".join([str(x) for x in success_cases]))
    logging.info("Collision cases: " + " ".join([str(x) for x in collision_cases]))
    logging.info("Timeout cases: " + " ".join([str(x) for x in timeout_cases]))
    logging.info("")
    logging.info("SCENARIO BREAKDOWN: ")
    log_events_dict(num_events, logging)
    metrics.add_metric("navigation time", success_times)
    metrics.add_metric("path length", path_lengths)
    metrics.add_metric("discounted reward", [x for key in bins for x in disc_sums[key]])
    metrics.add_metric("non-discounted rewards", [x for key in bins for x in raw_sums[key]])
    metrics.add_metric("cumulative heading change", chc_total)
    if config.test.social_metrics:
        metrics.add_metric("SM1 - personal space violation", pv_t)
        metrics.add_metric("SM2 - path violation", pathv_t)
        metrics.add_metric("SM3 - aggregate time", agg_t)
        metrics.add_metric("SM4 - jerk cost", jerk_t)
        metrics.add_metric("SM5 - speed violation", sv_t)
    if side:
        logging.info("")
        logging.info(f"Side Preference - {scenario} ======")
        logging.info(f"Left % = {100 * side_pref[scenario]['left'] / test_size:.3f}%")
        logging.info(f"Right % = {100 * side_pref[scenario]['right'] / test_size:.3f}%")
    metrics.log_metrics()
    eval_envs.close()
    evaluate.last = {"metrics": metrics, "num_events": num_events, "success_rate": success_rate,
                     "collision_rate": collision_rate, "timeout_rate": timeout_rate, "records": r,
                     "danger_steps": n_danger, "avg_min_dist": avg_min_dist,
                     "side_preferences": side_pref if side else None}
    return raw_rewards, discounted_rewards, dist_to_goal
