"""Device-resident rollout + PPO loop: the body of the reference's train.py:219-330, without host
round trips per step (train.py moves actions to the CPU, builds masks from Python lists and walks the
infos of every env at every step).

    trainer = RolloutTrainer(config, envs, actor_critic, agent)
    stats = trainer.update()      # num_steps env steps of every env + one PPO update

`envs` is a crowdnav_dsrnn_amd.envs.CrowdNavVecEnv (step_device path); episode returns are read from the
engine's Monitor counters where `done`.
"""
import time

import torch

from ..policy.utils import update_linear_schedule
from .storage import RolloutStorage, SRNNRolloutStorage


class RolloutTrainer:
    def __init__(self, config, envs, actor_critic, agent, deterministic=False, graphs=None):
        import os

        self.config = config
        # HIP-graph rollouts (collect); CN_NO_GRAPHS=1 or graphs=False: every rollout eager
        if graphs is None:
            graphs = envs.engine.device.type == "cuda" and os.environ.get("CN_NO_GRAPHS", "") in ("", "0")
        self.graphs = bool(graphs)
        self._graph, self._warm = None, False
        self.graph_audit = None   # node census of the captured rollout graph (collect)
        self._ones = self._ep_ret = None
        self.envs = envs
        self.ac = actor_critic
        self.agent = agent
        self.deterministic = deterministic
        dev = envs.engine.device
        self.device = dev
        if getattr(envs, "obs_mode", "srnn") == "convgru":   # train.py:157-172
            self.rollouts = RolloutStorage(config.ppo.num_steps, envs.num_envs, envs.observation_space.shape,
                                           envs.action_space, actor_critic.base.recurrent_hidden_state_size,
                                           device=dev, compact_hidden=True)
        else:
            self.rollouts = SRNNRolloutStorage(config.ppo.num_steps, envs.num_envs, envs.observation_space.spaces,
                                               envs.action_space, config.SRNN.human_node_rnn_size,
                                               config.SRNN.human_human_edge_rnn_size, "GRU", device=dev,
                                               compact_hidden=True)
        obs = envs.reset()
        if isinstance(self.rollouts.obs, dict):
            for k in self.rollouts.obs:
                self.rollouts.obs[k][0].copy_(obs[k])
        else:
            self.rollouts.obs[0].copy_(obs)
        self.srnn = getattr(actor_critic, "srnn", False) and isinstance(self.rollouts, SRNNRolloutStorage)
        self.episode_returns = []
        self.env_steps = 0
        # train.py:203-207: num_updates over the global env count (sharded runs: nenv of the engine)
        nenv = getattr(envs.engine.cfg, "nenv", envs.num_envs) or envs.num_envs
        self.num_updates = max(int(config.training.num_env_steps) // config.ppo.num_steps // nenv, 1)
        self.update_index = 0

    def _rollout(self):
        """num_steps env steps. Per step: act, cn_step, the storage writes (one multi-tensor copy) and one
        kernel of episode bookkeeping (the Monitor returns of the episodes that ended, into _ep_ret); collect()
        reduces the episode count and sum once per rollout, outside any captured graph."""
        r = self.rollouts
        T = r.num_steps
        if self._ones is None or self._ones.shape[0] != self.envs.num_envs:
            self._ones = torch.ones((self.envs.num_envs, 1), device=self.device)
            self._ep_ret = torch.zeros((T, self.envs.num_envs), dtype=torch.float64, device=self.device)
        for step in range(T):
            obs_s = {k: v[step] for k, v in r.obs.items()} if isinstance(r.obs, dict) else r.obs[step]
            hxs_s = r.hidden(step)
            # the new recurrent state goes straight into the storage slot insert() would copy it to
            value, action, logp, hxs = self.ac.act(obs_s, hxs_s, r.masks[step], deterministic=self.deterministic,
                                                   **({"out_hxs": r.hidden_slot()} if self.srnn else {}))
            obs, reward, done, _, _, ep_ret, _ = self.envs.step_device(action)
            masks = torch.rsub(done.unsqueeze(1), 1.0)   # 1 - done as float32 (one kernel)
            r.insert(obs, hxs, action, logp, value, reward.unsqueeze(1), masks, self._ones)
            torch.mul(ep_ret, done, out=self._ep_ret[step])   # Monitor return of the episodes that ended

    @torch.no_grad()
    def collect(self):
        """num_steps env steps of every env. With graphs (CUDA, the default): the first rollout runs eagerly
        (it also warms up the libraries), the second is captured once as one HIP graph -- act, cn_step (in
        graph mode: its launch sequence lives on the device, so its launches have no per-call arguments) and the storage
        writes of all steps -- and every rollout from then on is one replay of it: the same kernels on the
        same buffers in the same order, without the ~70 host-side launches per step."""
        r = self.rollouts
        if self.graphs and self._warm:
            if self._graph is None:
                import warnings

                from .. import _lib

                g = torch.cuda.CUDAGraph(keep_graph=True)   # kept until audited, then instantiated
                step0 = r.step
                try:
                    self.envs.engine.set_graph_mode(True)   # cn_step launches without per-call arguments
                    with torch.cuda.graph(g):   # records only; the replay below runs it
                        self._rollout()
                except RuntimeError as e:   # a capture-unsafe call on this path: stay eager
                    warnings.warn("rollout HIP-graph capture failed (%s); running eagerly" % e)
                    self.graphs = False
                    g = None
                    # eager cn_step launches take the host-sequenced kernels again (the capture recorded
                    # nothing that ran, so the device sequence words still equal the host's)
                    self.envs.engine.set_graph_mode(False)
                r.step = step0
                if g is not None:
                    # no memset nodes: this ROCm runtime can replay a memset node with stale bytes instead of its
                    # value (tools/graph_audit.py), e.g. the semaphore of a torch multi-block
                    # reduction, which then never writes its result
                    self.graph_audit = _lib.graph_node_counts(g.raw_cuda_graph())
                    if self.graph_audit.get("memset", 0):
                        warnings.warn("rollout HIP graph holds %d memset node(s) (%s); running eagerly"
                                      % (self.graph_audit["memset"], self.graph_audit))
                        self.graphs = False
                        g = None
                        self.envs.engine.set_graph_mode(False)
                    else:
                        g.instantiate()
                self._graph = g
        if self.graphs and self._graph is not None:
            self._graph.replay()   # (r.step is back at its start value: num_steps inserts wrap it)
        else:
            self._rollout()
            self._warm = True
        self.env_steps += r.num_steps * self.envs.num_envs
        # episode count and return sum of this rollout, reduced eagerly after it: the mask of slot s + 1 is 0
        # exactly when env step s ended an episode (insert() filled slots 1 .. T). Not in the captured graph:
        # torch's multi-block reductions zero their semaphore with hipMemsetAsync, i.e. a memset node, which
        # this runtime can replay with stale bytes -- round 4 saw the count reduction skip its write and the
        # count read the sum's bits from the recycled output block (profiles/r05/graph_audit/)
        return self._ep_ret.sum(), (r.masks[1:] == 0).sum()

    def update(self):
        """One rollout + PPO update. rollout_s / update_s are GPU time between HIP events recorded on the
        current stream (the mixed engine's side streams fork from and join back to it, so their work lies
        between the events); the update's one host sync (the losses) makes them
        readable at the end."""
        c = self.config
        if c.training.use_linear_lr_decay:   # train.py:216-222, before the rollout of update j
            update_linear_schedule(self.agent.optimizer, self.update_index, self.num_updates, c.training.lr)
        self.update_index += 1
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if self.device.type == "cuda" else None
        t0 = time.perf_counter()
        if ev:
            ev[0].record()
        ep_sum, ep_cnt = self.collect()
        r = self.rollouts
        with torch.no_grad():
            last = {k: v[-1] for k, v in r.obs.items()} if isinstance(r.obs, dict) else r.obs[-1]
            next_value = self.ac.get_value(last,
                                           r.hidden(r.num_steps),
                                           r.masks[-1]).detach()
        r.compute_returns(next_value, c.ppo.use_gae, c.reward.gamma, c.ppo.gae_lambda,
                          c.training.use_proper_time_limits)
        if ev:
            ev[1].record()
        t1 = time.perf_counter()
        losses = self.agent.update(r)
        r.after_update()
        if ev:
            ev[2].record()
        n = int(ep_cnt.item())
        t2 = time.perf_counter()
        if ev:
            ev[2].synchronize()
            rollout_s, update_s = ev[0].elapsed_time(ev[1]) / 1e3, ev[1].elapsed_time(ev[2]) / 1e3
        else:
            rollout_s, update_s = t1 - t0, t2 - t1
        return {"value_loss": losses[0], "action_loss": losses[1], "dist_entropy": losses[2],
                "episodes": n, "mean_episode_return": float(ep_sum.item()) / max(n, 1),
                "rollout_s": rollout_s, "update_s": update_s, "host_s": t2 - t0}
