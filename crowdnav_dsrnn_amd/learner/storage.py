"""SRNNRolloutStorage (pytorchBaselines/a2c_ppo_acktr/storage.py:14-292), device resident.

API and semantics as the reference: obs / recurrent_hidden_states dicts of (T+1, E, ...) tensors,
insert(), after_update(), compute_returns() (all four GAE / proper-time-limit branches, :132-177) and the
two minibatch generators. compact_hidden=True keeps 2 hidden-state slots instead of T+1
(slot 0 = rollout start, read by the recurrent generator; slot 1 = latest, carried by after_update): 96 MB
instead of 6.2 GB at 4096 envs x 128 steps. Its recurrent_hidden_states still index like the reference's
(T+1)-step tensors (CompactSteps): [0] is the rollout start, any other step the latest state -- what
train.py reads at [step] before act() and at [-1] for the next value -- so train.py runs unmodified.
The generators gather with index tensors instead of per-env Python loops; the
environment permutation is drawn with torch.randperm on the default CPU generator exactly as the
reference does (:231), so a seeded run produces the same minibatches.
"""
import torch


class CompactSteps:
    """A (2, ...) hidden-state tensor indexed as the (T+1, ...) one it replaces: integer index 0 (or
    -(T+1)) is slot 0 (the rollout start), every other step is slot 1 (the latest state, the only one a
    rollout reads after step 0); slices and every tensor attribute go to the 2-slot tensor itself."""

    def __init__(self, t, T):
        self.t, self.T = t, T

    def _slot(self, i):
        i = int(i)
        if not -(self.T + 1) <= i <= self.T:
            raise IndexError("step %d out of range for %d steps" % (i, self.T))
        return 0 if i in (0, -(self.T + 1)) else 1

    @staticmethod
    def _is_step(i):
        """A single step index: a Python / numpy integer or a 0-dim integer tensor (anything with
        __index__ that is not a slice or a multi-element tensor)."""
        if isinstance(i, torch.Tensor):
            return i.dim() == 0 and not i.is_floating_point() and not i.is_complex() and i.dtype != torch.bool
        return isinstance(i, int) or (hasattr(i, "__index__") and not isinstance(i, slice))

    def __getitem__(self, i):
        if self._is_step(i):
            return self.t[self._slot(i)]
        return self.t[i]

    def __setitem__(self, i, v):   # same step mapping as __getitem__ (numpy / tensor scalars included)
        if self._is_step(i):
            self.t[self._slot(i)] = v
        else:
            self.t[i] = v

    def __len__(self):   # the step count it stands for; .shape / .size() are the 2-slot tensor's own
        return self.T + 1

    def to(self, *a, **kw):
        return CompactSteps(self.t.to(*a, **kw), self.T)

    def __getattr__(self, n):
        return getattr(self.t, n)


def _raw(v):
    return v.t if isinstance(v, CompactSteps) else v


def _copy_all(dst, src):
    """dst[i].copy_(src[i]) for all i: one multi-tensor kernel when every pair has the same shape and
    dtype (the rollout's storage writes: one launch per step instead of ~10), else one copy each."""
    same = all(d.shape == x.shape and d.dtype == x.dtype and d.device == x.device for d, x in zip(dst, src))
    if same and dst and dst[0].is_cuda:
        torch._foreach_copy_(dst, src)
    else:
        for d, x in zip(dst, src):
            d.copy_(x)


def _flatten_helper(T, N, x):
    if isinstance(x, dict):
        return {k: v.reshape(T * N, *v.shape[2:]) for k, v in x.items()}
    return x.reshape(T * N, *x.shape[2:])


class SRNNRolloutStorage:
    def __init__(self, num_steps, num_processes, obs_shape, action_space, human_node_rnn_size,
                 human_human_edge_rnn_size, recurrent_cell_type="GRU", device=None, compact_hidden=False):
        T, E = num_steps, num_processes
        self.compact_hidden = bool(compact_hidden)
        TH = 2 if compact_hidden else T + 1
        dev = device
        self.obs = {k: torch.zeros(T + 1, E, *tuple(sp.shape), device=dev) for k, sp in obs_shape.items()}
        self.human_num = tuple(obs_shape["spatial_edges"].shape)[0]
        dbl = 1 if recurrent_cell_type == "GRU" else 2
        self.recurrent_hidden_states = {
            "human_node_rnn": torch.zeros(TH, E, 1, human_node_rnn_size * dbl, device=dev),
            "human_human_edge_rnn": torch.zeros(TH, E, self.human_num + 1, human_human_edge_rnn_size * dbl,
                                                device=dev),
        }
        if self.compact_hidden:
            self.recurrent_hidden_states = {k: CompactSteps(v, T) for k, v in self.recurrent_hidden_states.items()}
        self.rewards = torch.zeros(T, E, 1, device=dev)
        self.value_preds = torch.zeros(T + 1, E, 1, device=dev)
        self.returns = torch.zeros(T + 1, E, 1, device=dev)
        self.action_log_probs = torch.zeros(T, E, 1, device=dev)
        if action_space.__class__.__name__ == "Discrete":
            raise NotImplementedError("CrowdSimDict has a Box(2,) action space")
        self.actions = torch.zeros(T, E, action_space.shape[0], device=dev)
        self.masks = torch.ones(T + 1, E, 1, device=dev)
        self.bad_masks = torch.ones(T + 1, E, 1, device=dev)
        self.num_steps = T
        self.step = 0

    def to(self, device):
        for d in (self.obs, self.recurrent_hidden_states):
            for k in d:
                d[k] = d[k].to(device)
        for n in ("rewards", "value_preds", "returns", "action_log_probs", "actions", "masks", "bad_masks"):
            setattr(self, n, getattr(self, n).to(device))
        return self

    def insert(self, obs, recurrent_hidden_states, actions, action_log_probs, value_preds, rewards, masks,
               bad_masks):
        s = self.step
        dst = [self.obs[k][s + 1] for k in self.obs]
        src = [obs[k] for k in self.obs]
        for k in recurrent_hidden_states:
            d = self.recurrent_hidden_states[k][s + 1]
            if recurrent_hidden_states[k].data_ptr() != d.data_ptr():   # act(out_hxs=hidden_slot()) wrote it
                dst.append(d)
                src.append(recurrent_hidden_states[k])
        dst += [self.actions[s], self.action_log_probs[s], self.value_preds[s], self.rewards[s], self.masks[s + 1],
                self.bad_masks[s + 1]]
        src += [actions, action_log_probs, value_preds, rewards, masks, bad_masks]
        _copy_all(dst, src)
        self.step = (s + 1) % self.num_steps

    def hidden(self, step):
        """The recurrent state act() consumes at `step` (recurrent_hidden_states[k][step] in train.py:227)."""
        return {k: v[step] for k, v in self.recurrent_hidden_states.items()}

    def hidden_slot(self):
        """Where insert() puts the state produced at the current step (act's out_hxs target)."""
        return {k: v[self.step + 1] for k, v in self.recurrent_hidden_states.items()}

    def after_update(self):
        for d in (self.obs, self.recurrent_hidden_states):
            for k in d:
                d[k][0].copy_(d[k][-1])
        self.masks[0].copy_(self.masks[-1])
        self.bad_masks[0].copy_(self.bad_masks[-1])

    def compute_returns(self, next_value, use_gae, gamma, gae_lambda, use_proper_time_limits=True):
        """storage.py:132-177, same operation order (a backward scan over the steps)."""
        T = self.rewards.size(0)
        r, v, m, bm, ret = self.rewards, self.value_preds, self.masks, self.bad_masks, self.returns
        if use_gae and r.is_cuda and all(t.is_contiguous() and t.dtype == torch.float32 for t in (r, v, m, bm, ret)):
            # one HIP launch for the whole backward scan (cn_gae), same float32 operation order
            import ctypes

            from .. import _lib

            v[-1] = next_value
            E = r[0].numel()
            with torch.cuda.device(r.device):
                _lib.check(_lib.lib().cn_gae(ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream), T, E,
                                             float(gamma), float(gamma * gae_lambda), int(bool(use_proper_time_limits)),
                                             r.data_ptr(), v.data_ptr(), m.data_ptr(), bm.data_ptr(), ret.data_ptr()))
        elif use_gae:
            v[-1] = next_value
            gae = torch.zeros_like(next_value)
            for s in reversed(range(T)):
                delta = r[s] + gamma * v[s + 1] * m[s + 1] - v[s]
                gae = delta + gamma * gae_lambda * m[s + 1] * gae
                if use_proper_time_limits:
                    gae = gae * bm[s + 1]
                ret[s] = gae + v[s]
        else:
            ret[-1] = next_value
            for s in reversed(range(T)):
                if use_proper_time_limits:
                    ret[s] = (ret[s + 1] * gamma * m[s + 1] + r[s]) * bm[s + 1] + (1 - bm[s + 1]) * v[s]
                else:
                    ret[s] = ret[s + 1] * gamma * m[s + 1] + r[s]

    def recurrent_generator(self, advantages, num_mini_batch):
        """storage.py:223-292: minibatches of whole environments, (T*N, ...) in (step, env) order and the
        step-0 hidden states."""
        E = self.rewards.size(1)
        assert E >= num_mini_batch, "PPO requires num_processes >= num_mini_batch"
        n = E // num_mini_batch
        perm = torch.randperm(E)
        T = self.num_steps
        for start in range(0, E, n):
            ind = perm[start:start + n].to(self.rewards.device)
            obs_b = {k: v[:-1].index_select(1, ind) for k, v in self.obs.items()}
            hxs_b = {k: v[0].index_select(0, ind) for k, v in self.recurrent_hidden_states.items()}
            yield (_flatten_helper(T, n, obs_b), hxs_b,
                   _flatten_helper(T, n, self.actions.index_select(1, ind)),
                   _flatten_helper(T, n, self.value_preds[:-1].index_select(1, ind)),
                   _flatten_helper(T, n, self.returns[:-1].index_select(1, ind)),
                   _flatten_helper(T, n, self.masks[:-1].index_select(1, ind)),
                   _flatten_helper(T, n, self.action_log_probs.index_select(1, ind)),
                   _flatten_helper(T, n, advantages.index_select(1, ind)))

    def feed_forward_generator(self, advantages, num_mini_batch=None, mini_batch_size=None):
        """storage.py:179-221 (non-recurrent policies)."""
        from torch.utils.data.sampler import BatchSampler, SubsetRandomSampler

        T, E = self.rewards.shape[0:2]
        batch = T * E
        if mini_batch_size is None:
            assert batch >= num_mini_batch
            mini_batch_size = batch // num_mini_batch
        for indices in BatchSampler(SubsetRandomSampler(range(batch)), mini_batch_size, drop_last=True):
            idx = torch.as_tensor(indices, device=self.rewards.device)
            obs_b = {k: v[:-1].reshape(-1, *v.shape[2:])[idx] for k, v in self.obs.items()}
            if self.compact_hidden:
                raise NotImplementedError("feed_forward_generator needs every step's hidden state (compact_hidden=False)")
            hxs_b = {k: v[:-1].reshape(-1, v.shape[-1])[idx] for k, v in self.recurrent_hidden_states.items()}
            yield (obs_b, hxs_b, self.actions.reshape(-1, self.actions.shape[-1])[idx],
                   self.value_preds[:-1].reshape(-1, 1)[idx], self.returns[:-1].reshape(-1, 1)[idx],
                   self.masks[:-1].reshape(-1, 1)[idx], self.action_log_probs.reshape(-1, 1)[idx],
                   None if advantages is None else advantages.reshape(-1, 1)[idx])


class RolloutStorage(SRNNRolloutStorage):
    """RolloutStorage (pytorchBaselines/a2c_ppo_acktr/storage.py:295-508): the buffer train.py uses for the
    ConvGRU policy (train.py:157-172) — one observation tensor and one (E, H) recurrent state instead of the
    DSRNN's dicts. Returns, after_update and both generators follow the reference; compact_hidden as in
    SRNNRolloutStorage."""

    def __init__(self, num_steps, num_processes, obs_shape, action_space, recurrent_hidden_state_size, device=None,
                 compact_hidden=False):
        T, E = num_steps, num_processes
        dev = device
        self.compact_hidden = bool(compact_hidden)
        TH = 2 if compact_hidden else T + 1
        self.obs = torch.zeros(T + 1, E, *tuple(obs_shape), device=dev)
        self.recurrent_hidden_states = torch.zeros(TH, E, recurrent_hidden_state_size, device=dev)
        if self.compact_hidden:
            self.recurrent_hidden_states = CompactSteps(self.recurrent_hidden_states, T)
        self.rewards = torch.zeros(T, E, 1, device=dev)
        self.value_preds = torch.zeros(T + 1, E, 1, device=dev)
        self.returns = torch.zeros(T + 1, E, 1, device=dev)
        self.action_log_probs = torch.zeros(T, E, 1, device=dev)
        if action_space.__class__.__name__ == "Discrete":
            raise NotImplementedError("CrowdSimDict has a Box(2,) action space")
        self.actions = torch.zeros(T, E, action_space.shape[0], device=dev)
        self.masks = torch.ones(T + 1, E, 1, device=dev)
        self.bad_masks = torch.ones(T + 1, E, 1, device=dev)
        self.num_steps = T
        self.step = 0

    def to(self, device):
        for n in ("obs", "recurrent_hidden_states", "rewards", "value_preds", "returns", "action_log_probs",
                  "actions", "masks", "bad_masks"):
            setattr(self, n, getattr(self, n).to(device))
        return self

    def insert(self, obs, recurrent_hidden_states, actions, action_log_probs, value_preds, rewards, masks,
               bad_masks):
        s = self.step
        self.obs[s + 1].copy_(obs)
        self.recurrent_hidden_states[s + 1].copy_(recurrent_hidden_states)
        self.actions[s].copy_(actions)
        self.action_log_probs[s].copy_(action_log_probs)
        self.value_preds[s].copy_(value_preds)
        self.rewards[s].copy_(rewards)
        self.masks[s + 1].copy_(masks)
        self.bad_masks[s + 1].copy_(bad_masks)
        self.step = (s + 1) % self.num_steps

    def hidden(self, step):
        return self.recurrent_hidden_states[step]

    def after_update(self):
        self.obs[0].copy_(self.obs[-1])
        self.recurrent_hidden_states[0].copy_(self.recurrent_hidden_states[-1])
        self.masks[0].copy_(self.masks[-1])
        self.bad_masks[0].copy_(self.bad_masks[-1])

    def recurrent_generator(self, advantages, num_mini_batch):
        """storage.py:449-508 (same torch.randperm draw as the reference)."""
        E = self.rewards.size(1)
        assert E >= num_mini_batch, "PPO requires num_processes >= num_mini_batch"
        n = E // num_mini_batch
        perm = torch.randperm(E)
        T = self.num_steps
        for start in range(0, E, n):
            ind = perm[start:start + n].to(self.rewards.device)
            yield (_flatten_helper(T, n, self.obs[:-1].index_select(1, ind)),
                   self.recurrent_hidden_states[0].index_select(0, ind),
                   _flatten_helper(T, n, self.actions.index_select(1, ind)),
                   _flatten_helper(T, n, self.value_preds[:-1].index_select(1, ind)),
                   _flatten_helper(T, n, self.returns[:-1].index_select(1, ind)),
                   _flatten_helper(T, n, self.masks[:-1].index_select(1, ind)),
                   _flatten_helper(T, n, self.action_log_probs.index_select(1, ind)),
                   _flatten_helper(T, n, advantages.index_select(1, ind)))

    def feed_forward_generator(self, advantages, num_mini_batch=None, mini_batch_size=None):
        """storage.py:408-447."""
        from torch.utils.data.sampler import BatchSampler, SubsetRandomSampler

        T, E = self.rewards.shape[0:2]
        batch = T * E
        if mini_batch_size is None:
            assert batch >= num_mini_batch
            mini_batch_size = batch // num_mini_batch
        if self.compact_hidden:
            raise NotImplementedError("feed_forward_generator needs every step's hidden state (compact_hidden=False)")
        for indices in BatchSampler(SubsetRandomSampler(range(batch)), mini_batch_size, drop_last=True):
            idx = torch.as_tensor(indices, device=self.rewards.device)
            yield (self.obs[:-1].reshape(-1, *self.obs.shape[2:])[idx],
                   self.recurrent_hidden_states[:-1].reshape(-1, self.recurrent_hidden_states.shape[-1])[idx],
                   self.actions.reshape(-1, self.actions.shape[-1])[idx], self.value_preds[:-1].reshape(-1, 1)[idx],
                   self.returns[:-1].reshape(-1, 1)[idx], self.masks[:-1].reshape(-1, 1)[idx],
                   self.action_log_probs.reshape(-1, 1)[idx],
                   None if advantages is None else advantages.reshape(-1, 1)[idx])
