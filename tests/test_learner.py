"""On-device PPO learner vs the reference (tests/golden/ppo.npz: the reference's SRNNRolloutStorage +
compute_returns + PPO.update on procedural DSRNN weights, pytorchBaselines/a2c_ppo_acktr/storage.py,
algo/ppo.py). Same seeded minibatch permutation (torch.randperm on the default generator).
Tolerances: returns 1e-6 (same fp32 operation order); losses / parameters after one update 2e-6 / 1e-6
absolute on CPU (fp32 GEMM/GRU summation order), 5e-5 / 5e-6 on the GPU."""
import os

import numpy as np
import pytest
import torch

from crowdnav_dsrnn_amd.learner import PPO, SRNNRolloutStorage
from crowdnav_dsrnn_amd.spaces import Box
from tests.helpers import attention_pool_ref, edge_features_fp32, masked_gru_ref, load, make_policy

N, E, T = 5, 4, 8


@pytest.fixture(scope="module")
def fx():
    return load("ppo.npz")


def _spaces():
    return {"robot_node": Box(-np.inf, np.inf, (1, 7)), "temporal_edges": Box(-np.inf, np.inf, (1, 2)),
            "spatial_edges": Box(-np.inf, np.inf, (N, 2))}, Box(-np.inf, np.inf, (2,))


def _filled(fx, device="cpu", compact=False):
    obs_sp, act_sp = _spaces()
    rol = SRNNRolloutStorage(T, E, obs_sp, act_sp, 128, 256, "GRU", device=device, compact_hidden=compact)
    for k in rol.obs:
        rol.obs[k][0].copy_(torch.from_numpy(fx["obs0_" + k]))
    for t in range(T):
        g = lambda n: torch.from_numpy(fx["t%d_%s" % (t, n)]).to(device)  # noqa: E731
        rol.insert({k: g("obs_" + k) for k in rol.obs}, {k: g("hxs_" + k) for k in rol.recurrent_hidden_states},
                   g("actions"), g("logp"), g("values"), g("rewards"), g("masks"), g("bad_masks"))
    return rol


@pytest.mark.parametrize("use_gae,ptl,key", [(True, True, "returns_gae_ptl"), (False, True, "returns_nogae_ptl"),
                                             (True, False, "returns_gae"), (False, False, "returns_nogae")])
def test_compute_returns(fx, use_gae, ptl, key):
    rol = _filled(fx)
    rol.compute_returns(torch.from_numpy(fx["next_value"]), use_gae, 0.99, 0.95, ptl)
    # returns[-1] is only written by the non-GAE branches (the fixture ran the branches in sequence)
    np.testing.assert_allclose(rol.returns.numpy()[:-1], fx[key][:-1], atol=1e-6, rtol=0)
    if not use_gae:
        np.testing.assert_allclose(rol.returns.numpy()[-1], fx[key][-1], atol=0, rtol=0)


def test_recurrent_generator_layout(fx):
    rol = _filled(fx)
    adv = torch.arange(T * E, dtype=torch.float32).reshape(T, E, 1)
    torch.manual_seed(7)
    perm = torch.randperm(E)
    torch.manual_seed(7)
    batches = list(rol.recurrent_generator(adv, 2))
    assert len(batches) == 2
    obs_b, hxs_b, act_b, vp_b, ret_b, m_b, lp_b, adv_b = batches[0]
    ind = perm[:2]
    assert obs_b["spatial_edges"].shape == (T * 2, N, 2)
    assert hxs_b["human_human_edge_rnn"].shape == (2, N + 1, 256)
    np.testing.assert_array_equal(adv_b.numpy().reshape(T, 2), adv[:, ind, 0].numpy())
    np.testing.assert_array_equal(hxs_b["human_node_rnn"].numpy(), rol.recurrent_hidden_states["human_node_rnn"][0, ind].numpy())
    np.testing.assert_array_equal(obs_b["robot_node"].numpy().reshape(T, 2, 1, 7), rol.obs["robot_node"][:-1, ind].numpy())


def test_compact_hidden_same_minibatches(fx):
    """compact_hidden keeps slots {start, latest}: the generator and after_update see the same states."""
    full, comp = _filled(fx), _filled(fx, compact=True)
    assert comp.recurrent_hidden_states["human_human_edge_rnn"].shape[0] == 2
    for t in (0, 3, T):
        want = {k: v[t] for k, v in full.recurrent_hidden_states.items()} if t in (0, T) else None
        if want is not None:
            got = comp.hidden(t)
            for k in want:
                assert torch.equal(got[k], want[k])
    adv = torch.randn(T, E, 1)
    torch.manual_seed(3)
    a = list(full.recurrent_generator(adv, 2))
    torch.manual_seed(3)
    b = list(comp.recurrent_generator(adv, 2))
    for x, y in zip(a, b):
        for k in x[1]:
            assert torch.equal(x[1][k], y[1][k])
    full.after_update()
    comp.after_update()
    for k in full.recurrent_hidden_states:
        assert torch.equal(full.recurrent_hidden_states[k][0], comp.recurrent_hidden_states[k][0])


def test_compact_hidden_reference_indexing():
    """train.py:232-236,298-302 index the storage as (T+1)-step tensors -- [key][step] before act() and
    [key][-1] for the next value -- and insert the new state at step + 1: with compact_hidden the same
    code reads the same states as with the full buffer."""
    from crowdnav_dsrnn_amd import spaces

    obs_sp, act_sp = spaces.observation_space(N).spaces, spaces.action_space()
    full = SRNNRolloutStorage(T, E, obs_sp, act_sp, 128, 256, "GRU", device="cpu")
    comp = SRNNRolloutStorage(T, E, obs_sp, act_sp, 128, 256, "GRU", device="cpu", compact_hidden=True)
    g = torch.Generator().manual_seed(5)
    for rol in (full, comp):
        for k, v in rol.recurrent_hidden_states.items():
            v[0].copy_(torch.randn(v[0].shape, generator=torch.Generator().manual_seed(1)))
    for step in range(T):
        h_full = {k: full.recurrent_hidden_states[k][step] for k in full.recurrent_hidden_states}
        h_comp = {k: comp.recurrent_hidden_states[k][step] for k in comp.recurrent_hidden_states}
        for k in h_full:
            assert torch.equal(h_full[k], h_comp[k]), (step, k)
        new = {k: torch.randn(v.shape, generator=g) for k, v in h_full.items()}
        obs = {k: torch.zeros(v.shape[1:]) for k, v in full.obs.items()}
        args = (obs, new, torch.zeros(E, 2), torch.zeros(E, 1), torch.zeros(E, 1), torch.zeros(E, 1),
                torch.ones(E, 1), torch.ones(E, 1))
        full.insert(*args)
        comp.insert(*args)
    for k in full.recurrent_hidden_states:
        assert torch.equal(full.recurrent_hidden_states[k][-1], comp.recurrent_hidden_states[k][-1])
        assert len(comp.recurrent_hidden_states[k]) == T + 1


def _update(fx, device):
    pol = make_policy(N, E=E, T=T, device=device)
    pol.base.nminibatch = 2
    pol.train()
    rol = _filled(fx, device)
    rol.compute_returns(torch.from_numpy(fx["next_value"]).to(device), True, 0.99, 0.95, True)
    agent = PPO(pol, 0.2, 2, 2, 0.5, 0.01, lr=4e-5, eps=1e-5, max_grad_norm=0.5)
    torch.manual_seed(1234)
    losses = agent.update(rol)
    return pol, losses


def test_ppo_update_cpu(fx, monkeypatch):
    """The whole update on CPU (the fused input-layer kernel replaced by its fp32 torch restatement)."""
    from crowdnav_dsrnn_amd import ops

    monkeypatch.setattr(ops, "edge_features", edge_features_fp32)
    monkeypatch.setattr(ops, "masked_gru", masked_gru_ref)
    monkeypatch.setattr(ops, "attention_pool", attention_pool_ref)
    pol, losses = _update(fx, "cpu")
    np.testing.assert_allclose(losses, fx["update_losses"], atol=2e-6, rtol=1e-5)
    for k, v in pol.state_dict().items():
        np.testing.assert_allclose(v.numpy(), fx["param_" + k], atol=1e-6, rtol=0, err_msg=k)


@pytest.mark.gpu
def test_ppo_update_gpu(fx):
    pol, losses = _update(fx, "cuda:0")
    np.testing.assert_allclose(losses, fx["update_losses"], atol=5e-5, rtol=1e-4)
    for k, v in pol.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), fx["param_" + k], atol=5e-6, rtol=0, err_msg=k)


def _dist_worker(rank, world, port, out):
    import torch.distributed as dist

    from crowdnav_dsrnn_amd import ops

    ops.edge_features = edge_features_fp32
    ops.masked_gru = masked_gru_ref
    ops.attention_pool = attention_pool_ref
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fx = load("ppo.npz")
        torch.manual_seed(100 + rank)          # different initial weights per rank: PPO broadcasts rank 0's
        pol = make_policy(N, E=E, T=T)
        if rank == 1:
            for p in pol.parameters():
                p.data.add_(0.01)
        pol.base.nminibatch = 2
        pol.train()
        rol = _filled(fx)
        if rank == 1:                          # each rank holds different rollouts
            rol.rewards.mul_(-0.5)
        rol.compute_returns(torch.from_numpy(fx["next_value"]), True, 0.99, 0.95, True)
        agent = PPO(pol, 0.2, 1, 2, 0.5, 0.01, lr=4e-5, eps=1e-5, max_grad_norm=0.5)
        adv = agent._normalised_advantages(rol)
        torch.manual_seed(1234)
        agent.update(rol)
        flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
        raw = (rol.returns[:-1] - rol.value_preds[:-1]).reshape(-1)
        torch.save({"flat": flat, "adv": adv.reshape(-1), "raw": raw}, "%s.%d" % (out, rank))
    finally:
        dist.destroy_process_group()


def test_ppo_data_parallel_gloo(tmp_path):
    """world_size 2: ranks start identical (broadcast), stay identical after the all-reduced update, and
    normalise advantages with the global mean / unbiased std."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "r")
    mp.start_processes(_dist_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    r0, r1 = torch.load(out + ".0", weights_only=True), torch.load(out + ".1", weights_only=True)
    assert torch.equal(r0["flat"], r1["flat"])
    raw = torch.cat([r0["raw"], r1["raw"]]).double()
    mean, std = raw.mean(), raw.std()
    np.testing.assert_allclose(r0["adv"].numpy(), ((r0["raw"].double() - mean) / (std + 1e-5)).numpy(), atol=1e-5)
    np.testing.assert_allclose(r1["adv"].numpy(), ((r1["raw"].double() - mean) / (std + 1e-5)).numpy(), atol=1e-5)


def _rollout_storage(z, compact=False):
    from crowdnav_dsrnn_amd.learner import RolloutStorage

    T, E = 6, 4
    st = RolloutStorage(T, E, (1, 10), Box(-np.inf, np.inf, (2,)), 8, compact_hidden=compact)
    st.obs[0].copy_(torch.from_numpy(z["obs0"]))
    for t in range(T):
        st.insert(*[torch.from_numpy(z["t%d_%s" % (t, k)]) for k in ("obs", "hxs", "act", "logp", "val", "rew",
                                                                      "masks", "bad")])
    return st


def test_rollout_storage_vs_reference():
    """RolloutStorage (storage.py:295-508, the ConvGRU buffer) vs tests/golden/rollout_storage.npz."""
    z = load("rollout_storage.npz")
    for gae in (True, False):
        for ptl in (True, False):
            st = _rollout_storage(z)
            st.compute_returns(torch.from_numpy(z["next_value"]), gae, 0.99, 0.95, ptl)
            want = z["returns_%d%d" % (gae, ptl)]
            sl = slice(None) if not gae else slice(0, -1)   # returns[-1] is written by the non-GAE branches only
            np.testing.assert_allclose(st.returns.numpy()[sl], want[sl], atol=1e-6, rtol=0)
    for compact in (False, True):
        st = _rollout_storage(z, compact)
        adv = torch.from_numpy(z["adv"])
        torch.manual_seed(5)
        for i, b in enumerate(st.recurrent_generator(adv, 2)):
            for j, x in enumerate(b):
                np.testing.assert_array_equal(x.numpy(), z["rec%d_%d" % (i, j)], err_msg="rec %d %d" % (i, j))
        if not compact:
            torch.manual_seed(6)
            for i, b in enumerate(st.feed_forward_generator(adv, 3)):
                for j, x in enumerate(b):
                    np.testing.assert_array_equal(x.numpy(), z["ff%d_%d" % (i, j)], err_msg="ff %d %d" % (i, j))
        st.after_update()
        np.testing.assert_array_equal(st.obs[0].numpy(), z["after_obs0"])
        np.testing.assert_array_equal(st.recurrent_hidden_states[0].numpy(), z["after_hxs0"])


@pytest.mark.gpu
def test_rollout_trainer_matches_reference_train_loop():
    """RolloutTrainer (act -> step_device -> insert, masks from done on device, get_value,
    compute_returns, PPO.update, after_update) with base='srnn' against the reference's train.py:219-330
    loop body on real reference envs (tests/golden/train_loop.npz, oracle/gen_golden.py gen_train_loop):
    4 envs x 5 humans, ORCA, holonomic, 32 steps with two episode ends, procedural weights, policy-mode
    actions. Tolerances: actions / values 5e-5 (fp32 GEMM order, GPU vs CPU), rewards / returns 2e-4 (the
    env consumes the slightly different actions), losses 1e-3 relative, parameters 2e-5 absolute."""
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer

    z = load("train_loop.npz")
    Tn, En, ep = int(z["T"]), int(z["meta_E"]), int(z["epochs"])
    Nn = int(z["meta_N"])
    dev = "cuda:0"
    c = clone_config(Config())
    c.sim.human_num = Nn
    c.humans.policy = "orca"
    c.action_space.kinematics = "holonomic"
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    c.training.num_processes = En
    c.ppo.num_steps = Tn
    c.ppo.num_mini_batch = 1
    c.ppo.epoch = ep
    hp = z["hparams"]
    assert (c.ppo.clip_param, c.ppo.value_loss_coef, c.ppo.entropy_coef, c.training.lr, c.training.eps,
            c.training.max_grad_norm, c.reward.gamma, c.ppo.gae_lambda) == tuple(float(x) for x in hp[:8])
    envs = CrowdNavVecEnv(c, En, c.env.seed, dev, nenv=En, phase="train")
    pol = make_policy(Nn, E=En, T=Tn, device=dev)
    pol.train()
    agent = PPO(pol, c.ppo.clip_param, ep, 1, c.ppo.value_loss_coef, c.ppo.entropy_coef, lr=c.training.lr,
                eps=c.training.eps, max_grad_norm=c.training.max_grad_norm)
    tr = RolloutTrainer(c, envs, pol, agent, deterministic=True)
    torch.manual_seed(99)
    st = tr.update()
    r = tr.rollouts
    np.testing.assert_allclose(r.actions.cpu().numpy(), z["action"], atol=5e-5, rtol=0)
    np.testing.assert_allclose(r.value_preds[:Tn].cpu().numpy(), z["value"], atol=5e-5, rtol=1e-5)
    np.testing.assert_allclose(r.rewards.cpu().numpy(), z["reward"], atol=2e-4, rtol=0)
    np.testing.assert_array_equal((r.masks[1:].cpu().numpy()[..., 0] == 0).astype(np.uint8), z["done"])
    np.testing.assert_allclose(r.returns[:Tn].cpu().numpy(), z["returns"][:Tn], atol=2e-4, rtol=0)
    np.testing.assert_allclose([st["value_loss"], st["action_loss"], st["dist_entropy"]], z["update_losses"],
                               rtol=1e-3, atol=1e-5)
    assert st["episodes"] == int(z["done"].sum())
    for k, v in pol.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), z["param_" + k], atol=2e-5, rtol=0, err_msg=k)
    # train.py:216-222: with use_linear_lr_decay the lr of update j is lr * (1 - j / num_updates)
    c.training.use_linear_lr_decay = True
    tr.update_index = 1
    tr.num_updates = 4
    tr.update()
    assert abs(agent.optimizer.param_groups[0]["lr"] - c.training.lr * 0.75) < 1e-12
    envs.close()


def test_compact_steps_index_types():
    """CompactSteps maps every integer-like step (int, numpy integer, 0-dim integer tensor) to the same slot
    for reads AND writes: step 0 / -(T+1) -> slot 0, any other step -> slot 1."""
    import numpy as np
    import torch

    from crowdnav_dsrnn_amd.learner.storage import CompactSteps

    T = 5
    c = CompactSteps(torch.zeros(2, 3), T)
    for k, idx in enumerate((3, np.int64(4), torch.tensor(2), np.int32(T))):
        c[idx] = float(k + 1)
        assert float(c.t[1, 0]) == k + 1 and float(c.t[0, 0]) == 0.0
        assert float(c[idx][0]) == k + 1
    c[np.int64(0)] = 7.0
    assert float(c.t[0, 0]) == 7.0 and float(c[-(T + 1)][0]) == 7.0
    with pytest.raises(IndexError):
        c[np.int64(T + 1)] = 1.0
    assert len(c) == T + 1 and c.shape[0] == 2


@pytest.mark.gpu
def test_rollout_hip_graph_matches_eager():
    """RolloutTrainer's HIP-graph rollouts (captured at the second update, replayed after) == eager rollouts,
    bit for bit, over four updates from the same start (deterministic actions; the PPO updates in between
    change the weights the replays read). 64 envs x 5 humans, ORCA, holonomic, 16 steps; the engine's
    device-side launch sequence (spawn lists, launch ids, draw-all flag) makes cn_step capturable."""
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer

    def run(graphs):
        c = clone_config(Config())
        c.sim.human_num = 5
        c.humans.policy = "orca"
        c.action_space.kinematics = "holonomic"
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        c.training.num_processes = 64
        c.ppo.num_steps = 16
        c.ppo.num_mini_batch = 1
        c.ppo.epoch = 2
        torch.manual_seed(5)
        envs = CrowdNavVecEnv(c, 64, c.env.seed, "cuda:0", nenv=64, phase="train")
        pol = make_policy(5, E=64, T=16, device="cuda:0")
        agent = PPO(pol, c.ppo.clip_param, 2, 1, c.ppo.value_loss_coef, c.ppo.entropy_coef, lr=1e-3,
                    eps=c.training.eps, max_grad_norm=c.training.max_grad_norm)
        tr = RolloutTrainer(c, envs, pol, agent, deterministic=True, graphs=graphs)
        out = []
        for _ in range(4):
            st = tr.update()
            r = tr.rollouts
            out.append((r.actions.cpu().numpy().copy(), r.rewards.cpu().numpy().copy(),
                        r.value_preds.cpu().numpy().copy(), st["episodes"]))
        envs.close()
        return out, tr._graph is not None

    eager, g0 = run(False)
    graph, g1 = run(True)
    assert not g0 and g1
    for u, (a, b) in enumerate(zip(eager, graph)):
        for x, y in zip(a[:3], b[:3]):
            np.testing.assert_array_equal(x, y, err_msg="update %d" % u)
        assert a[3] == b[3]


@pytest.mark.gpu
def test_graph_node_counts_and_memset_free_engine_capture():
    """cn_graph_node_counts on captured graphs: a torch multi-block reduction (f64 sum of 524,288 values,
    the round-4 in-graph episode sum) brings memset nodes (its semaphore's hipMemsetAsync) -- the node type
    this runtime can replay with stale bytes (profiles/r05/graph_audit/memset.log), which RolloutTrainer
    therefore refuses; the engine's own graph-mode calls (cn_reset, whose draw-all flag is a kernel write,
    and cn_step) capture as kernel nodes only."""
    from crowdnav_dsrnn_amd import _lib
    from crowdnav_dsrnn_amd.engine import CrowdNavEngine

    x = torch.randn((128, 4096), dtype=torch.float64, device="cuda:0")
    acc = torch.zeros((), dtype=torch.float64, device="cuda:0")
    acc += x.sum()   # warm-up outside the capture
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        acc += x.sum()
    got = _lib.graph_node_counts(g.raw_cuda_graph())
    assert got.get("memset", 0) >= 1 and got["kernel"] >= 2 and got["total"] == sum(
        v for k, v in got.items() if k != "total"), got
    del g

    from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config

    c = clone_config(Config())
    c.sim.human_num = 5
    c.humans.policy = "orca"
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    eng = CrowdNavEngine(make_cn_config(c, num_envs=64, nenv=64, phase="train"), "cuda:0")
    eng.reset()
    a = torch.zeros((64, 2), device="cuda:0")
    eng.step(a)
    eng.set_graph_mode(True)
    g2 = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g2):
        eng.reset()
        eng.step(a)
        eng.step(a)
    got2 = _lib.graph_node_counts(g2.raw_cuda_graph())
    assert got2 == {"kernel": got2["total"], "total": got2["total"]} and got2["total"] >= 4, got2
    g2.replay()
    torch.cuda.synchronize()
    eng.close()


@pytest.mark.gpu
def test_c4_shape_update_properties():
    """C4's per-GPU shape: 4,096 envs x 10 humans, ORCA, holonomic, 128 steps, 5 epochs,
    2 minibatches, HIP-graph rollouts. Properties at that size (no reference fixture covers it):
    * graph == eager: four updates from the same start (the graph is captured at the second, replayed at
      the third and fourth) give the same rollouts, losses and parameters bit for bit (deterministic
      actions), and the captured graph holds no memset node;
    * finite losses and parameters after every update;
    * the Monitor's episode count of each rollout == the number of done flags it stored (masks == 0);
    * the minibatch split of storage.py:228-234: torch.randperm(E) cut into num_mini_batch blocks of
      E / num_mini_batch whole envs, every env exactly once, T * n rows per minibatch in (step, env) order,
      the step-0 hidden states of exactly those envs."""
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer

    E4, N4, T4, MB = 4096, 10, 128, 2

    def cfg():
        c = clone_config(Config())
        c.sim.human_num = N4
        c.humans.policy = "orca"
        c.action_space.kinematics = "holonomic"
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        c.training.num_processes = E4
        c.ppo.num_steps = T4
        c.ppo.epoch = 5
        c.ppo.num_mini_batch = MB
        c.training.lr = 4e-5
        c.training.eps = 1e-5
        c.training.max_grad_norm = 0.5
        return c

    def run(graphs, check_split=False):
        c = cfg()
        torch.manual_seed(11)
        envs = CrowdNavVecEnv(c, E4, c.env.seed, "cuda:0", nenv=E4, phase="train")
        from crowdnav_dsrnn_amd.policy import Policy
        from tests.helpers import BoxSpace, procedural_state_dict

        pol = Policy({}, BoxSpace((2,)), base="srnn", base_kwargs=c)   # nenv / num_mini_batch rows per minibatch
        pol.load_state_dict(procedural_state_dict(pol))
        pol = pol.to("cuda:0")
        agent = PPO(pol, c.ppo.clip_param, c.ppo.epoch, MB, c.ppo.value_loss_coef, c.ppo.entropy_coef,
                    lr=c.training.lr, eps=c.training.eps, max_grad_norm=c.training.max_grad_norm)
        tr = RolloutTrainer(c, envs, pol, agent, deterministic=True, graphs=graphs)
        out = []
        for u in range(4):
            st = tr.update()
            r = tr.rollouts
            for k in ("value_loss", "action_loss", "dist_entropy"):
                assert np.isfinite(st[k]), (u, k, st[k])
            assert all(bool(torch.isfinite(p).all()) for p in pol.parameters()), u
            dones = int((r.masks[1:] == 0).sum())
            assert st["episodes"] == dones, (u, st["episodes"], dones)
            out.append((r.actions.cpu().numpy().copy(), r.rewards.cpu().numpy().copy(),
                        r.value_preds.cpu().numpy().copy(), st["episodes"], st["value_loss"], st["action_loss"]))
        params = [p.detach().cpu().numpy().copy() for p in pol.parameters()]
        if check_split:
            r = tr.rollouts
            adv = r.returns[:-1] - r.value_preds[:-1]
            torch.manual_seed(123)
            perm = torch.randperm(E4)
            torch.manual_seed(123)
            seen = []
            h0 = r.recurrent_hidden_states["human_human_edge_rnn"][0]
            n = E4 // MB
            for b, mb in enumerate(r.recurrent_generator(adv, MB)):
                ind = perm[b * n:(b + 1) * n].to(h0.device)
                obs_b, hxs_b, act_b = mb[0], mb[1], mb[2]
                assert act_b.shape == (T4 * n, 2)
                assert obs_b["spatial_edges"].shape == (T4 * n, N4, 2)
                torch.testing.assert_close(hxs_b["human_human_edge_rnn"], h0.index_select(0, ind), rtol=0, atol=0)
                torch.testing.assert_close(act_b.view(T4, n, 2), r.actions.index_select(1, ind), rtol=0, atol=0)
                seen.append(ind.cpu())
            allv = torch.cat(seen)
            assert len(seen) == MB and allv.numel() == E4 and torch.equal(torch.sort(allv).values, torch.arange(E4))
        g = tr._graph is not None
        if graphs:
            assert tr.graph_audit is not None and not tr.graph_audit.get("memset"), tr.graph_audit
        envs.close()
        del tr, agent, pol, envs
        torch.cuda.empty_cache()
        return out, params, g

    eager, p_e, g0 = run(False)
    graph, p_g, g1 = run(True, check_split=True)
    assert not g0 and g1
    for u, (a, b) in enumerate(zip(eager, graph)):
        for x, y in zip(a[:3], b[:3]):
            np.testing.assert_array_equal(x, y, err_msg="update %d" % u)
        assert a[3:] == b[3:], u
    for x, y in zip(p_e, p_g):
        np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("E,T,ptl", [(4096, 128, True), (37, 5, False), (1, 1, True)])
def test_gae_kernel_matches_reference_loop(E, T, ptl):
    """compute_returns on the GPU (cn_gae, one launch) vs the reference's per-step torch loop
    (storage.py:132-177) on CPU copies of the same storage: bit-identical returns (same float32 operations in
    the same order; random episode ends and time-limit masks)."""
    from crowdnav_dsrnn_amd.learner.storage import SRNNRolloutStorage
    from tests.helpers import BoxSpace

    g = torch.Generator().manual_seed(E + T)
    obs_shape = {"robot_node": BoxSpace((1, 7)), "temporal_edges": BoxSpace((1, 2)), "spatial_edges": BoxSpace((3, 2))}
    st = {}
    for dev in ("cpu", "cuda:0"):
        s = SRNNRolloutStorage(T, E, obs_shape, BoxSpace((2,)), 8, 8, device=dev)
        st[dev] = s
    r = torch.randn((T, E, 1), generator=g)
    v = torch.randn((T + 1, E, 1), generator=g)
    m = (torch.rand((T + 1, E, 1), generator=g) > 0.1).float()
    bm = (torch.rand((T + 1, E, 1), generator=g) > 0.05).float()
    nv = torch.randn((E, 1), generator=g)
    for dev, s in st.items():
        s.rewards.copy_(r)
        s.value_preds.copy_(v)
        s.masks.copy_(m)
        s.bad_masks.copy_(bm)
        s.compute_returns(nv.to(dev), True, 0.99, 0.95, ptl)
    assert torch.equal(st["cuda:0"].returns[:-1].cpu(), st["cpu"].returns[:-1])
