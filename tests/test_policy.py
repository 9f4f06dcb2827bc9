"""DSRNN policy vs the reference (tests/golden/dsrnn.npz: reference Policy.act / evaluate_actions on
procedural weights, pytorchBaselines/a2c_ppo_acktr/model.py:63-104).

CPU tests check the module tree / state_dict against the reference's key list and run the whole
policy graph with the fused input-layer kernel replaced by its plain fp32 torch restatement; the GPU
tests run the real HIP kernel (cn_edge_features) and compare to the same fixture.
Tolerance: 2e-5 abs + 1e-4 rel on value / action / log-prob / hidden states (fp32 GEMM/GRU
summation-order differences between MIOpen/rocBLAS and the reference's CPU kernels)."""
import numpy as np
import pytest
import torch

from tests.helpers import (attention_pool_ref, edge_features_fp32, gru_infer_step_ref, masked_gru_ref, load,
                           make_policy)

ATOL, RTOL = 2e-5, 1e-4


@pytest.fixture(scope="module")
def dsrnn():
    return load("dsrnn.npz")


def _obs(d, p, dev):
    return {k: torch.from_numpy(d[p + k]).to(dev) for k in ("robot_node", "temporal_edges", "spatial_edges")}


def _run_act(d, N, dev, in_place=False, grad=False):
    """act() on the fixture; in_place: the new state is written over the input state tensors
    (out_hxs = rnn_hxs, the rollout loop's storage slot); grad: the autograd T = 1 path."""
    pol = make_policy(N, device=dev)
    p = "N%d_act_" % N
    obs = _obs(d, p + "obs_", dev)
    hxs = {k: torch.from_numpy(d[p + "hxs_" + k].copy()).to(dev) for k in ("human_node_rnn", "human_human_edge_rnn")}
    masks = torch.from_numpy(d[p + "masks"]).to(dev)
    if grad:
        v, a, lp, nh = pol.act(obs, hxs, masks, deterministic=True)
        return v.detach(), a.detach(), lp.detach(), {k: t.detach() for k, t in nh.items()}
    with torch.no_grad():
        out = dict(hxs) if in_place else None
        v, a, lp, nh = pol.act(obs, hxs, masks, deterministic=True, out_hxs=out)
        if in_place:
            assert all(nh[k].data_ptr() == out[k].data_ptr() for k in out)
    return v, a, lp, nh


def _check_act(d, N, out):
    v, a, lp, nh = out
    p = "N%d_act_" % N
    np.testing.assert_allclose(v.cpu().numpy(), d[p + "value"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(a.cpu().numpy(), d[p + "action"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(lp.cpu().numpy(), d[p + "logp"], atol=ATOL, rtol=RTOL)
    for k in ("human_node_rnn", "human_human_edge_rnn"):
        assert tuple(nh[k].shape) == d[p + "new_" + k].shape
        np.testing.assert_allclose(nh[k].cpu().numpy(), d[p + "new_" + k], atol=ATOL, rtol=RTOL)


def _run_eval(d, N, dev):
    pol = make_policy(N, device=dev)
    p = "N%d_ev_" % N
    obs = _obs(d, p + "obs_", dev)
    hxs = {k: torch.from_numpy(d[p + "hxs_" + k].copy()).to(dev) for k in ("human_node_rnn", "human_human_edge_rnn")}
    with torch.no_grad():
        return pol.evaluate_actions(obs, hxs, torch.from_numpy(d[p + "masks"]).to(dev),
                                    torch.from_numpy(d[p + "actions"]).to(dev))


def _check_eval(d, N, out):
    v, lp, ent, _ = out
    p = "N%d_ev_" % N
    np.testing.assert_allclose(v.cpu().numpy(), d[p + "value"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(lp.cpu().numpy(), d[p + "logp"], atol=ATOL, rtol=RTOL)
    np.testing.assert_allclose(float(ent), float(d[p + "entropy"]), atol=ATOL, rtol=RTOL)


@pytest.mark.parametrize("N", [5, 10, 25])
def test_state_dict_matches_reference_keys(dsrnn, N):
    pol = make_policy(N)
    sd = pol.state_dict()
    assert sorted(sd.keys()) == list(dsrnn["N%d_keys" % N])
    assert [str(tuple(v.shape)) for _, v in sorted(sd.items())] == list(dsrnn["N%d_shapes" % N])


def test_fused_kernel_is_mandatory():
    """On CPU tensors the product path fails loudly (no silent torch fallback)."""
    from crowdnav_dsrnn_amd import ops

    pol = make_policy(5)
    d = load("dsrnn.npz")
    with pytest.raises(ops.EdgeFeaturesUnavailable):
        _run_act(d, 5, "cpu")
    del pol


@pytest.mark.parametrize("N", [5, 10, 25])
def test_policy_graph_cpu_with_fp32_input_layers(dsrnn, N, monkeypatch):
    """Everything but the fused kernel, on CPU: act + evaluate_actions (mid-sequence episode starts)."""
    from crowdnav_dsrnn_amd import ops

    monkeypatch.setattr(ops, "edge_features", edge_features_fp32)
    monkeypatch.setattr(ops, "masked_gru", masked_gru_ref)
    monkeypatch.setattr(ops, "gru_infer_step", gru_infer_step_ref)
    monkeypatch.setattr(ops, "attention_pool", attention_pool_ref)
    _check_act(dsrnn, N, _run_act(dsrnn, N, "cpu"))
    _check_act(dsrnn, N, _run_act(dsrnn, N, "cpu", in_place=True))
    with torch.enable_grad():   # the autograd (training-graph) T = 1 path
        _check_act(dsrnn, N, _run_act(dsrnn, N, "cpu", grad=True))
    _check_eval(dsrnn, N, _run_eval(dsrnn, N, "cpu"))


@pytest.mark.gpu
@pytest.mark.parametrize("N", [5, 10, 25])
def test_policy_act_gpu(dsrnn, N):
    _check_act(dsrnn, N, _run_act(dsrnn, N, "cuda:0"))
    _check_act(dsrnn, N, _run_act(dsrnn, N, "cuda:0", in_place=True))
    with torch.enable_grad():
        _check_act(dsrnn, N, _run_act(dsrnn, N, "cuda:0", grad=True))


@pytest.mark.gpu
@pytest.mark.parametrize("N", [5, 10, 25])
def test_policy_evaluate_actions_gpu(dsrnn, N):
    _check_eval(dsrnn, N, _run_eval(dsrnn, N, "cuda:0"))


@pytest.mark.gpu
@pytest.mark.parametrize("E,N", [(1, 1), (7, 5), (4096, 10), (300, 20)])
def test_edge_features_kernel_vs_fp32(E, N):
    from crowdnav_dsrnn_amd import ops

    g = torch.Generator().manual_seed(E * 100 + N)
    dev = "cuda:0"
    args = [torch.randn(s, generator=g) * 2 for s in
            [(E, 1, 7), (E, 1, 2), (E, N, 2), (64, 2), (64,), (64, 2), (64,), (3, 7), (3,), (64, 3), (64,)]]
    ref = edge_features_fp32(*args)
    out = ops.edge_features(*[a.to(dev) for a in args])
    for r, o in zip(ref, out):
        # fp32: a few roundings of pre-activation terms as large as max|out| (inputs ~N(0, 2^2))
        tol = 8 * np.finfo(np.float32).eps * float(r.abs().max())
        np.testing.assert_allclose(o.cpu().numpy(), r.numpy(), atol=tol, rtol=1e-5)


@pytest.mark.gpu
def test_edge_features_backward_vs_fp32():
    from crowdnav_dsrnn_amd import ops

    g = torch.Generator().manual_seed(3)
    E, N = 33, 6
    shapes = [(E, 1, 7), (E, 1, 2), (E, N, 2), (64, 2), (64,), (64, 2), (64,), (3, 7), (3,), (64, 3), (64,)]
    base = [torch.randn(s, generator=g) for s in shapes]
    w = [torch.randn(s, generator=g) for s in [(E, 64), (E, N, 64), (E, 64)]]
    a_cpu = [b.clone().requires_grad_(True) for b in base]
    sum((o * wi).sum() for o, wi in zip(edge_features_fp32(*a_cpu), w)).backward()
    a_gpu = [b.to("cuda:0").requires_grad_(True) for b in base]
    sum((o * wi.to("cuda:0")).sum() for o, wi in zip(ops.edge_features(*a_gpu), w)).backward()
    for x, y in zip(a_cpu, a_gpu):
        np.testing.assert_allclose(y.grad.cpu().numpy(), x.grad.numpy(), atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("T,B,F,H", [(1, 45, 64, 256), (9, 33, 64, 256), (16, 70, 128, 128), (3, 1000, 32, 64),
                                     (4, 50, 16, 36), (5, 3000, 48, 256), (3, 40, 16, 64), (4, 9000, 64, 256)])
def test_masked_gru_kernels_vs_fp64(T, B, F, H):
    """ops.masked_gru vs the plain torch restatement of the mask-segmented GRU (srnn_model.py:52-104) in
    float64: outputs, final state and every input / weight gradient, with episode starts at step 0 and
    mid-sequence. Covers the sequence kernels' four forms -- 128-row tiles (>= 256 workgroups: B 3000 / 9000
    at H 256) and split-K 32-row tiles, each with the input projection in the kernel (F % 32 == 0) or a gi
    GEMM first (F 48 / 16) -- and the per-step path (H 36). fp32 GEMM/transcendental rounding: atol 2e-5
    (outputs), 1e-4 x scale (gradients)."""
    from crowdnav_dsrnn_amd import ops

    g = torch.Generator().manual_seed(T * 1000 + B)
    x = torch.randn(T, B, F, generator=g)
    h0 = torch.randn(B, H, generator=g) * 0.5
    masks = (torch.rand(T, B, generator=g) > 0.2).float()
    masks[:, 0] = 0.0
    gru = torch.nn.GRU(F, H)
    ws = [gru.weight_ih_l0.detach(), gru.weight_hh_l0.detach(),
          torch.randn(3 * H, generator=g) * 0.1, torch.randn(3 * H, generator=g) * 0.1]
    dout = torch.randn(T, B, H, generator=g)
    dhT = torch.randn(B, H, generator=g)

    def run(fn, dev, dt):
        leaves = [t.to(dev, dt).requires_grad_(True) for t in (x, h0, *ws)]
        out, hT = fn(leaves[0], leaves[1], masks.to(dev, dt), *leaves[2:])
        ((out * dout.to(dev, dt)).sum() + (hT * dhT.to(dev, dt)).sum()).backward()
        return [out.detach().cpu().double(), hT.detach().cpu().double()] + [l.grad.cpu().double() for l in leaves]

    got = run(ops.masked_gru, "cuda:0", torch.float32)
    want = run(masked_gru_ref, "cpu", torch.float64)
    names = ["out", "hT", "dx", "dh0", "dW_ih", "dW_hh", "db_ih", "db_hh"]
    for n, a, b in zip(names, got, want):
        tol = 2e-5 if n in ("out", "hT") else 1e-4 * max(1.0, float(b.abs().max()))
        np.testing.assert_allclose(a.numpy(), b.numpy(), atol=tol, rtol=0, err_msg=n)


def _gru_case(g, T, B, F, H):
    x = torch.randn(T, B, F, generator=g)
    h0 = torch.randn(B, H, generator=g) * 0.5
    masks = (torch.rand(T, B, generator=g) > 0.2).float()
    masks[:, 0] = 0.0
    gru = torch.nn.GRU(F, H)
    ws = [gru.weight_ih_l0.detach(), gru.weight_hh_l0.detach(),
          torch.randn(3 * H, generator=g) * 0.1, torch.randn(3 * H, generator=g) * 0.1]
    return x, h0, masks, ws, torch.randn(T, B, H, generator=g), torch.randn(B, H, generator=g)


@pytest.mark.gpu
@pytest.mark.parametrize("T,Bs,F,H", [(9, (300, 45), 64, 256), (3, (1, 129), 64, 128), (17, (2048 * 10, 2048), 64, 256),
                                      (2, (128, 256), 32, 64)])
def test_masked_gru_group_vs_fp64(T, Bs, F, H):
    """ops.masked_gru_group (two GRUs in shared cn_gru_fwd_seq / cn_gru_bwd_seq launches: the spatial and
    temporal edge RNNs) vs the float64 restatement of each GRU on its own: outputs, final states and every
    gradient of both. Ragged row tiles on either side of the boundary (1, 129, 45) and C4's minibatch shape
    (20,480 + 2,048 rows). Tolerances as test_masked_gru_kernels_vs_fp64."""
    from crowdnav_dsrnn_amd import ops

    g = torch.Generator().manual_seed(T * 7 + Bs[0])
    cases = [_gru_case(g, T, B, F, H) for B in Bs]

    def run(group, dev, dt):
        leaves, grus, loss = [], [], 0
        for x, h0, masks, ws, _, _ in cases:
            lv = [t.to(dev, dt).requires_grad_(True) for t in (x, h0, *ws)]
            leaves.append(lv)
            grus.append((lv[0], lv[1], masks.to(dev, dt), *lv[2:]))
        res = group(*grus)
        for (out, hT), (_, _, _, _, dout, dhT) in zip(res, cases):
            loss = loss + (out * dout.to(dev, dt)).sum() + (hT * dhT.to(dev, dt)).sum()
        loss.backward()
        return [[out.detach().cpu().double(), hT.detach().cpu().double()] + [l.grad.cpu().double() for l in lv]
                for (out, hT), lv in zip(res, leaves)]

    got = run(ops.masked_gru_group, "cuda:0", torch.float32)
    want = run(lambda *grus: [masked_gru_ref(*gr) for gr in grus], "cpu", torch.float64)
    names = ["out", "hT", "dx", "dh0", "dW_ih", "dW_hh", "db_ih", "db_hh"]
    for k in range(2):
        for n, a, b in zip(names, got[k], want[k]):
            tol = 2e-5 if n in ("out", "hT") else 1e-4 * max(1.0, float(b.abs().max()))
            np.testing.assert_allclose(a.numpy(), b.numpy(), atol=tol, rtol=0, err_msg="gru %d %s" % (k, n))


@pytest.mark.gpu
@pytest.mark.parametrize("Rg,G,F,H", [(4096, 10, 64, 256), (37, 1, 128, 128), (300, 5, 64, 256), (3, 2, 32, 64)])
def test_gru_infer_group_vs_infer_step(Rg, G, F, H):
    """ops.gru_infer_group (one launch for two GRUs, input projection in the kernel; split-K below one
    workgroup per CU) vs ops.gru_infer_step per GRU (gi GEMM + cn_gru_fwd_fused) on the same operands, the
    grouped copy into a (R', G + 1, H) state slice included (dest aliasing h0, as in act()). Only the
    summation order differs: atol 2e-6."""
    from crowdnav_dsrnn_amd import ops

    dev = "cuda:0"
    g = torch.Generator(device=dev)
    g.manual_seed(Rg + G + F + H)
    state = torch.randn((Rg, G + 1, H), generator=g, device=dev) * 0.5
    m = (torch.rand((Rg,), generator=g, device=dev) > 0.2).float()
    xs = [torch.randn((Rg * G, F), generator=g, device=dev), torch.randn((Rg, F), generator=g, device=dev)]
    ws = [[torch.randn(s, generator=g, device=dev) / s[-1] ** 0.5 for s in ((3 * H, F), (3 * H, H))] +
          [torch.randn((3 * H,), generator=g, device=dev) * 0.1 for _ in range(2)] for _ in range(2)]

    def args(st, i):
        sl = st[:, 1:, :] if i == 0 else st[:, 0:1, :]
        w_ih, w_hh, b_ih, b_hh = ws[i]
        return (xs[i], sl, m, w_ih, w_hh, b_ih, b_hh, sl)

    st_ref = state.clone()
    ref = [ops.gru_infer_step(*args(st_ref, i)) for i in range(2)]
    st_got = state.clone()
    got = ops.gru_infer_group(args(st_got, 0), args(st_got, 1))
    torch.cuda.synchronize()
    for a, b in zip(got + [st_got], ref + [st_ref]):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=2e-6, rtol=0)


@pytest.mark.gpu
def test_masked_gru_seq_matches_per_step_path():
    """The native sequence path (cn_gru_fwd_seq / cn_gru_bwd_seq) vs the per-step path it replaced
    (hipBLASLt gi = x W_ih^T + b_ih, then cn_gru_fwd_fused per step; cn_gru_bwd_step_gates + a library GEMM
    per step) on the same fp32 operands. The sequence forward accumulates x W_ih^T with hm W_hh^T in the
    step kernel and the backward's recurrent GEMM sums in another order: only the summation order differs
    (atol 2e-6 on the outputs, 2e-5 x scale on the gradients)."""
    from crowdnav_dsrnn_amd import ops

    g = torch.Generator().manual_seed(5)
    T, B, F, H = 12, 3000, 64, 256
    x, h0, masks, ws, dout, dhT = _gru_case(g, T, B, F, H)

    def run(fn):
        lv = [t.cuda().requires_grad_(True) for t in (x, h0, *ws)]
        out, hT = fn(lv[0], lv[1], masks.cuda(), *lv[2:])
        ((out * dout.cuda()).sum() + (hT * dhT.cuda()).sum()).backward()
        return [out.detach(), hT.detach()] + [l.grad for l in lv]

    got = run(ops.masked_gru)
    ref = run(ops._MaskedGRU.apply)
    for n, a, b in zip(["out", "hT"], got[:2], ref[:2]):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=2e-6, rtol=0, err_msg=n)
    for n, a, b in zip(["dx", "dh0", "dW_ih", "dW_hh", "db_ih", "db_hh"], got[2:], ref[2:]):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), atol=2e-5 * max(1.0, float(b.abs().max())),
                                   rtol=0, err_msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("K,m,n,relu", [(262144, 64, 2, True), (100003, 64, 3, True), (5000, 3, 7, False),
                                        (70001, 2, 256, False), (1, 1, 256, False), (33, 64, 2, True),
                                        (1000, 8, 8, True), (4097, 256, 1, False), (2621440, 64, 2, True)])
def test_wgrad_kernel_vs_fp64(K, m, n, relu):
    """cn_wgrad (ops.relu_wgrad): dW = (dy * (out > 0))^T x and db = its column sums vs float64. fp32 sums of
    K products in a fixed order: |error| <= ~K^0.5 eps of the absolute-value sum; tolerance 2e-6 x
    (|dy'|^T |x|) per entry (the bound a sequential fp32 sum of that length meets with room)."""
    from crowdnav_dsrnn_amd import ops

    g = torch.Generator().manual_seed(K + m + n)
    dy = torch.randn(K, m, generator=g)
    out = torch.randn(K, m, generator=g) if relu else None
    x = torch.randn(K, n, generator=g)
    dW, db = ops.relu_wgrad(dy.cuda(), out.cuda() if relu else None, x.cuda())
    d = dy.double() * (out > 0).double() if relu else dy.double()
    ref_w, ref_b = d.t() @ x.double(), d.sum(0)
    bw, bb = d.abs().t() @ x.double().abs(), d.abs().sum(0)
    np.testing.assert_array_less((dW.cpu().double() - ref_w).abs().numpy(), (2e-6 * bw + 1e-30).numpy())
    np.testing.assert_array_less((db.cpu().double() - ref_b).abs().numpy(), (2e-6 * bb + 1e-30).numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("R,N,H", [(1, 1, 256), (37, 10, 256), (300, 25, 128), (5, 3, 64)])
def test_attention_pool_kernels_vs_fp64(R, N, H):
    """cn_attn_pool_fwd / _bwd vs bmm(hs^T, attn) in float64 (srnn_model.py:320-333): output and both
    gradients; fp32 summation over N (forward) / H (d attn): atol 1e-5 x scale."""
    from crowdnav_dsrnn_amd import ops

    g = torch.Generator().manual_seed(R * 7 + N)
    hs = torch.randn(R, N, H, generator=g)
    attn = torch.softmax(torch.randn(R, N, generator=g), -1).reshape(R, N, 1)
    dout = torch.randn(R, H, generator=g)

    def run(fn, dev, dt):
        a, b = hs.to(dev, dt).requires_grad_(True), attn.to(dev, dt).requires_grad_(True)
        out = fn(a, b)
        (out * dout.to(dev, dt)).sum().backward()
        return [x.detach().cpu().double() for x in (out, a.grad, b.grad)]

    got = run(ops.attention_pool, "cuda:0", torch.float32)
    want = run(attention_pool_ref, "cpu", torch.float64)
    for n, a, b in zip(("out", "d_hs", "d_attn"), got, want):
        np.testing.assert_allclose(a.numpy(), b.numpy(), atol=1e-5 * max(1.0, float(b.abs().max())), rtol=0, err_msg=n)


def spatial_attention_ref(hs, te, ws, bs, scale):
    """EdgeAttention's spatial branch as the reference writes it (srnn_model.py:256-333): spatial_edge_layer,
    product with temporal_embed summed over the embedding, * scale, softmax over the edges, bmm pooling."""
    se = hs @ ws.t() + bs                                   # (R, N, A)
    attn = torch.softmax((se * te.unsqueeze(1)).sum(-1) * scale, -1).unsqueeze(-1)
    return torch.bmm(hs.transpose(1, 2), attn).squeeze(-1), attn


@pytest.mark.gpu
@pytest.mark.parametrize("R,N,H", [(1, 1, 256), (37, 10, 256), (300, 25, 128), (5, 3, 64), (4099, 20, 256),
                                   (9, 64, 64)])
def test_spatial_attention_kernels_vs_fp64(R, N, H):
    """cn_spatial_attn_fwd / _bwd (spatial_edge_layer folded into the score: reassociated) vs the
    reference's composition in float64: output, attention and the gradients of h_spatials, temporal_embed,
    the layer's weight and bias, with a gradient arriving on the returned attention too (N > 16 covers the
    reloaded tail of a row). fp32 accumulation over H and N: atol 2e-5 x scale."""
    from crowdnav_dsrnn_amd import ops

    A = 64
    g = torch.Generator().manual_seed(R * 11 + N)
    hs = torch.randn(R, N, H, generator=g)
    te = torch.relu(torch.randn(R, A, generator=g)) * 0.3
    ws = torch.randn(A, H, generator=g) / 16
    bs = torch.randn(A, generator=g) * 0.1
    dout = torch.randn(R, H, generator=g)
    datt = torch.randn(R, N, 1, generator=g)
    scale = N / np.sqrt(A)

    def run(fn, dev, dt):
        xs = [t.to(dev, dt).requires_grad_(True) for t in (hs, te, ws, bs)]
        out, att = fn(*xs, scale)
        ((out * dout.to(dev, dt)).sum() + (att * datt.to(dev, dt)).sum()).backward()
        return [x.detach().cpu().double() for x in [out, att] + [t.grad for t in xs]]

    got = run(ops.spatial_attention, "cuda:0", torch.float32)
    want = run(spatial_attention_ref, "cpu", torch.float64)
    for n, a, b in zip(("out", "attn", "d_hs", "d_te", "d_ws", "d_bs"), got, want):
        # d_bs is exactly 0 in exact arithmetic (te . bs shifts a row's scores uniformly; softmax ignores it):
        # both fp32 implementations return rounding noise of sums of te * dscore terms, which d_ws bounds
        ref = want[4] if n == "d_bs" else b
        tol = 2e-5 * max(1.0, float(ref.abs().max())) * (max(1.0, R / 256) if n in ("d_ws", "d_bs") else 1.0)
        np.testing.assert_allclose(a.numpy(), b.numpy(), atol=tol, rtol=0, err_msg=n)


@pytest.mark.gpu
def test_spatial_attention_rejects_bad_shapes():
    from crowdnav_dsrnn_amd import _lib

    L = _lib.lib()
    assert L.cn_spatial_attn_fwd(None, 4, 65, 256, 1.0, None, None, None, None, None) != 0   # N > 64
    assert L.cn_spatial_attn_fwd(None, 4, 10, 96, 1.0, None, None, None, None, None) != 0    # H not 64/128/256


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,G", [(20480, 256, 10), (4099, 128, 1), (1, 256, 1), (130, 64, 5)])
def test_gru_fused_step_vs_gemm_plus_gates(B, H, G):
    """cn_gru_fwd_fused (recurrent GEMM on the f32 MFMA + gate epilogue) vs torch.addmm + cn_gru_fwd_step_scatter
    on the same operands, every output: h_out, the grouped second copy h_out2, hm_next = h * m_next and the
    r | z | n | gh_n record. Only the GEMM's summation order differs (both f32 products / accumulation):
    atol 2e-6 on the gates and states of unit-scale operands. B = 20,480 x 256 is C4's spatial-edge step;
    4099 / 1 / 130 are ragged row tiles (128 rows per workgroup)."""
    from crowdnav_dsrnn_amd import _lib

    dev = "cuda:0"
    g = torch.Generator(device=dev)
    g.manual_seed(B + H)
    gi = torch.randn((B, 3 * H), generator=g, device=dev)
    hm = torch.randn((B, H), generator=g, device=dev) * 0.5
    w = torch.randn((3 * H, H), generator=g, device=dev) / H ** 0.5
    b = torch.randn((3 * H,), generator=g, device=dev) * 0.1
    m = (torch.rand((B,), generator=g, device=dev) > 0.3).float()
    Rg = (B + G - 1) // G
    L = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream

    def outs():
        return [torch.full((B, H), float("nan"), device=dev), torch.full((B, H), float("nan"), device=dev),
                torch.full((B, 4 * H), float("nan"), device=dev), torch.zeros((Rg, G + 1, H), device=dev)]

    ref = outs()
    gh = torch.addmm(b, hm, w.t())
    _lib.check(L.cn_gru_fwd_step_scatter(st, B, H, gi.data_ptr(), gh.data_ptr(), hm.data_ptr(), m.data_ptr(),
                                         ref[0].data_ptr(), ref[1].data_ptr(), ref[2].data_ptr(), ref[3].data_ptr(),
                                         G, (G + 1) * H))
    got = outs()
    _lib.check(L.cn_gru_fwd_fused(st, B, H, gi.data_ptr(), hm.data_ptr(), w.data_ptr(), b.data_ptr(), m.data_ptr(),
                                  got[0].data_ptr(), got[1].data_ptr(), got[2].data_ptr(), got[3].data_ptr(), G,
                                  (G + 1) * H))
    torch.cuda.synchronize()
    for n, a, r in zip(("h_out", "hm_next", "save", "h_out2"), got, ref):
        assert torch.isfinite(a).all(), n
        np.testing.assert_allclose(a.cpu().numpy(), r.cpu().numpy(), atol=2e-6, rtol=0, err_msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("E,A,det", [(4096, 2, False), (37, 2, True), (5, 3, False)])
def test_gaussian_act_kernel_vs_torch(E, A, det):
    """cn_gaussian_act (ops.gaussian_act) vs DiagGaussian -> FixedNormal.sample / mode + log_probs in torch
    on the same N(0, 1) draw (same generator state): action and summed log-probability, float32 (exp / log of
    the device math library on both sides; atol 2e-6 x scale)."""
    from crowdnav_dsrnn_amd import ops
    from crowdnav_dsrnn_amd.policy.distributions import FixedNormal

    g = torch.Generator(device="cuda:0")
    g.manual_seed(E + A)
    mean = torch.randn((E, A), generator=g, device="cuda:0")
    logstd = torch.randn((A,), generator=g, device="cuda:0") * 0.5
    torch.manual_seed(11)
    act, lp = ops.gaussian_act(mean, logstd, det)
    torch.manual_seed(11)
    d = FixedNormal(mean, (torch.zeros_like(mean) + logstd.view(1, -1)).exp())
    ref = d.mode() if det else d.sample()
    ref_lp = d.log_probs(ref)
    np.testing.assert_allclose(act.cpu().numpy(), ref.cpu().numpy(), atol=2e-6 * max(1.0, float(ref.abs().max())), rtol=0)
    np.testing.assert_allclose(lp.cpu().numpy(), ref_lp.cpu().numpy(), atol=2e-6 * max(1.0, float(ref_lp.abs().max())),
                               rtol=0)
