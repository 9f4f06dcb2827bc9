"""Torch-facing wrappers of the native kernels (no compute in Python; the HIP kernels are mandatory).

edge_features(...)  — the fused DSRNN input layers (cn_edge_features, include/crowdnav.h): one launch
                      computes relu(temporal encoder), relu(spatial encoder) and
                      relu(node encoder(robot_linear(robot_node))) for every env (and time step).
linear(...)         — nn.Linear with a split-K weight gradient (library GEMMs; for the layers applied to
                      T*B or T*B*N rows in training, where dW = dY^T X has a tiny output and K ~ 10^6).
attention_pool(...) — EdgeAttention's weighted sum of the spatial edge states (cn_attn_pool_*).
masked_gru(...)     — the mask-segmented GRU of the three DSRNN RNNs over a (T, B) sequence
                      (cn_gru_fwd_fused: recurrent GEMM on the f32 matrix cores + gates in one launch per
                      step; cn_gru_bwd_step + library GEMMs backward), with its own backward.
gru_infer_step(...) — one no-autograd step of the same GRU for act(): reads the state through strided views
                      and writes the new state straight into the (B, N + 1, H) layout (cn_gru_fwd_fused).
"""
import torch

from . import _lib


class EdgeFeaturesUnavailable(RuntimeError):
    pass


def _stream(device):
    import ctypes

    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _c(t):
    return t.contiguous().float() if (not t.is_contiguous() or t.dtype != torch.float32) else t


class _EdgeFeatures(torch.autograd.Function):
    """Forward = fused HIP kernel. Backward = the matching gradients of the three tiny input layers
    (recomputed from the saved inputs with torch ops on the same device; these layers are
    <2% of the DSRNN FLOPs)."""

    @staticmethod
    def forward(ctx, robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn):
        E = temporal.shape[0]
        N = spatial.shape[1]
        dev = temporal.device
        t_out = torch.empty((E, 64), dtype=torch.float32, device=dev)
        s_out = torch.empty((E, N, 64), dtype=torch.float32, device=dev)
        n_out = torch.empty((E, 64), dtype=torch.float32, device=dev)
        args = [_c(x) for x in (robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn)]
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().cn_edge_features(_stream(dev), E, N, *[a.data_ptr() for a in args],
                                                   t_out.data_ptr(), s_out.data_ptr(), n_out.data_ptr()))
        ctx.save_for_backward(*args, t_out, s_out, n_out)
        return t_out, s_out, n_out

    @staticmethod
    def backward(ctx, g_t, g_s, g_n):
        robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn, t_out, s_out, n_out = ctx.saved_tensors
        E, N = temporal.shape[0], spatial.shape[1]
        x_t = temporal.reshape(E, 2)
        x_s = spatial.reshape(E * N, 2)
        x_r = robot_node.reshape(E, 7)
        # weight / bias gradients through the ReLUs: cn_wgrad, one HBM pass each (the ReLU mask applied on
        # the fly); the node encoder's input h = robot_linear(x_r) is recomputed (E x 3)
        dWt, dbt = relu_wgrad(g_t, t_out, x_t)
        dWs, dbs = relu_wgrad(g_s.reshape(E * N, 64), s_out.reshape(E * N, 64), x_s)
        h = torch.addmm(br, x_r, Wr.t())
        dWn, dbn = relu_wgrad(g_n, n_out, h)
        gn = g_n * (n_out > 0)
        g_h = gn @ Wn
        dWr, dbr = relu_wgrad(g_h, None, x_r)
        need = ctx.needs_input_grad
        # the observations carry no gradient in training; computed only when asked for
        d_rn = (g_h @ Wr).reshape(robot_node.shape) if need[0] else None
        d_t = ((g_t * (t_out > 0)) @ Wt).reshape(temporal.shape) if need[1] else None
        d_s = ((g_s * (s_out > 0)).reshape(E * N, 64) @ Ws).reshape(spatial.shape) if need[2] else None
        return d_rn, d_t, d_s, dWt, dbt, dWs, dbs, dWr, dbr, dWn, dbn


def edge_features(robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn):
    """robot_node (E,1,7) temporal (E,1,2) spatial (E,N,2) -> (E,64), (E,N,64), (E,64)."""
    if not robot_node.is_cuda:
        raise EdgeFeaturesUnavailable("the DSRNN edge-feature layers run only as the fused HIP kernel "
                                      "(tensors are on %s)" % robot_node.device)
    return _EdgeFeatures.apply(robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn)


def relu_wgrad(dy, relu_out, x):
    """(dW, db) = ((dy * (relu_out > 0))^T x, column sums of the same) over K rows, on cn_wgrad (one pass;
    relu_out None: plain dy). dy, relu_out (K, m), x (K, n), min(m, n) <= 8, max(m, n) <= 256."""
    dy, x = _c(dy), _c(x)
    K, m = dy.shape
    n = x.shape[1]
    mo = _c(relu_out) if relu_out is not None else None
    L = _lib.lib()
    dW = torch.empty((m, n), dtype=torch.float32, device=dy.device)
    db = torch.empty((m,), dtype=torch.float32, device=dy.device)
    work = torch.empty((max(1, L.cn_wgrad_work_elems(K, m, n)),), dtype=torch.float32, device=dy.device)
    with torch.cuda.device(dy.device):
        _lib.check(L.cn_wgrad(_stream(dy.device), K, m, n, dy.data_ptr(), mo.data_ptr() if mo is not None else None,
                              x.data_ptr(), dW.data_ptr(), db.data_ptr(), work.data_ptr()))
    return dW, db


def skinny(m, n):
    """The Linear weight gradients cn_wgrad serves (one side tiny)."""
    return min(m, n) <= 8 and max(m, n) <= 256


def wgrad(dy, x, chunk=16384):
    """dy^T @ x for (K, m), (K, n) with K >> m, n: K split into S chunks (one batched GEMM, then a sum over
    S) so the reduction fills the GPU instead of m*n/tile workgroups walking all of K."""
    K = dy.shape[0]
    S = K // chunk
    if S < 4:
        return dy.t() @ x
    Kc = K // S

    def chunks(t):   # (S, Kc, n) view of a row-strided (K, n) matrix (unit column stride)
        return t.as_strided((S, Kc, t.shape[1]), (Kc * t.stride(0), t.stride(0), t.stride(1)))

    main = torch.bmm(chunks(dy).transpose(1, 2), chunks(x)).sum(0)
    if S * Kc < K:
        main = main + dy[S * Kc:].t() @ x[S * Kc:]
    return main


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        x2 = x.reshape(-1, x.shape[-1])
        y = torch.addmm(b, x2, W.t()) if b is not None else x2 @ W.t()
        ctx.save_for_backward(x2, W)
        ctx.has_b = b is not None
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], W.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, W = ctx.saved_tensors
        dy2 = dy.reshape(-1, W.shape[0]).contiguous()
        dx = (dy2 @ W).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dW = db = None
        if ctx.needs_input_grad[1] and dy2.is_cuda and skinny(dy2.shape[1], x2.shape[1]):
            dW, db = relu_wgrad(dy2, None, x2)   # one pass for both
        elif ctx.needs_input_grad[1]:
            dW = wgrad(dy2, x2)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = db if db is not None else dy2.sum(0)
        else:
            db = None
        return dx, dW, db


def linear(x, W, b=None):
    """y = x W^T + b (torch.nn.functional.linear) with the split-K weight gradient."""
    return _Linear.apply(x, W, b)


# Optional in-loop timing of the fused recurrent steps (bench.py's C4 roofline): a list that receives
# (rows B, steps T, start event, end event) for every training forward with B >= FUSED_TIMING_MIN_ROWS.
FUSED_TIMING = None
FUSED_TIMING_MIN_ROWS = 8192


class _MaskedGRU(torch.autograd.Function):
    """srnn_model.py:52-104 (RNNBase._forward_gru): h <- h * mask[t] before step t, then one nn.GRU step.

    Forward: gi = x W_ih^T + b_ih as one GEMM over all T*B rows; per step one cn_gru_fwd_fused (the
    recurrent GEMM gh = hm W_hh^T + b_hh on the f32 matrix cores with the gates, new state, next masked
    state and the r|z|n|gh_n record for backward in its epilogue; H % 32 != 0: a library GEMM + the
    cn_gru_fwd_step gate kernel). Backward: per step (reversed) one cn_gru_bwd_step and one GEMM acc += dgh W_hh, then the
    weight / input gradients as single GEMMs over all T*B rows.

    masked_gru sends only H % 32 != 0 here (every other H runs _MaskedGRUSeq), so in production this class
    serves those sizes through its `nblk == 0` branches. The `nblk > 0` branch (cn_gru_bwd_step_gates + a
    library GEMM per step, H in {64, 128, 256}) is kept as the per-step reference composition the sequence
    kernels are tested against (tests/test_policy.py::test_masked_gru_seq_matches_per_step_path); nothing else reaches it."""

    @staticmethod
    def forward(ctx, x, h0, masks, w_ih, w_hh, b_ih, b_hh):
        T, B, F = x.shape
        H = w_hh.shape[1]
        dev = x.device
        need = any(ctx.needs_input_grad)
        L = _lib.lib()
        st = _stream(dev)
        x2 = _c(x).reshape(T * B, F)
        m = _c(masks).reshape(T, B)
        gi = torch.addmm(b_ih, x2, w_ih.t()).reshape(T, B, 3 * H)
        out = torch.empty((T, B, H), dtype=torch.float32, device=dev)
        if need:
            hm = torch.empty((T, B, H), dtype=torch.float32, device=dev)
            save = torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev)
        else:
            hm = torch.empty((min(T, 2), B, H), dtype=torch.float32, device=dev)
            save = None
        torch.mul(h0, m[0].unsqueeze(-1), out=hm[0])
        fused = H % 32 == 0
        gh = None if fused else torch.empty((B, 3 * H), dtype=torch.float32, device=dev)
        whh, bhh = _c(w_hh), _c(b_hh)
        nh = hm.shape[0]
        timing = FUSED_TIMING if (FUSED_TIMING is not None and fused and B >= FUSED_TIMING_MIN_ROWS) else None
        if timing is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        with torch.cuda.device(dev):
            for t in range(T):
                cur = hm[t % nh]
                last = t + 1 == T
                mn = None if last else m[t + 1].data_ptr()
                hn = None if last else hm[(t + 1) % nh].data_ptr()
                sv = save[t].data_ptr() if need else None
                if fused:
                    _lib.check(L.cn_gru_fwd_fused(st, B, H, gi[t].data_ptr(), cur.data_ptr(), whh.data_ptr(),
                                                  bhh.data_ptr(), mn, out[t].data_ptr(), hn, sv, None, 1, 0))
                else:
                    torch.addmm(b_hh, cur, w_hh.t(), out=gh)
                    _lib.check(L.cn_gru_fwd_step(st, B, H, gi[t].data_ptr(), gh.data_ptr(), cur.data_ptr(), mn,
                                                 out[t].data_ptr(), hn, sv))
        if timing is not None:
            ev1.record()
            timing.append((B, H, T, ev0, ev1, 0))
        if need:
            ctx.save_for_backward(x2, m, w_ih, w_hh, hm, save)
        return out, out[-1].clone()

    @staticmethod
    def backward(ctx, dout, dhT):
        x2, m, w_ih, w_hh, hm, save = ctx.saved_tensors
        T, B, H = hm.shape
        dev = x2.device
        L = _lib.lib()
        st = _stream(dev)
        acc = dhT.contiguous().clone() if dhT is not None else torch.zeros((B, H), dtype=torch.float32, device=dev)
        dout = dout.contiguous() if dout is not None else None
        # bias gradients folded into the step kernel (column sums per 16-row block, reduced once at the end);
        # the gate gradients stored once per row, g = [dn | dr | dz | dhn] (cn_gru_bwd_step_gates):
        # dgh = g[:, H:4H], dgi = g[:, 0:3H] in gate order (n, r, z)
        nblk = L.cn_gru_bias_blocks(B) if H in (64, 128, 256) else 0
        if nblk:
            part = torch.empty((T, nblk, 4 * H), dtype=torch.float32, device=dev)
            g = torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev)
        else:
            dgi = torch.empty((T, B, 3 * H), dtype=torch.float32, device=dev)
            dgh = torch.empty((T, B, 3 * H), dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            for t in reversed(range(T)):
                args = (st, B, H, acc.data_ptr(), None if t + 1 == T else m[t + 1].data_ptr(),
                        dout[t].data_ptr() if dout is not None else None, save[t].data_ptr(), hm[t].data_ptr())
                if nblk:
                    _lib.check(L.cn_gru_bwd_step_gates(*args, g[t].data_ptr(), part[t].data_ptr()))
                    acc.addmm_(g[t][:, H:], w_hh)
                else:
                    _lib.check(L.cn_gru_bwd_step(*args, dgi[t].data_ptr(), dgh[t].data_ptr()))
                    acc.addmm_(dgh[t], w_hh)
            if nblk:
                db_ih = torch.empty((3 * H,), dtype=torch.float32, device=dev)
                db_hh = torch.empty((3 * H,), dtype=torch.float32, device=dev)
                work = torch.empty((L.cn_gru_bias_work_elems(H),), dtype=torch.float32, device=dev)
                _lib.check(L.cn_gru_bias_reduce(st, T * nblk, H, part.data_ptr(), db_ih.data_ptr(), db_hh.data_ptr(),
                                                work.data_ptr()))
        dh0 = acc * m[0].unsqueeze(-1)
        hm2 = hm.reshape(T * B, H)
        if nblk:
            g2 = g.view(T * B, 4 * H)
            dgi_nrz, dgh2 = g2[:, :3 * H], g2[:, H:]
            w_ih_nrz = torch.cat((w_ih[2 * H:], w_ih[:2 * H]), 0)   # W_ih's rows in gate order n, r, z
            dx = (dgi_nrz @ w_ih_nrz).reshape(T, B, -1) if ctx.needs_input_grad[0] else None
            dw = wgrad(dgi_nrz, x2)
            dw_ih = torch.cat((dw[H:], dw[:H]), 0)                   # back to r, z, n
            return (dx, dh0, None, dw_ih, wgrad(dgh2, hm2), db_ih, db_hh)
        dgi2 = dgi.reshape(T * B, 3 * H)
        dgh2 = dgh.reshape(T * B, 3 * H)
        db_ih, db_hh = dgi2.sum(0), dgh2.sum(0)
        dx = (dgi2 @ w_ih).reshape(T, B, -1) if ctx.needs_input_grad[0] else None
        return (dx, dh0, None, wgrad(dgi2, x2), wgrad(dgh2, hm2), db_ih, db_hh)


def _a16(t):
    """t contiguous fp32 with a 16-byte aligned base (the sequence kernels' float4 accesses)."""
    t = _c(t)
    return t if t.data_ptr() % 16 == 0 else t.clone()


class _MaskedGRUSeq(torch.autograd.Function):
    """srnn_model.py:52-104 for one or two GRUs of the same T and H (H % 32 == 0) at once: the T-step loops
    run in native code (cn_gru_fwd_seq / cn_gru_bwd_seq, one launch per step for both GRUs: the DSRNN's
    spatial and temporal edge RNNs share every launch instead of running on two streams). Forward: the fused
    recurrent steps (cn_gru_fwd_fused's kernel), which also project the inputs (x W_ih^T on the MFMA ahead of
    hm W_hh^T) when F % 32 == 0 (else gi = x W_ih^T + b_ih as one GEMM over all T*B rows first).
    Backward: T + 1 launches of the fused recurrent-GEMM + gate-gradient kernel and the bias reduction
    (cn_gru_bwd_seq), then the weight / input gradients as single GEMMs over all T*B rows.
    Inputs: nseg, then per GRU (x, h0, masks, w_ih, w_hh, b_ih, b_hh); outputs per GRU (out, h_T)."""

    @staticmethod
    def forward(ctx, nseg, *args):
        segs = [args[7 * i:7 * i + 7] for i in range(nseg)]
        need = any(ctx.needs_input_grad)
        L = _lib.lib()
        T, H = segs[0][0].shape[0], segs[0][4].shape[1]
        dev = segs[0][0].device
        fs = (_lib.GruSeqFwd * nseg)()
        outs, saved, rows = [], [], 0
        # every input width F % 32 == 0: the step kernel projects x itself (x W_ih^T on the MFMA, gi never
        # stored); otherwise gi = x W_ih^T + b_ih first as one GEMM over all T*B rows (one mode per call).
        # (For the split-K node GRU the in-kernel projection makes each step 7.5 -> 10.6 us but drops a
        # 262,144 x 128 -> 384 GEMM and its gi buffer: C4 793.5 k with it, 787.7 k without.)
        xm = all(sg[0].shape[2] % 32 == 0 for sg in segs)
        fl = segs[0][0].shape[2] if xm else 0
        for i, (x, h0, masks, w_ih, w_hh, b_ih, b_hh) in enumerate(segs):
            if x.shape[0] != T or w_hh.shape[1] != H:
                raise ValueError("masked_gru_group: every GRU needs the same T and H")
            B, F = x.shape[1], x.shape[2]
            x2 = _a16(x).reshape(T * B, F)
            m = _c(masks).reshape(T, B)
            gi = None if xm else torch.addmm(b_ih, x2, w_ih.t())
            wih, bih = (_a16(w_ih), _a16(b_ih)) if xm else (None, None)
            out = torch.empty((T, B, H), dtype=torch.float32, device=dev)
            nh = T if need else min(T, 2)
            hm = torch.empty((nh, B, H), dtype=torch.float32, device=dev)
            torch.mul(h0, m[0].unsqueeze(-1), out=hm[0])
            save = torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev) if need else None
            whh, bhh = _a16(w_hh), _a16(b_hh)
            fs[i] = _lib.GruSeqFwd(B, gi.data_ptr() if gi is not None else None, whh.data_ptr(), bhh.data_ptr(),
                                   m.data_ptr(), out.data_ptr(), hm.data_ptr(),
                                   save.data_ptr() if save is not None else None, nh,
                                   x2.data_ptr() if xm else None, wih.data_ptr() if xm else None,
                                   bih.data_ptr() if xm else None, F if xm else 0)
            outs += [out, gi, whh, bhh, wih, bih]
            saved += [x2, m, w_ih, w_hh, hm, save]
            rows += B
        timing = FUSED_TIMING if (FUSED_TIMING is not None and rows >= FUSED_TIMING_MIN_ROWS) else None
        if timing is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        with torch.cuda.device(dev):
            _lib.check(L.cn_gru_fwd_seq(_stream(dev), T, H, nseg, fs))
        if timing is not None:
            ev1.record()
            timing.append((rows, H, T, ev0, ev1, fl))
        ctx.nseg = nseg
        if need:
            ctx.save_for_backward(*saved)
        res = []
        for i in range(nseg):
            out = outs[6 * i]
            res += [out, out[-1].clone()]
        return tuple(res)

    @staticmethod
    def backward(ctx, *grads):
        nseg = ctx.nseg
        sv = ctx.saved_tensors
        L = _lib.lib()
        dev = sv[0].device
        st = _stream(dev)
        bs = (_lib.GruSeqBwd * nseg)()
        keep = []
        T, H = sv[4].shape[0], sv[4].shape[2]
        for i in range(nseg):
            x2, m, w_ih, w_hh, hm, save = sv[6 * i:6 * i + 6]
            dout, dhT = grads[2 * i], grads[2 * i + 1]
            B = hm.shape[1]
            acc = dhT.float().clone(memory_format=torch.contiguous_format) if dhT is not None else \
                torch.zeros((B, H), dtype=torch.float32, device=dev)
            acc = _a16(acc)
            dout = _a16(dout) if dout is not None else None
            g = torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev)
            db = torch.empty((2, 3 * H), dtype=torch.float32, device=dev)
            wt = w_hh.t().contiguous()
            bs[i] = _lib.GruSeqBwd(B, wt.data_ptr(), m.data_ptr(), dout.data_ptr() if dout is not None else None,
                                   save.data_ptr(), hm.data_ptr(), acc.data_ptr(), g.data_ptr(), db[0].data_ptr(),
                                   db[1].data_ptr())
            keep.append((acc, dout, g, db, wt))
        with torch.cuda.device(dev):   # the workspace size follows the device the backward runs on
            nw = L.cn_gru_bwd_seq_work_elems(T, H, nseg, bs)
            work = torch.empty((nw,), dtype=torch.float32, device=dev)
            _lib.check(L.cn_gru_bwd_seq(st, T, H, nseg, bs, work.data_ptr(), nw))
            res = [None]
            for i in range(nseg):
                x2, m, w_ih, w_hh, hm, save = sv[6 * i:6 * i + 6]
                acc, _, g, db, _ = keep[i]
                B = hm.shape[1]
                dh0 = acc * m[0].unsqueeze(-1)
                g2 = g.view(T * B, 4 * H)
                dgi_nrz, dgh2 = g2[:, :3 * H], g2[:, H:]
                idx = 7 * i + 1   # needs_input_grad index of this GRU's x (after nseg)
                dx = None
                if ctx.needs_input_grad[idx]:
                    w_ih_nrz = torch.cat((w_ih[2 * H:], w_ih[:2 * H]), 0)   # W_ih's rows in gate order n, r, z
                    dx = (dgi_nrz @ w_ih_nrz).reshape(T, B, -1)
                dw = wgrad(dgi_nrz, x2)
                dw_ih = torch.cat((dw[H:], dw[:H]), 0)                       # back to r, z, n
                res += [dx, dh0, None, dw_ih, wgrad(dgh2, hm.reshape(T * B, H)), db[0], db[1]]
        return tuple(res)


def masked_gru(x, h0, masks, w_ih, w_hh, b_ih, b_hh):
    """x (T,B,F), h0 (B,H), masks (T,B) -> out (T,B,H), h_T (B,H); the weights of a 1-layer nn.GRU.
    H % 32 == 0: the native sequence kernels (_MaskedGRUSeq); otherwise per-step launches (_MaskedGRU)."""
    if not x.is_cuda:
        raise EdgeFeaturesUnavailable("the DSRNN GRUs run only through the HIP step kernels (cn_gru_*); "
                                      "tensors are on %s" % x.device)
    if x.dtype != torch.float32 or w_hh.shape[1] % 4:
        raise ValueError("masked_gru: fp32 operands and a hidden size divisible by 4 required")
    if w_hh.shape[1] % 32 == 0:
        return _MaskedGRUSeq.apply(1, x, h0, masks, w_ih, w_hh, b_ih, b_hh)
    return _MaskedGRU.apply(x, h0, masks, w_ih, w_hh, b_ih, b_hh)


def masked_gru_group(*grus):
    """Two (or one) independent masked GRUs of the same T and H (H % 32 == 0) in shared launches: each
    argument is (x, h0, masks, w_ih, w_hh, b_ih, b_hh) as for masked_gru; returns ((out, h_T), ...)."""
    if not 1 <= len(grus) <= 2:
        raise ValueError("masked_gru_group: one or two GRUs")
    for gr in grus:
        if not gr[0].is_cuda:
            raise EdgeFeaturesUnavailable("the DSRNN GRUs run only through the HIP step kernels (cn_gru_*); "
                                          "tensors are on %s" % gr[0].device)
        if gr[0].dtype != torch.float32 or gr[4].shape[1] % 32:
            raise ValueError("masked_gru_group: fp32 operands and a hidden size divisible by 32 required")
    flat = [t for gr in grus for t in gr]
    r = _MaskedGRUSeq.apply(len(grus), *flat)
    return tuple((r[2 * i], r[2 * i + 1]) for i in range(len(grus)))


def gru_infer_step(x, h0, m, w_ih, w_hh, b_ih, b_hh, dest):
    """One masked GRU step without autograd (the T = 1 inference path of srnn_model.py:52-104).

    x (R, F); h0 (R', G, H) or (R, H), any strides with a unit last stride (e.g. a slice of the
    (B, N + 1, H) edge-state tensor, R = R' * G); m (R') per group row; dest: a (R', G, H) view with
    the same grouping, or None. h0 * m is formed in a contiguous buffer first, so dest may alias h0.
    Returns the new state (R, H) contiguous; the kernel also writes it into dest (cn_gru_fwd_step_scatter)."""
    if not x.is_cuda:
        raise EdgeFeaturesUnavailable("gru_infer_step runs only through the HIP step kernels; tensors are on %s"
                                      % x.device)
    H = w_hh.shape[1]
    h0g = h0 if h0.dim() == 3 else h0.unsqueeze(1)
    Rg, G = h0g.shape[0], h0g.shape[1]
    R = Rg * G
    dev = x.device
    hm = torch.empty((Rg, G, H), dtype=torch.float32, device=dev)
    torch.mul(h0g, m.reshape(Rg, 1, 1), out=hm)
    gi = torch.addmm(b_ih, _c(x).reshape(R, -1), w_ih.t())
    fused = H % 32 == 0
    gh = None if fused else torch.addmm(b_hh, hm.view(R, H), w_hh.t())
    out = torch.empty((R, H), dtype=torch.float32, device=dev)
    d_ptr, ld = None, 0
    if dest is not None:
        dg = dest if dest.dim() == 3 else dest.unsqueeze(1)
        if tuple(dg.shape) != (Rg, G, H) or dg.stride(2) != 1 or dg.stride(1) != H or dg.dtype != torch.float32:
            raise ValueError("gru_infer_step: dest must be a float32 (R', G, H) view with rows of H contiguous")
        d_ptr, ld = dg.data_ptr(), dg.stride(0)
    with torch.cuda.device(dev):
        if fused:
            _lib.check(_lib.lib().cn_gru_fwd_fused(_stream(dev), R, H, gi.data_ptr(), hm.data_ptr(), _c(w_hh).data_ptr(),
                                                   _c(b_hh).data_ptr(), None, out.data_ptr(), None, None, d_ptr, G,
                                                   ld))
        else:
            _lib.check(_lib.lib().cn_gru_fwd_step_scatter(_stream(dev), R, H, gi.data_ptr(), gh.data_ptr(),
                                                          hm.data_ptr(), None, out.data_ptr(), None, None, d_ptr, G,
                                                          ld))
    return out


def gru_infer_group(*grus):
    """gru_infer_step for one or two GRUs of the same H (H % 32 == 0) in one launch (cn_gru_fwd_step_group):
    each argument is (x, h0, m, w_ih, w_hh, b_ih, b_hh, dest) as for gru_infer_step; the input projection runs
    in the kernel when every x has F % 32 == 0. Returns the new states (R, H) in order."""
    if not 1 <= len(grus) <= 2:
        raise ValueError("gru_infer_group: one or two GRUs")
    x0 = grus[0][0]
    if not x0.is_cuda:
        raise EdgeFeaturesUnavailable("gru_infer_group runs only through the HIP step kernels; tensors are on %s"
                                      % x0.device)
    H = grus[0][4].shape[1]
    xm = all(gr[0].shape[-1] % 32 == 0 for gr in grus)
    segs = (_lib.GruStepSeg * len(grus))()
    keep, outs = [], []
    for i, (x, h0, m, w_ih, w_hh, b_ih, b_hh, dest) in enumerate(grus):
        if w_hh.shape[1] != H or H % 32:
            raise ValueError("gru_infer_group: every GRU needs the same H, a multiple of 32")
        h0g = h0 if h0.dim() == 3 else h0.unsqueeze(1)
        Rg, G = h0g.shape[0], h0g.shape[1]
        R = Rg * G
        dev = x.device
        hm = torch.empty((Rg, G, H), dtype=torch.float32, device=dev)
        torch.mul(h0g, m.reshape(Rg, 1, 1), out=hm)
        x2 = _a16(x).reshape(R, -1)
        F = x2.shape[1]
        gi = None if xm else torch.addmm(b_ih, x2, w_ih.t())
        out = torch.empty((R, H), dtype=torch.float32, device=dev)
        d_ptr, ld = None, 0
        if dest is not None:
            dg = dest if dest.dim() == 3 else dest.unsqueeze(1)
            if tuple(dg.shape) != (Rg, G, H) or dg.stride(2) != 1 or dg.stride(1) != H or dg.dtype != torch.float32:
                raise ValueError("gru_infer_group: dest must be a float32 (R', G, H) view with rows of H contiguous")
            d_ptr, ld = dg.data_ptr(), dg.stride(0)
        wih, bih, whh, bhh = _a16(w_ih), _a16(b_ih), _a16(w_hh), _a16(b_hh)
        segs[i] = _lib.GruStepSeg(R, gi.data_ptr() if gi is not None else None, x2.data_ptr() if xm else None,
                                  wih.data_ptr() if xm else None, bih.data_ptr() if xm else None, F if xm else 0,
                                  hm.data_ptr(), whh.data_ptr(), bhh.data_ptr(), out.data_ptr(), d_ptr, G, ld)
        keep += [hm, x2, gi, wih, bih, whh, bhh]
        outs.append(out)
    dev = x0.device
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().cn_gru_fwd_step_group(_stream(dev), H, len(grus), segs))
    return outs


def gaussian_act(mean, logstd, deterministic=False):
    """The no-grad act() tail of DiagGaussian (distributions.py:74-94) in one launch: returns
    (action, log_prob) with action = mean (deterministic) or eps * exp(logstd) + mean, eps = torch.randn
    (the same draw FixedNormal.sample makes), log_prob summed over the action dims (cn_gaussian_act)."""
    if not mean.is_cuda:
        raise EdgeFeaturesUnavailable("gaussian_act runs only as the HIP kernel (tensors are on %s)" % mean.device)
    mean = _c(mean)
    E, A = mean.shape
    eps = None if deterministic else torch.randn((E, A), dtype=mean.dtype, device=mean.device)
    action = torch.empty_like(mean)
    logp = torch.empty((E, 1), dtype=torch.float32, device=mean.device)
    with torch.cuda.device(mean.device):
        _lib.check(_lib.lib().cn_gaussian_act(_stream(mean.device), E, A, mean.data_ptr(), _c(logstd).data_ptr(),
                                              eps.data_ptr() if eps is not None else None, action.data_ptr(),
                                              logp.data_ptr()))
    return action, logp


class _AttnPool(torch.autograd.Function):
    """srnn_model.py:320-333: weighted = bmm(h_spatials^T, attn) as one HBM pass (cn_attn_pool_fwd) and
    a one-pass backward (cn_attn_pool_bwd: d h_spatials and d attn together)."""

    @staticmethod
    def forward(ctx, hs, attn):
        R, N, H = hs.shape
        hs, attn = _c(hs), _c(attn).reshape(R, N)
        out = torch.empty((R, H), dtype=torch.float32, device=hs.device)
        with torch.cuda.device(hs.device):
            _lib.check(_lib.lib().cn_attn_pool_fwd(_stream(hs.device), R, N, H, hs.data_ptr(), attn.data_ptr(),
                                                   out.data_ptr()))
        ctx.save_for_backward(hs, attn)
        return out

    @staticmethod
    def backward(ctx, dout):
        hs, attn = ctx.saved_tensors
        R, N, H = hs.shape
        dout = _c(dout)
        dhs = torch.empty_like(hs)
        dattn = torch.empty((R, N), dtype=torch.float32, device=hs.device)
        with torch.cuda.device(hs.device):
            _lib.check(_lib.lib().cn_attn_pool_bwd(_stream(hs.device), R, N, H, hs.data_ptr(), attn.data_ptr(),
                                                   dout.data_ptr(), dhs.data_ptr(), dattn.data_ptr()))
        return dhs, dattn.reshape(R, N, 1)


def attention_pool(hs, attn):
    """hs (R, N, H), attn (R, N, 1) -> (R, H) = sum_n hs[:, n, :] * attn[:, n] (bmm(hs^T, attn))."""
    if not hs.is_cuda:
        raise EdgeFeaturesUnavailable("the DSRNN attention pooling runs only as the HIP kernel (cn_attn_pool_*); "
                                      "tensors are on %s" % hs.device)
    return _AttnPool.apply(hs, attn)


class _SpatialAttn(torch.autograd.Function):
    """srnn_model.py:256-333 (EdgeAttention.att_func + the bmm pooling) for the spatial edges, with the
    spatial_edge_layer folded into the score: score = scale * (hs . (te Ws) + te . bs), the same quantity
    as scale * sum_k te_k (Ws hs + bs)_k reassociated, so the (R*N, 64) spatial embedding, its product with
    temporal_embed and the second read of hs for the pooling are never formed (cn_spatial_attn_fwd: one
    pass over hs). Backward: cn_spatial_attn_bwd (one pass: dhs, du, dc), then the small host GEMMs
    d te = du Ws^T + dc bs^T, dWs = te^T du, dbs = te^T dc."""

    @staticmethod
    def forward(ctx, hs, te, ws, bs, scale):
        R, N, H = hs.shape
        hs, te = _c(hs), _c(te)
        u = torch.mm(te, ws)                 # (R, H)
        c = torch.mv(te, bs)                 # (R,)
        out = torch.empty((R, H), dtype=torch.float32, device=hs.device)
        attn = torch.empty((R, N), dtype=torch.float32, device=hs.device)
        with torch.cuda.device(hs.device):
            _lib.check(_lib.lib().cn_spatial_attn_fwd(_stream(hs.device), R, N, H, float(scale), hs.data_ptr(),
                                                      u.data_ptr(), c.data_ptr(), out.data_ptr(), attn.data_ptr()))
        ctx.scale = float(scale)
        ctx.save_for_backward(hs, te, ws, bs, u, attn)
        return out, attn.reshape(R, N, 1)

    @staticmethod
    def backward(ctx, dout, dattn):
        hs, te, ws, bs, u, attn = ctx.saved_tensors
        R, N, H = hs.shape
        dev = hs.device
        dout = _c(dout) if dout is not None else torch.zeros((R, H), dtype=torch.float32, device=dev)
        da = _c(dattn).reshape(R, N) if dattn is not None else None
        dhs = torch.empty_like(hs)
        ld = H + 4                           # [du | dc | pad] rows: dWs and dbs from one split-K GEMM
        due = torch.empty((R, ld), dtype=torch.float32, device=dev)
        du, dc = due[:, :H], due[:, H]
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().cn_spatial_attn_bwd(_stream(dev), R, N, H, ctx.scale, hs.data_ptr(), u.data_ptr(),
                                                      attn.data_ptr(), dout.data_ptr(),
                                                      da.data_ptr() if da is not None else None, dhs.data_ptr(),
                                                      due.data_ptr(), ld, due.data_ptr() + 4 * H, ld))
        dte = torch.addmm(torch.outer(dc, bs), du, ws.t()) if ctx.needs_input_grad[1] else None
        dws = dbs = None
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            g = wgrad(te, due)               # (A, H + 4) = te^T [du | dc | pad]; the pad columns are dropped
            dws, dbs = g[:, :H].contiguous(), g[:, H].contiguous()
        return dhs, dte, dws, dbs, None


def spatial_attention(hs, te, ws, bs, scale):
    """hs (R, N, H) spatial edge states, te (R, A) temporal_embed, ws (A, H) / bs (A,) spatial_edge_layer
    -> weighted (R, H), attn (R, N, 1) of EdgeAttention (srnn_model.py:256-333), one HIP pass over hs."""
    if not hs.is_cuda:
        raise EdgeFeaturesUnavailable("the DSRNN spatial attention runs only as the HIP kernel (cn_spatial_attn_*); "
                                      "tensors are on %s" % hs.device)
    return _SpatialAttn.apply(hs, te, ws, bs, scale)
