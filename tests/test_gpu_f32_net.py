"""Reference-precision (fp32 MFMA) network kernels vs plain PyTorch references.

Every layer of ``F32DuelingNet`` (f32_kernels.hip) is compared with an fp64 PyTorch
reference computed from the SAME layer input (the previous kernel's output), so each
kernel's own error is measured: fp32 accumulation over K <= 3136 stays far below the
rtol 1e-4 per layer / 1e-3 per parameter gradient required here."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _model(dev, A=18, seed=0):
    from apex_amd.models.dqn import DuelingDQN

    torch.manual_seed(seed)
    m = DuelingDQN.from_shapes((4, 84, 84), A).to(dev)
    with torch.no_grad():  # random biases: the reference init zeroes them
        for mod in list(m.features) + list(m.advantage) + list(m.value):
            if getattr(mod, "bias", None) is not None:
                mod.bias.uniform_(-0.1, 0.1)
    m.flatten_parameters()
    return m


def _rel(got, ref):
    return float((got.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))


def _nchw(t, B, C, H):
    return t.view(B, H, H, C).permute(0, 3, 1, 2).double()


@pytest.mark.parametrize("B", [37, 64])
def test_f32_layers_match_fp64(cuda, B):
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    m = _model(cuda)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = F32Workspace(B, 18, cuda, keep_for_backward=True)
    net(x, ws)
    torch.cuda.synchronize()
    f = m.features
    d = lambda t: t.detach().double()  # noqa: E731
    r1 = F.relu(F.conv2d(x.double(), d(f[0].weight), d(f[0].bias), stride=4))
    g1 = _nchw(ws.a1, B, 32, 20)
    assert _rel(g1, r1) < 1e-5
    r2 = F.relu(F.conv2d(g1, d(f[2].weight), d(f[2].bias), stride=2))
    g2 = _nchw(ws.a2, B, 64, 9)
    assert _rel(g2, r2) < 1e-5
    r3 = F.relu(F.conv2d(g2, d(f[4].weight), d(f[4].bias), stride=1))
    g3 = _nchw(ws.a3, B, 64, 7)
    assert _rel(g3, r3) < 1e-5
    hflat = g3.reshape(B, -1)
    ha = F.relu(F.linear(hflat, d(m.advantage[0].weight), d(m.advantage[0].bias)))
    hv = F.relu(F.linear(hflat, d(m.value[0].weight), d(m.value[0].bias)))
    assert _rel(ws.h[:, :128], ha) < 1e-5 and _rel(ws.h[:, 128:], hv) < 1e-5
    adv = F.linear(ha, d(m.advantage[2].weight), d(m.advantage[2].bias))
    val = F.linear(hv, d(m.value[2].weight), d(m.value[2].bias))
    q_ref = val + adv - adv.mean(1, keepdim=True)
    torch.testing.assert_close(ws.q.double(), q_ref, rtol=1e-4, atol=1e-4 * float(q_ref.abs().max()))
    # end to end against the fp32 module itself
    with torch.no_grad():
        q32 = m(x.float())
    assert float((ws.q - q32).norm() / q32.norm()) < 1e-5


@pytest.mark.parametrize("B", [37, 300])
def test_conv1_exact_split_is_fp32_class(cuda, B):
    """conv1 on bf16 MFMA with the exact three-term weight split (f32_conv1_fwd_x3_k):
    per-element error against fp64, scaled by sum_k |x_k w_k| (the fp32 dot-product error
    scale), stays in the fp32 class -- every product is exact, only the fp32 accumulation
    rounds (the retired fp32-MFMA conv1 kernel measured 1.5e-7 on the same test)."""
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    m = _model(cuda, seed=3)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    f = m.features
    d = lambda t: t.detach().double()  # noqa: E731
    pre = F.conv2d(x.double(), d(f[0].weight), d(f[0].bias), stride=4)
    scale = F.conv2d(x.double(), d(f[0].weight).abs(), None, stride=4) + d(f[0].bias).abs().view(1, -1, 1, 1)
    ref = F.relu(pre)
    ws = F32Workspace(B, 18, cuda, keep_for_backward=True)
    net(x, ws)
    torch.cuda.synchronize()
    g = _nchw(ws.a1, B, 32, 20)
    assert bool((g >= 0).all())
    # fp32 unit roundoff 6e-8: a K = 256 accumulation stays within a few ulps of sum|x w|
    assert float(((g - ref).abs() / scale).max()) < 4e-7


def test_f32_frame_ring_and_multi_pass(cuda):
    """conv1 reading the HBM frame ring by id (rows picked by idx) == dense input, and the
    3-problem launch == three single launches (bit-identical)."""
    from apex_amd.models.fused import forward_multi
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    m, mt = _model(cuda, A=6, seed=1), _model(cuda, A=6, seed=2)
    net, tnet = F32DuelingNet(m), F32DuelingNet(mt)
    B, F_ = 48, 300
    frames = torch.randint(0, 256, (F_, 84 * 84), dtype=torch.uint8, device=cuda)
    ids = torch.randint(0, F_, (100, 4), dtype=torch.int32, device=cuda)
    idx = torch.randint(0, 100, (B,), dtype=torch.int32, device=cuda)
    dense = frames[ids[idx.long()].long()].view(B, 4, 84, 84).contiguous()
    wss = [F32Workspace(B, 6, cuda) for _ in range(3)]
    forward_multi([(net, frames, wss[0], ids, idx), (net, dense, wss[1], None, None),
                   (tnet, frames, wss[2], ids, idx)])
    single = F32Workspace(B, 6, cuda)
    tnet(dense, single)
    torch.cuda.synchronize()
    assert torch.equal(wss[0].q, wss[1].q)
    assert torch.equal(wss[2].q, single.q)
    with torch.no_grad():
        assert float((wss[0].q - m(dense.float())).norm() / m(dense.float()).norm()) < 1e-5


@pytest.mark.parametrize("B", [29, 128])
def test_f32_backward_matches_fp64_autograd(cuda, B):
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    A = 18
    m = _model(cuda, A=A, seed=3)
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = F32Workspace(B, A, cuda, keep_for_backward=True)
    net(x, ws)
    dq = torch.randn(B, A, device=cuda) / B
    # poison the grads: every parameter gradient must be written (no accumulate / no zeroing pass)
    for p in m.parameters():
        p.grad.fill_(float("nan"))
    net.backward(dq, x, ws)
    torch.cuda.synchronize()
    m64 = _model(cuda, A=A, seed=3).double()
    m64.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
    q = m64(x.double())
    (q * dq.double()).sum().backward()
    for (name, p), p64 in zip(m.named_parameters(), m64.parameters()):
        ref = p64.grad
        err = float((p.grad.double() - ref).norm() / ref.norm().clamp_min(1e-30))
        assert err < 1e-4, (name, err)
        torch.testing.assert_close(p.grad.double(), ref, rtol=1e-3, atol=1e-4 * float(ref.abs().max()),
                                   msg=lambda s, n=name: f"{n}: {s}")


@pytest.mark.parametrize("B", [29, 256])
def test_conv1_wgrad_exact_split_is_fp32_class(cuda, B):
    """conv1 weight gradient on bf16 MFMA with dy split exactly into three bf16 terms
    (f32_conv1_wgrad_x3_k) against fp64 on the SAME conv1 output gradient, per element
    scaled by sum |dy x| (weights) / sum |dy| (bias)."""
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    A = 18
    m = _model(cuda, A=A, seed=5)
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = F32Workspace(B, A, cuda, keep_for_backward=True)
    net(x, ws)
    dq = torch.randn(B, A, device=cuda) / B
    f = m.features
    net.backward(dq, x, ws)
    torch.cuda.synchronize()
    dy = _nchw(ws.dy1, B, 32, 20)
    ref = torch.nn.grad.conv2d_weight(x.double(), f[0].weight.shape, dy, stride=4)
    scale = torch.nn.grad.conv2d_weight(x.double(), f[0].weight.shape, dy.abs(), stride=4)
    err = float(((f[0].weight.grad.double() - ref).abs() / scale.clamp_min(1e-30)).max())
    bref = dy.sum((0, 2, 3))
    berr = float(((f[0].bias.grad.double() - bref).abs() / dy.abs().sum((0, 2, 3))).max())
    assert err < 4e-7 and berr < 4e-7, (err, berr)


def test_f32_finalize_norm_partials(cuda):
    """trunk_backward's grad_finalize sum-of-squares partials cover every trunk + FC1
    weight gradient (the FC1 weights through their slice-transpose jobs)."""
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    B, A = 64, 6
    m = _model(cuda, A=A, seed=4)
    flat = m.flatten_parameters()
    g = torch.zeros_like(flat)
    off = 0
    for p in m.parameters():
        p.grad = g[off:off + p.numel()].view_as(p)
        off += p.numel()
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = F32Workspace(B, A, cuda, keep_for_backward=True)
    net(x, ws)
    ws.dz.normal_()
    ws.dz.mul_((ws.h > 0).float())
    sumsq = torch.zeros(8192, dtype=torch.float64, device=cuda)
    n = net.trunk_backward(x, ws, sumsq=sumsq)
    torch.cuda.synchronize()
    trunk = [m.features[i].weight.grad for i in (0, 2, 4)] + [m.features[i].bias.grad for i in (0, 2, 4)]
    trunk += [m.advantage[0].weight.grad, m.value[0].weight.grad]
    want = sum(float(t.double().pow(2).sum()) for t in trunk)
    got = float(sumsq[:n].sum())
    assert abs(got - want) <= 1e-6 * want


def test_f32_packed_arena_stays_exact_under_training(cuda):
    """The optimizer's fp32 PackMap / FcPack writes keep every packed copy EXACTLY equal to
    a fresh permutation of the master weights (online net), and target sync / actor
    publish copy the forward part (the kernels never see a stale or rounded weight)."""
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=64, replay_capacity=8192, threshold_size=2048, publish_param_interval=2,
                       target_update_interval=3, learner=LearnerConfig(batch_size=64, forward="hip", dtype="fp32"))
    eng = ApexEngine(cfg, cuda)
    eng.fill()
    for _ in range(2):
        eng.train_step()
    eng.capture()
    for _ in range(4):
        eng.train_step()
    torch.cuda.synchronize()
    L = eng.learner
    got = L.net.arena.clone()
    L.net.repack()
    assert torch.equal(got, L.net.arena)
    for net in (L.tnet, eng.actor_net):  # forward part matches its own master
        fwd = net.arena[:net.fwd_numel].clone()
        net.repack()
        assert torch.equal(fwd, net.arena[:net.fwd_numel])
    assert int(L.step_counter.item()) == 2 + 3 + 4


def test_gemm_layers_are_fp32_class(cuda):
    """Every gemm_body layer (conv2 / conv3 / FC1 forward; FC1, conv3, conv2 input and weight
    gradients) against fp64 on the SAME layer inputs, per element scaled by the fp32
    dot-product error scale sum_k |a_k b_k|.  The GEMMs run on v_mfma_f32_32x32x16_bf16 through
    the exact three-term split of every fp32 operand (six products per 16 k, every dropped term
    below 2^-23 |a b|); they must stay within a few fp32 ulps of that scale, like the fp32-MFMA
    kernels they replaced (round-5 table of both: profiles/r5_x6.md)."""
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    B, A = 96, 18
    m = _model(cuda, A=A, seed=7)
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = F32Workspace(B, A, cuda, keep_for_backward=True)
    net(x, ws)
    dq = torch.randn(B, A, device=cuda) / B
    net.backward(dq, x, ws)
    torch.cuda.synchronize()
    f = m.features
    d = lambda t: t.detach().double()  # noqa: E731
    errs = {}

    def scaled(name, got, ref, scale):
        errs[name] = float(((got.double() - ref).abs() / scale.clamp_min(1e-30)).max())

    g1, g2, g3 = _nchw(ws.a1, B, 32, 20), _nchw(ws.a2, B, 64, 9), _nchw(ws.a3, B, 64, 7)
    for name, xin, L, out in (("conv2", g1, 2, g2), ("conv3", g2, 4, g3)):
        st = 2 if L == 2 else 1
        pre = F.conv2d(xin, d(f[L].weight), d(f[L].bias), stride=st)
        sc = F.conv2d(xin.abs(), d(f[L].weight).abs(), d(f[L].bias).abs(), stride=st)
        mask = pre > 1e-6 * sc  # ReLU-active outputs (the clamped ones are exact zeros)
        scaled(name + "_fwd", out[mask], pre[mask], sc[mask])
    hflat = g3.reshape(B, -1)
    W = torch.cat([d(m.advantage[0].weight), d(m.value[0].weight)])
    bb = torch.cat([d(m.advantage[0].bias), d(m.value[0].bias)])
    pre = hflat @ W.t() + bb
    sc = hflat.abs() @ W.abs().t() + bb.abs()
    mask = pre > 1e-6 * sc
    scaled("fc1_fwd", ws.h.double()[mask], pre[mask], sc[mask])
    # backward: weight gradients from the kernels' own output gradients
    dz = ws.dz.double()  # [B, 256] (post-ReLU-mask FC1 output gradient)
    gW = torch.cat([m.advantage[0].weight.grad, m.value[0].weight.grad]).double()
    scaled("fc1_wgrad", gW, dz.t() @ hflat, dz.abs().t() @ hflat.abs())
    dy3 = _nchw(ws.dy3, B, 64, 7)
    ref = (dz @ W).view(B, 64, 7, 7) * (g3 > 0)
    sc = (dz.abs() @ W.abs()).view(B, 64, 7, 7)
    mask = g3 > 0
    scaled("fc1_dgrad", dy3[mask], ref[mask], sc[mask])
    for name, xin, L, dy, st in (("conv3", g2, 4, dy3, 1), ("conv2", g1, 2, _nchw(ws.dy2, B, 64, 9), 2)):
        ref = torch.nn.grad.conv2d_weight(xin, f[L].weight.shape, dy, stride=st)
        sc = torch.nn.grad.conv2d_weight(xin.abs(), f[L].weight.shape, dy.abs(), stride=st)
        scaled(name + "_wgrad", f[L].weight.grad, ref, sc)
        dx = torch.nn.grad.conv2d_input(xin.shape, d(f[L].weight), dy, stride=st)
        dxs = torch.nn.grad.conv2d_input(xin.shape, d(f[L].weight).abs(), dy.abs(), stride=st)
        got = _nchw(ws.dy2 if L == 4 else ws.dy1, B, xin.shape[1], xin.shape[2])
        mask = xin > 0
        scaled(name + "_dgrad", got[mask], dx[mask], dxs[mask])
    print({k: f"{v:.2e}" for k, v in errs.items()})
    # fp32 unit roundoff 6e-8: K <= 3136 accumulations stay within a few ulps of sum |a b|
    assert max(errs.values()) < 1e-6, errs



@pytest.mark.parametrize("B", [96, 384])
def test_stage_split_gemms_bit_identical(cuda, B):
    """The stage-split GEMM form (each staged fp32 element split once into bf16 hi / mid / lo
    planes in LDS, fragments read back as ready MFMA operands -- ds_read_b128 for K-major,
    ds_read_b64_tr_b16 for MN-major operands) against the per-wave register split: the same
    terms in the same MFMA k-slots, so every forward activation (3-problem learner launch:
    B = 384 takes the learner-sized tiles), every input gradient and every weight gradient is
    BIT-identical."""
    from apex_amd import ops
    from apex_amd.models.fused import forward_multi
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    hip = ops.hip()
    A = 18
    m, mt = _model(cuda, A=A, seed=11), _model(cuda, A=A, seed=12)
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    net, tnet = F32DuelingNet(m), F32DuelingNet(mt)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    x2 = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    dq = torch.randn(B, A, device=cuda) / B
    prev = hip.f32_stage_split()
    outs = []
    try:
        for mode in (0, 1 + 4, 2 + 8, 3 + 12):  # register split | stage-split, 2 LDS images | 1 | 1, 3 waves
            hip.f32_set_stage_split(mode)
            wss = [F32Workspace(B, A, cuda, keep_for_backward=(i == 0)) for i in range(3)]
            forward_multi([(net, x, wss[0], None, None), (net, x2, wss[1], None, None), (tnet, x2, wss[2], None, None)])
            net.backward(dq, x, wss[0])
            torch.cuda.synchronize()
            ws = wss[0]
            outs.append([t.clone() for t in (ws.a1, ws.a2, ws.a3, ws.h, ws.q, wss[1].q, wss[2].q, ws.dz, ws.dy3,
                                              ws.dy2, ws.dy1)] + [p.grad.clone() for p in m.parameters()])
    finally:
        hip.f32_set_stage_split(prev)
    for m, out in enumerate(outs[1:], 1):
        for i, (a, b) in enumerate(zip(outs[0], out)):
            assert torch.equal(a, b), (m, i, float((a - b).abs().max()))
