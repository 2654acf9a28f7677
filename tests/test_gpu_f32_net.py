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
    """conv1 on bf16 MFMA with the exact three-term weight split (f32_conv1_fwd_x3_k, knob
    (1, 2)) vs the fp32-MFMA kernel (knob (1, 0)): per-element error against fp64, scaled by
    sum_k |x_k w_k| (the fp32 dot-product error scale), stays in the fp32 class -- every
    product is exact, only the fp32 accumulation rounds."""
    from apex_amd import ops
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    hip = ops.hip()
    m = _model(cuda, seed=3)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    f = m.features
    d = lambda t: t.detach().double()  # noqa: E731
    pre = F.conv2d(x.double(), d(f[0].weight), d(f[0].bias), stride=4)
    scale = F.conv2d(x.double(), d(f[0].weight).abs(), None, stride=4) + d(f[0].bias).abs().view(1, -1, 1, 1)
    ref = F.relu(pre)
    errs = {}
    try:
        for v in (0, 2):
            hip.f32_set_variant(1, v)
            ws = F32Workspace(B, 18, cuda, keep_for_backward=True)
            net(x, ws)
            torch.cuda.synchronize()
            g = _nchw(ws.a1, B, 32, 20)
            errs[v] = float(((g - ref).abs() / scale).max())
            assert bool((g >= 0).all())
    finally:
        hip.f32_set_variant(1, 2)  # the default
    # fp32 unit roundoff 6e-8: a K = 256 accumulation stays within a few ulps of sum|x w|
    assert errs[2] < 4e-7, errs
    assert errs[2] <= 2.0 * errs[0] + 1e-7, errs


@pytest.mark.parametrize("B", [37, 200])
def test_x9_gemm_forward_is_fp32_class(cuda, B):
    """conv2 / conv3 / FC1 forward on the exact-split bf16 GEMM body (both operands split
    into three bf16 terms, all 9 products exact, fp32 accumulation; knob (10, 1)) vs the
    fp32-MFMA body (knob (10, 0)): per-element error against fp64 from the SAME layer input,
    scaled by sum_k |a_k w_k|."""
    from apex_amd import ops
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    hip = ops.hip()
    m = _model(cuda, seed=7)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    f = m.features
    d = lambda t: t.detach().double()  # noqa: E731
    errs = {}
    try:
        for v in (0, 1):
            hip.f32_set_variant(10, v)
            ws = F32Workspace(B, 18, cuda, keep_for_backward=True)
            net(x, ws)
            torch.cuda.synchronize()
            g1, g2, g3 = _nchw(ws.a1, B, 32, 20), _nchw(ws.a2, B, 64, 9), _nchw(ws.a3, B, 64, 7)
            for name, inp, got, k, st in (("conv2", g1, g2, 2, 2), ("conv3", g2, g3, 4, 1)):
                ref = F.relu(F.conv2d(inp, d(f[k].weight), d(f[k].bias), stride=st))
                sc = F.conv2d(inp.abs(), d(f[k].weight).abs(), d(f[k].bias).abs(), stride=st)
                errs[(name, v)] = float(((got - ref).abs() / sc.clamp_min(1e-30)).max())
            hflat = g3.reshape(B, -1)
            for name, lin, sl in (("fc1a", m.advantage[0], slice(0, 128)), ("fc1v", m.value[0], slice(128, 256))):
                ref = F.relu(F.linear(hflat, d(lin.weight), d(lin.bias)))
                sc = F.linear(hflat.abs(), d(lin.weight).abs(), d(lin.bias).abs())
                errs[(name, v)] = float(((ws.h[:, sl].double() - ref).abs() / sc.clamp_min(1e-30)).max())
    finally:
        hip.f32_set_variant(10, 0)  # the default
    for name in ("conv2", "conv3", "fc1a", "fc1v"):
        e1, e0 = errs[(name, 1)], errs[(name, 0)]
        assert e1 < 1e-6, (name, errs)
        assert e1 <= 2.0 * e0 + 1e-7, (name, errs)


@pytest.mark.parametrize("B", [37, 300])
def test_direct_conv_forward_is_fp32_class(cuda, B):
    """conv2 / conv3 forward on the sample-resident kernel (f32_conv_fwd_direct_k, knob
    (25, 1): input samples in an LDS ring, weights in registers, v_mfma_f32_16x16x4_f32) vs
    the GEMM body (knob (25, 0)), per problem of a 3-problem launch (online / online on other
    frames / target net: the persistent workgroups split each problem's tiles, ranges start
    mid-sample): error against fp64 from the SAME layer input, scaled by sum_k |a_k w_k|;
    the single-problem launch is bit-identical to the 3-problem one."""
    from apex_amd import ops
    from apex_amd.models.fused import forward_multi
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    hip = ops.hip()
    m, mt = _model(cuda, seed=11), _model(cuda, seed=12)
    net, tnet = F32DuelingNet(m), F32DuelingNet(mt)
    xs = [torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda) for _ in range(2)]
    d = lambda t: t.detach().double()  # noqa: E731
    errs, q = {}, {}
    try:
        for v in (0, 1, 2, 3):
            hip.f32_set_variant(25, v)
            wss = [F32Workspace(B, 18, cuda, keep_for_backward=True) for _ in range(3)]
            forward_multi([(net, xs[0], wss[0], None, None), (net, xs[1], wss[1], None, None),
                           (tnet, xs[0], wss[2], None, None)])
            single = F32Workspace(B, 18, cuda, keep_for_backward=True)
            tnet(xs[0], single)
            torch.cuda.synchronize()
            assert torch.equal(single.a2, wss[2].a2) and torch.equal(single.a3, wss[2].a3), v
            for i, (mod, ws) in enumerate(zip((m, m, mt), wss)):
                f = mod.features
                g1, g2, g3 = _nchw(ws.a1, B, 32, 20), _nchw(ws.a2, B, 64, 9), _nchw(ws.a3, B, 64, 7)
                for name, inp, got, k, st in (("conv2", g1, g2, 2, 2), ("conv3", g2, g3, 4, 1)):
                    ref = F.relu(F.conv2d(inp, d(f[k].weight), d(f[k].bias), stride=st))
                    sc = F.conv2d(inp.abs(), d(f[k].weight).abs(), d(f[k].bias).abs(), stride=st)
                    errs[(name, i, v)] = float(((got - ref).abs() / sc.clamp_min(1e-30)).max())
                q[(i, v)] = ws.q.clone()
    finally:
        hip.f32_set_variant(25, 0)
    for key in [k for k in errs if k[2] > 0]:
        e1, e0 = errs[key], errs[key[:2] + (0,)]
        assert e1 < 1e-6, (key, errs)
        assert e1 <= 2.0 * e0 + 1e-7, (key, errs)
    for i in range(3):
        assert torch.equal(q[(i, 1)], q[(i, 2)]) and torch.equal(q[(i, 1)], q[(i, 3)])  # same per-row k order
        assert float((q[(i, 1)] - q[(i, 0)]).norm() / q[(i, 0)].norm()) < 1e-5


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
    (f32_conv1_wgrad_x3_k, knob (9, 1)) vs the fp32-MFMA kernel (knob (9, 0)), both against
    fp64 on the SAME conv1 output gradient, per element scaled by sum |dy x|."""
    from apex_amd import ops
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    hip = ops.hip()
    A = 18
    m = _model(cuda, A=A, seed=5)
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = F32Workspace(B, A, cuda, keep_for_backward=True)
    net(x, ws)
    dq = torch.randn(B, A, device=cuda) / B
    errs, f = {}, m.features
    try:
        for v in (0, 1):
            hip.f32_set_variant(9, v)
            net.backward(dq, x, ws)
            torch.cuda.synchronize()
            dy = _nchw(ws.dy1, B, 32, 20)
            ref = torch.nn.grad.conv2d_weight(x.double(), f[0].weight.shape, dy, stride=4)
            scale = torch.nn.grad.conv2d_weight(x.double(), f[0].weight.shape, dy.abs(), stride=4)
            errs[v] = float(((f[0].weight.grad.double() - ref).abs() / scale.clamp_min(1e-30)).max())
            bref = dy.sum((0, 2, 3))
            errs[f"b{v}"] = float(((f[0].bias.grad.double() - bref).abs() / dy.abs().sum((0, 2, 3))).max())
    finally:
        hip.f32_set_variant(9, 1)  # the default
    for v in (1,):
        assert errs[v] < 4e-7 and errs[f"b{v}"] < 4e-7, errs
        assert errs[v] <= 2.0 * errs[0] + 1e-7, errs


@pytest.mark.parametrize("B", [29, 512])
def test_f32_fc1_wgrad_slices_match_in_place(cuda, B):
    """FC1 weight gradient in batch slices (knob 15: natural-order partials summed +
    transposed by grad_finalize's FC1 row job) vs the in-place reference-layout pass: one
    slice is bit-identical, more slices differ only by the fp32 slice-sum order."""
    from apex_amd import ops
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    hip = ops.hip()
    A = 18
    m = _model(cuda, A=A, seed=7)
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    net = F32DuelingNet(m)
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = F32Workspace(B, A, cuda, keep_for_backward=True)
    net(x, ws)
    net.backward(torch.randn(B, A, device=cuda) / B, x, ws)  # fills ws.dz
    ga, gv = m.advantage[0].weight.grad, m.value[0].weight.grad
    net._fc1_bwd(ws, in_place=True)
    torch.cuda.synchronize()
    ref_a, ref_v = ga.clone(), gv.clone()
    try:
        for G in (1, 2, 4):
            hip.f32_set_variant(15, G)
            net._ws_B = None
            net.enable_backward(B)
            ga.fill_(float("nan"))
            gv.fill_(float("nan"))
            jobs = net._fc1_bwd(ws)
            assert len(jobs) == 2 and net._fc1_G == min(G, (B + 31) // 32)
            hip.grad_finalize(jobs, net._s(), 0)
            torch.cuda.synchronize()
            if G == 1:
                assert torch.equal(ga, ref_a) and torch.equal(gv, ref_v)
            else:
                torch.testing.assert_close(ga, ref_a, rtol=1e-5, atol=1e-6 * float(ref_a.abs().max()))
                torch.testing.assert_close(gv, ref_v, rtol=1e-5, atol=1e-6 * float(ref_v.abs().max()))
    finally:
        hip.f32_set_variant(15, 1)  # the default
        net._ws_B = None


def test_f32_finalize_norm_partials(cuda):
    """trunk_backward's grad_finalize sum-of-squares partials cover every trunk + FC1
    weight gradient (the FC1 weights through norm-only jobs)."""
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
