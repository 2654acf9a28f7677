"""Pre-split exact ("px") forward GEMMs (px_kernels.hip, knob (19, 1)): conv2 / conv3 / FC1
on bf16 MFMA with operands that arrive as three bf16 planes (hi + mid + lo == the fp32
value), six exact term products per element pair, fp32 accumulation.

* the planes the producers write are exact splits (conv1 epilogue, optimizer, split kernel);
* every layer's error against fp64 from the SAME layer input, scaled by sum_k |a_k w_k|,
  is fp32-class and within 2x of the fp32-MFMA body's;
* after learner steps with px on, the optimizer-maintained weight planes equal a fresh
  split of the fp32 packed weights (the optimizer writes them in its update pass)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _model(dev, A=18, seed=0):
    from apex_amd.models.dqn import DuelingDQN

    torch.manual_seed(seed)
    m = DuelingDQN.from_shapes((4, 84, 84), A).to(dev)
    with torch.no_grad():
        for mod in list(m.features) + list(m.advantage) + list(m.value):
            if getattr(mod, "bias", None) is not None:
                mod.bias.uniform_(-0.1, 0.1)
    m.flatten_parameters()
    return m


def _nchw(t, B, C, H):
    return t.view(B, H, H, C).permute(0, 3, 1, 2).double()


def _sum_planes(x, n=None):
    """fp64 sum of the three bf16 planes [3, N] (each term exact in fp64), first n elements."""
    x = x[:, :n] if n is not None else x
    return x[0].double() + x[1].double() + x[2].double()


@pytest.fixture
def px(cuda):
    from apex_amd import ops

    hip = ops.hip()
    hip.f32_set_variant(19, 1)
    yield hip
    hip.f32_set_variant(19, 0)


@pytest.mark.parametrize("B", [37, 200])
def test_px_forward_is_fp32_class(cuda, B):
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
            hip.f32_set_variant(19, v)
            ws = F32Workspace(B, 18, cuda, keep_for_backward=True)
            assert ws.px == bool(v)
            net(x, ws)
            torch.cuda.synchronize()
            if v:  # the activation planes are exact splits of the fp32 activations
                for full, planes in ((ws.a1, ws.a1x), (ws.a2, ws.a2x), (ws.a3, ws.a3x)):
                    assert torch.equal(_sum_planes(planes, full.numel()), full.reshape(-1).double())
                assert torch.equal(_sum_planes(net.arena_x.view(3, -1), net.arena.numel()), net.arena.double())
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
        hip.f32_set_variant(19, 0)
    print("px errors (scaled, vs fp64):", {k: f"{e:.2e}" for k, e in errs.items()})
    for name in ("conv2", "conv3", "fc1a", "fc1v"):
        e1, e0 = errs[(name, 1)], errs[(name, 0)]
        assert e1 < 1e-6, (name, errs)
        assert e1 <= 2.0 * e0 + 1e-7, (name, errs)


def test_px_multi_pass_equals_single(cuda, px):
    """The 3-problem px launch == three single launches (bit-identical)."""
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace, forward_multi_f32

    m, mt = _model(cuda, A=6, seed=1), _model(cuda, A=6, seed=2)
    net, tnet = F32DuelingNet(m), F32DuelingNet(mt)
    B = 96
    xs = [torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda) for _ in range(3)]
    wss = [F32Workspace(B, 6, cuda) for _ in range(3)]
    forward_multi_f32([(net, xs[0], wss[0], None, None), (net, xs[1], wss[1], None, None),
                       (tnet, xs[2], wss[2], None, None)])
    singles = [F32Workspace(B, 6, cuda) for _ in range(3)]
    for n_, x_, w_ in ((net, xs[0], singles[0]), (net, xs[1], singles[1]), (tnet, xs[2], singles[2])):
        forward_multi_f32([(n_, x_, w_, None, None)])
    torch.cuda.synchronize()
    for a, b in zip(wss, singles):
        assert torch.equal(a.q, b.q) and torch.equal(a.a3, b.a3)


def test_px_optimizer_keeps_weight_planes(cuda, px):
    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=64, replay_capacity=16384, threshold_size=2048, use_graphs=False,
                       learner=LearnerConfig(batch_size=128, forward="hip"))
    eng = ApexEngine(cfg, cuda)
    eng.fill()
    net = eng.learner.net
    before = net.arena_x.clone()
    for _ in range(3):
        eng.train_step()
    torch.cuda.synchronize()
    assert not torch.equal(before, net.arena_x)  # the weights moved
    fresh = torch.empty_like(net.arena_x)
    n = net.arena.numel()
    eng.learner.net.hip.f32_split_planes(net.arena.data_ptr(), fresh.data_ptr(), n, net.x_plane,
                                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(fresh.view(3, -1)[:, :n], net.arena_x.view(3, -1)[:, :n])
    st = eng.learner.stats()
    assert st["loss"] == st["loss"]


@pytest.mark.parametrize("B,terms,fc1_slices", [(29, 1, 1), (128, 2, 1), (128, 1, 0)])
def test_pxb_backward_matches_fp64_autograd(cuda, B, terms, fc1_slices):
    """Pre-split exact backward (pxb_kernels.hip, knobs (19, terms) + (20, 1)): every parameter
    gradient against fp64 autograd, next to the fp32-MFMA backward's own error; the output
    gradients' planes the FC1 / conv3 input-gradient epilogues write are exact splits."""
    from apex_amd import ops
    from apex_amd.models.fused_f32 import F32DuelingNet, F32Workspace

    hip = ops.hip()
    A = 18
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    dq = torch.randn(B, A, device=cuda) / B
    m64 = _model(cuda, A=A, seed=3).double()
    (m64(x.double()) * dq.double()).sum().backward()
    errs = {}
    try:
        hip.f32_set_variant(15, fc1_slices)
        for v in (0, terms):
            hip.f32_set_variant(19, v)
            hip.f32_set_variant(20, 1 if v else 0)
            m = _model(cuda, A=A, seed=3)
            for p in m.parameters():
                p.grad = torch.full_like(p, float("nan"))  # every gradient must be written
            net = F32DuelingNet(m)
            ws = F32Workspace(B, A, cuda, keep_for_backward=True)
            assert ws.pxb == bool(v)
            net(x, ws)
            net.backward(dq, x, ws)
            torch.cuda.synchronize()
            if v:
                for full, planes in ((ws.dz, ws.dzx), (ws.dy3, ws.dy3x), (ws.dy2, ws.dy2x)):
                    assert torch.equal(_sum_planes(planes, full.numel()), full.reshape(-1).double())
            for (name, p), p64 in zip(m.named_parameters(), m64.parameters()):
                ref = p64.grad
                errs[(name, v)] = float((p.grad.double() - ref).norm() / ref.norm().clamp_min(1e-30))
    finally:
        hip.f32_set_variant(19, 0)
        hip.f32_set_variant(20, 0)
        hip.f32_set_variant(15, 1)
    print("pxb grad errors (rel, vs fp64):", {k: f"{e:.2e}" for k, e in errs.items()})
    for (name, v), e in errs.items():
        if v:
            assert e < 1e-4, (name, e)
            assert e <= 3.0 * errs[(name, 0)] + 1e-6, (name, e, errs[(name, 0)])
