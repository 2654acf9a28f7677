"""HIP MFMA network kernels vs plain PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _model(dev, A=18, seed=0):
    from apex_amd.models.dqn import DuelingDQN

    torch.manual_seed(seed)
    m = DuelingDQN.from_shapes((4, 84, 84), A).to(dev)
    # random biases (the reference init zeroes them) so the bias paths are exercised
    with torch.no_grad():
        for mod in list(m.features) + list(m.advantage) + list(m.value):
            if hasattr(mod, "bias") and mod.bias is not None:
                mod.bias.uniform_(-0.1, 0.1)
    m.flatten_parameters()
    return m


def test_conv_layers_match_torch(cuda):
    from apex_amd.models.fused import HipDuelingNet, NetWorkspace

    m = _model(cuda)
    net = HipDuelingNet(m)
    B = 10
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = NetWorkspace(B, 18, cuda)
    net(x, ws)
    torch.cuda.synchronize()
    f = m.features
    # layer-by-layer reference in fp32 on bf16-rounded operands (our kernels: bf16 x bf16 -> fp32 acc)
    r1 = F.relu(F.conv2d(x.float(), _bf(f[0].weight), f[0].bias, stride=4))
    got1 = ws.a1.float().view(B, 20, 20, 32).permute(0, 3, 1, 2)
    torch.testing.assert_close(got1, _bf(r1), rtol=1e-2, atol=1e-2)
    r2 = F.relu(F.conv2d(got1, _bf(f[2].weight), f[2].bias, stride=2))
    got2 = ws.a2.float().view(B, 9, 9, 64).permute(0, 3, 1, 2)
    torch.testing.assert_close(got2, _bf(r2), rtol=1e-2, atol=1e-2)
    r3 = F.relu(F.conv2d(got2, _bf(f[4].weight), f[4].bias, stride=1))
    got3 = ws.a3.float().view(B, 7, 7, 64).permute(0, 3, 1, 2)
    torch.testing.assert_close(got3, _bf(r3), rtol=1e-2, atol=1e-2)
    # heads on the same a3
    hflat = got3.reshape(B, -1)
    adv = F.linear(F.relu(F.linear(hflat, _bf(m.advantage[0].weight), m.advantage[0].bias)), m.advantage[2].weight,
                   m.advantage[2].bias)
    val = F.linear(F.relu(F.linear(hflat, _bf(m.value[0].weight), m.value[0].bias)), m.value[2].weight,
                   m.value[2].bias)
    q_ref = val + adv - adv.mean(1, keepdim=True)
    torch.testing.assert_close(ws.q, q_ref, rtol=1e-3, atol=1e-3)


def test_forward_close_to_fp32_module(cuda):
    from apex_amd.models.fused import HipDuelingNet, NetWorkspace

    m = _model(cuda, A=6)
    net = HipDuelingNet(m)
    B = 64
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = NetWorkspace(B, 6, cuda)
    q = net(x, ws).clone()
    with torch.no_grad():
        q_ref = m(x.float())
    err = (q - q_ref).norm() / q_ref.norm()
    assert err < 2e-2, float(err)


def test_backward_grads_close_to_autograd(cuda):
    from apex_amd.models.fused import HipDuelingNet, NetWorkspace

    m = _model(cuda, A=18, seed=1)
    P = sum(p.numel() for p in m.parameters())
    flat_grad = torch.full((P,), float("nan"), device=cuda)  # every grad must be written
    off = 0
    for p in m.parameters():
        p.grad = flat_grad[off:off + p.numel()].view_as(p)
        off += p.numel()
    net = HipDuelingNet(m)
    B = 128
    x = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    ws = NetWorkspace(B, 18, cuda, keep_for_backward=True)
    net(x, ws)
    dq = torch.randn(B, 18, device=cuda) / B
    net.backward(dq, x, ws)
    torch.cuda.synchronize()
    assert torch.isfinite(flat_grad).all()
    ours = {n: p.grad.clone() for n, p in m.named_parameters()}
    ref = _model(cuda, A=18, seed=1)
    ref.load_state_dict(m.state_dict())
    q = ref(x.float())
    q.backward(dq)
    for n, p in ref.named_parameters():
        g = ours[n]
        # bf16 activations flip a few ReLU masks vs the fp32 reference: expect a few % of
        # relative error (measured 0.3-7%); a wrong kernel gives O(1)
        rel = (g - p.grad).norm() / (p.grad.norm() + 1e-12)
        assert rel < 0.15, (n, float(rel))


def test_hip_learner_engine_step(cuda):
    import numpy as np

    from apex_amd.engine.apex import ApexEngine, EngineConfig
    from apex_amd.engine.learner import LearnerConfig

    cfg = EngineConfig(n_envs=64, replay_capacity=16384, threshold_size=2048,
                       learner=LearnerConfig(batch_size=128, forward="hip"))
    eng = ApexEngine(cfg, cuda)
    eng.fill()
    before = eng.learner.flat.clone()
    for _ in range(3):
        eng.train_step()
    eng.capture()
    for _ in range(5):
        eng.train_step()
    torch.cuda.synchronize()
    st = eng.learner.stats()
    assert np.isfinite(st["loss"]) and st["grad_norm_l2"] > 0
    assert not torch.equal(before, eng.learner.flat)


def _rand_bf16(shape, dev, scale=1.0, g=None):
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(dev)


@pytest.mark.parametrize("layer,masked", [(1, False), (2, False), (3, False), (1, True), (2, True)])
def test_wgrad_kernel_matches_torch(cuda, layer, masked):
    """MFMA weight/bias gradient vs torch fp32 on identical bf16-valued operands (with the
    optional ReLU mask of dy applied while staging)."""
    from apex_amd import ops

    hip = ops.hip()
    g = torch.Generator().manual_seed(layer)
    geo = {1: (4, 84, 32, 8, 4, 20), 2: (32, 20, 64, 4, 2, 9), 3: (64, 9, 64, 3, 1, 7)}[layer]
    C, H, N, KS, S, OH = geo
    B = 37
    if layer == 1:
        x = torch.randint(0, 256, (B, 4, H, H), generator=g, dtype=torch.uint8).to(cuda)
        x_f = x.float()
        xptr = x.data_ptr()
    else:
        x_nhwc = _rand_bf16((B, H, H, C), cuda, 1.0, g)
        x_f = x_nhwc.float().permute(0, 3, 1, 2)
        xptr = x_nhwc.data_ptr()
    dy = _rand_bf16((B, OH, OH, N), cuda, 0.1, g)
    mask = _rand_bf16((B, OH, OH, N), cuda, 1.0, g) if masked else None
    ws = torch.empty(hip.wgrad_workspace_floats(layer), device=cuda)
    gw = torch.empty(N, C, KS, KS, device=cuda)
    gb = torch.empty(N, device=cuda)
    hip.conv_wgrad(layer, xptr, 0, 0, dy.data_ptr(), 0 if mask is None else mask.data_ptr(), B, ws.data_ptr(),
                   gw.data_ptr(), gb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    dy_eff = dy.float() if mask is None else dy.float() * (mask.float() > 0)
    dy_f = dy_eff.permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(x_f, (N, C, KS, KS), dy_f, stride=S)
    ref_b = dy_f.sum((0, 2, 3))
    torch.testing.assert_close(gw, ref_w, rtol=2e-3, atol=2e-3 * ref_w.abs().max().item())
    torch.testing.assert_close(gb, ref_b, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("layer", [2, 3])
def test_dgrad_kernel_matches_torch(cuda, layer):
    """MFMA input gradient vs torch fp32, with both optional ReLU masks (dy while staged,
    the output in the epilogue)."""
    from apex_amd import ops

    hip = ops.hip()
    g = torch.Generator().manual_seed(10 + layer)
    C, H, N, KS, S, OH = {2: (32, 20, 64, 4, 2, 9), 3: (64, 9, 64, 3, 1, 7)}[layer]
    B = 21
    w = torch.randn(N, C, KS, KS, generator=g).to(cuda) * 0.1
    wt = torch.empty(KS, KS, C, N, dtype=torch.bfloat16, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    hip.pack_conv_wt(w.data_ptr(), wt.data_ptr(), N, C, KS, KS, s)
    dy = _rand_bf16((B, OH, OH, N), cuda, 1.0, g)
    act = _rand_bf16((B, OH, OH, N), cuda, 1.0, g)  # ~half positive: exercises the input mask
    act_below = _rand_bf16((B, H, H, C), cuda, 1.0, g)  # epilogue (output) mask
    out = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=cuda)
    hip.conv_dgrad(layer, dy.data_ptr(), act.data_ptr(), wt.data_ptr(), out.data_ptr(), act_below.data_ptr(), B, s)
    dy_m = dy.float() * (act.float() > 0)
    ref = torch.nn.grad.conv2d_input((B, C, H, H), _bf(w), dy_m.permute(0, 3, 1, 2), stride=S)
    ref = (ref.permute(0, 2, 3, 1) * (act_below.float() > 0)).to(torch.bfloat16).float()
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2)


def test_frame_ring_input_matches_dense(cuda):
    """conv1 reading stacks in place from the frame ring (ids + idx) == dense input."""
    from apex_amd.models.fused import HipDuelingNet, NetWorkspace

    m = _model(cuda, A=18, seed=3)
    net = HipDuelingNet(m)
    g = torch.Generator().manual_seed(0)
    frames = torch.randint(0, 256, (50, 84 * 84), generator=g, dtype=torch.uint8).to(cuda)
    table = torch.randint(0, 50, (30, 4), generator=g, dtype=torch.int32).to(cuda)
    idx = torch.randint(0, 30, (12,), generator=g, dtype=torch.int32).to(cuda)
    dense = frames[table[idx.long()].long()].view(12, 4, 84, 84).contiguous()
    ws1, ws2 = NetWorkspace(12, 18, cuda), NetWorkspace(12, 18, cuda)
    q1 = net(dense, ws1).clone()
    q2 = net(frames, ws2, table, idx).clone()
    assert torch.equal(q1, q2)


@pytest.mark.parametrize("tiles", [False, True])
@pytest.mark.parametrize("opt", ["rmsprop", "adam"])
def test_fused_optimizer_packing_matches_repack(cuda, opt, tiles):
    """The optimizer's PackMap stores (and, with ``tiles``, the LDS-transposed FC1 tile
    path) leave the bf16 arena exactly as repack() would."""
    from apex_amd import ops
    from apex_amd.models.fused import HipDuelingNet

    hip = ops.hip()
    m = _model(cuda)
    flat = m.flatten_parameters()
    net = HipDuelingNet(m)
    net.enable_backward()
    d1, d2 = net.pack_maps()
    P = flat.numel()
    assert int((d1 >= 0).sum()) == net.fwd_numel
    assert int((d2 >= 0).sum()) == net.arena.numel() - net.fwd_numel
    g = torch.randn(P, device=cuda)
    s1, s2 = torch.zeros(P, device=cuda), torch.zeros(P, device=cuda)
    partials = torch.zeros(hip.grad_norm_partials(), dtype=torch.float64, device=cuda)
    norms = torch.zeros(4, device=cuda)
    step = torch.zeros(1, dtype=torch.int64, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    net.arena.zero_()
    hip.grad_sumsq(g.data_ptr(), P, partials.data_ptr(), s)
    fc = net.fc_pack_args() if tiles else {}
    if opt == "rmsprop":
        hp = hip.RMSpropParams(1e-3, 0.95, 1.5e-7, 40.0, 1.0, 0, 0, True)
        hip.rmsprop_step(flat.data_ptr(), g.data_ptr(), s1.data_ptr(), s2.data_ptr(), P, partials.data_ptr(),
                         partials.numel(), hp, step.data_ptr(), norms.data_ptr(), s, d1.data_ptr(), d2.data_ptr(),
                         net.arena.data_ptr(), **fc)
    else:
        hp = hip.AdamParams(1e-3, max_norm=40.0)
        hip.adam_step(flat.data_ptr(), g.data_ptr(), s1.data_ptr(), s2.data_ptr(), P, partials.data_ptr(),
                      partials.numel(), hp, step.data_ptr(), norms.data_ptr(), s, d1.data_ptr(), d2.data_ptr(),
                      net.arena.data_ptr(), **fc)
    fused = net.arena.clone()
    net.repack()
    assert torch.equal(fused.view(torch.int16), net.arena.view(torch.int16))


def test_optimizer_tiles_and_grad_scale_bit_exact(cuda):
    """FC1 tile path == scatter-map path elementwise, and grad_scale=1/k on a k-times
    gradient (the DP all-reduce SUM) == the plain update, bit for bit."""
    from apex_amd import ops
    from apex_amd.models.fused import HipDuelingNet

    hip = ops.hip()
    m = _model(cuda)
    flat0 = m.flatten_parameters().clone()
    net = HipDuelingNet(m)
    net.enable_backward()
    d1, d2 = net.pack_maps()
    P = flat0.numel()
    g = torch.randn(P, device=cuda) * 0.3
    s = torch.cuda.current_stream().cuda_stream
    s10, s20 = torch.rand(P, device=cuda), torch.randn(P, device=cuda) * 0.1
    outs = []
    for tiles, k in ((False, 1), (True, 1), (True, 4)):
        flat, s1, s2 = flat0.clone(), s10.clone(), s20.clone()
        gk = g * k
        partials = torch.zeros(hip.grad_norm_partials(), dtype=torch.float64, device=cuda)
        norms = torch.zeros(4, device=cuda)
        step = torch.zeros(1, dtype=torch.int64, device=cuda)
        hip.grad_sumsq(gk.data_ptr(), P, partials.data_ptr(), s)
        hp = hip.RMSpropParams(1e-3, 0.95, 1.5e-7, 1.0, 1.0, 0, 0, True)  # clipping active
        hp.grad_scale = 1.0 / k
        hip.rmsprop_step(flat.data_ptr(), gk.data_ptr(), s1.data_ptr(), s2.data_ptr(), P, partials.data_ptr(),
                         partials.numel(), hp, step.data_ptr(), norms.data_ptr(), s, d1.data_ptr(), d2.data_ptr(),
                         net.arena.data_ptr(), **(net.fc_pack_args() if tiles else {}))
        outs.append((flat, s1, s2, norms.clone()))
    for j, o in enumerate(outs[1:], 1):
        for name, a, b in zip(("param", "s1", "s2", "norms"), outs[0], o):
            bad = (a != b).nonzero().flatten()
            assert bad.numel() == 0, (j, name, bad.numel(), bad[:8].tolist(), (a - b).abs().max().item())


@pytest.mark.parametrize("B", [1536, 512, 256, 37])
def test_fc1_splitk_matches_torch(cuda, B):
    """Split-K FC1 partials sum to the fp32 GEMM of the same bf16 operands (ragged batch
    included: the last 32-row tile is clamped on load and masked on store)."""
    from apex_amd import ops
    from apex_amd.models.fused import FC1_SPLITS, FEAT

    hip = ops.hip()
    g = torch.Generator().manual_seed(B)
    a = _rand_bf16((B, FEAT), cuda, g=g)
    w = _rand_bf16((256, FEAT), cuda, scale=0.02, g=g)
    part = torch.full((FC1_SPLITS, B, 256), float("nan"), device=cuda)
    S = hip.fc1_fwd(a.data_ptr(), w.data_ptr(), part.data_ptr(), B, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert S == hip.fc1_splits_for(B) and 1 <= S <= FC1_SPLITS
    want = a.float() @ w.float().t()
    got = part[:S].sum(0)
    assert torch.isfinite(part[:S]).all()
    assert (got - want).abs().max().item() <= 1e-4 * max(1.0, want.abs().max().item())


@pytest.mark.parametrize("B", [512, 37])
def test_forward_multi_equals_single_passes(cuda, B):
    """One launch per layer for 3 passes (two nets, ring input via ids/idx) gives the
    same activations as three single-pass forwards."""
    from apex_amd.models.fused import HipDuelingNet, NetWorkspace, forward_multi

    m1, m2 = _model(cuda, seed=1), _model(cuda, seed=2)
    n1, n2 = HipDuelingNet(m1), HipDuelingNet(m2)
    F = 4 * B + 8
    g = torch.Generator(device=cuda).manual_seed(B)
    frames = torch.randint(0, 256, (F, 84 * 84), dtype=torch.uint8, device=cuda, generator=g)
    s_ids = torch.randint(0, F, (3 * B, 4), dtype=torch.int32, device=cuda, generator=g)
    s2_ids = torch.randint(0, F, (3 * B, 4), dtype=torch.int32, device=cuda, generator=g)
    idx = torch.randperm(3 * B, device=cuda)[:B].int()
    ws = [NetWorkspace(B, 18, cuda, keep_for_backward=(i == 0)) for i in range(6)]
    forward_multi([(n1, frames, ws[0], s_ids, idx), (n1, frames, ws[1], s2_ids, idx),
                   (n2, frames, ws[2], s2_ids, idx)])
    n1(frames, ws[3], s_ids, idx)
    n1(frames, ws[4], s2_ids, idx)
    n2(frames, ws[5], s2_ids, idx)
    torch.cuda.synchronize()
    for a, b in ((0, 3), (1, 4), (2, 5)):
        # conv activations bit-identical; FC1's split-K slab count follows the launch's
        # total rows, so Q may differ by fp32 summation order only
        assert torch.equal(ws[a].a1, ws[b].a1) and torch.equal(ws[a].a3, ws[b].a3)
        torch.testing.assert_close(ws[a].q, ws[b].q, rtol=1e-5, atol=1e-6 * ws[b].q.abs().max().item())
    assert not torch.equal(ws[1].q, ws[2].q)  # different nets really ran


@pytest.mark.parametrize("B", [512, 100])
def test_fc1_backward_matches_torch(cuda, B):
    """fc1_bwd: dy3 = relu_mask(dz . W, a3) in bf16 and the dW slabs reduced + scattered by
    grad_finalize into the reference [n][c*49+p] layout, vs torch fp32 on the same
    bf16-valued operands."""
    from apex_amd import ops
    from apex_amd.models.fused import C3, FEAT, P3

    hip = ops.hip()
    g = torch.Generator().manual_seed(B)
    dz = _rand_bf16((B, 256), cuda, scale=0.1, g=g)
    a3 = torch.relu(_rand_bf16((B, FEAT), cuda, g=g))  # post-ReLU activations (zeros included)
    w = _rand_bf16((256, FEAT), cuda, scale=0.05, g=g)  # packed [n][p*64+c]
    wt = w.t().contiguous()
    dy3 = torch.full((B, FEAT), 7.0, dtype=torch.bfloat16, device=cuda)
    ws = torch.full((hip.fc1_bwd_workspace_floats(),), float("nan"), device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    hip.fc1_bwd(dz.data_ptr(), a3.data_ptr(), wt.data_ptr(), dy3.data_ptr(), ws.data_ptr(), B, s)
    ga = torch.zeros(128, FEAT, device=cuda)
    gv = torch.zeros(128, FEAT, device=cuda)
    hip.grad_finalize([hip.fc1_finalize_job(0, ws.data_ptr(), ga.data_ptr()),
                       hip.fc1_finalize_job(1, ws.data_ptr(), gv.data_ptr())], s)
    torch.cuda.synchronize()
    dx = (dz.float() @ w.float()) * (a3.float() > 0)
    torch.testing.assert_close(dy3.float(), dx, rtol=1e-2, atol=1e-3)
    gw = dz.float().t() @ a3.float()  # [256][p*64+c]
    ref = gw.view(256, P3, C3).permute(0, 2, 1).reshape(256, FEAT)  # -> [n][c*49+p]
    torch.testing.assert_close(ga, ref[:128], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gv, ref[128:], rtol=1e-4, atol=1e-4)
