"""Where do write_batch and the sequential writes disagree (test_batched_tree_write_equals_sequential_writes)?"""
import torch

from apex_amd.engine.hbm_replay import HBMReplay

cuda = torch.device("cuda")
C, B, E = 4096, 512, 256
g = torch.Generator(device=cuda).manual_seed(11)
rp1 = HBMReplay(C, E, 3, 0.6, cuda)
rp2 = HBMReplay(C, E, 3, 0.6, cuda)
c1, c2 = torch.zeros(1, dtype=torch.int64, device=cuda), torch.zeros(1, dtype=torch.int64, device=cuda)
slots = torch.arange(E, device=cuda, dtype=torch.int32)
aprio = torch.rand(E, device=cuda, generator=g) * 2 + 0.05
idx = torch.randint(0, C, (B,), device=cuda, generator=g, dtype=torch.int32)
idx[:E // 4] = slots[:E // 4]
idx[E // 4:E // 2] = idx[:E // 4]
delta = torch.rand(B, device=cuda, generator=g) * 3
lw = torch.rand(B, device=cuda, generator=g)
p1, p2 = torch.zeros(B, device=cuda), torch.zeros(B, device=cuda)
l1, l2 = torch.zeros(1, device=cuda), torch.zeros(1, device=cuda)
rp1.write_priorities(slots, aprio, dedup=False, bumps=((rp1.filled, E),))
torch.cuda.synchronize()
after_actor = rp1.leaf_sum.clone()
rp1.write_priorities(idx, None, dedup=True, bumps=((c1, 1),), mix=(delta, lw, p1, l1))
rp2.write_batch(pre=(slots, aprio, rp2.filled), idx=idx, bump=c2, mix=(delta, lw, p2, l2))
torch.cuda.synchronize()
print("prio equal", torch.equal(p1, p2), "loss", l1.item(), l2.item())
d = (rp1.leaf_sum != rp2.leaf_sum).nonzero().flatten()
print("differing leaves", d.numel(), d[:20].tolist())
for j in d[:10].tolist():
    pos = (idx == j).nonzero().flatten().tolist()
    print(j, "seq", rp1.leaf_sum[j].item(), "batch", rp2.leaf_sum[j].item(), "actor-only", after_actor[j].item(),
          "positions", pos, "p at last", p1[pos[-1]].item() ** 0.6 if pos else None, "in slots", j < E)
dk = (p1 != p2).nonzero().flatten()
dm = delta.max()
ref = (0.9 * dm + 0.1 * delta) + 1e-6
print("prio diffs", dk.numel(), "seq==torch", torch.equal(p1, ref), "batch==torch", torch.equal(p2, ref))
for k in dk[:5].tolist():
    print(k, p1[k].item(), p2[k].item(), ref[k].item(), delta[k].item())
