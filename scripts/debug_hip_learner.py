"""Diagnostics for the HIP learner path: per-param grad error vs fp32 autograd on the
same sampled batch, then a few eager training steps printing loss / grad norms."""
import sys

import torch

sys.path.insert(0, ".")
from apex_amd.engine.apex import ApexEngine, EngineConfig  # noqa: E402
from apex_amd.engine.learner import LearnerConfig  # noqa: E402
from apex_amd.models.dqn import DuelingDQN  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
E = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = EngineConfig(n_envs=E, replay_capacity=200_000, threshold_size=50_000,
                   learner=LearnerConfig(batch_size=B, forward="hip"))
eng = ApexEngine(cfg, dev)
eng.fill()
L = eng.learner
L.sample_and_forward()
torch.cuda.synchronize()
print("loss", L.loss.item(), "q range", L.ws_s.q.min().item(), L.ws_s.q.max().item())
ours = {n: p.grad.clone() for n, p in L.model.named_parameters()}
ref = DuelingDQN.from_shapes((4, 84, 84), 18).to(dev)
ref.load_state_dict(L.model.state_dict())
q = ref(L.s.float())
print("fwd rel err", ((q - L.ws_s.q).norm() / q.norm()).item())
q.backward(L.dq)
for n, p in ref.named_parameters():
    g = ours[n]
    print(f"{n:22s} ref_norm {p.grad.norm().item():12.4e} ours_norm {g.norm().item():12.4e} "
          f"rel {((g - p.grad).norm() / (p.grad.norm() + 1e-30)).item():.3e}")
# fp32 conv backward through the same NHWC views for conv1 only
for step in range(30):
    eng.train_step()
    torch.cuda.synchronize()
    st = L.stats()
    print(step, {k: round(v, 5) if abs(v) < 1e6 else v for k, v in st.items()},
          "param absmax", L.flat.abs().max().item())

eng.capture()
for step in range(300):
    eng.train_step()
    if step % 20 == 0:
        torch.cuda.synchronize()
        st = L.stats()
        bad = {n: f"{p.grad.norm().item():.3e}" for n, p in L.model.named_parameters()}
        print("graphed", step, bad, {k: round(v, 5) if abs(v) < 1e6 else v for k, v in st.items()},
              "param absmax", L.flat.abs().max().item(), "q absmax", L.ws_s.q.abs().max().item())
