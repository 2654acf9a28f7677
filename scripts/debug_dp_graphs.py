"""Graph-vs-eager equality probe for the engine's learner paths (single-process and the
data-parallel phase split with a world-1 all-reduce)."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests.test_gpu_overlap import _engine  # noqa: E402

dev = torch.device("cuda:0")
for dp in (False, True):
    for overlap in (True, False):
        for first_eager in (False, True):
            g = _engine(dev, overlap, True, dp=dp)
            e = _engine(dev, overlap, False, dp=dp)
            for eng in (g, e):
                eng.fill()
            if first_eager:
                g.train_step()
                e.train_step()
            g.capture()
            for _ in range(3):
                e.train_step()
            res = []
            for k in range(6):
                g.train_step()
                e.train_step()
                torch.cuda.synchronize()
                res.append(int(torch.equal(g.learner.flat, e.learner.flat)))
            print(f"dp={dp} overlap={overlap} first_eager={first_eager} equal-per-step={res} "
                  f"leaf_eq={torch.equal(g.replay.leaf_sum, e.replay.leaf_sum)}", flush=True)
