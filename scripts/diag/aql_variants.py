#!/usr/bin/env python
"""Which AQL learner-step variants agree bit for bit with the reference launch sequence (per
tensor), without stopping at the first difference: ``python scripts/diag/aql_variants.py``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def run(**kw):
    from apex_amd.engine.aql import AQLEngine, AQLEngineConfig
    cfg = AQLEngineConfig(env_id="BipedalWalker-v3", n_envs=64, capacity=8192, batch_size=32, seed=9, **kw)
    eng = AQLEngine(cfg, "cuda")
    L = eng.learner
    eng.fill(1024)
    for _ in range(int(os.environ.get("ITERS", "5"))):
        eng.iteration()
    torch.cuda.synchronize()
    r = eng.replay
    return dict(idx=L.idx.clone(), w=L.w.clone(), flat=L.flat.clone(), prio=L.prio.clone(), step=L.step_ctr.clone(),
                leaf_sum=r.leaf_sum.clone(), root=r.node_sum[-1].clone(), nodes1=r.node_sum[0].clone())


ref = run(fused_sample=False, fused_tree=False, split_tree=False, fused_step=False, bwd_tree=False, fused_update=False)
for name, kw in (("update, draw in update", dict(fused_update=True, tree_levels_in_grad=False, draw_in_grad=False)),
                 ("update, draw in grad", dict(fused_update=True, tree_levels_in_grad=False, draw_in_grad=True)),
                 ("update, levels+draw in grad", dict(fused_update=True, tree_levels_in_grad=True, draw_in_grad=True)),
                 ("bwd_tree only", dict(fused_update=False, bwd_tree=True))):
    out = run(**kw)
    diffs = [k for k in ref if not torch.equal(ref[k], out[k])]
    print(f"{name:32s}", "OK" if not diffs else "DIFF " + " ".join(
        f"{k}({(ref[k].double() - out[k].double()).abs().max().item():.3g})" for k in diffs), flush=True)
