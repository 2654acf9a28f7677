"""Bit-reproducibility check of the HIP fp32 learner: run the learning-parity harness for a
few steps and dump the HIP learner's per-step loss / priority sums (run twice per build, and
for two builds via PYTHONPATH, to tell a kernel change from run-to-run nondeterminism)."""
import json
import sys

import torch

sys.path.insert(0, "tests")
sys.path.append(".")  # after PYTHONPATH: an A/B build given there wins
import test_gpu_learning as T  # noqa: E402

dev = torch.device("cuda", 0)
traj = T._run(dev, "fp32", steps=int(sys.argv[2]) if len(sys.argv) > 2 else 30)
out = [{"hip_loss": r["hip_loss"], "hip_prio": float(r["hip_prio"].sum()), "t32_loss": r["t32_loss"],
        "hip_vs_64": r["hip_vs_64"], "t32_vs_64": r["t32_vs_64"]} for r in traj]
import apex_amd
out.append({"pkg": apex_amd.__file__})
json.dump(out, open(sys.argv[1], "w"))
