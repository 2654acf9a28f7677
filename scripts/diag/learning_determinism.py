"""The HIP learner's trajectory is bit-identical run to run; torch fp32's is not (its conv
backward): three short runs of tests/test_gpu_learning.py's setup in one process."""
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
import test_gpu_learning as T
cuda = torch.device("cuda:0")
for rep in range(3):
    tr = T._run(cuda, "fp32", steps=12)
    print(rep, [f"{tr[i]['hip_vs_64']:.3g}/{tr[i]['t32_vs_64']:.3g}" for i in (0, 2, 5, 8, 10, 11)],
          float(tr[-1]["hip_loss"]))
