"""bench.py with the fp32 GEMM arithmetic forced: ``python scripts/ab/x6_bench.py X6 <bench args>``
(X6 = 1: exact-split bf16 MFMA, 0: f32 MFMA) -- the whole-step A/B of f32_set_x6."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from apex_amd import ops  # noqa: E402

ops.hip().f32_set_x6(int(sys.argv[1]))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
