"""Micro-benchmark of the FC1 GEMM shapes (hipBLASLt through torch) on the GPU."""
import torch

dev = torch.device("cuda")
B, K, N = 512, 3136, 256
a3 = torch.randn(B, K, device=dev).bfloat16()
w = torch.randn(N, K, device=dev).bfloat16()
dz = torch.randn(B, N, device=dev).bfloat16()
z = torch.empty(B, N, device=dev)
zt = torch.empty(N, B, device=dev)


def t(fn, it=200):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1000


cases = {
    "fwd a3@w^T f32out": lambda: torch.mm(a3, w.t(), out_dtype=torch.float32, out=z),
    "fwd w@a3^T f32out": lambda: torch.mm(w, a3.t(), out_dtype=torch.float32, out=zt),
    "fwd a3@w^T bf16": lambda: torch.mm(a3, w.t()),
    "fwd linear bf16": lambda: torch.nn.functional.linear(a3, w),
    "dW dz^T@a3 f32": lambda: torch.mm(dz.t(), a3, out_dtype=torch.float32),
    "dW a3^T@dz f32 (transposed out)": lambda: torch.mm(a3.t(), dz, out_dtype=torch.float32),
    "dX dz@w bf16": lambda: torch.mm(dz, w),
    "dX w^T@dz^T bf16": lambda: torch.mm(w.t(), dz.t()),
}
for name, fn in cases.items():
    print(f"{name:40s} {t(fn):8.2f} us", flush=True)
