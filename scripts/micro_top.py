#!/usr/bin/env python3
"""Time the fused output-layer kernels in isolation (Reddit shape 10000 x 128 -> 41)."""
import sys
import pathlib

import torch

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
from nts.hip import HipContext  # noqa: E402

dev = "cuda:0"
h = HipContext(0, seed=1)
n, K, C = 10000, 128, 41
Y = torch.randn(n, K, device=dev)
W = torch.randn(K, C, device=dev) * 0.1
lab = torch.randint(0, C, (n,), device=dev)
loss = torch.empty((), device=dev)
dY, dW = torch.empty(n, K, device=dev), torch.empty(K, C, device=dev)
one = torch.ones((), device=dev)
for name, f in (("train", lambda: h.linear_xent_train(Y, W, lab, loss, dY, dW)),
                ("fwd", lambda: h.linear_xent_fwd(Y, W, lab, loss)),
                ("bwd", lambda: h.linear_xent_bwd(Y, W, lab, one, dY, dW))):
    for _ in range(5):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us/call")
