"""C3 / C4 bottom-layer GEMMs (aggregate-first: Z = relu/dropout(Y W0), dW0 =
Y^T (dZ ⊙ mask)) on each GEMM mode, timed alone: Y [140,390 x 100] (C3's
bottom dst rows), W0 [100 x 256].  One JSON line per (kernel, mode, pitch)."""
import json
import sys

import torch

sys.path.insert(0, "sample-based-gnn_amd")
from nts import _abi  # noqa: E402
from nts.hip import HipContext  # noqa: E402

DEV = torch.device("cuda:0")


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    M, K, N = 140390, 100, 256
    g = torch.Generator(device=DEV).manual_seed(1)
    modes = {"f32": _abi.NTS_GEMM_F32, "split3": _abi.NTS_GEMM_SPLIT3, "split3_all": _abi.NTS_GEMM_SPLIT3_ALL}
    for pitch in (100, 128):
        Y = torch.empty(M, pitch, device=DEV)[:, :K]
        Y.copy_(torch.randn(M, K, device=DEV, generator=g))
        W = torch.randn(K, N, device=DEV, generator=g)
        Z = torch.empty(M, N, device=DEV)
        G = torch.randn(M, N, device=DEV, generator=g)
        dW = torch.empty(K, N, device=DEV)
        for name, mode in modes.items():
            ctx = HipContext(0, seed=2000)
            ctx.set_gemm_mode(mode)
            nn = timeit(lambda: ctx.gemm_relu_dropout(Y, W, Z, p=0.5, seed=7, offset=1))
            tn = timeit(lambda: ctx.gemm_tn_masked(Y, G, Z, dW, scale=2.0))
            nnp = timeit(lambda: ctx.gemm(Y, W, Z))
            tnp = timeit(lambda: ctx.gemm(Y, G, dW, trans_a=True))
            for k, us in (("nn_relu_dropout", nn), ("tn_masked", tn), ("nn_plain", nnp), ("tn_plain", tnp)):
                print(json.dumps({"kernel": k, "mode": name, "pitch": pitch, "us": round(us, 1)}), flush=True)
            ctx.close()


if __name__ == "__main__":
    main()
