"""Synthetic graphs shaped like the BASELINE configs (no datasets can be fetched).

Chung–Lu power-law multigraph, symmetrised, plus one self-loop per vertex, in
the reference's edge-file order: for every sampled pair k the edges
(u_k, v_k), (v_k, u_k), then the self-loops (i, i).  Expected degrees follow
w_i = (i + i0)^-1/2 with i0 chosen so max/mean matches the real dataset;
vertex ids are randomly permuted.  Features N(0,1) fp32, labels uniform,
masks 65/10/25 % by vertex id (GNNDatum::random_generate, core/ntsDataloador.hpp:835-861).
Everything is generated with torch on the target device from fixed seeds
(graph 2024, features 7).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

# name: (V, total edges incl. self-loops, feature dim, classes, max/mean degree)
SHAPES = {
    "reddit": (232_965, 114_848_857, 602, 41, 44.0),
    "products": (2_449_029, 126_167_309, 100, 47, 350.0),
    "papers100m": (111_059_956, 3_339_184_668, 128, 172, 1000.0),
    "tiny": (2_000, 40_000, 32, 8, 10.0),
}


def _solve_i0(V: int, ratio: float) -> float:
    # ratio(x) = 1 / (2 sqrt(x) (sqrt(1+x) - sqrt(x))), x = i0 / V; bisect on log x
    lo, hi = 1e-12, 10.0
    for _ in range(200):
        mid = math.sqrt(lo * hi)
        r = 1.0 / (2 * math.sqrt(mid) * (math.sqrt(1 + mid) - math.sqrt(mid)))
        if r > ratio:
            lo = mid
        else:
            hi = mid
    return max(lo * V, 1e-3)


@dataclass
class SyntheticGraph:
    n_vertices: int
    src: torch.Tensor  # int32 [E]  (uint32 ids)
    dst: torch.Tensor  # int32 [E]

    @property
    def n_edges(self) -> int:
        return self.src.numel()


def chung_lu(V: int, total_edges: int, max_over_mean: float, device="cuda", seed: int = 2024,
             chunk: int = 1 << 24) -> SyntheticGraph:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    i0 = _solve_i0(V, max_over_mean)
    w = (torch.arange(V, device=device, dtype=torch.float64) + i0).pow(-0.5)
    cdf = torch.cumsum(w, 0)
    cdf = (cdf / cdf[-1]).to(torch.float64)
    perm = torch.randperm(V, generator=g, device=device).to(torch.int32)
    M = max((total_edges - V) // 2, 0)
    src = torch.empty(2 * M + V, dtype=torch.int32, device=device)
    dst = torch.empty_like(src)
    for s in range(0, M, chunk):
        n = min(chunk, M - s)
        ru = torch.rand(n, generator=g, device=device, dtype=torch.float64)
        rv = torch.rand(n, generator=g, device=device, dtype=torch.float64)
        u = perm[torch.searchsorted(cdf, ru).clamp_(max=V - 1)]
        v = perm[torch.searchsorted(cdf, rv).clamp_(max=V - 1)]
        # interleave (u,v),(v,u)
        src[2 * s:2 * (s + n):2] = u
        dst[2 * s:2 * (s + n):2] = v
        src[2 * s + 1:2 * (s + n):2] = v
        dst[2 * s + 1:2 * (s + n):2] = u
    ar = torch.arange(V, dtype=torch.int32, device=device)
    src[2 * M:] = ar
    dst[2 * M:] = ar
    return SyntheticGraph(V, src, dst)


def features(V: int, F: int, device="cuda", seed: int = 7, dtype=torch.float32) -> torch.Tensor:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randn(V, F, generator=g, device=device, dtype=dtype)


def labels_masks(V: int, C: int, device="cuda", seed: int = 11):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    labels = torch.randint(0, C, (V,), generator=g, device=device, dtype=torch.int64)
    masks = torch.full((V,), 2, dtype=torch.int32, device=device)
    max_train = int(V * 0.65)
    max_val = int(V * 0.10 + max_train)
    masks[:max_train] = 0
    masks[max_train:max_val] = 1
    return labels, masks


def shaped(name: str, device="cuda", scale: float = 1.0) -> tuple[SyntheticGraph, int, int]:
    V, E, F, C, ratio = SHAPES[name]
    V = max(int(V * scale), 16)
    E = max(int(E * scale), 2 * V)
    return chung_lu(V, E, ratio, device=device), F, C
