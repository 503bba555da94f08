"""Thin Python handle over the C-ABI (one `nts_hip_ctx` per stream).

Used by the kernel-level parity tests and by the data-preparation helpers;
the training path itself runs in the C++ host layer (nts/host).  All methods
take torch tensors already resident on the GPU and enqueue work on the
context's stream; nothing here falls back to the CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import torch

from . import _abi
from ._abi import check, ptr


def _u32(n, device):
    return torch.empty(int(n), dtype=torch.int32, device=device)


class HipContext:
    """Owns an nts_hip_ctx bound to a torch stream (Cuda_Stream equivalent)."""

    def __init__(self, device: int = 0, stream: torch.cuda.Stream | None = None, seed: int = 2000):
        self.lib = _abi.lib()
        self.device = device
        self.stream = stream if stream is not None else torch.cuda.current_stream(device)
        h = C.c_void_p()
        check(self.lib.nts_hip_ctx_create(C.byref(h), device, C.c_void_p(self.stream.cuda_stream), seed))
        self.h = h

    def set_gemm_mode(self, mode: int):
        """NTS_GEMM_F32 (fp32-input MFMA) or NTS_GEMM_SPLIT3 (fp32-accurate
        three-piece bf16 split on the bf16 MFMA) for this context's GEMMs."""
        check(self.lib.nts_hip_ctx_set_gemm_mode(self.h, int(mode)))

    def close(self):
        if self.h:
            self.lib.nts_hip_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- context -------------------------------------------------------------
    def reserve(self, n_vertices: int, max_items: int):
        check(self.lib.nts_hip_ctx_reserve(self.h, n_vertices, max_items))

    def rng_seed(self, seed: int):
        check(self.lib.nts_hip_rng_seed(self.h, seed))

    def rng_state(self) -> torch.Tensor:
        out = torch.empty(625, dtype=torch.int32)
        check(self.lib.nts_hip_rng_state(self.h, C.c_void_p(out.data_ptr())))
        return out

    # ---- graph ---------------------------------------------------------------
    def degrees(self, src: torch.Tensor, dst: torch.Tensor, V: int):
        out_deg = _u32(V, src.device)
        in_deg = _u32(V, src.device)
        check(self.lib.nts_hip_degrees(self.h, ptr(src), ptr(dst), src.numel(), V,
                                       ptr(out_deg), ptr(in_deg)))
        return out_deg, in_deg

    def build_csc(self, src: torch.Tensor, dst: torch.Tensor, V: int):
        col = torch.empty(V + 1, dtype=torch.int64, device=src.device)
        rows = _u32(src.numel(), src.device)
        check(self.lib.nts_hip_build_csc(self.h, ptr(src), ptr(dst), src.numel(), V,
                                         ptr(col), ptr(rows)))
        return col, rows

    # ---- sampler -------------------------------------------------------------
    def sample_layer(self, graph: "DeviceGraph", lay: "LayerBuffers", fanout: int, layer: int,
                     batch_seq: int, rng_mode: int, weight_type: int):
        g = graph.as_struct()
        o = lay.as_struct()
        check(self.lib.nts_hip_sample_layer(self.h, C.byref(g), fanout, layer, batch_seq,
                                            rng_mode, weight_type, C.byref(o)))

    # ---- movement / aggregation ------------------------------------------------
    def gather_rows(self, table, index, n_dev, n_cap, out):
        F = table.shape[1]
        check(self.lib.nts_hip_gather_rows(self.h, ptr(table), table.stride(0), ptr(index),
                                           ptr(n_dev), n_cap, F, ptr(out), out.stride(0)))

    def cache_select(self, out_degree, n_vertices: int, n_cache: int, cache_map, cache_ids):
        check(self.lib.nts_hip_cache_select(self.h, ptr(out_degree), n_vertices, n_cache,
                                            ptr(cache_map), ptr(cache_ids)))

    def gather_rows_cached(self, cache, cache_map, host: "HostTable", index, n_dev, n_cap, out):
        F = host.shape[1]
        check(self.lib.nts_hip_gather_rows_cached(
            self.h, ptr(cache), cache.stride(0) if cache is not None else host.ld, ptr(cache_map),
            host.dev_ptr, host.ld, ptr(index), ptr(n_dev), n_cap, F, ptr(out), out.stride(0)))

    def stage_uncached_rows(self, cache_map, host: "HostTable", index, n_dev, n_cap, stage):
        F = host.shape[1]
        check(self.lib.nts_hip_stage_uncached_rows(self.h, ptr(cache_map), host.dev_ptr, host.ld,
                                                   ptr(index), ptr(n_dev), n_cap, F, ptr(stage),
                                                   stage.stride(0)))

    def spmm_csc_fwd_cached(self, co, ri, w, v_dev, v_cap, cache, cache_map, host: "HostTable",
                            row_map, y, stage=None):
        """stage: rows staged by local src id (stage_uncached_rows), else the host table."""
        F = host.shape[1]
        spill, ld = (stage.data_ptr(), stage.stride(0)) if stage is not None else (host.dev_ptr, host.ld)
        check(self.lib.nts_hip_spmm_csc_fwd_cached(
            self.h, ptr(co), ptr(ri), ptr(w), ptr(v_dev), v_cap, ptr(cache),
            cache.stride(0) if cache is not None else ld, ptr(cache_map), spill, ld,
            int(stage is not None), ptr(row_map), F, ptr(y), y.stride(0)))

    def gat_forward(self, co, ri, dl, v, H, att, m, a, Y):
        F = H.shape[1]
        check(self.lib.nts_hip_gat_forward(self.h, ptr(co), ptr(ri), ptr(dl), v, ptr(H), H.stride(0),
                                           F, ptr(att), ptr(m), ptr(a), ptr(Y), Y.stride(0)))

    def gat_backward(self, co, ri, dl, v, ro, ci, ceid, s, H, att, a, m, Y, GY, du, ds2, dH, dS,
                     GM=None):
        F = H.shape[1]
        if GM is None:
            GM = torch.empty(max(v, 1), F, device=H.device)
        check(self.lib.nts_hip_gat_backward(
            self.h, ptr(co), ptr(ri), ptr(dl), v, ptr(ro), ptr(ci), ptr(ceid), s, ptr(H), H.stride(0),
            F, ptr(att), ptr(a), ptr(m), ptr(Y), Y.stride(0), ptr(GY), GY.stride(0), ptr(du), ptr(ds2),
            ptr(GM), GM.stride(0), ptr(dH), dH.stride(0), ptr(dS)))

    def gather_labels(self, labels, index, n_dev, n_cap, out):
        check(self.lib.nts_hip_gather_labels(self.h, ptr(labels), ptr(index), ptr(n_dev),
                                             n_cap, ptr(out)))

    def spmm_csc_fwd(self, co, ri, w, v_dev, v_cap, x, y, row_map=None):
        F = x.shape[1]
        check(self.lib.nts_hip_spmm_csc_fwd(self.h, ptr(co), ptr(ri), ptr(w), ptr(v_dev), v_cap,
                                            ptr(x), x.stride(0), ptr(row_map), F, ptr(y),
                                            y.stride(0)))

    def spmm_csc_fwd_act(self, co, ri, w, v_dev, v_cap, x, y, p=0.0, seed=0, offset=0):
        """y = dropout(relu(A x), p) (transform-first bottom layer)."""
        F = x.shape[1]
        check(self.lib.nts_hip_spmm_csc_fwd_act(self.h, ptr(co), ptr(ri), ptr(w), ptr(v_dev), v_cap,
                                                ptr(x), x.stride(0), F, ptr(y), y.stride(0),
                                                float(p), int(seed), int(offset)))

    def act_bits_words(self, F):
        return int(self.lib.nts_hip_act_bits_words(F))

    def spmm_csc_fwd_act_bits(self, co, ri, w, v_dev, v_cap, x, y, bits, p=0.0, seed=0, offset=0):
        """spmm_csc_fwd_act that also writes the keep mask [y > 0] as bits
        (act_bits_words(F) int32 words per row)."""
        F = x.shape[1]
        check(self.lib.nts_hip_spmm_csc_fwd_act_bits(self.h, ptr(co), ptr(ri), ptr(w), ptr(v_dev),
                                                     v_cap, ptr(x), x.stride(0), F, ptr(y),
                                                     y.stride(0), float(p), int(seed), int(offset),
                                                     ptr(bits)))

    def spmm_csr_bwd_postmask_bits(self, ro, ci, wb, s_dev, s_cap, g_out, bits, g_in, scale=1.0):
        """spmm_csr_bwd_postmask with the mask from spmm_csc_fwd_act_bits."""
        F = g_out.shape[1]
        check(self.lib.nts_hip_spmm_csr_bwd_postmask_bits(self.h, ptr(ro), ptr(ci), ptr(wb),
                                                          ptr(s_dev), s_cap, ptr(g_out),
                                                          g_out.stride(0), ptr(bits), float(scale), F,
                                                          ptr(g_in), g_in.stride(0)))

    def spmm_csr_bwd_postmask(self, ro, ci, wb, s_dev, s_cap, g_out, x_act, g_in, scale=1.0):
        """g_in = (A^T g_out) ⊙ (x_act > 0) * scale, x_act indexed by g_in's rows."""
        F = g_out.shape[1]
        check(self.lib.nts_hip_spmm_csr_bwd_postmask(self.h, ptr(ro), ptr(ci), ptr(wb), ptr(s_dev),
                                                     s_cap, ptr(g_out), g_out.stride(0), ptr(x_act),
                                                     x_act.stride(0), float(scale), F, ptr(g_in),
                                                     g_in.stride(0)))

    def spmm_csr_bwd_masked(self, ro, ci, wb, s_dev, s_cap, g_out, x_act, g_in, scale=1.0):
        """g_in = A^T (g_out * (x_act > 0) * scale) over the CSR."""
        F = g_out.shape[1]
        check(self.lib.nts_hip_spmm_csr_bwd_masked(self.h, ptr(ro), ptr(ci), ptr(wb), ptr(s_dev),
                                                   s_cap, ptr(g_out), g_out.stride(0), ptr(x_act),
                                                   x_act.stride(0), float(scale), F, ptr(g_in),
                                                   g_in.stride(0)))

    def spmm_csr_bwd(self, ro, ci, wb, s_dev, s_cap, g_out, g_in):
        F = g_out.shape[1]
        check(self.lib.nts_hip_spmm_csr_bwd(self.h, ptr(ro), ptr(ci), ptr(wb), ptr(s_dev), s_cap,
                                            ptr(g_out), g_out.stride(0), F, ptr(g_in),
                                            g_in.stride(0)))

    def colmax_rows_per_part(self, F):
        return int(self.lib.nts_hip_csr_bwd_colmax_rows_per_part(F))

    def spmm_csr_bwd_colmax(self, ro, ci, wb, s_dev, s_cap, g_out, g_in, parts, rs=None,
                            rows=None):
        """spmm_csr_bwd + parts[p, c] (int32 bits) = max |rs(s) g_in[s, c]| over
        the part's rows s in [p R, (p+1) R), R = colmax_rows_per_part(F),
        rs(s) = rs[rows[s]] (rows None: rs[s]; rs None: 1)."""
        F = g_out.shape[1]
        check(self.lib.nts_hip_spmm_csr_bwd_colmax(self.h, ptr(ro), ptr(ci), ptr(wb), ptr(s_dev), s_cap,
                                                   ptr(g_out), g_out.stride(0), F, ptr(g_in),
                                                   g_in.stride(0), ptr(parts), ptr(rs), ptr(rows)))

    def spmm_csc_bwd_atomic(self, co, ri, w, v_dev, v_cap, g_out, g_in):
        F = g_out.shape[1]
        check(self.lib.nts_hip_spmm_csc_bwd_atomic(self.h, ptr(co), ptr(ri), ptr(w), ptr(v_dev),
                                                   v_cap, ptr(g_out), g_out.stride(0), F,
                                                   ptr(g_in), g_in.stride(0)))

    def gemm(self, A, B, C, trans_a=False):
        """C = A @ B (trans_a: A.T @ B) on the MFMA fp32 kernels."""
        if trans_a:
            K, M = A.shape
        else:
            M, K = A.shape
        N = B.shape[1]
        check(self.lib.nts_hip_gemm_f32(self.h, int(trans_a), M, N, K, ptr(A), A.stride(0), ptr(B),
                                        B.stride(0), ptr(C), C.stride(0)))

    def act_backward(self, g, x_act, out, scale=1.0):
        """out = g * (x_act > 0) * scale."""
        rows, F = g.shape
        check(self.lib.nts_hip_act_backward(self.h, rows, F, ptr(g), g.stride(0), ptr(x_act),
                                            x_act.stride(0), float(scale), ptr(out), out.stride(0)))

    # ---- PD cache ----------------------------------------------------------------
    def presample_counts(self, graph: "DeviceGraph", seeds, layers: int, counts, tmp):
        g = graph.as_struct()
        check(self.lib.nts_hip_presample_counts(self.h, C.byref(g), ptr(seeds), seeds.numel(),
                                                layers, ptr(counts), ptr(tmp)))

    def presample_select(self, counts, cache_rate: float, out_ids, out_n):
        check(self.lib.nts_hip_presample_select(self.h, ptr(counts), counts.numel(),
                                                float(cache_rate), ptr(out_ids), ptr(out_n)))

    def pd_set_cache(self, ids, key: int, cache_map, cache_location):
        check(self.lib.nts_hip_pd_set_cache(self.h, ptr(ids), ids.numel(), key, ptr(cache_map),
                                            ptr(cache_location)))

    def pd_load_share(self, omit_row, v_dev, v_cap, share, emb):
        F = emb.shape[1]
        check(self.lib.nts_hip_pd_load_share(self.h, ptr(omit_row), ptr(v_dev), v_cap, ptr(share),
                                             share.stride(0), F, ptr(emb), emb.stride(0)))

    def relu_dropout(self, x, y, p=0.0, seed=0, offset=0):
        rows, F = x.shape
        check(self.lib.nts_hip_relu_dropout_f32(self.h, rows, F, ptr(x), x.stride(0), float(p),
                                                int(seed), int(offset), ptr(y), y.stride(0)))

    def gemm_gather(self, A, rows, B, C):
        """C = A[rows] @ B (rows: int32 device tensor of row ids)."""
        M, K, N = rows.numel(), A.shape[1], B.shape[1]
        check(self.lib.nts_hip_gemm_gather_f32(self.h, M, N, K, ptr(A), A.stride(0), ptr(rows),
                                               ptr(B), B.stride(0), ptr(C), C.stride(0)))

    def gemm_tn_gather(self, A, rows, B, C):
        """C = A[rows].T @ B."""
        K, M, N = rows.numel(), A.shape[1], B.shape[1]
        check(self.lib.nts_hip_gemm_tn_gather_f32(self.h, M, N, K, ptr(A), A.stride(0), ptr(rows),
                                                  ptr(B), B.stride(0), ptr(C), C.stride(0)))

    # ---- two-piece f16 pair tables (csrc/gemmh2.hip) ---------------------------
    def h2_split_rows(self, X, pad_to=32):
        """X [R, K] fp32 -> (P int32 [R, Kp] pair words, rs fp32 [R] row scales)."""
        R, K = X.shape
        Kp = (K + pad_to - 1) // pad_to * pad_to
        P = torch.empty(R, Kp, dtype=torch.int32, device=X.device)
        rs = torch.empty(R, dtype=torch.float32, device=X.device)
        check(self.lib.nts_hip_h2_split_rows(self.h, R, K, ptr(X), X.stride(0), Kp, ptr(P),
                                             P.stride(0), ptr(rs)))
        return P, rs

    def h2_split_rows_planar(self, X, pad_to=32, tail=False):
        """X [R, K] fp32 -> (Q int16 [R, 2 Kp]: y0 plane then y1 plane per row, rs [R]).
        tail: rows padded to 2560 bytes (Q a view of them) with the row scale in
        the tail, as the driver builds the table (the four-stage forward GEMM)."""
        R, K = X.shape
        Kp = (K + pad_to - 1) // pad_to * pad_to
        if tail and 4 * Kp + 8 <= 2560:
            Q = torch.empty(R, 1280, dtype=torch.int16, device=X.device)[:, :2 * Kp]
        else:
            Q = torch.empty(R, 2 * Kp, dtype=torch.int16, device=X.device)
        rs = torch.empty(R, dtype=torch.float32, device=X.device)
        check(self.lib.nts_hip_h2_split_rows_planar(self.h, R, K, ptr(X), X.stride(0), Kp, ptr(Q),
                                                    Q.stride(0), ptr(rs)))
        return Q, rs

    def gemm_h2p_gather(self, Q, rs, rows, W, C, relu_dropout=False, p=0.0, seed=0, offset=0):
        """C = act(X[rows] @ W), X given as its planar pair table (rows None: all rows)."""
        K, N = W.shape
        M = rows.numel() if rows is not None else Q.shape[0]
        check(self.lib.nts_hip_gemm_h2p_gather(self.h, int(relu_dropout), M, N, Q.shape[1] // 2, ptr(Q),
                                               Q.stride(0), ptr(rs), ptr(rows), ptr(W), W.stride(0), K,
                                               ptr(C), C.stride(0), float(p), int(seed), int(offset)))

    def gemm_h2p_tn_gather(self, Q, rs, rows, B, C, M, parts=None, rows_per_part=0):
        """C = X[rows, :M].T @ B with X given as its planar pair table."""
        N = B.shape[1]
        Kr = rows.numel() if rows is not None else B.shape[0]
        if parts is not None:  # B's per-part column maxima given (spmm_csr_bwd_colmax)
            check(self.lib.nts_hip_gemm_h2p_tn_gather_cm(self.h, M, N, Kr, ptr(Q), Q.stride(0),
                                                         Q.shape[1] // 2, ptr(rs), ptr(rows), ptr(B),
                                                         B.stride(0), ptr(C), C.stride(0), ptr(parts),
                                                         rows_per_part))
            return
        check(self.lib.nts_hip_gemm_h2p_tn_gather(self.h, M, N, Kr, ptr(Q), Q.stride(0),
                                                  Q.shape[1] // 2, ptr(rs), ptr(rows), ptr(B),
                                                  B.stride(0), ptr(C), C.stride(0)))

    def gemm_h2d_act(self, A, W, C, relu_dropout=False, p=0.0, seed=0, offset=0, Q=None, rs=None):
        """C = act(A @ W) with A (K <= 128) split into f16 pairs in the kernel;
        Q/rs: A's planar pair table written on the way."""
        K, N = W.shape
        M = A.shape[0]
        check(self.lib.nts_hip_gemm_h2d_act(self.h, int(relu_dropout), M, N, K, ptr(A), A.stride(0),
                                            ptr(W), W.stride(0), ptr(C), C.stride(0), float(p), int(seed),
                                            int(offset), ptr(Q) if Q is not None else None,
                                            Q.stride(0) if Q is not None else 0,
                                            ptr(rs) if rs is not None else None))

    def gemm_h2_gather(self, P, rs, rows, W, C, relu_dropout=False, p=0.0, seed=0, offset=0):
        """C = act(X[rows] @ W), X given as its pair table (rows None: all rows)."""
        K, N = W.shape
        M = rows.numel() if rows is not None else P.shape[0]
        check(self.lib.nts_hip_gemm_h2_gather(self.h, int(relu_dropout), M, N, P.shape[1], ptr(P),
                                              P.stride(0), ptr(rs), ptr(rows), ptr(W), W.stride(0),
                                              K, ptr(C), C.stride(0), float(p), int(seed),
                                              int(offset)))

    def gemm_h2_tn_gather(self, P, rs, rows, B, C, M, X=None, bscale=1.0):
        """C = X[rows, :M].T @ op(B), op(B) = B or B * (X_mask > 0) * bscale."""
        N = B.shape[1]
        Kr = rows.numel() if rows is not None else B.shape[0]
        check(self.lib.nts_hip_gemm_h2_tn_gather(self.h, M, N, Kr, ptr(P), P.stride(0), ptr(rs),
                                                 ptr(rows), ptr(B), B.stride(0), ptr(X),
                                                 X.stride(0) if X is not None else 0, float(bscale),
                                                 ptr(C), C.stride(0)))

    def gemm_relu_dropout(self, A, B, C, p=0.0, seed=0, offset=0):
        """C = dropout(relu(A @ B), p) with the Philox mask of (seed, offset)."""
        M, K = A.shape
        N = B.shape[1]
        check(self.lib.nts_hip_gemm_relu_dropout_f32(self.h, M, N, K, ptr(A), A.stride(0), ptr(B),
                                                     B.stride(0), ptr(C), C.stride(0), float(p),
                                                     int(seed), int(offset)))

    def gemm_tn_masked(self, A, G, X, C, scale=1.0):
        """C = A.T @ (G * (X > 0) * scale)."""
        K, M = A.shape
        N = G.shape[1]
        check(self.lib.nts_hip_gemm_tn_masked_f32(self.h, M, N, K, ptr(A), A.stride(0), ptr(G),
                                                  G.stride(0), ptr(X), X.stride(0), float(scale),
                                                  ptr(C), C.stride(0)))

    def linear_xent_fwd(self, Y, W, labels, loss, correct=None):
        """loss = nll_loss(log_softmax(log_softmax(Y @ W)), labels) (mean), fused;
        correct (int32 device scalar) += rows whose argmax is the label."""
        n, K = Y.shape
        check(self.lib.nts_hip_linear_xent_fwd(self.h, ptr(Y), Y.stride(0), n, K, ptr(W), W.shape[1],
                                               ptr(labels), ptr(loss), ptr(correct)))

    def linear_xent_bwd(self, Y, W, labels, grad_loss, dY, dW):
        n, K = Y.shape
        check(self.lib.nts_hip_linear_xent_bwd(self.h, ptr(Y), Y.stride(0), n, K, ptr(W), W.shape[1],
                                               ptr(labels), ptr(grad_loss), ptr(dY), ptr(dW)))

    def linear_xent_train(self, Y, W, labels, loss, dY, dW, correct=None):
        """The loss and its gradients for d loss = 1 in one pass (== fwd + bwd(1))."""
        n, K = Y.shape
        check(self.lib.nts_hip_linear_xent_train(self.h, ptr(Y), Y.stride(0), n, K, ptr(W),
                                                 W.shape[1], ptr(labels), ptr(loss), ptr(dY),
                                                 ptr(dW), ptr(correct)))

    def adam(self, w, g, m, v, alpha, beta1, beta2, eps, wd, beta1_t, beta2_t, bias_correction):
        check(self.lib.nts_hip_adam(self.h, ptr(w), ptr(g), ptr(m), ptr(v), w.numel(), alpha,
                                    beta1, beta2, eps, wd, beta1_t, beta2_t, int(bias_correction)))


class HostTable:
    """fp32 [rows, cols] table in pinned host memory mapped into the device
    address space (nts_hip_host_alloc), row pitch `ld` floats.  `.tensor` is a
    CPU view for filling it; `.dev_ptr` is what kernels read (zero-copy)."""

    def __init__(self, rows: int, cols: int, ld: int | None = None):
        lib = _abi.lib()
        self.shape = (rows, cols)
        self.ld = ld or cols
        nbytes = max(rows * self.ld * 4, 4)
        hp = C.c_void_p()
        check(lib.nts_hip_host_alloc(nbytes, C.byref(hp)))
        self._host = hp.value
        dp = C.c_void_p()
        check(lib.nts_hip_host_device_pointer(hp, C.byref(dp)))
        self.dev_ptr = dp.value
        buf = (C.c_float * (nbytes // 4)).from_address(self._host)
        self.tensor = torch.frombuffer(buf, dtype=torch.float32).view(-1, self.ld)[:rows, :cols]

    def close(self):
        if getattr(self, "_host", None):
            self.tensor = None
            _abi.lib().nts_hip_host_free(C.c_void_p(self._host))
            self._host = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class DeviceGraph:
    """FullyRepGraph + degrees resident in HBM."""
    n_vertices: int
    n_edges: int
    column_offset: torch.Tensor  # int64 [V+1]
    row_indices: torch.Tensor    # int32 [E]
    in_degree: torch.Tensor      # int32 [V]
    out_degree: torch.Tensor     # int32 [V]

    def as_struct(self) -> _abi.GraphDev:
        return _abi.GraphDev(self.n_vertices, self.n_edges, ptr(self.column_offset),
                             ptr(self.row_indices), ptr(self.in_degree), ptr(self.out_degree))


@dataclass
class LayerBuffers:
    """Device arrays of one sampCSC (capacity-sized)."""
    v_cap: int
    e_cap: int
    s_cap: int
    destination: torch.Tensor
    v_size: torch.Tensor
    device: torch.device
    csr: bool = True
    weights: bool = True
    merge: bool = False  # dsts merged into the frontier (GAT): dst_local_id + csr_edge_id
    omit_map: torch.Tensor | None = None  # PD cache: dsts with omit_map[d] == omit_key sample nothing
    omit_key: int = 0
    omit_loc: torch.Tensor | None = None  # ... their cache rows, recorded per dst in t["omit_row"]
    t: dict = field(default_factory=dict)

    def __post_init__(self):
        d = self.device
        self.t["column_offset"] = _u32(self.v_cap + 1, d)
        self.t["row_indices"] = _u32(max(self.e_cap, 1), d)
        self.t["sample_ans"] = _u32(max(self.e_cap, 1), d)
        self.t["edge_dst"] = _u32(max(self.e_cap, 1), d)
        self.t["source"] = _u32(max(self.s_cap, 1), d)
        self.t["sizes"] = torch.zeros(4, dtype=torch.int32, device=d)
        self.t["edge_weight_forward"] = (torch.empty(max(self.e_cap, 1), dtype=torch.float32, device=d)
                                         if self.weights else None)
        if self.csr:
            self.t["row_offset"] = _u32(self.s_cap + 1, d)
            self.t["column_indices"] = _u32(max(self.e_cap, 1), d)
            self.t["edge_weight_backward"] = (torch.empty(max(self.e_cap, 1), dtype=torch.float32, device=d)
                                              if self.weights else None)
        else:
            self.t["row_offset"] = self.t["column_indices"] = self.t["edge_weight_backward"] = None
        self.t["dst_local_id"] = _u32(max(self.v_cap, 1), d) if self.merge else None
        self.t["csr_edge_id"] = _u32(max(self.e_cap, 1), d) if (self.merge and self.csr) else None
        self.t["omit_row"] = _u32(max(self.v_cap, 1), d) if self.omit_map is not None else None

    def __getattr__(self, k):
        t = self.__dict__.get("t")
        if t is not None and k in t:
            return t[k]
        raise AttributeError(k)

    def as_struct(self) -> _abi.SampCSCDev:
        t = self.t
        return _abi.SampCSCDev(
            self.v_cap, self.e_cap, self.s_cap, ptr(self.destination), ptr(self.v_size),
            ptr(t["column_offset"]), ptr(t["row_indices"]), ptr(t["sample_ans"]), ptr(t["edge_dst"]),
            ptr(t["source"]), ptr(t["edge_weight_forward"]), ptr(t["row_offset"]),
            ptr(t["column_indices"]), ptr(t["edge_weight_backward"]), ptr(t["sizes"]),
            ptr(t["dst_local_id"]), ptr(t["csr_edge_id"]), ptr(self.omit_map), self.omit_key,
            ptr(self.omit_loc), ptr(t.get("omit_row")))

    def sizes_host(self):
        s = self.t["sizes"].cpu().tolist()
        return s[0], s[1], s[2], s[3]


def layer_caps(batch: int, fanouts, n_vertices: int, n_edges: int, merge: bool = False):
    """Upper bounds (v_cap, e_cap, s_cap) per layer: v_0 = B, e_l <= v_l * f_l
    (or the edge count for fanout -1), s_l <= min(e_l (+ v_l when the dsts are
    merged into the frontier), V), v_{l+1} = s_l."""
    caps = []
    v = batch
    for f in fanouts:
        e = n_edges if f < 0 else min(v * f, n_edges)
        s = min(e + (v if merge else 0), n_vertices)
        caps.append((v, e, s))
        v = s
    return caps
