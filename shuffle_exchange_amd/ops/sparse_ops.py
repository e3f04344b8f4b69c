"""Standalone block-sparse MatMul (sdd / dsd / dds) and block-sparse Softmax.

Parity: reference ops/sparse_attention/matmul.py:628 ``MatMul`` (modes ``sdd``: sparse = dense x
dense, ``dsd``: dense = sparse x dense, ``dds``: dense = dense x sparse; ``trans_a`` / ``trans_b``)
and softmax.py:224 ``Softmax`` (scale, rpe, key-padding and attention masks in add / mul mode).
Sparse tensors use the reference format: ``[B, nnz, block, block]``, the non-zero blocks of the
layout ``[H, M, N]`` in ``layout.nonzero()`` (head, block-row, block-column) order.

MI355X path: no Triton. bf16 / fp16 GPU inputs run the HIP block-sparse kernels
(csrc/kernels/bsmm.hip: MFMA 16x16x32 tiles that read the dense operands in place through their
strides -- transposes and broadcast heads included -- and, for ``dsd`` / ``dds``, sum a block row's /
column's products in registers over the layout's CSR / CSC lists); their backward runs the same
three kernels with the reference's mode / transpose algebra (matmul.py:628 ``_sparse_matmul``).
Other dtypes and devices take the batched-GEMM form: ``sdd`` gathers the block rows of A and block
columns of B per non-zero and multiplies [nnz] (block x K) x (K x block) pairs; ``dsd`` / ``dds``
multiply each non-zero block by its dense panel and sum the partial products per output block row /
column with one ``index_add``. Softmax works on the compact blocks only: on the GPU one HIP kernel
(csrc/kernels/bsoftmax.hip) walks each block row's CSR list per query row (forward and backward);
elsewhere per-row max and sum are segment reductions over the blocks of one (head, block-row) group
(``scatter_reduce`` / ``index_add``), so memory stays O(nnz block^2) -- the dense S x S score matrix
is never formed. Gradients flow through the same ops (autograd). Block-sparse attention itself does not use these: it runs fused in the
flash kernels (ops/sparse_attention.py ``block_sparse_attention``), which never write the scores.
"""
import torch


def _coords(layout):
    lay = layout if layout.dim() == 3 else layout.unsqueeze(0)
    nz = lay.nonzero(as_tuple=False)
    return lay, nz[:, 0], nz[:, 1], nz[:, 2]


def _pad4(x):
    while x.dim() < 4:
        x = x.unsqueeze(0)
    return x


class MatMul:
    """Block-sparse matrix multiplication; see the module docstring for the tensor formats."""

    def __init__(self, layout, block, mode, trans_a=False, trans_b=False, bench=False):
        if mode not in ("sdd", "dsd", "dds"):
            raise NotImplementedError("Supported modes are: sdd, dsd, dds")
        assert layout.dim() in (2, 3), "Layout should be a 2 or 3 dimensional tensor of 0s and 1s"
        self.layout, self.block, self.mode = layout, int(block), mode
        self.trans_a, self.trans_b = trans_a, trans_b
        self.lay, h, i, j = _coords(layout.long())
        self.spdims = tuple(self.lay.shape)
        self._idx = {}
        self._hij = (h, i, j)

    def _index(self, device):
        if device not in self._idx:
            self._idx[device] = tuple(t.to(device) for t in self._hij)
        return self._idx[device]

    # ---------------------------------------------------------------- HIP kernels (bsmm.hip)
    def _hip_ok(self, a, b):
        from . import native
        if not (a.is_cuda and b.is_cuda and a.dtype == b.dtype and a.dtype in (torch.bfloat16, torch.float16)
                and self.block in (16, 32, 64, 128) and native.use_hip(a)):
            return False
        dense = b if self.mode == "dsd" else a
        if self.mode == "sdd":  # the reduction dim is the backward's dense width
            A = _pad4(a)
            return (A.shape[-2] if self.trans_a else A.shape[-1]) % 16 == 0
        d = _pad4(dense)
        d = d.transpose(-1, -2) if (self.trans_b if self.mode == "dsd" else self.trans_a) else d
        return (d.shape[-1] if self.mode == "dsd" else d.shape[-2]) % 16 == 0

    def _lists(self, device, kind, trans):
        """CSR (kind 'row', dsd) / CSC (kind 'col', dds) lists of the output blocks: ptr [H*R + 1],
        ent [nnz, 2] = (non-zero index, reduction block) -- built once per device."""
        key = (device, kind, bool(trans))
        if key not in self._idx:
            h, i, j = self._index(device)
            H, M, N = self.spdims
            if (kind == "row") != bool(trans):
                out, red, R = i, j, M
            else:
                out, red, R = j, i, N
            g = h * R + out
            order = torch.argsort(g, stable=True)
            cnt = torch.bincount(g, minlength=H * R)
            ptr = torch.zeros(H * R + 1, dtype=torch.int32, device=device)
            ptr[1:] = cnt.cumsum(0).to(torch.int32)
            nzid = torch.arange(h.numel(), device=device)
            ent = torch.stack([nzid[order], red[order]], 1).to(torch.int32).contiguous()
            self._idx[key] = (ptr, ent, R)
        return self._idx[key]

    def _hij32(self, device):
        key = (device, "hij")
        if key not in self._idx:
            h, i, j = self._index(device)
            self._idx[key] = torch.stack([h, i, j], 1).to(torch.int32).contiguous()
        return self._idx[key]

    def _k_sdd(self, A, B):
        return torch.ops.sxe.bsmm_sdd(A, B, self._hij32(A.device), self.block)

    def _k_dsd(self, S, trans, D):
        ptr, ent, R = self._lists(S.device, "row", trans)
        return torch.ops.sxe.bsmm_dsd(_pad4(S).contiguous(), bool(trans), D, ptr, ent, self.spdims[0], R, self.block)

    def _k_dds(self, D, S, trans):
        ptr, ent, R = self._lists(S.device, "col", trans)
        return torch.ops.sxe.bsmm_dds(D, _pad4(S).contiguous(), bool(trans), ptr, ent, self.spdims[0], R, self.block)

    def __call__(self, a, b):
        if self._hip_ok(a, b):
            nd = max(a.dim(), b.dim()) if self.mode == "sdd" else (b if self.mode == "dsd" else a).dim()
            c = _BSMM.apply(self, a, b)
            while c.dim() > nd and c.shape[0] == 1:
                c = c.squeeze(0)
            return c
        nd = max(a.dim(), b.dim())
        if self.mode != "sdd":
            nd = (b if self.mode == "dsd" else a).dim()
        a, b = _pad4(a), _pad4(b)
        if a.dtype != b.dtype:
            raise ValueError(f"Inputs must be the same dtype; got {a.dtype} for A and {b.dtype} for B")
        h, i, j = self._index(a.device)
        H, M, N = self.spdims
        blk = self.block
        if self.mode == "sdd":
            A = a.transpose(-1, -2) if self.trans_a else a          # [B, H, M*blk, K]
            Bm = b.transpose(-1, -2) if self.trans_b else b         # [B, H, K, N*blk]
            Bsz, _, _, K = A.shape
            Ar = A.reshape(Bsz, A.shape[1], M, blk, K)[:, h if A.shape[1] > 1 else 0 * h, i]   # [B, nnz, blk, K]
            Bc = Bm.reshape(Bsz, Bm.shape[1], K, N, blk).transpose(2, 3)[:, h if Bm.shape[1] > 1 else 0 * h, j]
            # Bc: [B, nnz, K, blk]
            c = torch.matmul(Ar, Bc)
        elif self.mode == "dsd":
            # sparse A [B, nnz, blk, blk] (transposed: each block transposed, block coords swapped)
            As = a.transpose(-1, -2) if self.trans_a else a
            ri, ci = (j, i) if self.trans_a else (i, j)
            D = b.transpose(-1, -2) if self.trans_b else b          # [B, H, (cols of A)*blk, Nd]
            Bsz, Hd, _, Nd = D.shape
            rows = M if not self.trans_a else N
            cols = N if not self.trans_a else M
            Dp = D.reshape(Bsz, Hd, cols, blk, Nd)[:, h if Hd > 1 else 0 * h, ci]  # [B, nnz, blk, Nd]
            part = torch.matmul(As, Dp)                              # [B, nnz, blk, Nd]
            out = torch.zeros(Bsz, H * rows, blk, Nd, dtype=part.dtype, device=part.device)
            out = out.index_add(1, h * rows + ri, part)
            c = out.view(Bsz, H, rows * blk, Nd)
        else:  # dds
            D = a.transpose(-1, -2) if self.trans_a else a          # [B, H, Md, (rows of Bs)*blk]
            Bs = b.transpose(-1, -2) if self.trans_b else b
            ri, ci = (j, i) if self.trans_b else (i, j)
            Bsz, Hd, Md, _ = D.shape
            rows = M if not self.trans_b else N
            cols = N if not self.trans_b else M
            Dp = D.reshape(Bsz, Hd, Md, rows, blk).transpose(2, 3)[:, h if Hd > 1 else 0 * h, ri]  # [B, nnz, Md, blk]
            part = torch.matmul(Dp, Bs)                              # [B, nnz, Md, blk]
            out = torch.zeros(Bsz, H * cols, Md, blk, dtype=part.dtype, device=part.device)
            out = out.index_add(1, h * cols + ci, part)
            c = out.view(Bsz, H, cols, Md, blk).permute(0, 1, 3, 2, 4).reshape(Bsz, H, Md, cols * blk)
        while c.dim() > nd and c.shape[0] == 1:
            c = c.squeeze(0)
        return c


def _t(x):
    return x.transpose(-1, -2)


def _fit(g, like):
    """Sum a gradient over the dims its (padded 4-D) input broadcast, then give it the input's shape."""
    ref = _pad4(like)
    for d in range(g.dim()):
        if ref.shape[d] == 1 and g.shape[d] != 1:
            g = g.sum(d, keepdim=True)
    return g.reshape(like.shape).to(like.dtype)


class _BSMM(torch.autograd.Function):
    """The HIP block-sparse products with their backward (reference matmul.py ``_sparse_matmul``
    backward: the gradient of each mode is two products of the other modes)."""

    @staticmethod
    def forward(ctx, mm, a, b):
        ctx.mm = mm
        ctx.save_for_backward(a, b)
        A, B = _pad4(a), _pad4(b)
        if mm.mode == "sdd":
            return mm._k_sdd(_t(A) if mm.trans_a else A, _t(B) if mm.trans_b else B)
        if mm.mode == "dsd":
            return mm._k_dsd(A, mm.trans_a, _t(B) if mm.trans_b else B)
        return mm._k_dds(_t(A) if mm.trans_a else A, B, mm.trans_b)

    @staticmethod
    def backward(ctx, g):
        mm = ctx.mm
        a, b = ctx.saved_tensors
        A, B = _pad4(a), _pad4(b)
        g = _pad4(g).contiguous()
        da = db = None
        if mm.mode == "sdd":  # C = A' B' (sparse)
            Ap, Bp = (_t(A) if mm.trans_a else A), (_t(B) if mm.trans_b else B)
            if ctx.needs_input_grad[1]:
                dA = mm._k_dsd(g, False, _t(Bp))
                da = _fit(_t(dA) if mm.trans_a else dA, a)
            if ctx.needs_input_grad[2]:
                dB = mm._k_dds(_t(Ap), g, False)
                db = _fit(_t(dB) if mm.trans_b else dB, b)
        elif mm.mode == "dsd":  # C = S' D'
            Dp = _t(B) if mm.trans_b else B
            if ctx.needs_input_grad[1]:
                dS = mm._k_sdd(Dp, _t(g)) if mm.trans_a else mm._k_sdd(g, _t(Dp))
                da = _fit(dS, a)
            if ctx.needs_input_grad[2]:
                dD = mm._k_dsd(A, not mm.trans_a, g)
                db = _fit(_t(dD) if mm.trans_b else dD, b)
        else:  # dds: C = D' S'
            Dp = _t(A) if mm.trans_a else A
            if ctx.needs_input_grad[1]:
                dD = mm._k_dds(g, B, not mm.trans_b)
                da = _fit(_t(dD) if mm.trans_a else dD, a)
            if ctx.needs_input_grad[2]:
                dS = mm._k_sdd(_t(g), Dp) if mm.trans_b else mm._k_sdd(_t(Dp), g)
                db = _fit(dS, b)
        return None, da, db


class Softmax:
    """Row softmax of a block-sparse score tensor [B, nnz, block, block] (rows = queries), with the
    reference's optional scale, relative position embedding, key-padding mask [B, S] and attention
    mask [S, S] (each in 'add' or 'mul' mode). Returns a new tensor of the same format."""

    def __init__(self, layout, block, bench=False):
        self.layout, self.block = layout, int(block)
        self.lay, h, i, j = _coords(layout.long())
        self.spdims = tuple(self.lay.shape)
        self.num_blocks = int(h.numel())
        self._hij = (h, i, j)
        self._idx = {}

    def _index(self, device):
        if device not in self._idx:
            self._idx[device] = tuple(t.to(device) for t in self._hij)
        return self._idx[device]

    def _blocks_of(self, t, h, i, j, batched):
        """Dense [.., S, S] (per head when 3-D / 4-D) -> its non-zero blocks [.., nnz, blk, blk]."""
        blk = self.block
        H, M, N = self.spdims
        if t.dim() == 2:
            return t.reshape(M, blk, N, blk).permute(0, 2, 1, 3)[i, j]
        x = t.reshape(*t.shape[:-2], M, blk, N, blk).transpose(-3, -2)  # [.., M, N, blk, blk]
        if batched:  # [B, H, ...]
            return x[:, h if x.shape[1] > 1 else 0 * h, i, j]
        return x[h if x.shape[0] > 1 else 0 * h, i, j]

    def _csr(self, device):
        """Block-row pointer [H M + 1] and block column [nnz] (int32) of the layout on ``device``."""
        key = ("csr", device)
        if key not in self._idx:
            h, i, j = self._hij
            H, M, _ = self.spdims
            cnt = torch.bincount(h * M + i, minlength=H * M)
            ptr = torch.zeros(H * M + 1, dtype=torch.int64)
            ptr[1:] = torch.cumsum(cnt, 0)
            self._idx[key] = (ptr.int().to(device), j.int().to(device))
        return self._idx[key]

    def _hip_ok(self, x):
        from . import native
        return (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and self.block % 8 == 0
                and x.dim() == 4 and x.shape[1] == self.num_blocks and native.use_hip(x))

    def __call__(self, x, scale=1.0, rpe=None, key_padding_mask=None, attn_mask=None, key_padding_mask_mode="add",
                 attn_mask_mode="add"):
        for name, t in (("relative position embedding", rpe), ("Attention mask", attn_mask),
                        ("Key padding mask", key_padding_mask)):
            if t is not None and t.dtype != x.dtype:
                raise ValueError(f"{name} must be {x.dtype}")
        if self._hip_ok(x):  # csrc/kernels/bsoftmax.hip (gradient w.r.t. x only, as the reference)
            f32 = lambda t: None if t is None else t.detach().float().contiguous()  # noqa: E731
            r = f32(rpe)
            if r is not None and r.dim() == 2:
                r = r.unsqueeze(0)
            kp = f32(key_padding_mask)
            return _BSoftmax.apply(x.contiguous(), self, float(scale), r, f32(attn_mask), attn_mask_mode == "mul",
                                   None if kp is None else kp.reshape(x.shape[0], -1), key_padding_mask_mode == "mul")
        h, i, j = self._index(x.device)
        H, M, N = self.spdims
        blk = self.block
        ct = torch.promote_types(x.dtype, torch.float32)  # compute in fp32 (fp64 stays fp64)
        s = x.to(ct) * scale
        if rpe is not None:
            s = s + self._blocks_of(rpe.to(ct), h, i, j, batched=rpe.dim() == 4)
        if attn_mask is not None:
            am = self._blocks_of(attn_mask.to(ct), h, i, j, batched=False)
            s = s * am if attn_mask_mode == "mul" else s + am
        if key_padding_mask is not None:
            kp = key_padding_mask.to(ct).reshape(x.shape[0], N, blk)[:, j].unsqueeze(2)  # [B, nnz, 1, blk]
            s = s * kp if key_padding_mask_mode == "mul" else s + kp
        g = h * M + i                                                # block-row group of each non-zero
        Bsz = s.shape[0]
        rmax = s.amax(-1)                                            # [B, nnz, blk]
        gmax = torch.full((Bsz, H * M, blk), float("-inf"), dtype=ct, device=s.device).scatter_reduce(
            1, g.view(1, -1, 1).expand_as(rmax), rmax, "amax", include_self=True)
        mx = gmax[:, g].unsqueeze(-1)
        mx = torch.where(torch.isinf(mx), torch.zeros_like(mx), mx)
        e = torch.exp(s - mx)
        rsum = torch.zeros(Bsz, H * M, blk, dtype=ct, device=s.device).index_add(1, g, e.sum(-1))
        den = rsum[:, g].unsqueeze(-1)
        y = torch.where(den > 0, e / den.clamp_min(1e-30), torch.zeros_like(e))
        return y.to(x.dtype)


def dense_to_block_sparse(x, layout, block):
    """Helper (tests, conversions): dense [B, H, S, S] -> [B, nnz, block, block] in layout order."""
    lay, h, i, j = _coords(layout.long())
    H, M, N = lay.shape
    xb = x.reshape(x.shape[0], x.shape[1], M, block, N, block).transpose(3, 4)
    return xb[:, h if x.shape[1] > 1 else 0 * h, i, j]


def block_sparse_to_dense(xs, layout, block, fill=0.0):
    """Inverse of ``dense_to_block_sparse`` (missing blocks filled with ``fill``)."""
    lay, h, i, j = _coords(layout.long())
    H, M, N = lay.shape
    out = torch.full((xs.shape[0], H, M, N, block, block), fill, dtype=xs.dtype, device=xs.device)
    out[:, h, i, j] = xs
    return out.transpose(3, 4).reshape(xs.shape[0], H, M * block, N * block)


class _BSoftmax(torch.autograd.Function):
    """HIP block-sparse softmax (bsoftmax.hip); backward dx = y (dy - rowsum(dy y)) * ds/dx."""

    @staticmethod
    def forward(ctx, x, sm, scale, rpe, am, am_mul, kpm, kpm_mul):
        ptr, col = sm._csr(x.device)
        H, M, N = sm.spdims
        y = torch.ops.sxe.bsparse_softmax_fwd(x, ptr, col, H, M, N, scale, rpe, am, am_mul, kpm, kpm_mul)
        ctx.save_for_backward(y)
        ctx.meta = (sm, scale, am, am_mul, kpm, kpm_mul)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        sm, scale, am, am_mul, kpm, kpm_mul = ctx.meta
        ptr, col = sm._csr(y.device)
        H, M, N = sm.spdims
        dx = torch.ops.sxe.bsparse_softmax_bwd(y, dy.contiguous(), ptr, col, H, M, N, scale, am, am_mul, kpm, kpm_mul)
        return dx, None, None, None, None, None, None, None
