"""Transformer ops (LayerNorm(+residual), masked softmax, embedding) on ``csrc/transformer.hip``.

GPU path: the HIP kernels (bf16 activations, fp32 statistics; parameter
gradients accumulate straight into the variables' fp32 grad slots when
available).  CPU path: PyTorch reference implementations.
"""
import math
import os

import torch
import torch.nn.functional as F

from . import _native as N
from ..train import variables as V

N.register("mdtf_ln_fwd", [N.P, N.P, N.P, N.P, N.P, N.P, N.P, N.P, N.L, N.I, N.F, N.F, N.U, N.P, N.P])
N.register("mdtf_ln_bwd", [N.P, N.P, N.P, N.P, N.P, N.P, N.P, N.P, N.P, N.P, N.L, N.I, N.F, N.U, N.P, N.P])
N.register("mdtf_ln_bwd_ws", [N.L, N.I], restype=N.L)
N.register("mdtf_set_ln_reduce_stream", [N.P])
N.register("mdtf_softmax_fwd", [N.P, N.P, N.P, N.L, N.I, N.F, N.L, N.P])
N.register("mdtf_softmax_bwd", [N.P, N.P, N.P, N.L, N.I, N.F, N.P])
N.register("mdtf_embed_fwd", [N.P, N.P, N.P, N.L, N.I, N.L, N.P])
N.register("mdtf_embed_bwd", [N.P, N.P, N.P, N.L, N.I, N.L, N.P])
N.register("mdtf_embed_bwd_ws_floats", [N.L, N.I, N.L], N.L)
N.register("mdtf_embed_bwd_ws", [N.P, N.P, N.P, N.L, N.I, N.L, N.P, N.P])
# MDTF_EMBED_SMALL_2PASS=0: small tables (token types) by the one-pass atomic kernel instead of partial rows + one
# reduction
EMBED_SMALL_2PASS = os.environ.get("MDTF_EMBED_SMALL_2PASS", "1") != "0"
N.register("mdtf_attn_fwd", [N.P, N.P, N.P, N.P, N.I, N.I, N.I, N.I, N.F, N.F, N.U, N.P, N.P])
N.register("mdtf_attn_bwd", [N.P, N.P, N.P, N.P, N.P, N.P, N.I, N.I, N.I, N.I, N.F, N.F, N.U, N.P, N.P])
N.register("mdtf_set_attn_bwd", [N.I], N.I)     # S = 128 backward kernel: 1 = v1 ([q][k] images), 2 = v2, 3 = v2s
N.register("mdtf_set_attn_pp", [N.I], N.I)      # S = 128 persistent kernels: 0 off, 1 on, n >= 2 on, grid <= n


def effective_seed(seed, device):
    """The seed the dropout kernels hash with: ``seed ^ (step_counter * 0x85EBCA6B)`` (32-bit)."""
    from ..train.graph import rng_offset_tensor
    off = int(rng_offset_tensor(device).item())
    return (int(seed) ^ ((off * 0x85EBCA6B) & 0xFFFFFFFF)) & 0xFFFFFFFF


def _seed_off(p_drop, device):
    """Device step counter mixed into the dropout hash (advanced by hipGraph replays,
    see mdtf.train.graph); None without dropout."""
    if not p_drop:
        return None
    from ..train.graph import rng_offset_tensor
    return rng_offset_tensor(device)


def _sink_or_zeros(t, n, device):
    var = V.grad_sink(t) if t is not None else None
    if var is not None:
        return var, var.grad
    return None, torch.zeros(n, dtype=torch.float32, device=device)


class _LayerNorm(torch.autograd.Function):
    """y = LN(dropout_p(x) + residual) with the dropout mask regenerated from a counter hash."""

    @staticmethod
    def forward(ctx, x, res, gamma, beta, eps, p_drop, seed):
        from . import actsink
        ctx.set_materialize_grads(False)
        # the residual is usually the previous LayerNorm's output, which also feeds a dense layer:
        # hand d(residual) to its sink (the dense dgrad then accumulates in its GEMM).  Only with
        # dropout: without it dx and d(residual) are one tensor that autograd still passes on.
        ctx.res_sink = actsink.sink_of(res) if (res is not None and p_drop > 0) else None
        if ctx.res_sink is not None:
            ctx.res_sink.register()
        x = x.contiguous()
        H = x.shape[-1]
        rows = x.numel() // H
        y = torch.empty_like(x)
        s = torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        g = gamma.detach().float().contiguous()
        b = beta.detach().float().contiguous()
        r = res.contiguous() if res is not None else None
        N.check(N.fn("mdtf_ln_fwd")(N.ptr(x), N.ptr(r), N.ptr(g), N.ptr(b), N.ptr(y), N.ptr(s), N.ptr(mean),
                                    N.ptr(rstd), rows, H, float(eps), float(p_drop), seed,
                                    N.ptr(_seed_off(p_drop, x.device)), N.stream_ptr()), "ln_fwd")
        ctx.save_for_backward(s, g, mean, rstd)
        ctx.has_res = res is not None
        ctx.drop = (float(p_drop), seed)
        ctx.sinks = (V.grad_sink(gamma), V.grad_sink(beta))
        ctx.like = (gamma, beta)
        ctx.out_sink = actsink.attach(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        s, g, mean, rstd = ctx.saved_tensors
        if ctx.out_sink is not None:
            dy = ctx.out_sink.take(dy)
        if dy is None:
            return None, None, None, None, None, None, None
        dy = dy.contiguous()
        H = s.shape[-1]
        rows = s.numel() // H
        p_drop, seed = ctx.drop
        ds = torch.empty_like(s)
        dxb = torch.empty_like(s) if p_drop > 0 else None     # gradient of the dropped-out branch input
        sg, sb = ctx.sinks
        dg = sg.grad if sg is not None else torch.zeros(H, dtype=torch.float32, device=s.device)
        db = sb.grad if sb is not None else torch.zeros(H, dtype=torch.float32, device=s.device)
        ws = torch.empty(N.fn("mdtf_ln_bwd_ws")(rows, H), dtype=torch.float32, device=s.device)
        from . import conv as _conv
        # gamma / beta in grad slots (read after the join at the end of backward): the partial reduction may leave
        # the chain on the side stream (MDTF_SLAB_SIDE)
        with _conv.slab_side(ws if (sg is not None and sb is not None) else None, "mdtf_set_ln_reduce_stream"):
            N.check(N.fn("mdtf_ln_bwd")(N.ptr(dy), N.ptr(s), N.ptr(g), N.ptr(mean), N.ptr(rstd), N.ptr(ds),
                                        N.ptr(dxb), N.ptr(dg), N.ptr(db), N.ptr(ws), rows, H, p_drop, seed,
                                        N.ptr(_seed_off(p_drop, s.device)), N.stream_ptr()),
                    "ln_bwd")
        gamma, beta = ctx.like
        rg = V.grad_marker(gamma) if sg is not None else dg
        rb = V.grad_marker(beta) if sb is not None else db
        dx = dxb if dxb is not None else ds
        dres = ds if ctx.has_res else None
        if ctx.res_sink is not None:
            ctx.res_sink.adopt_or_add(ds.view(s.shape))
            dres = None
        return dx, dres, rg, rb, None, None, None


def layer_norm(x, gamma, beta, eps=1e-12, residual=None, dropout=0.0):
    """LayerNorm over the last axis of ``dropout(x) (+ residual)`` (dropout fused on the GPU)."""
    if N.use_native(x):
        if x.dtype != torch.bfloat16:
            raise TypeError("mdtf LayerNorm kernel expects bf16, got %s" % x.dtype)
        if residual is not None and residual.dtype != x.dtype:
            residual = residual.to(x.dtype)
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if dropout else 0
        return _LayerNorm.apply(x, residual, gamma, beta, float(eps), float(dropout), seed)
    if dropout:
        x = F.dropout(x, dropout, True)
    s = x if residual is None else x + residual
    return F.layer_norm(s.float(), (s.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


class _Softmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, scale, rows_per_batch):
        x = x.contiguous()
        cols = x.shape[-1]
        rows = x.numel() // cols
        y = torch.empty_like(x)
        m = mask.float().contiguous() if mask is not None else None
        N.check(N.fn("mdtf_softmax_fwd")(N.ptr(x), N.ptr(m), N.ptr(y), rows, cols, float(scale), int(rows_per_batch),
                                         N.stream_ptr()), "softmax_fwd")
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        cols = y.shape[-1]
        dx = torch.empty_like(y)
        N.check(N.fn("mdtf_softmax_bwd")(N.ptr(dy), N.ptr(y), N.ptr(dx), y.numel() // cols, cols, float(ctx.scale),
                                         N.stream_ptr()), "softmax_bwd")
        return dx, None, None, None


def masked_softmax(scores, mask=None, scale=1.0):
    """softmax(scale * scores + mask) over the last axis.

    ``scores``: [B, heads, Sq, Sk]; ``mask``: additive [B, Sk] (0 / -10000) or None.
    """
    if N.use_native(scores):
        b = scores.shape[0]
        rows_per_batch = scores.numel() // scores.shape[-1] // b
        return _Softmax.apply(scores, mask, float(scale), rows_per_batch)
    s = scores.float() * scale
    if mask is not None:
        s = s + mask.float()[:, None, None, :]
    return torch.softmax(s, -1).to(scores.dtype)


class _Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, ids):
        ids = ids.to(torch.int64).contiguous()
        vocab, H = table.shape
        out = torch.empty(tuple(ids.shape) + (H,), dtype=table.dtype, device=table.device)
        N.check(N.fn("mdtf_embed_fwd")(N.ptr(table), N.ptr(ids), N.ptr(out), ids.numel(), H, vocab, N.stream_ptr()),
                "embed_fwd")
        ctx.save_for_backward(ids)
        ctx.shape = (vocab, H)
        ctx.sink = V.grad_sink(table)
        ctx.like = table
        return out

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        vocab, H = ctx.shape
        dy = dy.contiguous()
        sink = ctx.sink
        dt = sink.grad if sink is not None else torch.zeros((vocab, H), dtype=torch.float32, device=dy.device)
        if N.deterministic():
            # sorted (deterministic) scatter-add instead of the atomic kernel
            prev = torch.are_deterministic_algorithms_enabled()
            torch.use_deterministic_algorithms(True)
            try:
                dt.index_add_(0, ids.reshape(-1), dy.reshape(-1, H).float())
            finally:
                torch.use_deterministic_algorithms(prev)
        else:
            nws = int(N.fn("mdtf_embed_bwd_ws_floats")(ids.numel(), H, vocab)) if EMBED_SMALL_2PASS else 0
            if nws > 0:
                ws = torch.empty(nws, dtype=torch.float32, device=dy.device)
                N.check(N.fn("mdtf_embed_bwd_ws")(N.ptr(dy), N.ptr(ids), N.ptr(dt), ids.numel(), H, vocab, N.ptr(ws),
                                                  N.stream_ptr()), "embed_bwd_ws")
            else:
                N.check(N.fn("mdtf_embed_bwd")(N.ptr(dy), N.ptr(ids), N.ptr(dt), ids.numel(), H, vocab,
                                               N.stream_ptr()), "embed_bwd")
        if sink is not None:
            return V.grad_marker(ctx.like), None
        return dt.to(ctx.like.dtype), None


def embedding_lookup(table, ids):
    """``tf.nn.embedding_lookup``: rows of ``table`` [V, H] for integer ``ids``."""
    if N.use_native(table):
        return _Embed.apply(table, ids)
    return F.embedding(ids.long(), table)


N.register("mdtf_bert_embed_fwd", [N.P] * 6 + [N.L, N.I, N.I, N.L, N.I, N.I, N.P])
N.register("mdtf_bert_embed_bwd", [N.P] * 6 + [N.I, N.I, N.I, N.L, N.I, N.P])


class _BertEmbed(torch.autograd.Function):
    """word[ids] + position[s] + token_type[types] in one kernel each way (``csrc/transformer.hip``)."""

    @staticmethod
    def forward(ctx, word, pos, typ, ids, types):
        B, S_ = ids.shape
        H = word.shape[1]
        ids = ids.to(torch.int64).contiguous()
        types = types.to(torch.int64).contiguous()
        out = torch.empty((B, S_, H), dtype=word.dtype, device=word.device)
        rc = N.fn("mdtf_bert_embed_fwd")(N.ptr(word), N.ptr(pos), N.ptr(typ), N.ptr(ids), N.ptr(types), N.ptr(out),
                                         B * S_, S_, H, word.shape[0], pos.shape[0], typ.shape[0], N.stream_ptr())
        N.check(rc, "bert_embed_fwd")
        ctx.save_for_backward(ids, types)
        ctx.like = (word, pos, typ)
        ctx.sinks = tuple(V.grad_sink(t) for t in (word, pos, typ))
        return out

    @staticmethod
    def backward(ctx, dy):
        ids, types = ctx.saved_tensors
        B, S_ = ids.shape
        word, pos, typ = ctx.like
        H = word.shape[1]
        dy = dy.contiguous()
        bufs = [sk.grad if sk is not None else torch.zeros(t.shape, dtype=torch.float32, device=dy.device)
                for sk, t in zip(ctx.sinks, ctx.like)]
        N.check(N.fn("mdtf_bert_embed_bwd")(N.ptr(dy), N.ptr(ids), N.ptr(types), N.ptr(bufs[0]), N.ptr(bufs[1]),
                                            N.ptr(bufs[2]), B, S_, H, word.shape[0], typ.shape[0], N.stream_ptr()),
                "bert_embed_bwd")
        out = [V.grad_marker(t) if sk is not None else b.to(t.dtype) for t, sk, b in zip(ctx.like, ctx.sinks, bufs)]
        return out[0], out[1], out[2], None, None


class _AddPositions(torch.autograd.Function):
    """``e + pos[0..S)`` broadcast over the batch for ``e`` [B, S, H].  The position table's gradient is the
    column sum of ``dy`` over the batch (``mdtf_colsum`` of dy viewed [B, S*H] into slot rows 0..S-1), not a
    scatter of B*S rows onto S rows with atomics; no position-id tensor and no gather either way."""

    @staticmethod
    def forward(ctx, e, pos):
        S_ = e.shape[1]
        ctx.S = S_
        ctx.like = pos
        ctx.sink = V.grad_sink(pos)
        return e + pos[:S_]

    @staticmethod
    def backward(ctx, dy):
        from . import kernels as K
        B, S_, H = dy.shape
        dy = dy.contiguous()
        sink = ctx.sink
        dt = sink.grad if sink is not None else torch.zeros(ctx.like.shape, dtype=torch.float32, device=dy.device)
        K.colsum_into(dy.view(B, S_ * H), dt[:S_].view(S_ * H))
        if sink is not None:
            return dy, V.grad_marker(ctx.like)
        return dy, dt.to(ctx.like.dtype)


# MDTF_BERT_EMBED=1: the one-kernel embedding (bert_embeddings)
BERT_EMBED_FUSED = os.environ.get("MDTF_BERT_EMBED", "0") == "1"
# MDTF_POS_BCAST=0: the position embedding as a gather of arange ids (atomic scatter backward), for A/B
POS_BCAST = os.environ.get("MDTF_POS_BCAST", "1") == "1"


def bert_embeddings(word, pos, typ, ids, types):
    """BERT input embedding ``word[ids] + pos[0..S) + typ[types]`` for ``ids``/``types`` [B, S]: one fused kernel
    each way on the GPU (not in deterministic mode: the backward scatters with atomics); else three lookups."""
    B, S_ = ids.shape
    if (BERT_EMBED_FUSED and N.use_native(word) and not N.deterministic() and word.dtype == torch.bfloat16 and pos.dtype == word.dtype
            and typ.dtype == word.dtype and word.shape[1] % 8 == 0 and S_ <= pos.shape[0] and typ.shape[0] <= 4):
        return _BertEmbed.apply(word, pos, typ, ids, types)
    e = embedding_lookup(word, ids)
    if (POS_BCAST and N.use_native(word) and pos.dtype == e.dtype and pos.dim() == 2 and S_ <= pos.shape[0]
            and (S_ * pos.shape[1]) % 8 == 0 and e.dtype == torch.bfloat16):
        return _AddPositions.apply(e, pos) + embedding_lookup(typ, types)
    pos_ids = torch.arange(S_, device=ids.device).unsqueeze(0).expand(B, S_)
    return e + embedding_lookup(pos, pos_ids) + embedding_lookup(typ, types)


def attention(q, k, v, mask=None, dropout=0.0):
    """Multi-head attention core: q, k, v [B, heads, S, d] -> [B, heads, S, d].

    Unfused path: two batched GEMMs (hipBLASLt on the GPU) around the scaled
    masked softmax kernel; attention-probability dropout as in TF BERT.
    """
    scale = 1.0 / math.sqrt(q.shape[-1])
    scores = torch.matmul(q, k.transpose(-1, -2))
    p = masked_softmax(scores, mask, scale)
    if dropout:
        p = F.dropout(p, dropout, True)
    return torch.matmul(p, v)


FUSED_SEQ, FUSED_DIM = 128, 64      # shapes csrc/attention.hip is built for
N.register("mdtf_attn_fwd_flash", [N.P, N.P, N.P, N.P, N.I, N.I, N.I, N.I, N.F, N.F, N.U, N.P, N.P])
N.register("mdtf_attn_bwd_flash", [N.P, N.P, N.P, N.P, N.P, N.P, N.P, N.I, N.I, N.I, N.I, N.F, N.F, N.U, N.P, N.P])
# MDTF_ATTN_FLASH=1: the tiled kernels (csrc/attention_flash.hip) at S = 128 too (A/B)
FLASH_ALWAYS = os.environ.get("MDTF_ATTN_FLASH", "0") == "1"


def flash_ok(seq, dh):
    """Shapes of the tiled kernels: any S % 64 == 0 (192, 384, 512, ...), head dim 64 or 128."""
    return seq % 64 == 0 and seq >= 64 and dh in (64, 128)


class _FusedAttention(torch.autograd.Function):
    """softmax(Q K^T / sqrt(d) + mask) V for all heads, straight from/to the fused QKV layout."""

    @staticmethod
    def forward(ctx, qkv, mask, B, S_, nh, p_drop, seed):
        qkv = qkv.contiguous()
        dh = qkv.shape[-1] // 3 // nh
        H = nh * dh
        out = torch.empty((B * S_, H), dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty((B * nh, S_), dtype=torch.float32, device=qkv.device)
        m = mask.float().contiguous() if mask is not None else None
        scale = 1.0 / math.sqrt(dh)
        ctx.flash = FLASH_ALWAYS or not (S_ == FUSED_SEQ and dh == FUSED_DIM)
        name = "mdtf_attn_fwd_flash" if ctx.flash else "mdtf_attn_fwd"
        N.check(N.fn(name)(N.ptr(qkv), N.ptr(m), N.ptr(out), N.ptr(lse), B, S_, nh, dh, scale,
                           float(p_drop), seed, N.ptr(_seed_off(p_drop, qkv.device)), N.stream_ptr()), name)
        ctx.save_for_backward(qkv, out, lse)
        ctx.mask = m
        ctx.args = (B, S_, nh, float(p_drop), seed, scale, dh)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        B, S_, nh, p_drop, seed, scale, dh = ctx.args
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        if ctx.flash:
            ws = torch.empty((B * nh * S_,), dtype=torch.float32, device=qkv.device)
            N.check(N.fn("mdtf_attn_bwd_flash")(N.ptr(qkv), N.ptr(ctx.mask), N.ptr(out), N.ptr(dout), N.ptr(lse),
                                                N.ptr(dqkv), N.ptr(ws), B, S_, nh, dh, scale, p_drop, seed,
                                                N.ptr(_seed_off(p_drop, qkv.device)), N.stream_ptr()),
                    "attn_bwd_flash")
            return dqkv, None, None, None, None, None, None
        N.check(N.fn("mdtf_attn_bwd")(N.ptr(qkv), N.ptr(ctx.mask), N.ptr(out), N.ptr(dout), N.ptr(lse), N.ptr(dqkv),
                                      B, S_, nh, FUSED_DIM, scale, p_drop, seed, N.ptr(_seed_off(p_drop, qkv.device)),
                                      N.stream_ptr()), "attn_bwd")
        return dqkv, None, None, None, None, None, None


def fused_attention(qkv, batch, seq, heads, mask=None, dropout=0.0):
    """Self-attention from the fused projection ``qkv`` [B*S, 3H] (q | k | v, heads
    contiguous inside each) to the context [B*S, H].

    GPU, S = 128, head dim 64: one fused HIP kernel per direction (``csrc/attention.hip``);
    any other S % 64 == 0 with head dim 64 / 128 (SQuAD seq 384, phase-2 seq 512, BERT-large heads):
    the tiled online-softmax kernels (``csrc/attention_flash.hip``); otherwise the unfused
    matmul/softmax path.
    ``mask``: additive [B, S] key mask (0 keep, -10000 drop) or None.
    """
    H3 = qkv.shape[-1]
    H = H3 // 3
    dh = H // heads
    if N.use_native(qkv) and qkv.dtype == torch.bfloat16 and ((seq == FUSED_SEQ and dh == FUSED_DIM)
                                                              or flash_ok(seq, dh)):
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if dropout else 0
        return _FusedAttention.apply(qkv.reshape(batch * seq, H3), mask, batch, seq, heads, float(dropout), seed)
    q, k, v = qkv.reshape(batch, seq, 3, heads, dh).unbind(2)
    ctx = attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), mask, dropout)
    return ctx.transpose(1, 2).reshape(batch * seq, H)
