"""Fused BatchNorm(+residual)(+ReLU) autograd op on the HIP kernels of ``csrc/bn.hip``."""
import os

import torch

from . import _native as N
from ..train import variables as V

N.register("mdtf_bn_workspace_floats", [N.L, N.I], N.L)
N.register("mdtf_bn_fwd_train", [N.P, N.P, N.P, N.P, N.L, N.I, N.P, N.P, N.P, N.P, N.F, N.F, N.I, N.P, N.P, N.P, N.P])
N.register("mdtf_bn_fwd_eval", [N.P, N.P, N.P, N.L, N.I, N.P, N.P, N.P, N.P, N.F, N.I, N.P, N.P])
N.register("mdtf_bn_bwd", [N.P, N.P, N.P, N.P, N.P, N.L, N.I, N.P, N.P, N.P, N.P, N.P, N.I, N.P, N.I, N.P])
N.register("mdtf_bn_bwd_stats", [N.P, N.P, N.P, N.P, N.P, N.L, N.I, N.P, N.P, N.P, N.P, N.P, N.I, N.P, N.P, N.I,
                                 N.P, N.I, N.P])
N.register("mdtf_bn_fwd_dual", [N.P, N.P, N.P, N.P, N.L, N.I] + [N.P] * 6 + [N.I, N.P, N.P] + [N.P] * 6 + [N.I, N.P, N.P]
           + [N.F, N.F, N.P, N.P])
N.register("mdtf_bn_fwd_stats", [N.P, N.P, N.P, N.P, N.L, N.I, N.P, N.P, N.P, N.P, N.F, N.F, N.I, N.P, N.P, N.P, N.P,
                                 N.I, N.P, N.P])
N.register("mdtf_bn_relu_maxpool_fwd", [N.P, N.P, N.P] + [N.I] * 12 + [N.P] * 4 + [N.F, N.F] + [N.P] * 4 + [N.I]
           + [N.P, N.P])
N.register("mdtf_maxpool_bn_bwd", [N.P] * 4 + [N.I] * 12 + [N.P] * 8 + [N.P])
N.register("mdtf_bn_bwd_dual", [N.P] * 6 + [N.L, N.I] + [N.P] * 7 + [N.I] + [N.P] * 6 + [N.P])
N.register("mdtf_bn_bwd_finalize_ws", [N.L, N.I, N.P, N.P, N.P, N.P, N.P, N.I, N.P, N.P])
N.register("mdtf_bn_dx_ws", [N.P, N.P, N.P, N.P, N.P, N.L, N.I, N.P, N.P, N.P, N.I, N.I, N.P])
N.register("mdtf_bn_fwd_coeffs", [N.L, N.I, N.P, N.P, N.P, N.P, N.F, N.F, N.P, N.P, N.P, N.P, N.I, N.P, N.P])
N.register("mdtf_bn_apply_ss", [N.P, N.P, N.P, N.L, N.I, N.P, N.I, N.P])


FUSED_BWD = [0]      # backward passes that took their statistics from the dgrad epilogue (tests)
# MDTF_BN_EARLY_FIN=1: the backward finalize runs on a side stream right after the data gradient that completes its
# statistics instead of in the BN's backward (after the conv's weight gradient).  Measured -3 % in the captured
# ResNet-50 step (the 45 fork / join pairs cost more than the finalize latency they hide, profiles/ab_r5.md): off.
EARLY_FIN = os.environ.get("MDTF_BN_EARLY_FIN", "0") == "1"
# MDTF_BN_WG_FIN=1 (default): the backward finalize runs as extra workgroups of the conv's weight-gradient launch that
# follows the data gradient completing the statistics (csrc/conv_igemm.hip fin_bwd_block) -- same stream, no launch
# and no fork of its own; the BN backward then runs only its input-gradient pass (mdtf_bn_dx_ws).
WG_FIN = os.environ.get("MDTF_BN_WG_FIN", "1") == "1"
WG_FIN_USED = [0]    # backward passes whose finalize rode on a weight-gradient launch (tests)
EARLY_USED = [0]     # backward passes that used an early finalize (tests)
_FIN_SIDE = {}


def _early_finalize(sbuf, g, mean, invstd, M, C):
    """Issue the backward finalize of statistics ``sbuf`` ([2, slots, C], complete) on a side stream forked from
    the current one: k1..k3 | dgamma | dbeta into a fresh workspace, the partial rows re-zeroed.  The conv's
    weight gradient that follows on the main stream hides its latency; the BN backward waits for the returned
    event before its input-gradient pass (csrc/bn.hip mdtf_bn_bwd_finalize_ws / mdtf_bn_dx_ws)."""
    dev = sbuf.device
    main = torch.cuda.current_stream(dev)
    side = _FIN_SIDE.get(dev)
    if side is None:
        side = _FIN_SIDE[dev] = torch.cuda.Stream(device=dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        ws = torch.empty(5 * C, dtype=torch.float32, device=dev)
        N.check(N.fn("mdtf_bn_bwd_finalize_ws")(M, C, N.ptr(g), N.ptr(mean), N.ptr(invstd), N.ptr(sbuf[0]),
                                                N.ptr(sbuf[1]), int(sbuf.shape[1]), N.ptr(ws), N.stream_ptr()),
                "bn_bwd_finalize_ws")
        ev = torch.cuda.Event()
        ev.record(side)
    ws.record_stream(main)
    for t in (sbuf, g, mean, invstd):
        if t is not None:
            t.record_stream(side)
    return ws, ev
# projection-shortcut BNs applied inside the residual BN's pass (MDTF_DEFER_SHORTCUT_BN=0: separate apply)
DEFER_SHORTCUT = os.environ.get("MDTF_DEFER_SHORTCUT_BN", "1") != "0"
# MDTF_BN_ON_CONSUMER=1: a BN + ReLU whose only consumer is a 1x1 / stride-1 conv on the weight-stationary kernel
# with K <= 128 (ResNet's conv2 -> BN -> ReLU -> conv3 in stages 1 and 2) runs its finalize only; the conv applies
# scale / shift / ReLU to its operand as it loads it and writes the BN output and ReLU mask for the backward
# (csrc/conv_ws.hip mdtf_conv_ws_bna): the apply pass's read of x and the conv's re-read of its output are gone.
# Any other consumer gets the separate apply first (take_pending / apply_pending).
ON_CONSUMER = os.environ.get("MDTF_BN_ON_CONSUMER", "0") == "1"
_PENDING = {}        # data_ptr of an unwritten BN output -> (y, x, scale|shift [2C], mask)
ON_CONSUMER_USED = [0]   # BN outputs applied by their consumer conv (tests)


def take_pending(y):
    """The pending apply of BN output ``y`` (removed), or None."""
    if not _PENDING:
        return None
    ent = _PENDING.get(y.data_ptr())
    if ent is None or ent[0].shape != y.shape or ent[0].dtype != y.dtype:
        return None
    del _PENDING[y.data_ptr()]
    return ent


def apply_pending(ent):
    """Run a pending BN + ReLU apply as its own pass (the consumer could not fuse it)."""
    y, x, ss, mask = ent
    C = x.shape[-1]
    N.check(N.fn("mdtf_bn_apply_ss")(N.ptr(x), N.ptr(y), N.ptr(mask), x.numel() // C, C, N.ptr(ss), 1,
                                     N.stream_ptr()), "bn_apply_ss")


def materialize(y):
    """Make sure BN output ``y`` is written (a consumer that reads it as a plain tensor)."""
    ent = take_pending(y)
    if ent is not None:
        apply_pending(ent)
    return y


def _check(x):
    if x.dtype != torch.bfloat16:
        raise TypeError("mdtf BN kernel expects bf16 NHWC activations, got %s" % x.dtype)
    if x.shape[-1] % 8:
        raise ValueError("mdtf BN kernel needs C % 8 == 0 (C=%d)" % x.shape[-1])


def _f32(t):
    return None if t is None else t.detach().float().contiguous()


# MDTF_BN_TRACE=1: record (input shape, has residual, how the backward statistics were obtained) per BN backward
BWD_TRACE = [] if os.environ.get("MDTF_BN_TRACE") == "1" else None
DUAL_DZ = os.environ.get("MDTF_DUAL_DZ", "0") == "1"
# the dual BN's two input gradients in one pass (csrc/bn.hip mdtf_bn_bwd_dual); MDTF_DUAL_BWD_FUSED=0: two bn_dx
# passes.  ResNet-50 A/B with the fused stem: 11102 / 11121 vs 10949 / 10983 img/s (profiles/resnet_fusions_r3.md)
DUAL_FUSED = os.environ.get("MDTF_DUAL_BWD_FUSED", "1") != "0"
DUAL_BWD = [0]       # one-pass dual backward launches (tests)


class _BNTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, mm, mv, decay, eps, relu, stats, on_consumer=False):
        from . import actsink
        ctx.set_materialize_grads(False)
        ctx.res_sink = actsink.sink_of(residual)       # residual fan-out: write dres into the producer's sink
        if ctx.res_sink is not None:
            ctx.res_sink.register()
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        y = torch.empty_like(x)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        # ReLU: 1-bit-per-element mask for the backward (instead of keeping / re-reading y)
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=x.device) if relu else None
        g, b = _f32(gamma), _f32(beta)
        res = residual.contiguous() if residual is not None else None
        if stats is not None and on_consumer and relu and res is None:
            # finalize only: the consumer conv applies scale / shift / ReLU to its operand and writes y and mask
            psum, psq, P = stats
            ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_bn_fwd_coeffs")(M, C, N.ptr(g), N.ptr(b), N.ptr(mm), N.ptr(mv), float(decay),
                                               float(eps), N.ptr(mean), N.ptr(invstd), N.ptr(psum), N.ptr(psq),
                                               int(P), N.ptr(ws), N.stream_ptr()), "bn_fwd_coeffs")
            from . import conv as _conv
            _conv.stats_consumed(x.device)
            _PENDING[y.data_ptr()] = (y, x, ws, mask)
        elif stats is not None:
            # Σx / Σx² already produced by the conv epilogue: finalize + apply only
            psum, psq, P = stats
            ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_bn_fwd_stats")(N.ptr(x), N.ptr(res), N.ptr(y), N.ptr(mask), M, C, N.ptr(g), N.ptr(b),
                                              N.ptr(mm), N.ptr(mv), float(decay), float(eps), int(relu), N.ptr(mean),
                                              N.ptr(invstd), N.ptr(psum), N.ptr(psq), int(P), N.ptr(ws),
                                              N.stream_ptr()), "bn_fwd_stats")
            from . import conv as _conv
            _conv.stats_consumed(x.device)           # the finalize kernel re-zeroed the partials
        else:
            ws = torch.empty(int(N.fn("mdtf_bn_workspace_floats")(M, C)), dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_bn_fwd_train")(N.ptr(x), N.ptr(res), N.ptr(y), N.ptr(mask), M, C, N.ptr(g), N.ptr(b),
                                              N.ptr(mm), N.ptr(mv), float(decay), float(eps), int(relu), N.ptr(mean),
                                              N.ptr(invstd), N.ptr(ws), N.stream_ptr()), "bn_fwd_train")
        ctx.save_for_backward(x, mask if mask is not None else y.new_empty(0), g, mean, invstd)
        ctx.has_res = residual is not None
        ctx.relu = relu
        ctx.has_gamma = gamma is not None
        ctx.has_beta = beta is not None
        ctx.sinks = (V.grad_sink(gamma) if gamma is not None else None,
                     V.grad_sink(beta) if beta is not None else None)
        ctx.like = (gamma, beta)
        ctx.out_sink = actsink.attach(y)             # this output's consumers may accumulate here
        if ctx.out_sink is not None:
            # the consumer that completes dy may emit Σ dy·mask, Σ dy·mask·x for this backward, and start its
            # finalize right away
            fin = None
            if EARLY_FIN and x.is_cuda and not N.deterministic():
                def fin(sbuf, g=g, mean=mean, invstd=invstd, M=M, C=C):
                    return _early_finalize(sbuf, g, mean, invstd, M, C)
            # the weight-gradient launch that follows the completing data gradient may run this BN's finalize
            # (ops.conv _Conv.backward): the arguments it needs
            wgf = (g, mean, invstd, M, C) if (WG_FIN and x.is_cuda and not N.deterministic()) else None
            ctx.out_sink.stat_req = (x, mask, fin, wgf)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, g, mean, invstd = ctx.saved_tensors
        pstats = None
        early = None
        why = "no_sink"
        if ctx.out_sink is not None:
            pstats = ctx.out_sink.take_stats()
            early = ctx.out_sink.take_early()
            why = "no_epilogue_stats" if pstats is None else "fused"
            if early is not None and (pstats is None or dy is not None):
                # finalized early from statistics that turned out incomplete: wait for it (it re-zeroed the
                # partial rows) and drop its workspace -- nothing reached the slots
                if early[1] is not None:
                    torch.cuda.current_stream(x.device).wait_event(early[1])
                early = None
            if pstats is not None and dy is not None:
                # part of dy came through plain autograd: the epilogue statistics are incomplete
                from . import conv as _conv
                _conv.bwd_stats_release(pstats, False)
                pstats = None
                why = "autograd_part"
            dy = ctx.out_sink.take(dy)
            ctx.out_sink.stat_req = None
        if BWD_TRACE is not None:
            BWD_TRACE.append((tuple(x.shape), ctx.has_res, why))
        if dy is None:
            if early is not None and early[1] is not None:   # join the side stream (captures must not end forked)
                torch.cuda.current_stream(x.device).wait_event(early[1])
            return (None,) * 11
        dy = dy.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        dx = torch.empty_like(x)
        dres, accum = None, 0
        rs = ctx.res_sink if ctx.needs_input_grad[3] else None
        pending = False
        if ctx.has_res:
            from . import actsink
            if (rs is not None and ctx.relu and actsink.MASKED_RESIDUAL and rs.idle()
                    and not rs.completing()):
                # identity shortcut: its gradient dy * mask is left pending in the sink; the conv dgrad that
                # completes the sum folds it into its epilogue (never written / re-read here)
                pending = True
            else:
                if rs is not None:
                    dres, acc = rs.target()
                    accum = int(acc)
                if dres is None:
                    dres = torch.empty_like(x)
        sg, sb = ctx.sinks
        # dgamma/dbeta accumulate straight into the fp32 grad slots when available
        dgamma = sg.grad if sg is not None else torch.zeros(C, dtype=torch.float32, device=x.device)
        dbeta = sb.grad if sb is not None else torch.zeros(C, dtype=torch.float32, device=x.device)
        if pstats is not None and early is not None:
            from . import conv as _conv
            ws, ev = early
            if ev is not None:                           # side-stream early finalize (EARLY_FIN)
                torch.cuda.current_stream(x.device).wait_event(ev)
                EARLY_USED[0] += 1
            else:                                        # rode on the conv's weight-gradient launch (WG_FIN)
                WG_FIN_USED[0] += 1
            N.check(N.fn("mdtf_bn_dx_ws")(N.ptr(dy), N.ptr(x), N.ptr(mask if ctx.relu else None), N.ptr(dx),
                                          N.ptr(dres), M, C, N.ptr(ws), N.ptr(dgamma), N.ptr(dbeta), int(ctx.relu),
                                          accum, N.stream_ptr()), "bn_dx_ws")
            _conv.bwd_stats_release(pstats, True)        # the early finalize re-zeroed it
            FUSED_BWD[0] += 1
        elif pstats is not None:
            from . import conv as _conv
            ws = torch.empty(3 * C, dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_bn_bwd_stats")(N.ptr(dy), N.ptr(x), N.ptr(mask if ctx.relu else None), N.ptr(dx),
                                              N.ptr(dres), M, C, N.ptr(g), N.ptr(mean), N.ptr(invstd), N.ptr(dgamma),
                                              N.ptr(dbeta), int(ctx.relu), N.ptr(pstats[0]), N.ptr(pstats[1]),
                                              int(pstats.shape[1]), N.ptr(ws), accum, N.stream_ptr()), "bn_bwd_stats")
            _conv.bwd_stats_release(pstats, True)        # the finalize re-zeroed it
            FUSED_BWD[0] += 1
        else:
            ws = torch.empty(int(N.fn("mdtf_bn_workspace_floats")(M, C)), dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_bn_bwd")(N.ptr(dy), N.ptr(x), N.ptr(mask if ctx.relu else None), N.ptr(dx), N.ptr(dres), M,
                                        C, N.ptr(g),
                                        N.ptr(mean), N.ptr(invstd), N.ptr(dgamma), N.ptr(dbeta), int(ctx.relu),
                                        N.ptr(ws), accum, N.stream_ptr()), "bn_bwd")
        if pending:
            rs.defer_masked(dy, mask)
        elif rs is not None and dres is not None:
            rs.written(dres)
            dres = None                                  # delivered through the sink
        gamma, beta = ctx.like
        rg = (V.grad_marker(gamma) if sg is not None else dgamma) if ctx.has_gamma else None
        rb = (V.grad_marker(beta) if sb is not None else dbeta) if ctx.has_beta else None
        return (dx, rg, rb, dres, None, None, None, None, None, None, None)


class DeferredBN(object):
    """A training BatchNorm (no ReLU, no residual) whose apply is deferred into its consumer: the projection
    shortcut of a ResNet block.  The residual BN that adds it applies both normalisations in one pass
    (``csrc/bn.hip`` bn_apply_dual_kernel), so the shortcut's normalised tensor is never written or re-read."""

    def __init__(self, x, gamma, beta, moving_mean, moving_var, decay, epsilon, stats):
        self.x, self.gamma, self.beta = x, gamma, beta
        self.moving_mean, self.moving_var = moving_mean, moving_var
        self.decay, self.epsilon, self.stats = decay, epsilon, stats
        self.shape = x.shape
        self.dtype = x.dtype

    def materialize(self):
        return _BNTrain.apply(self.x, self.gamma, self.beta, None, self.moving_mean, self.moving_var, self.decay,
                              self.epsilon, False, self.stats)


class _BNTrainDual(torch.autograd.Function):
    """relu(BN(x) + BN2(r)): the last BN of a projection-shortcut block with the shortcut's BN fused in."""

    @staticmethod
    def forward(ctx, x, gamma, beta, mm, mv, r, gamma2, beta2, mm2, mv2, decay, eps, stats, stats2):
        from . import actsink
        ctx.set_materialize_grads(False)
        x = x.contiguous()
        r = r.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        y = torch.empty_like(x)
        mean, invstd = (torch.empty(C, dtype=torch.float32, device=x.device) for _ in range(2))
        mean2, invstd2 = (torch.empty(C, dtype=torch.float32, device=x.device) for _ in range(2))
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=x.device)
        g, b, g2, b2 = _f32(gamma), _f32(beta), _f32(gamma2), _f32(beta2)
        ws = torch.empty(4 * C, dtype=torch.float32, device=x.device)
        (ps, pq, P), (ps2, pq2, P2) = stats, stats2
        N.check(N.fn("mdtf_bn_fwd_dual")(N.ptr(x), N.ptr(r), N.ptr(y), N.ptr(mask), M, C, N.ptr(g), N.ptr(b),
                                         N.ptr(mm), N.ptr(mv), N.ptr(ps), N.ptr(pq), int(P), N.ptr(mean),
                                         N.ptr(invstd), N.ptr(g2), N.ptr(b2), N.ptr(mm2), N.ptr(mv2), N.ptr(ps2),
                                         N.ptr(pq2), int(P2), N.ptr(mean2), N.ptr(invstd2), float(decay), float(eps),
                                         N.ptr(ws), N.stream_ptr()), "bn_fwd_dual")
        from . import conv as _conv
        _conv.stats_consumed(x.device)               # both finalizes re-zeroed their partials
        ctx.save_for_backward(x, mask, g, mean, invstd, r, g2, mean2, invstd2)
        ctx.sinks = tuple(V.grad_sink(t) for t in (gamma, beta, gamma2, beta2))
        ctx.like = (gamma, beta, gamma2, beta2)
        ctx.out_sink = actsink.attach(y)
        if ctx.out_sink is not None:
            ctx.out_sink.stat_req = (x, mask)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, g, mean, invstd, r, g2, mean2, invstd2 = ctx.saved_tensors
        pstats = None
        if ctx.out_sink is not None:
            pstats = ctx.out_sink.take_stats()
            if pstats is not None and dy is not None:
                from . import conv as _conv
                _conv.bwd_stats_release(pstats, False)
                pstats = None
            dy = ctx.out_sink.take(dy)
            ctx.out_sink.stat_req = None
        if dy is None:
            return (None,) * 14
        dy = dy.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        dx = torch.empty_like(x)
        if DUAL_FUSED and not DUAL_DZ:
            grads = [sk.grad if sk is not None else torch.zeros(C, dtype=torch.float32, device=x.device)
                     for sk in ctx.sinks]
            dr = torch.empty_like(r)
            ws = torch.empty(2 * int(N.fn("mdtf_bn_workspace_floats")(M, C)), dtype=torch.float32, device=x.device)
            ps, pq, P = (pstats[0], pstats[1], int(pstats.shape[1])) if pstats is not None else (None, None, 0)
            N.check(N.fn("mdtf_bn_bwd_dual")(N.ptr(dy), N.ptr(x), N.ptr(r), N.ptr(mask), N.ptr(dx), N.ptr(dr), M, C,
                                             N.ptr(g), N.ptr(mean), N.ptr(invstd), N.ptr(grads[0]), N.ptr(grads[1]),
                                             N.ptr(ps), N.ptr(pq), P, N.ptr(g2), N.ptr(mean2), N.ptr(invstd2),
                                             N.ptr(grads[2]), N.ptr(grads[3]), N.ptr(ws), N.stream_ptr()),
                    "bn_bwd_dual")
            DUAL_BWD[0] += 1
            if pstats is not None:
                from . import conv as _conv
                _conv.bwd_stats_release(pstats, True)
                FUSED_BWD[0] += 1
            out = [V.grad_marker(t) if sk is not None else gr for t, sk, gr in zip(ctx.like, ctx.sinks, grads)]
            return (dx, out[0], out[1], None, None, dr, out[2], out[3], None, None, None, None, None, None)
        # the shortcut BN's output gradient is dy * mask: its backward reads dy and the ReLU mask itself
        # (no masked copy dz is written and re-read); MDTF_DUAL_DZ=1: the written-copy path (A/B, tests)
        dz = torch.empty_like(x) if DUAL_DZ else None
        grads = [sk.grad if sk is not None else torch.zeros(C, dtype=torch.float32, device=x.device)
                 for sk in ctx.sinks]
        if pstats is not None:
            from . import conv as _conv
            ws = torch.empty(3 * C, dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_bn_bwd_stats")(N.ptr(dy), N.ptr(x), N.ptr(mask), N.ptr(dx), N.ptr(dz), M, C, N.ptr(g),
                                              N.ptr(mean), N.ptr(invstd), N.ptr(grads[0]), N.ptr(grads[1]), 1,
                                              N.ptr(pstats[0]), N.ptr(pstats[1]), int(pstats.shape[1]), N.ptr(ws), 0,
                                              N.stream_ptr()), "bn_bwd_stats")
            _conv.bwd_stats_release(pstats, True)
            FUSED_BWD[0] += 1
        else:
            ws = torch.empty(int(N.fn("mdtf_bn_workspace_floats")(M, C)), dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_bn_bwd")(N.ptr(dy), N.ptr(x), N.ptr(mask), N.ptr(dx), N.ptr(dz), M, C, N.ptr(g),
                                        N.ptr(mean), N.ptr(invstd), N.ptr(grads[0]), N.ptr(grads[1]), 1, N.ptr(ws), 0,
                                        N.stream_ptr()), "bn_bwd")
        dr = torch.empty_like(r)
        ws2 = torch.empty(int(N.fn("mdtf_bn_workspace_floats")(M, C)), dtype=torch.float32, device=x.device)
        N.check(N.fn("mdtf_bn_bwd")(N.ptr(dz if dz is not None else dy), N.ptr(r),
                                    N.ptr(mask) if dz is None else None, N.ptr(dr), None, M, C, N.ptr(g2),
                                    N.ptr(mean2), N.ptr(invstd2), N.ptr(grads[2]), N.ptr(grads[3]), int(dz is None),
                                    N.ptr(ws2), 0, N.stream_ptr()), "bn_bwd")
        out = []
        for t, sk, gr in zip(ctx.like, ctx.sinks, grads):
            out.append(V.grad_marker(t) if sk is not None else gr)
        return (dx, out[0], out[1], None, None, dr, out[2], out[3], None, None, None, None, None, None)


# the stem's BN + ReLU + max pool as one pass (bn_relu_maxpool_nhwc); MDTF_FUSED_STEM=0: BN apply + max pool
FUSED_STEM = os.environ.get("MDTF_FUSED_STEM", "1") != "0"
# its backward's BN statistics from the pooled tensors (dy, pooled y: x recovered from y at each window's argmax)
# instead of a gather pass over the 4x larger input; MDTF_STEM_POOLED_STATS=0: the input-row pass
STEM_POOLED_STATS = os.environ.get("MDTF_STEM_POOLED_STATS", "1") != "0"


class _BNReluMaxPool(torch.autograd.Function):
    """maxpool(relu(BN(x))) with the BN statistics from the conv epilogue (``csrc/bn.hip``
    mdtf_bn_relu_maxpool_fwd / mdtf_maxpool_bn_bwd): the normalised activation is never materialised; the
    backward recomputes the ReLU mask from x and the saved scale/shift."""

    @staticmethod
    def forward(ctx, x, gamma, beta, mm, mv, decay, eps, stats, geo):
        from . import actsink
        ctx.set_materialize_grads(False)
        x = x.contiguous()
        n, h, w, c = x.shape
        oh, ow, kh, kw, sh, sw, pt, pl = geo
        y = torch.empty((n, oh, ow, c), dtype=x.dtype, device=x.device)
        arg = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        mean, invstd = (torch.empty(c, dtype=torch.float32, device=x.device) for _ in range(2))
        ss = torch.empty(2 * c, dtype=torch.float32, device=x.device)
        psum, psq, P = stats
        g, b = _f32(gamma), _f32(beta)
        N.check(N.fn("mdtf_bn_relu_maxpool_fwd")(N.ptr(x), N.ptr(y), N.ptr(arg), n, h, w, c, oh, ow, kh, kw, sh, sw,
                                                 pt, pl, N.ptr(g), N.ptr(b), N.ptr(mm), N.ptr(mv), float(decay),
                                                 float(eps), N.ptr(mean), N.ptr(invstd), N.ptr(psum), N.ptr(psq),
                                                 int(P), N.ptr(ss), N.stream_ptr()), "bn_relu_maxpool_fwd")
        from . import conv as _conv
        _conv.stats_consumed(x.device)
        ctx.save_for_backward(x, arg, g, mean, invstd, ss, y if STEM_POOLED_STATS else None)
        ctx.geo = geo
        ctx.sinks = (V.grad_sink(gamma) if gamma is not None else None,
                     V.grad_sink(beta) if beta is not None else None)
        ctx.like = (gamma, beta)
        ctx.out_sink = actsink.attach(y)         # the pooled output feeds conv1 and the projection shortcut
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.out_sink is not None:
            dy = ctx.out_sink.take(dy)
        if dy is None:
            return (None,) * 9
        x, arg, g, mean, invstd, ss, yp = ctx.saved_tensors
        dy = dy.contiguous()
        n, h, w, c = x.shape
        oh, ow, kh, kw, sh, sw, pt, pl = ctx.geo
        dx = torch.empty_like(x)
        sg, sb = ctx.sinks
        dgamma = sg.grad if sg is not None else torch.zeros(c, dtype=torch.float32, device=x.device)
        dbeta = sb.grad if sb is not None else torch.zeros(c, dtype=torch.float32, device=x.device)
        ws = torch.empty(int(N.fn("mdtf_bn_workspace_floats")(n * h * w, c)), dtype=torch.float32, device=x.device)
        N.check(N.fn("mdtf_maxpool_bn_bwd")(N.ptr(dy), N.ptr(arg), N.ptr(x), N.ptr(dx), n, h, w, c, oh, ow, kh, kw,
                                            sh, sw, pt, pl, N.ptr(g), N.ptr(mean), N.ptr(invstd), N.ptr(dgamma),
                                            N.ptr(dbeta), N.ptr(ss), N.ptr(ws), N.ptr(yp), N.stream_ptr()),
                "maxpool_bn_bwd")
        gamma, beta = ctx.like
        rg = (V.grad_marker(gamma) if sg is not None else dgamma) if gamma is not None else None
        rb = (V.grad_marker(beta) if sb is not None else dbeta) if beta is not None else None
        return (dx, rg, rb, None, None, None, None, None, None)


def bn_relu_maxpool_nhwc(x, gamma, beta, moving_mean, moving_var, decay, epsilon, stats, geo):
    """Training ``max_pool(relu(BN(x)))``; ``geo = (oh, ow, kh, kw, sh, sw, pad_top, pad_left)``."""
    _check(x)
    return _BNReluMaxPool.apply(x, gamma, beta, moving_mean, moving_var, decay, epsilon, stats, geo)


def batch_norm_nhwc(x, gamma, beta, moving_mean, moving_var, training, decay, epsilon, relu, residual, stats=None,
                    on_consumer=False):
    """``on_consumer`` (training, ReLU, no residual, conv-epilogue statistics): the output may be left unwritten
    for the 1x1 conv consuming it to apply (``ON_CONSUMER``); every other reader must go through
    :func:`materialize`."""
    _check(x)
    if isinstance(residual, DeferredBN):
        d = residual
        if training and relu and stats is not None and d.stats is not None and d.x.shape == x.shape:
            return _BNTrainDual.apply(x, gamma, beta, moving_mean, moving_var, d.x, d.gamma, d.beta, d.moving_mean,
                                      d.moving_var, decay, epsilon, stats, d.stats)
        residual = d.materialize()
    if residual is not None and residual.dtype != x.dtype:
        residual = residual.to(x.dtype)
    if training:
        oc = bool(on_consumer and ON_CONSUMER and relu and residual is None and stats is not None
                  and not N.deterministic())
        return _BNTrain.apply(x, gamma, beta, residual, moving_mean, moving_var, decay, epsilon, bool(relu), stats,
                              oc)
    x = x.contiguous()
    C = x.shape[-1]
    M = x.numel() // C
    y = torch.empty_like(x)
    ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    res = residual.contiguous() if residual is not None else None
    N.check(N.fn("mdtf_bn_fwd_eval")(N.ptr(x), N.ptr(res), N.ptr(y), M, C, N.ptr(_f32(gamma)), N.ptr(_f32(beta)),
                                     N.ptr(moving_mean), N.ptr(moving_var), float(epsilon), int(bool(relu)),
                                     N.ptr(ws), N.stream_ptr()), "bn_fwd_eval")
    return y
