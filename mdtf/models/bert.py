"""BERT (base / large) pre-training model on mdtf kernels.

BASELINE config "BERT-base data-parallel 8×MI355X (MFMA bf16 GEMM + fused
Adam)".  Variable names follow Google's TF BERT checkpoints
(``bert/encoder/layer_0/attention/self/query/kernel`` ...), so checkpoints
written by the tensor-bundle Saver line up with the TF layout.

Compute: dense layers are bf16 GEMMs (hipBLASLt) with the fused bias(+GELU)
epilogue kernel; Q/K/V projections run as ONE GEMM on the concatenated
kernels; residual add + LayerNorm, the scaled masked softmax and the
embedding gather/scatter-add are HIP kernels; the MLM decoder is tied to the
word embeddings; the optimizer is the fused AdamWeightDecay kernel.

Inputs (packed so the framework's (raw_data, ground_truth) tower API carries
them): ``raw_data`` int64 ``[B, 3*S + P]`` = input_ids | token_type_ids |
input_mask | masked_lm_positions; ``ground_truth`` int64 ``[B, P + 1]`` =
masked_lm_ids | next_sentence_label.
"""
import math
import os

import torch

from ..layers import tools
from ..ops import nn as ops
from ..ops import transformer as T
from ..runtime.model import Loss, Model
from ..train import step as S
from ..train import variables as V

CONFIGS = {
    "base": dict(hidden=768, layers=12, heads=12, intermediate=3072),
    "large": dict(hidden=1024, layers=24, heads=16, intermediate=4096),
    "tiny": dict(hidden=128, layers=2, heads=2, intermediate=512),
}


def _init(std=0.02):
    return V.truncated_normal_initializer(stddev=std)


_DENSE_VIEW = os.environ.get("MDTF_BERT_DENSE_VIEW", "0") == "1"


def _dense(name, x, out, act=None):
    with V.variable_scope(name):
        w = V.get_variable("kernel", [x.shape[-1], out], initializer=_init())
        b = V.get_variable("bias", [out], initializer=V.constant_initializer(0.0))
    # x goes in unreshaped: a reshaped view would hide the activation-gradient sink attached to a
    # LayerNorm output, and autograd would then add this layer's dx to the residual's separately
    # (MDTF_BERT_DENSE_VIEW=1 restores the view, for A/B runs)
    if _DENSE_VIEW:
        shp = x.shape
        return ops.dense(x.reshape(-1, shp[-1]), w, b, act=act).reshape(*shp[:-1], out)
    return ops.dense(x, w, b, act=act)


def _ln(name, x, residual=None, eps=1e-12, dropout=0.0):
    """LayerNorm(dropout(x) + residual): the dropout of TF BERT's dense outputs is fused into the LN kernel."""
    with V.variable_scope(name):
        g = V.get_variable("gamma", [x.shape[-1]], initializer=V.constant_initializer(1.0), keep_fp32=True)
        b = V.get_variable("beta", [x.shape[-1]], initializer=V.constant_initializer(0.0), keep_fp32=True)
    return T.layer_norm(x, g, b, eps, residual=residual, dropout=dropout if S.is_training() else 0.0)


def _dropout(x, rate):
    if rate and S.is_training():
        return torch.nn.functional.dropout(x, rate, True)
    return x


class Bert(Model):
    def __init__(self, size="base", vocab_size=30522, max_position=512, type_vocab=2, max_predictions=20,
                 seq_len=128, dropout=0.1):
        cfg = CONFIGS[size]
        self.H = cfg["hidden"]
        self.L = cfg["layers"]
        self.heads = cfg["heads"]
        self.I = cfg["intermediate"]
        self.vocab = vocab_size
        self.max_position = max_position
        self.type_vocab = type_vocab
        self.P = max_predictions
        self.S = seq_len
        self.dropout = dropout

    def unpack(self, raw):
        S_, P = self.S, self.P
        return raw[:, :S_], raw[:, S_:2 * S_], raw[:, 2 * S_:3 * S_], raw[:, 3 * S_:3 * S_ + P]

    def inference(self, raw):
        ids, types, mask, positions = self.unpack(raw)
        B, S_ = ids.shape
        store = V.get_store()
        H, nh = self.H, self.heads
        dh = H // nh
        with V.variable_scope("bert"):
            with V.variable_scope("embeddings"):
                word = V.get_variable("word_embeddings", [self.vocab, H], initializer=_init())
                word_obj = V.find_variable("word_embeddings")
                pos = V.get_variable("position_embeddings", [self.max_position, H], initializer=_init())
                typ = V.get_variable("token_type_embeddings", [self.type_vocab, H], initializer=_init())
                e = T.bert_embeddings(word, pos, typ, ids, types)      # one fused kernel each way on the GPU
                x = _ln("LayerNorm", e)
                x = _dropout(x, self.dropout)
            # additive attention mask over keys: 0 keep, -10000 masked
            amask = (1.0 - mask.float()) * -10000.0
            with V.variable_scope("encoder"):
                for l in range(self.L):
                    with V.variable_scope("layer_%d" % l):
                        x = self._layer(x, amask, B, S_, H, nh, dh)
            with V.variable_scope("pooler"):
                first = x[:, 0, :].contiguous()
                pooled = torch.tanh(_dense("dense", first, H).float()).to(x.dtype)
        # ---- pre-training heads
        with V.variable_scope("cls"):
            with V.variable_scope("predictions"):
                flat = x.reshape(B * S_, H)
                idx = (positions + torch.arange(B, device=ids.device).unsqueeze(1) * S_).reshape(-1)
                h = flat.index_select(0, idx)
                with V.variable_scope("transform"):
                    h = _dense("dense", h, H, act="gelu")
                    h = _ln("LayerNorm", h)
                out_bias = V.get_variable("output_bias", [self.vocab], initializer=V.constant_initializer(0.0))
                # tied decoder on its own read of the embedding variable: both consumers then accumulate straight
                # into the fp32 gradient slot (one shared read made autograd add their two zero-stride markers into
                # a materialised [vocab, H] tensor and add that into the slot: two extra passes per step)
                wvar = getattr(word, "_mdtf_var", None)
                bias_obj = V.find_variable("output_bias")
                if word_obj is not None and bias_obj is not None:
                    # zero rows after the embedding and the bias in the flat buffers: the decoder's products run
                    # over a 30720-wide vocabulary (ops.tied_decoder); checkpoints keep the [30522, H] shapes.
                    # Set on the build pass, before the flat parameter space exists.
                    word_obj.pad_rows = bias_obj.pad_rows = ops.decoder_pad_rows(self.vocab)
                word_dec = wvar.read(store.compute_dtype) if wvar is not None else word
                mlm = ops.tied_decoder(h, word_dec, out_bias)
            with V.variable_scope("seq_relationship"):
                w = V.get_variable("output_weights", [2, H], initializer=_init())
                b = V.get_variable("output_bias", [2], initializer=V.constant_initializer(0.0))
                nsp = ops.dense_transposed(pooled, w, b)
        return mlm, nsp

    def _layer(self, x, amask, B, S_, H, nh, dh):
        with V.variable_scope("attention"):
            with V.variable_scope("self"):
                ws, bs = {}, {}
                # created value, key, query: the flat parameter space lays variables out in reverse
                # creation order, so the three biases (and their fp32 gradient slots) end up adjacent
                # in q|k|v order -- one fused bias view / one column-sum for the fused projection
                for nm in ("value", "key", "query"):
                    with V.variable_scope(nm):
                        ws[nm] = V.get_variable("kernel", [H, H], initializer=_init())
                        bs[nm] = V.get_variable("bias", [H], initializer=V.constant_initializer(0.0))
                order = ("query", "key", "value")
                qkv = ops.dense_multi(x, [ws[n] for n in order], [bs[n] for n in order])   # one GEMM
                qkv = qkv.reshape(-1, 3 * H)
                drop = self.dropout if S.is_training() else 0.0
                ctx = T.fused_attention(qkv, B, S_, nh, amask, drop).reshape(B, S_, H)
            with V.variable_scope("output"):
                a = _dense("dense", ctx, H)
                x = _ln("LayerNorm", a, residual=x, dropout=self.dropout)
        with V.variable_scope("intermediate"):
            with V.variable_scope("dense"):
                w1 = V.get_variable("kernel", [H, self.I], initializer=_init())
                b1 = V.get_variable("bias", [self.I], initializer=V.constant_initializer(0.0))
        with V.variable_scope("output"):
            with V.variable_scope("dense"):
                w2 = V.get_variable("kernel", [self.I, H], initializer=_init())
                b2 = V.get_variable("bias", [H], initializer=V.constant_initializer(0.0))
            # one feed-forward op: the GELU backward rides in the second layer's data-gradient epilogue
            o = ops.ffn(x, w1, b1, w2, b2, act="gelu")
            x = _ln("LayerNorm", o, residual=x, dropout=self.dropout)
        return x


class BertPretrainingLoss(Loss):
    """Masked-LM cross entropy + next-sentence cross entropy (fp32)."""

    def __init__(self, max_predictions=20):
        self.P = max_predictions

    def loss(self, predict, ground_truth):
        mlm, nsp = predict
        lm_ids = ground_truth[:, :self.P].reshape(-1)
        ns = ground_truth[:, self.P]
        l1 = ops.sparse_softmax_cross_entropy_with_logits(lm_ids, mlm.reshape(-1, mlm.shape[-1])).mean()
        l2 = ops.sparse_softmax_cross_entropy_with_logits(ns, nsp).mean()
        return l1 + l2


class SyntheticBertLoader(object):
    """Synthetic pre-training batches of the packed BERT layout (device resident)."""
    type = "SyntheticDataLoader"

    def __init__(self, seq_len=128, max_predictions=20, vocab=30522, seed=0):
        self.S, self.P, self.vocab, self.seed = seq_len, max_predictions, vocab, seed
        self.batch_size = 32
        self._batch = None

    def _make(self):
        g = torch.Generator().manual_seed(self.seed)
        B, S_, P = self.batch_size, self.S, self.P
        ids = torch.randint(0, self.vocab, (B, S_), generator=g)
        types = (torch.arange(S_) >= S_ // 2).long().unsqueeze(0).expand(B, S_)
        mask = torch.ones(B, S_, dtype=torch.long)
        pos = torch.stack([torch.randperm(S_, generator=g)[:P].sort().values for _ in range(B)])
        raw = torch.cat([ids, types, mask, pos], 1)
        gt = torch.cat([torch.randint(0, self.vocab, (B, P), generator=g), torch.randint(0, 2, (B, 1), generator=g)], 1)
        dev = V.get_store().device
        return raw.to(dev), gt.to(dev)

    def _next(self):
        if self._batch is None:
            self._batch = self._make()
        return self._batch

    def load_train_batch(self, name_queue=None, *args, **kwargs):
        return S.BatchSource(self._next, name="synthetic-bert").outputs(2)

    def load_eval_batch(self, *args, **kwargs):
        return self.load_train_batch()
