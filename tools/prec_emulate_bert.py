#!/usr/bin/env python3
"""CPU emulation of the HIP BERT fp16 forward with per-site rounding switches (round 5).

Restates the fp16 transformer path in torch fp64 on the CPU:
fp32 residual stream and LayerNorm, fp16 GEMM operands with exact products and wide
accumulation, fp16 Q / K / V, fp16 P for the P.V product, fp16 attention context, fp16 GELU
output.  Each rounding site can be switched off (kept exact) to rank the sites by the error
they carry against the fp32 oracle (HF BertModel), e.g. on the wide-init (std 0.05) three-layer
model of tests/test_parity_gpu.py::test_transformer_layernorm_fold.

sites: w (all GEMM weights), ln (LayerNorm output copy feeding QKV / FFN1), qkv (Q, K, V
stored), p (softmax P for P.V), ctx (attention output feeding the out-projection), gelu
(FFN1 output feeding FFN2), fold (the LayerNorm consumer fold: QKV / FFN1 read the fp16 copy of
the PRE-LayerNorm rows and normalise after the GEMM)
usage: python tools/prec_emulate_bert.py --exact '' --exact gelu --exact p,ctx ...
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SITES = ["w", "wq", "wo", "w1", "w2", "ln", "qkv", "p", "ctx", "gelu"]


def r16(x, on):
    return x.half().double() if on else x


def ln(x, w, b, eps):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def forward(bert, ids, mask, exact, fold=False):
    """exact: the set of sites kept exact (everything else rounded as the HIP fp16 path)."""
    rd = {s: s not in exact for s in SITES}
    sd = {k: v.detach().double() for k, v in bert.state_dict().items()}
    cfg = bert.config
    eps = cfg.layer_norm_eps
    H, D = cfg.num_attention_heads, cfg.hidden_size
    hd = D // H
    B, S = ids.shape
    site = {"query": "wq", "key": "wq", "value": "wq", "attention.output": "wo", "intermediate": "w1",
            "output.dense": "w2"}

    def W(k):  # a GEMM's weight: rounded unless "w" or its own site is exact
        own = next(v for n, v in site.items() if n in k)
        return r16(sd[k], rd["w"] and rd[own])
    x = sd["embeddings.word_embeddings.weight"][ids] + sd["embeddings.position_embeddings.weight"][:S][None] + \
        sd["embeddings.token_type_embeddings.weight"][0][None, None]
    x = ln(x, sd["embeddings.LayerNorm.weight"], sd["embeddings.LayerNorm.bias"], eps)
    bias = (1.0 - mask.double())[:, None, None, :] * torch.finfo(torch.float32).min
    def consume(xn, pre, g_, b_, wk, bk):
        """LN(pre) W^T + b as the HIP path runs it: on the fp16 copy of LN(pre) (unfused), or
        folded (ln_fold.hpp: rstd (fp16(pre) W'^T - mean c1) + b + W beta, W' = fp16(W diag(g)),
        c1 = the row sums of W' as packed; layer 0 and the embeddings always unfused)."""
        if not fold or pre is None:
            return r16(xn, rd["ln"]) @ W(wk).T + sd[bk]
        mu = pre.mean(-1, keepdim=True)
        rstd = 1.0 / torch.sqrt(((pre - mu) ** 2).mean(-1, keepdim=True) + eps)
        wf = r16(sd[wk] * g_[None, :], rd["w"] and rd[next(v for n_, v in site.items() if n_ in wk)])
        c1 = wf.sum(1)
        return rstd * (r16(pre, rd["ln"]) @ wf.T - mu * c1) + sd[bk] + sd[wk] @ b_

    pre = None  # the rows before the LayerNorm that produced x (None: not foldable)
    g_prev = b_prev = None
    for i in range(cfg.num_hidden_layers):
        p = f"encoder.layer.{i}."
        q = r16(consume(x, pre, g_prev, b_prev, p + "attention.self.query.weight", p + "attention.self.query.bias"), rd["qkv"])
        k = r16(consume(x, pre, g_prev, b_prev, p + "attention.self.key.weight", p + "attention.self.key.bias"), rd["qkv"])
        v = r16(consume(x, pre, g_prev, b_prev, p + "attention.self.value.weight", p + "attention.self.value.bias"), rd["qkv"])
        q, k, v = (t.view(B, S, H, hd).transpose(1, 2) for t in (q, k, v))
        s = q @ k.transpose(-1, -2) / hd ** 0.5 + bias
        m = s.max(-1, keepdim=True).values
        e = torch.exp(s - m)
        l_ = e.sum(-1, keepdim=True)
        ctx = (r16(e, rd["p"]) @ v) / l_
        ctx = r16(ctx.transpose(1, 2).reshape(B, S, D), rd["ctx"])
        y = ctx @ W(p + "attention.output.dense.weight").T + sd[p + "attention.output.dense.bias"] + x
        g1, b1 = sd[p + "attention.output.LayerNorm.weight"], sd[p + "attention.output.LayerNorm.bias"]
        x = ln(y, g1, b1, eps)
        h = consume(x, y, g1, b1, p + "intermediate.dense.weight", p + "intermediate.dense.bias")
        h = r16(0.5 * h * (1.0 + torch.erf(h / 2 ** 0.5)), rd["gelu"])
        y = h @ W(p + "output.dense.weight").T + sd[p + "output.dense.bias"] + x
        g_prev, b_prev = sd[p + "output.LayerNorm.weight"], sd[p + "output.LayerNorm.bias"]
        x = ln(y, g_prev, b_prev, eps)
        pre = y
    return x.float().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--init-std", type=float, default=0.05)
    ap.add_argument("--exact", action="append", default=[])
    ap.add_argument("--fold", action="store_true", help="the LayerNorm consumer fold on QKV / FFN1")
    a = ap.parse_args()
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    m = zoo.bert(layers=a.layers, init_std=a.init_std)
    rng = np.random.default_rng(13)  # test_transformer_layernorm_fold's inputs
    ids = rng.integers(0, 30522, size=(3, 80), dtype=np.int64)
    mask = np.ones((3, 80), dtype=np.int64)
    mask[-1, 50:] = 0
    with torch.inference_mode():
        ref = m(torch.from_numpy(ids), torch.from_numpy(mask))
        ref = (ref[0] if isinstance(ref, tuple) else ref).numpy()
    ids_t, mask_t = torch.from_numpy(ids), torch.from_numpy(mask)
    for ex in a.exact or ["", "w,ln,qkv,p,ctx,gelu"]:
        exact = set(filter(None, ex.split(",")))
        got = forward(m.bert, ids_t, mask_t, exact, fold=a.fold)
        err = np.abs(got.astype(np.float64) - ref).max() / np.abs(ref).max()
        print(f"exact={ex or '-':30s} err {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
