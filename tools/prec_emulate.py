#!/usr/bin/env python3
"""CPU emulation of the HIP ResNet forward under per-layer precision plans (round 5).

The HIP path folds eval BatchNorm into the conv weights (fp64), multiplies fp16 (or split
hi + lo) operands exactly with fp32 accumulation, and rounds each conv's epilogue output to
its storage format.  This restates that arithmetic in torch fp32/fp64 on the CPU so a plan
-- which operands are fp16, which are ~fp32 (split), which outputs are stored fp32 -- can be
ranked by its normalised max error against the fp32 oracle before it is built.

Classes of layers: stem, c1 (bottleneck 1x1 reduce), c2 (3x3), c3 (1x1 expand), ds (the
downsample 1x1), fc; storage of the block output (the residual stream) 'S'.
A plan is a set of tokens, e.g. 'w32:stem,ds,fc a32:stem out32:ds' :
  w32:<classes>   weights split hi + lo (~fp32) instead of fp16
  a32:<classes>   the A operand read as fp32 (split at fragment read) instead of fp16
  out32:<classes> the output stored fp32 instead of fp16 (ds: its output feeds the residual)
  s32             the block output kept fp32 for the next block's residual add (conv1 / ds
                  still read an fp16 copy unless a32 says otherwise)
usage: python tools/prec_emulate.py --model resnet152 --batch 4 --plan f16m --plan 'f16m s32' ...
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PRESETS = {
    "f16": "",
    "f16m": "w32:stem,ds,fc a32:stem,fc out32:ds",  # the round-2 ResNet-18 mode
    "f32": "w32:stem,c1,c2,c3,ds,fc a32:stem,c1,c2,c3,ds,fc out32:stem,c1,c2,c3,ds s32",
}


def parse_plan(text):
    toks = []
    for t in text.split():
        toks += PRESETS[t].split() if t in PRESETS else [t]
    plan = {"w32": set(), "a32": set(), "out32": set(), "s32": False, "exact": set()}
    for t in toks:
        if t == "s32":
            plan["s32"] = True
            continue
        if t.startswith("exact:"):  # every conv of these stages (1..4) fp32-grade
            plan["exact"] |= {int(v) for v in t[6:].split(",")}
            continue
        k, _, v = t.partition(":")
        plan[k] |= set(filter(None, v.split(",")))
    return plan


def fold(conv, bn):
    w = conv.weight.detach().double()
    s = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    b = bn.bias.detach().double() - bn.running_mean.detach().double() * s
    return (w * s.view(-1, 1, 1, 1)).float(), b.float()


def r16(x):
    return x.half().float()


class Emu:
    def __init__(self, model, plan):
        self.m = model
        self.p = plan

    def conv(self, x, conv, bn, cls, res=None, relu=True):
        w, b = fold(conv, bn)
        ex = self.stage in self.p["exact"]
        if cls not in self.p["w32"] and not ex:
            w = r16(w)
        if cls not in self.p["a32"] and not ex:
            x = r16(x)
        y = F.conv2d(x, w, b, conv.stride, conv.padding)
        if res is not None:
            y = y + res
        if relu:
            y = F.relu(y)
        return y if cls in self.p["out32"] or ex else r16(y)

    def forward(self, x):
        m = self.m
        self.stage = 0
        x = self.conv(x, m.conv1, m.bn1, "stem")
        x = F.max_pool2d(x, 3, 2, 1)
        for si, layer in enumerate((m.layer1, m.layer2, m.layer3, m.layer4)):
            self.stage = si + 1
            for blk in layer:
                x = self.block(blk, x)
        # the residual stream is stored as the block output format; avgpool reads it, fp32 out
        f = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        w = m.fc.weight.detach().float()
        if "fc" not in self.p["w32"]:
            w = r16(w)
        if "fc" not in self.p["a32"]:
            f = r16(f)
        return F.linear(f, w, m.fc.bias.detach().float())

    def block(self, blk, x):
        # x: the block input as stored (fp32 if s32 else fp16-valued)
        xa = x  # what conv1 / ds read (their a32 decides the rounding)
        if hasattr(blk, "conv3"):
            o = self.conv(xa, blk.conv1, blk.bn1, "c1")
            o = self.conv(o, blk.conv2, blk.bn2, "c2")
            last, lbn, lcls = blk.conv3, blk.bn3, "c3"
        else:
            o = self.conv(xa, blk.conv1, blk.bn1, "c2")
            last, lbn, lcls = blk.conv2, blk.bn2, "c2"
        if blk.downsample is not None:
            ident = self.conv(xa, blk.downsample[0], blk.downsample[1], "ds", relu=False)
        else:
            ident = x
        w, b = fold(last, lbn)
        ex = self.stage in self.p["exact"]
        if lcls not in self.p["w32"] and not ex:
            w = r16(w)
        if lcls not in self.p["a32"] and not ex:
            o = r16(o)
        y = F.relu(F.conv2d(o, w, b, last.stride, last.padding) + ident)
        return y if self.p["s32"] or ex else r16(y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet152")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seeds", default="0")
    ap.add_argument("--plan", action="append", default=[])
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    zoo = importlib.import_module("starpu-inference-server_amd.zoo")
    model = zoo.build(a.model, seed=0)
    plans = a.plan or ["f16", "f16m"]
    for seed in (int(s) for s in a.seeds.split(",")):
        x = torch.from_numpy(np.random.default_rng(seed).random((a.batch, 3, 224, 224), dtype=np.float32))
        with torch.no_grad():
            ref = model(x).numpy()
            for p in plans:
                got = Emu(model, parse_plan(p)).forward(x).numpy()
                err = np.abs(got.astype(np.float64) - ref).max() / np.abs(ref).max()
                top1 = float((got.argmax(1) == ref.argmax(1)).mean())
                print(f"seed {seed} {p:60s} err {err:.3e} top1 {top1:.2f}", flush=True)


if __name__ == "__main__":
    main()
