"""Model zoo: the architectures the reference serves, with seeded random weights.

The reference exports TorchScript files from torchvision / HF
(models/import_resnet.py:25-73, models/import_vit.py:10-62,
models/import_bert-base-uncased.py:8-39).  torchvision is not installed and
nothing can be downloaded, so the ResNet and ViT graphs are re-declared here in
plain ``torch.nn`` with torchvision's parameter names and forward, and BERT is
HF ``transformers.BertModel`` built from a local ``BertConfig`` (bert-base
defaults: 768/12/12/3072/30522, LN eps 1e-12, erf-GELU), wrapped exactly like
the reference's ``BertWrapper`` (returns ``last_hidden_state``).

Weights are random (no checkpoints offline) but deterministic: ``torch`` CPU RNG
seeded per model, then BatchNorm running statistics are calibrated on a seeded
synthetic batch so activations stay O(1) through 150+ layers (as with trained
statistics).  These modules are what the host loads into the HIP replicas and
what the CPU codelet (and the test oracle) runs.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Sequence

import torch
from torch import nn


# ---------------------------------------------------------------------------
# ResNet (torchvision.models.resnet naming)
# ---------------------------------------------------------------------------
class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class ResNet(nn.Module):
    def __init__(self, block, layers: Sequence[int], num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.inplanes = width
        self.conv1 = nn.Conv2d(3, width, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, width, layers[0])
        self.layer2 = self._make_layer(block, width * 2, layers[1], 2)
        self.layer3 = self._make_layer(block, width * 4, layers[2], 2)
        self.layer4 = self._make_layer(block, width * 8, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(width * 8 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def _randomize_bn_and_calibrate(model: nn.Module, image: int, seed: int, calib_batch: int = 4) -> None:
    g = torch.Generator().manual_seed(seed + 1)
    # The last BN of each residual branch gets a small gamma, as in trained
    # ResNets (torchvision's zero_init_residual idea, kept non-zero): with unit
    # gammas a random 50-block ResNet-152 amplifies fp32 rounding to ~5e-4
    # (fp32 vs fp64 on CPU), which would make any parity check meaningless.
    last_bn = set()
    for blk in model.modules():
        if isinstance(blk, Bottleneck):
            last_bn.add(id(blk.bn3))
        elif isinstance(blk, BasicBlock):
            last_bn.add(id(blk.bn2))
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d):
            with torch.no_grad():
                if id(m) in last_bn:
                    m.weight.copy_(0.1 + 0.3 * torch.rand(m.num_features, generator=g))
                else:
                    m.weight.copy_(0.75 + 0.5 * torch.rand(m.num_features, generator=g))
                m.bias.copy_(0.2 * torch.rand(m.num_features, generator=g) - 0.1)
            m.momentum = None  # cumulative average: one pass = that batch's statistics
            m.reset_running_stats()
    x = torch.rand(calib_batch, 3, image, image, generator=g)
    model.train()
    with torch.no_grad():
        model(x)
    model.eval()


def resnet(layers: Sequence[int], bottleneck: bool, seed: int = 0, image: int = 224,
           num_classes: int = 1000, calibrate: bool = True) -> ResNet:
    torch.manual_seed(seed)
    model = ResNet(Bottleneck if bottleneck else BasicBlock, layers, num_classes)
    if calibrate:
        _randomize_bn_and_calibrate(model, image, seed)
    return model.eval()


def resnet18(seed: int = 0, image: int = 224, **kw) -> ResNet:
    return resnet([2, 2, 2, 2], False, seed, image, **kw)


def resnet152(seed: int = 0, image: int = 224, **kw) -> ResNet:
    return resnet([3, 8, 36, 3], True, seed, image, **kw)


# ---------------------------------------------------------------------------
# Vision Transformer (torchvision.models.vision_transformer naming)
# ---------------------------------------------------------------------------
class MLPBlock(nn.Sequential):
    def __init__(self, dim: int, mlp_dim: int):
        super().__init__(nn.Linear(dim, mlp_dim), nn.GELU(), nn.Dropout(0.0), nn.Linear(mlp_dim, dim),
                         nn.Dropout(0.0))


class EncoderBlock(nn.Module):
    def __init__(self, heads: int, dim: int, mlp_dim: int):
        super().__init__()
        self.ln_1 = nn.LayerNorm(dim, eps=1e-6)
        self.self_attention = nn.MultiheadAttention(dim, heads, dropout=0.0, batch_first=True)
        self.dropout = nn.Dropout(0.0)
        self.ln_2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = MLPBlock(dim, mlp_dim)

    def forward(self, inp):
        x = self.ln_1(inp)
        x, _ = self.self_attention(x, x, x, need_weights=False)
        x = self.dropout(x) + inp
        y = self.mlp(self.ln_2(x))
        return x + y


class Encoder(nn.Module):
    def __init__(self, seq: int, layers: int, heads: int, dim: int, mlp_dim: int):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq, dim).normal_(std=0.02))
        self.dropout = nn.Dropout(0.0)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", EncoderBlock(heads, dim, mlp_dim)) for i in range(layers)))
        self.ln = nn.LayerNorm(dim, eps=1e-6)

    def forward(self, x):
        return self.ln(self.layers(self.dropout(x + self.pos_embedding)))


class VisionTransformer(nn.Module):
    def __init__(self, image: int, patch: int, layers: int, heads: int, dim: int, mlp_dim: int,
                 num_classes: int = 1000):
        super().__init__()
        self.image_size, self.patch_size, self.hidden_dim = image, patch, dim
        self.conv_proj = nn.Conv2d(3, dim, patch, patch)
        self.class_token = nn.Parameter(torch.zeros(1, 1, dim))
        seq = (image // patch) ** 2 + 1
        self.encoder = Encoder(seq, layers, heads, dim, mlp_dim)
        self.heads = nn.Sequential(OrderedDict(head=nn.Linear(dim, num_classes)))

    def _process_input(self, x):
        n = x.shape[0]
        x = self.conv_proj(x)
        x = x.reshape(n, self.hidden_dim, -1)
        return x.permute(0, 2, 1)

    def forward(self, x):
        x = self._process_input(x)
        cls = self.class_token.expand(x.shape[0], -1, -1)
        x = self.encoder(torch.cat([cls, x], dim=1))
        return self.heads(x[:, 0])


def vit(image: int = 224, patch: int = 16, layers: int = 24, heads: int = 16, dim: int = 1024,
        mlp_dim: int = 4096, num_classes: int = 1000, seed: int = 0) -> VisionTransformer:
    torch.manual_seed(seed)
    model = VisionTransformer(image, patch, layers, heads, dim, mlp_dim, num_classes)
    with torch.no_grad():
        # torchvision zero-initialises class_token and the head, which would make
        # every logit equal; random values keep the parity check meaningful.
        model.class_token.normal_(std=0.02)
        model.heads.head.weight.normal_(std=0.02)
        model.heads.head.bias.normal_(std=0.02)
        for m in model.modules():
            if isinstance(m, nn.LayerNorm):
                m.weight.copy_(1.0 + 0.1 * torch.randn_like(m.weight))
                m.bias.copy_(0.05 * torch.randn_like(m.bias))
    return model.eval()


def vit_l_16(seed: int = 0, image: int = 224, **kw) -> VisionTransformer:
    return vit(image, 16, 24, 16, 1024, 4096, seed=seed, **kw)


# ---------------------------------------------------------------------------
# BERT (HF transformers BertModel, wrapped like models/import_bert-base-uncased.py)
# ---------------------------------------------------------------------------
class BertWrapper(nn.Module):
    def __init__(self, bert: nn.Module):
        super().__init__()
        self.bert = bert

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
        return self.bert(input_ids=input_ids, attention_mask=attention_mask, return_dict=False)[0]


def bert(layers: int = 12, hidden: int = 768, heads: int = 12, intermediate: int = 3072,
         vocab: int = 30522, max_position: int = 512, seed: int = 0, init_std: float = 0.02) -> BertWrapper:
    import logging

    from transformers import BertConfig, BertModel
    from transformers.utils import logging as hf_logging

    hf_logging.set_verbosity_error()
    logging.getLogger("transformers").setLevel(logging.ERROR)
    torch.manual_seed(seed)
    cfg = BertConfig(num_hidden_layers=layers, hidden_size=hidden, num_attention_heads=heads,
                     intermediate_size=intermediate, vocab_size=vocab, max_position_embeddings=max_position,
                     initializer_range=init_std, torchscript=True)
    model = BertWrapper(BertModel(cfg))
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, nn.LayerNorm):
                m.weight.copy_(1.0 + 0.1 * torch.randn_like(m.weight))
                m.bias.copy_(0.05 * torch.randn_like(m.bias))
    return model.eval()


def bert_base(seed: int = 0, **kw) -> BertWrapper:
    return bert(seed=seed, **kw)


class AddConstant(nn.Module):
    """The reference's toy TorchScript models (tests/e2e/fixtures/simple_model.ts: x + 1)."""

    def __init__(self, value: float = 1.0):
        super().__init__()
        self.value = value

    def forward(self, x):
        return x + self.value


def build(name: str, seed: int = 0, **kw) -> nn.Module:
    """Named constructors for the BASELINE.json configs."""
    table = {
        "resnet18": resnet18,
        "resnet152": resnet152,
        "vit_l_16": vit_l_16,
        "bert-base-uncased": bert_base,
        "bert_base": bert_base,
    }
    if name not in table:
        raise KeyError(f"unknown model {name!r}; known: {sorted(table)}")
    return table[name](seed=seed, **kw)


# TorchScript names a class by its Python module path; this package's directory
# name is not an identifier, so give the zoo's modules a loadable qualified name
# (a traced/scripted model must round-trip through .pt like the reference's).
for _cls in (BasicBlock, Bottleneck, ResNet, MLPBlock, EncoderBlock, Encoder, VisionTransformer, BertWrapper,
             AddConstant):
    _cls.__module__ = "spi_zoo"
