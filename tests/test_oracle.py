"""The CPU oracle against the reference's golden vectors (and the committed
model fixtures that pin the oracle + weight generator across machines)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle.cpu_codelet import OracleError, cpu_inference, flatten_ivalue, normalized_max_error, top1_agreement

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def toy_modules():
    def script(src):
        return torch.jit.CompilationUnit(src)

    class Wrap(torch.nn.Module):
        def __init__(self, fn):
            super().__init__()
            self.fn = fn

        def forward(self, x):
            return self.fn(x)

    return {
        "add_one": Wrap(lambda x: x + 1),
        "add_one_point_five": Wrap(lambda x: x + 1.5),
        "mul_two": Wrap(lambda x: x * 2),
        "identity": Wrap(lambda x: x),
        "tuple_x_xplus1": Wrap(lambda x: (x, x + 1)),
        "list_x_xplus1": Wrap(lambda x: [x, x + 1]),
    }


def test_oracle_reproduces_reference_toy_vectors():
    vecs = json.load(open(os.path.join(GOLDEN, "toy.json")))
    mods = toy_modules()
    for name, v in vecs.items():
        outs = cpu_inference(mods[name], [np.array(v["input"], dtype=np.float32)], num_outputs=len(v["outputs"]))
        assert [o.tolist() for o in outs] == v["outputs"], name


def test_oracle_on_the_reference_e2e_fixture():
    """tests/e2e/fixtures/simple_model.ts is `def forward(self, x): return x + 1` (TorchScript source)."""
    class SimpleModel(torch.nn.Module):
        def forward(self, x):
            return x + 1

    out = cpu_inference(torch.jit.script(SimpleModel()), [np.array([1, 2, 3], dtype=np.float32)])[0]
    assert out.tolist() == [2.0, 3.0, 4.0]


def test_oracle_error_paths():
    class Const(torch.nn.Module):
        def forward(self, x):
            return 5

    with pytest.raises(OracleError, match="Unsupported model output type"):
        cpu_inference(Const(), [np.ones(3, np.float32)])
    with pytest.raises(OracleError, match="Mismatch between model outputs"):
        cpu_inference(toy_modules()["tuple_x_xplus1"], [np.ones(3, np.float32)], num_outputs=1)
    with pytest.raises(OracleError, match="size mismatch"):
        cpu_inference(toy_modules()["add_one"], [np.ones(3, np.float32)], output_nbytes=[16])
    with pytest.raises(OracleError, match="layout mismatch"):
        cpu_inference(toy_modules()["add_one"], [np.ones(3, np.float32)], dims=[[4]])


def test_flatten_ivalue_order():
    """append_ivalue: depth-first, dict insertion order (unit_starpu_setup.cpp:3979-4063)."""
    t = [torch.tensor([float(i)]) for i in range(5)]
    nested = (t[0], [t[1], {"b": t[2], "a": [t[3]]}], t[4])
    assert [int(x.item()) for x in flatten_ivalue(nested, [])] == [0, 1, 2, 3, 4]


def test_dims_view_uses_layout_not_buffer_length():
    """dims come from params.layout (dims[0] = effective batch), not from the buffer size."""
    buf = np.arange(12, dtype=np.float32)
    out = cpu_inference(toy_modules()["mul_two"], [buf], dims=[[2, 3]])[0]
    np.testing.assert_array_equal(out, (buf[:6] * 2).reshape(2, 3))


@pytest.mark.parametrize("name", ["resnet18_img64_b2", "resnet_bottleneck_1221_img64_b2", "bert_L2_S16_b2_masked",
                                  "vit_img32_p16_L2_D128_b2"])
def test_oracle_reproduces_model_fixtures(zoo, name):
    import importlib
    import sys
    sys.path.insert(0, GOLDEN)
    mk = importlib.import_module("make_golden")
    g = np.load(os.path.join(GOLDEN, "models.npz"))
    model, _ = mk.SMALL[name]()
    inputs = [g[f"{name}__in{i}"] for i in range(2) if f"{name}__in{i}" in g]
    out = cpu_inference(model, inputs)[0]
    ref = g[f"{name}__out"]
    assert normalized_max_error(out, ref) < 1e-5
    if ref.ndim == 2:
        assert top1_agreement(out, ref) == 1.0


# Graph fidelity of the oracle's ResNet / ViT restatements (torchvision itself is
# not importable here).  torchvision publishes, in each pretrained weights enum's
# metadata, the parameter count and the multiply-add count ("_ops", GMACs at 224^2)
# of exactly the graphs models/import_resnet.py and models/import_vit.py export:
#   ResNet18_Weights.IMAGENET1K_V1   num_params 11,689,512   _ops 1.814
#   ResNet152_Weights.IMAGENET1K_V1  num_params 60,192,808   _ops 11.514
#   ViT_L_16_Weights.IMAGENET1K_V1   num_params 304,326,632  _ops 61.555
# Matching both (per-tensor names follow torchvision's state_dict keys) pins the
# layer structure the parity tests compare against; the arithmetic per layer is
# ATen's.  BERT uses transformers' own BertModel, so it needs no such pin.
TORCHVISION_META = {"resnet18": (11_689_512, 1.814), "resnet152": (60_192_808, 11.514),
                    "vit_l_16": (304_326_632, 61.555)}


@pytest.mark.parametrize("name", sorted(TORCHVISION_META))
def test_restated_graphs_match_torchvision_metadata(zoo, name):
    from torch.utils.flop_counter import FlopCounterMode

    params, gmacs = TORCHVISION_META[name]
    model = zoo.build(name, seed=0)
    assert sum(p.numel() for p in model.parameters()) == params
    sd = model.state_dict()
    if name.startswith("resnet"):
        for key in ("conv1.weight", "bn1.running_var", "layer1.0.conv1.weight", "layer4.0.downsample.0.weight",
                    "layer4.0.downsample.1.running_mean", "fc.weight", "fc.bias"):
            assert key in sd, key
    else:
        for key in ("class_token", "conv_proj.weight", "encoder.pos_embedding",
                    "encoder.layers.encoder_layer_23.self_attention.in_proj_weight",
                    "encoder.layers.encoder_layer_23.mlp.3.weight", "encoder.ln.weight", "heads.head.weight"):
            assert key in sd, key
    # grad mode on: nn.MultiheadAttention's fused inference fast path is invisible to the counter
    with FlopCounterMode(display=False) as fc:
        model(torch.zeros(1, 3, 224, 224))
    # torchvision's _ops counts the conv / linear / attention-matmul multiply-adds; the counter
    # does not see scaled_dot_product_attention's CPU matmuls, added here (QK^T and PV per layer)
    attn = 24 * 2 * 197 * 197 * 1024 / 1e9 if name == "vit_l_16" else 0.0
    assert abs(fc.get_total_flops() / 2e9 + attn - gmacs) / gmacs < 2e-3
