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
