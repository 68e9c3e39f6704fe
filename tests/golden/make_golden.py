#!/usr/bin/env python3
"""Regenerate the committed golden fixtures (run from the repo root, CPU only).

toy.json      -- the reference's own boundary golden vectors, restated as data:
                 x+1 on {1,2,3} -> {2,3,4} (tests/integration/starpu/integration_starpu_setup.cpp:42-60),
                 x+1.5 (tests/unit/core/unit_starpu_setup.cpp:2332-2433), x*2 / identity / (x, x+1) /
                 [x, x+1] (tests/common/test_inference_runner.hpp:22-70,
                 tests/integration/core/integration_inference_runner.cpp:67-123).
models.npz    -- seeded inputs and CPU-oracle outputs for reduced model configs (no reference fixture
                 pins ResNet/BERT/ViT numerics): they pin the oracle + weight generator
                 across machines and give the GPU tests fixed expected outputs.
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle.cpu_codelet import cpu_inference  # noqa: E402

zoo = importlib.import_module("starpu-inference-server_amd.zoo")
HERE = os.path.dirname(os.path.abspath(__file__))

SMALL = {
    # name: (constructor kwargs, input builder)
    "resnet18_img64_b2": lambda: (zoo.resnet18(image=64), [np.random.default_rng(10).random((2, 3, 64, 64),
                                                                                            dtype=np.float32)]),
    "resnet_bottleneck_1221_img64_b2": lambda: (zoo.resnet([1, 2, 2, 1], True, image=64),
                                                [np.random.default_rng(11).random((2, 3, 64, 64), dtype=np.float32)]),
    "bert_L2_S16_b2_masked": lambda: (zoo.bert(layers=2, init_std=0.05), [
        np.random.default_rng(12).integers(0, 30522, size=(2, 16), dtype=np.int64),
        np.array([[1] * 16, [1] * 10 + [0] * 6], dtype=np.int64)]),
    "vit_img32_p16_L2_D128_b2": lambda: (zoo.vit(image=32, patch=16, layers=2, heads=2, dim=128, mlp_dim=256),
                                         [np.random.default_rng(13).random((2, 3, 32, 32), dtype=np.float32)]),
}


def toy_vectors():
    x = [1.0, 2.0, 3.0]
    return {
        "add_one": {"input": x, "outputs": [[2.0, 3.0, 4.0]]},
        "add_one_point_five": {"input": x, "outputs": [[2.5, 3.5, 4.5]]},
        "mul_two": {"input": x, "outputs": [[2.0, 4.0, 6.0]]},
        "identity": {"input": x, "outputs": [x]},
        "tuple_x_xplus1": {"input": x, "outputs": [x, [2.0, 3.0, 4.0]]},
        "list_x_xplus1": {"input": x, "outputs": [x, [2.0, 3.0, 4.0]]},
    }


def main():
    torch.set_num_threads(8)
    with open(os.path.join(HERE, "toy.json"), "w") as f:
        json.dump(toy_vectors(), f, indent=1)
    arrays = {}
    for name, build in SMALL.items():
        model, inputs = build()
        out = cpu_inference(model, inputs)[0]
        for i, x in enumerate(inputs):
            arrays[f"{name}__in{i}"] = x
        arrays[f"{name}__out"] = out
        print(name, out.shape, float(np.abs(out).max()))
    np.savez_compressed(os.path.join(HERE, "models.npz"), **arrays)


if __name__ == "__main__":
    main()
