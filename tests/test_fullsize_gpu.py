"""Full-size parity for the remaining BASELINE configs at their stated batches, through the
C-ABI codelet: C4 ResNet-152 @224 bs=32 and C5 ViT-L/16 @224 bs=16 (the GEMM plans -- tile size,
split-K, halo bands -- depend on M = batch x pixels, so the stated batch is what must be checked).
dims[0] = the effective batch (inference_task.cpp:606-613)."""
import numpy as np
import pytest
import torch

from oracle.cpu_codelet import cpu_inference, normalized_max_error, top1_agreement

pytestmark = pytest.mark.gpu


def run(spi, rep, x, out_shape):
    xin = torch.from_numpy(x).cuda()
    out = torch.full(out_shape, float("nan"), device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    spi.run_hip(rep, [xin], out, stream=s.cuda_stream)
    return out.cpu().numpy()


@pytest.fixture(scope="module")
def resnet152(zoo):
    torch.set_num_threads(16)
    return zoo.resnet152()


@pytest.fixture(scope="module")
def resnet152_refs(resnet152):
    """fp32 oracle and its fp64 restatement (truth) on the same input."""
    import copy
    x = np.random.default_rng(21).random((32, 3, 224, 224), dtype=np.float32)
    ref32 = cpu_inference(resnet152, [x])[0]
    # fp64 truth on the first 4 images only (ATen's fp64 convs are slow on the host)
    with torch.inference_mode():
        ref64 = copy.deepcopy(resnet152).double()(torch.from_numpy(x[:4]).double()).numpy()
    return x, ref32, ref64


@pytest.mark.parametrize("prec", ["fp32", "fp16x3", "fp16"])
def test_resnet152_224(spi, gpu, resnet152, resnet152_refs, prec):
    """50 bottleneck blocks: the oracle's own fp32 result sits ~8e-6 from fp64, so fp32-grade
    modes are held to 'as close to fp64 as the reference's fp32 CPU codelet' (and 3e-5 vs it);
    plain fp16 operands are bounded by their format floor (CPU emulation 1.06e-2)."""
    x, ref32, ref64 = resnet152_refs
    rep = spi.ModelReplica(resnet152, 0, prec, max_batch=32)
    got = run(spi, rep, x, ref32.shape)
    err32 = normalized_max_error(got, ref32)
    err64 = normalized_max_error(got[:4], ref64)
    oracle64 = normalized_max_error(ref32[:4], ref64)
    print(f"resnet152 bs32 {prec} err_vs_fp32_oracle={err32:.3e} err_vs_fp64={err64:.3e} oracle_vs_fp64={oracle64:.3e}")
    if prec == "fp16":
        assert err32 < 2e-2
    else:
        assert err32 < 3e-5
        assert err64 <= 3 * oracle64 + 1e-6
        assert top1_agreement(got, ref32) == 1.0


@pytest.fixture(scope="module")
def vit_l(zoo):
    torch.set_num_threads(16)
    return zoo.vit_l_16()


@pytest.fixture(scope="module")
def vit_l_ref(vit_l):
    x = np.random.default_rng(22).random((16, 3, 224, 224), dtype=np.float32)
    return x, cpu_inference(vit_l, [x])[0]


@pytest.mark.parametrize("prec,tol", [("fp32", 1e-5), ("fp16", 1e-3)])
def test_vit_l_16_224(spi, gpu, vit_l, vit_l_ref, prec, tol):
    x, ref = vit_l_ref
    rep = spi.ModelReplica(vit_l, 0, prec, max_batch=16)
    got = run(spi, rep, x, ref.shape)
    err = normalized_max_error(got, ref)
    print(f"vit_l_16 bs16 {prec} err={err:.3e}")
    assert err < tol
    assert top1_agreement(got, ref) == 1.0
