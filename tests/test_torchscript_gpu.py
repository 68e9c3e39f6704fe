"""F2 end to end: the reference's on-disk model format (a TorchScript .pt, exported with
torch.jit.trace as models/import_resnet.py:25-73 / models/import_bert-base-uncased.py:8-39 do)
loaded through ModelReplica(path) -- torch::jit::load + weight extraction
(inference_runner.cpp:243-275) -- and the HIP codelet's output checked against the CPU codelet
oracle running the SAME loaded TorchScript module."""
import numpy as np
import pytest
import torch

from oracle.cpu_codelet import cpu_inference, normalized_max_error, top1_agreement

pytestmark = pytest.mark.gpu


def hip(spi, rep, inputs, shape):
    ins = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in inputs]
    out = torch.full(shape, float("nan"), device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    spi.run_hip(rep, ins, out, stream=s.cuda_stream)
    return out.cpu().numpy()


@pytest.mark.parametrize("prec,tol", [("fp32", 1e-5), ("fp16x3", 1e-5)])
def test_traced_resnet18_pt(spi, zoo, gpu, tmp_path, prec, tol):
    m = zoo.resnet18(image=64)
    path = str(tmp_path / "resnet18.pt")
    torch.jit.trace(m, torch.rand(1, 3, 64, 64)).save(path)
    loaded = spi.load_model(path)
    x = np.random.default_rng(11).random((4, 3, 64, 64), dtype=np.float32)
    ref = cpu_inference(loaded, [x])[0]
    rep = spi.ModelReplica(path, 0, prec, max_batch=4, image_size=64)
    got = hip(spi, rep, [x], ref.shape)
    err = normalized_max_error(got, ref)
    print(f".pt resnet18@64 {prec} err={err:.3e}")
    assert err < tol and top1_agreement(got, ref) == 1.0


@pytest.mark.parametrize("prec,tol", [("fp32", 1e-5), ("fp16", 1e-3)])
def test_traced_bert_pt(spi, zoo, gpu, tmp_path, prec, tol):
    m = zoo.bert(layers=2, init_std=0.05)
    path = str(tmp_path / "bert.pt")
    ex = (torch.randint(0, 30522, (1, 16)), torch.ones(1, 16, dtype=torch.int64))
    torch.jit.trace(m, ex, strict=False).save(path)
    loaded = spi.load_model(path)
    rng = np.random.default_rng(12)
    ids = rng.integers(0, 30522, (2, 16), dtype=np.int64)
    mask = np.ones((2, 16), dtype=np.int64)
    ref = cpu_inference(loaded, [ids, mask])[0]
    rep = spi.ModelReplica(path, 0, prec, max_batch=2, seq_len=128)
    got = hip(spi, rep, [ids, mask], ref.shape)
    err = normalized_max_error(got, ref)
    print(f".pt bert L2 S16 {prec} err={err:.3e}")
    assert err < tol
