"""GPU parity: the HIP codelet (through the C-ABI) vs the CPU codelet oracle.

Metric: normalised max-abs error max|hip - ref| / max|ref| plus top-1
agreement for classifiers (hard part 3).  Tolerances
(BASELINE.json north_star): fp32 1e-5; fp16 compute (fp16 MFMA operands, fp32
accumulation, fp32 residual stream / LN / softmax) 1e-3 for the model families
at the reference configs.  Inputs are seeded synthetic data shaped like the
reference's input generator (src/utils/input_generator.hpp:22-88).
"""
import numpy as np
import pytest
import torch

from oracle.cpu_codelet import cpu_inference, normalized_max_error, top1_agreement

pytestmark = pytest.mark.gpu

TOL = {"fp32": 1e-5, "fp16": 1e-3, "fp16x3": 1e-5, "fp16m": 1e-3}  # fp16x3 measures 1.6e-6 .. 3.2e-6 (fp32-grade)
# Plain fp16 operands on the random-init ResNets: rounding the MFMA operands
# alone gives ~1.7e-3 normalised max error (CPU emulation: fp16 weights 1.4e-3,
# fp16 activations 1.2e-3, both 1.67e-3 at ResNet-18 bs8@224).  That is the
# format's floor, not a kernel defect; fp16x3 (split-fp16 MFMA) is the
# parity-grade fp16 mode and is held to the 1e-3 bar (it lands near 1e-6).
TOL_RESNET_PLAIN_FP16 = 3e-3
# fp16m (SPI_PREC_F16M): plain fp16 everywhere except the stem (fp16 image x hi + lo weights)
# and the downsample convs (hi + lo weights); the FC on plain fp16 weights since round 5
# (DESIGN.md 3.2).  CPU emulation on ResNet-18 bs8@224 (tools/prec_emulate.py): worst case
# 0.74e-3 over eight input seeds (plain fp16 0.94e-3 .. 1.04e-3), GPU 0.60e-3 .. 0.69e-3;
# held to the north_star 1e-3 bar.
# Deep bottleneck nets amplify fp16 rounding (ResNet-152 emulated: fp16 11e-3, fp16m
# 6-7e-3), so C4 is served in fp16x3 and fp16m is held to the plain-fp16 bound there.
TOL_RESNET18_FP16M = 1e-3


def hip_forward(spi, replica, inputs, out_shape, graphs=False):
    ins = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in inputs]
    out = torch.full(out_shape, float("nan"), device="cuda", dtype=torch.float32)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    replica.set_graphs(graphs)
    spi.run_hip(replica, ins, out, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def image(rng, b, size):
    return rng.random((b, 3, size, size), dtype=np.float32)


def resnet_tol(prec, at_config=True):
    """at_config: ResNet-18 at the reference resolution (224), where fp16m is held to 1e-3.
    The reduced 64x64 / bottleneck cases sit at 1.1e-3 in fp16m (emulated 1.06e-3: activation
    rounding spread over every layer, no single layer dominates) and keep the plain-fp16 bound."""
    if prec == "fp16m":
        return TOL_RESNET18_FP16M if at_config else TOL_RESNET_PLAIN_FP16
    return TOL_RESNET_PLAIN_FP16 if prec == "fp16" else TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp16x3", "fp16m"])
def test_resnet18_small_image(spi, zoo, gpu, prec):
    rng = np.random.default_rng(0)
    m = zoo.resnet18(image=64)
    x = image(rng, 3, 64)
    ref = cpu_inference(m, [x])[0]
    rep = spi.ModelReplica(m, 0, prec, max_batch=4, image_size=64)
    got = hip_forward(spi, rep, [x], ref.shape)
    err = normalized_max_error(got, ref)
    print(f"resnet18@64 {prec} err={err:.3e}")
    assert np.isfinite(got).all()
    assert err < resnet_tol(prec, at_config=False)
    assert top1_agreement(got, ref) == 1.0


@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp16x3", "fp16m"])
def test_resnet_bottleneck_small(spi, zoo, gpu, prec):
    rng = np.random.default_rng(1)
    m = zoo.resnet([1, 2, 2, 1], True, image=64)
    x = image(rng, 2, 64)
    ref = cpu_inference(m, [x])[0]
    rep = spi.ModelReplica(m, 0, prec, max_batch=2, image_size=64)
    got = hip_forward(spi, rep, [x], ref.shape)
    err = normalized_max_error(got, ref)
    print(f"resnet-bottleneck@64 {prec} err={err:.3e}")
    assert err < resnet_tol(prec, at_config=False)


@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp16x3", "fp16m"])
def test_resnet18_full_bs8(spi, zoo, gpu, prec):
    """C2: ResNet-18 bs=8 at 224x224."""
    rng = np.random.default_rng(2)
    m = zoo.resnet18()
    x = image(rng, 8, 224)
    ref = cpu_inference(m, [x])[0]
    rep = spi.ModelReplica(m, 0, prec, max_batch=8)
    got = hip_forward(spi, rep, [x], ref.shape)
    got_g = hip_forward(spi, rep, [x], ref.shape, graphs=True)
    err = normalized_max_error(got, ref)
    print(f"resnet18@224 bs8 {prec} err={err:.3e}")
    assert err < resnet_tol(prec)
    assert top1_agreement(got, ref) == 1.0
    np.testing.assert_array_equal(got, got_g)


@pytest.mark.parametrize("seed", [3, 7, 11])
def test_resnet18_fp16m_c2_seeds(spi, zoo, gpu, seed):
    """C2 in the fp16m mode over more input draws (the 1e-3 bar, top-1 agreement)."""
    m = zoo.resnet18()
    x = image(np.random.default_rng(seed), 8, 224)
    ref = cpu_inference(m, [x])[0]
    rep = spi.ModelReplica(m, 0, "fp16m", max_batch=8)
    got = hip_forward(spi, rep, [x], ref.shape, graphs=True)
    err = normalized_max_error(got, ref)
    print(f"resnet18@224 bs8 fp16m seed{seed} err={err:.3e}")
    assert err < TOL_RESNET18_FP16M
    assert top1_agreement(got, ref) == 1.0


@pytest.mark.parametrize("win", ["2", "3"])
def test_resnet18_fp16m_window_kgroups(spi, zoo, gpu, win, monkeypatch):
    """C2 with the layer-2..4 3x3 convs on the window kind's two-K-group (8-wave) tiles
    (SPI_GEMM_WIN=2: the 4-wave plan's split-K slices, 3: half of them)."""
    m = zoo.resnet18()
    x = image(np.random.default_rng(5), 8, 224)
    ref = cpu_inference(m, [x])[0]
    monkeypatch.setenv("SPI_GEMM_WIN", win)
    spi.lib.spi_debug_gemm_reload_env()
    try:
        rep = spi.ModelReplica(m, 0, "fp16m", max_batch=8)
        got = hip_forward(spi, rep, [x], ref.shape)
        got_g = hip_forward(spi, rep, [x], ref.shape, graphs=True)
    finally:
        monkeypatch.delenv("SPI_GEMM_WIN")
        spi.lib.spi_debug_gemm_reload_env()
    err = normalized_max_error(got, ref)
    print(f"resnet18@224 bs8 fp16m win={win} err={err:.3e}")
    assert err < TOL_RESNET18_FP16M
    assert top1_agreement(got, ref) == 1.0
    np.testing.assert_array_equal(got, got_g)


def bert_inputs(rng, b, s, vocab=30522, pad_from=None):
    ids = rng.integers(0, vocab, size=(b, s), dtype=np.int64)
    mask = np.ones((b, s), dtype=np.int64)
    if pad_from is not None:
        mask[-1, pad_from:] = 0
    return ids, mask


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
def test_bert_two_layers_masked(spi, zoo, gpu, prec):
    rng = np.random.default_rng(3)
    m = zoo.bert(layers=2, init_std=0.05)
    ids, mask = bert_inputs(rng, 3, 80, pad_from=50)
    ref = cpu_inference(m, [ids, mask])[0]
    rep = spi.ModelReplica(m, 0, prec, max_batch=3, seq_len=128)
    got = hip_forward(spi, rep, [ids, mask], ref.shape)
    err = normalized_max_error(got, ref)
    print(f"bert L2 S80 masked {prec} err={err:.3e}")
    assert err < TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp16m"])
def test_bert_base_seq128_bs8(spi, zoo, gpu, prec):
    """C3: bert-base-uncased seq=128 bs=8 (mask all ones)."""
    rng = np.random.default_rng(4)
    m = zoo.bert_base()
    ids, mask = bert_inputs(rng, 8, 128)
    ref = cpu_inference(m, [ids, mask])[0]
    rep = spi.ModelReplica(m, 0, prec, max_batch=8, seq_len=128)
    got = hip_forward(spi, rep, [ids, mask], ref.shape)
    err = normalized_max_error(got, ref)
    print(f"bert-base S128 bs8 {prec} err={err:.3e}")
    assert err < TOL[prec]


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
def test_vit_small_seq197(spi, zoo, gpu, prec):
    """ViT at 224/16 (S=197: three full 64-key tiles + a 5-key tail), small width."""
    rng = np.random.default_rng(5)
    m = zoo.vit(image=224, patch=16, layers=2, heads=2, dim=128, mlp_dim=256)
    x = image(rng, 2, 224)
    ref = cpu_inference(m, [x])[0]
    rep = spi.ModelReplica(m, 0, prec, max_batch=2)
    got = hip_forward(spi, rep, [x], ref.shape)
    err = normalized_max_error(got, ref)
    print(f"vit-small S197 {prec} err={err:.3e}")
    assert err < TOL[prec]


@pytest.mark.parametrize("prec", ["fp16", "fp16m"])
@pytest.mark.parametrize("family", ["bert", "vit"])
def test_transformer_layernorm_fold(spi, zoo, gpu, family, prec, monkeypatch):
    """The LayerNorm fold (ln_fold.hpp, DESIGN.md 3.6: statistics from the producing GEMM's
    epilogue, gain folded into the consuming GEMM's weights, post-LN residuals recomputed
    element-wise, the two-plane residual rows of round 6) against the separate LayerNorm launches
    (SPI_LN_FOLD=0) and the oracle, every path at the 1e-3 bar; the folded forward runs at most two
    LayerNorm launches.  fp16m's BERT is drawn wider than HF's init (std 0.05: larger activations
    and row means), where plain fp16 arithmetic itself -- folded or not -- sits at the bar (CPU
    emulation, tools/prec_emulate_bert.py: unfused 1.00e-3, folded 1.04e-3, spread over every
    rounding site); plain fp16 runs HF's init here, and its fold is stressed by the
    outlier-dimension and large-row-mean fixtures of test_bert_layernorm_fold_outliers."""
    rng = np.random.default_rng(13)
    if family == "bert":
        m = zoo.bert(layers=3, init_std=0.05 if prec == "fp16m" else 0.02)
        ids, mask = bert_inputs(rng, 3, 80, pad_from=50)
        inputs, kw = [ids, mask], dict(max_batch=3, seq_len=128)
    else:
        m = zoo.vit(image=224, patch=16, layers=3, heads=2, dim=128, mlp_dim=256)
        inputs, kw = [image(rng, 2, 224)], dict(max_batch=2)
    ref = cpu_inference(m, inputs)[0]
    monkeypatch.setenv("SPI_LN_FOLD", "1")  # whatever the family's default
    rep = spi.ModelReplica(m, 0, prec, **kw)
    folded = hip_forward(spi, rep, inputs, ref.shape, graphs=True)
    ins = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in inputs]
    out = torch.empty(ref.shape, device="cuda")
    ops = rep.profile(ins, out, torch.cuda.current_stream().cuda_stream)
    n_ln = sum(1 for o in ops if o["name"].startswith("layernorm"))
    monkeypatch.setenv("SPI_LN_FOLD", "0")
    plain = hip_forward(spi, spi.ModelReplica(m, 0, prec, **kw), inputs, ref.shape)
    d = normalized_max_error(folded, plain)
    e_f, e_p = normalized_max_error(folded, ref), normalized_max_error(plain, ref)
    print(f"{family} {prec} LN fold: vs unfused {d:.3e}, vs oracle {e_f:.3e} (unfused {e_p:.3e}), LN launches {n_ln}")
    assert n_ln <= 2
    assert e_f < 1e-3 and e_p < 1e-3 and d < 1e-3, (e_f, e_p, d)


def bert_with_outliers(zoo, kind, layers=3):
    """BERT at HF's init (std 0.02) with the LayerNorm structure that makes trained checkpoints hard
    for fp16: "dims" -- three outlier dimensions (gain 8, bias +-3 in every
    LayerNorm: the residual stream carries a few features an order of magnitude above the rest,
    as in pretrained BERT); "offset" -- every LayerNorm bias shifted by +2 (rows whose mean is twice
    their spread: the folded form's cancellation case, rstd (x W' - mean c1))."""
    m = zoo.bert(layers=layers)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.LayerNorm):
                if kind == "dims":
                    for d, sgn in ((17, 1.0), (308, -1.0), (555, 1.0)):
                        mod.weight[d] = 8.0
                        mod.bias[d] = 3.0 * sgn
                else:
                    mod.bias.add_(2.0)
    return m


@pytest.mark.parametrize("kind", ["dims", "offset"])
def test_bert_layernorm_fold_outliers(spi, zoo, gpu, kind, monkeypatch):
    """The plain-fp16 LayerNorm fold (C3's serving path) on outlier-dimension and large-row-mean
    BERT (bert_with_outliers) against the separate LayerNorm launches and the oracle, at the
    north_star 1e-3 bar."""
    rng = np.random.default_rng(17)
    m = bert_with_outliers(zoo, kind)
    ids, mask = bert_inputs(rng, 3, 80, pad_from=50)
    ref = cpu_inference(m, [ids, mask])[0]
    kw = dict(max_batch=3, seq_len=128)
    monkeypatch.setenv("SPI_LN_FOLD", "1")
    folded = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", **kw), [ids, mask], ref.shape, graphs=True)
    monkeypatch.setenv("SPI_LN_FOLD", "0")
    plain = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", **kw), [ids, mask], ref.shape)
    d = normalized_max_error(folded, plain)
    e_f, e_p = normalized_max_error(folded, ref), normalized_max_error(plain, ref)
    # the outlier features set max|ref|: hold the ordinary features to the bar on their own scale too
    keep = np.ones(ref.shape[-1], bool)
    keep[[17, 308, 555]] = False
    e_k = normalized_max_error(folded[..., keep], ref[..., keep])
    print(f"bert outliers {kind} fp16 LN fold: vs unfused {d:.3e}, vs oracle {e_f:.3e} (unfused {e_p:.3e}), "
          f"ordinary features {e_k:.3e}")
    assert e_f < 1e-3 and e_p < 1e-3 and d < 1e-3 and e_k < 1e-3, (e_f, e_p, d, e_k)


@pytest.mark.parametrize("family", ["vit", "bert"])
@pytest.mark.parametrize("route", ["0,1,3", "0,1,2", "1"], ids=["bm128", "bm128b2", "bm256"])
def test_transformer_layernorm_fold_on_gemm256(spi, zoo, gpu, family, route, monkeypatch):
    """The LayerNorm fold's gemm256 epilogues (consumer statistics + c1 on QKV / FFN1, producer
    chunk statistics + fp16 copy on ViT's out-proj / FFN2; BERT's post-LN producers stay on the
    general kernel) at width 256, every eligible GEMM forced onto gemm256 at tile height 128
    (SPI_GEMM_256_MIN=0,1) or 256 (=1), 394 / 240 token rows (ragged last tile row): folded
    vs the separate LayerNorm launches on the same kernels, and both vs the oracle."""
    rng = np.random.default_rng(29)
    if family == "bert":
        m = zoo.bert(layers=2, hidden=256, heads=4, intermediate=1024)
        ids, mask = bert_inputs(rng, 3, 80, pad_from=50)
        inputs, kw = [ids, mask], dict(max_batch=3, seq_len=128)
    else:
        m = zoo.vit(image=224, patch=16, layers=2, heads=4, dim=256, mlp_dim=512)
        inputs, kw = [image(rng, 2, 224)], dict(max_batch=2)
    ref = cpu_inference(m, inputs)[0]
    monkeypatch.setenv("SPI_GEMM_256_MIN", route)
    monkeypatch.setenv("SPI_LN_FOLD", "1")
    spi.lib.spi_debug_gemm_reload_env()
    try:
        folded = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", **kw), inputs, ref.shape)
        monkeypatch.setenv("SPI_LN_FOLD", "0")
        plain = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", **kw), inputs, ref.shape)
    finally:
        monkeypatch.delenv("SPI_GEMM_256_MIN")
        spi.lib.spi_debug_gemm_reload_env()
    d = normalized_max_error(folded, plain)
    e_f, e_p = normalized_max_error(folded, ref), normalized_max_error(plain, ref)
    print(f"{family} gemm256 {route} LN fold: vs unfused {d:.3e}, vs oracle {e_f:.3e} (unfused {e_p:.3e})")
    assert e_f < 1e-3 and e_p < 1e-3 and d < 1e-3, (e_f, e_p, d)


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("S,pad_from", [(128, None), (80, 50), (16, 9), (128, 100)])
def test_bert_qkv_attention_fused(spi, zoo, gpu, S, pad_from, fold, monkeypatch):
    """The fused QKV projection + attention kernel (qkv_attn.hip: one workgroup per (sequence,
    head), the head's q | k | v GEMM, then the attention on the LDS-resident Q / K / V) against
    the QKV GEMM + attention launches it replaces (SPI_QKV_ATTN=0) and the oracle: full and
    ragged sequences (S < 128: rows past S clamped and zeroed), padding masks, with and without
    the LayerNorm consumer fold on the QKV GEMM."""
    rng = np.random.default_rng(31 + S)
    m = zoo.bert(layers=2)
    ids, mask = bert_inputs(rng, 3, S, pad_from=pad_from)
    ref = cpu_inference(m, [ids, mask])[0]
    monkeypatch.setenv("SPI_LN_FOLD", fold)
    fused = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", max_batch=3, seq_len=128), [ids, mask], ref.shape)
    monkeypatch.setenv("SPI_QKV_ATTN", "0")
    plain = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", max_batch=3, seq_len=128), [ids, mask], ref.shape)
    d = normalized_max_error(fused, plain)
    e = normalized_max_error(fused, ref)
    print(f"qkv+attention fused S{S} pad{pad_from} fold{fold}: vs unfused {d:.3e} (identical: {np.array_equal(fused, plain)}), "
          f"vs oracle {e:.3e}")
    assert e < 1e-3 and d < 2e-4, (e, d)


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("S,pad_from", [(128, None), (80, 50), (16, 9)])
def test_bert_qkv_attention_two_heads_per_workgroup(spi, zoo, gpu, S, pad_from, fold, monkeypatch):
    """SPI_QKV_HP=2 (round 6): two heads per 16-wave workgroup, the A rows staged once for both
    heads' W rows; each head's arithmetic is the one-head kernel's, so the outputs are identical."""
    rng = np.random.default_rng(41 + S)
    m = zoo.bert(layers=2)
    ids, mask = bert_inputs(rng, 3, S, pad_from=pad_from)
    ref = cpu_inference(m, [ids, mask])[0]
    monkeypatch.setenv("SPI_LN_FOLD", fold)
    outs = {}
    try:
        for hp in ("2", "1"):
            monkeypatch.setenv("SPI_QKV_HP", hp)
            spi.lib.spi_debug_gemm_reload_env()
            outs[hp] = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", max_batch=3, seq_len=128), [ids, mask],
                                   ref.shape)
    finally:
        monkeypatch.delenv("SPI_QKV_HP")
        spi.lib.spi_debug_gemm_reload_env()
    e = normalized_max_error(outs["2"], ref)
    assert np.array_equal(outs["2"], outs["1"]) and e < 1e-3, e


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("img,patch", [(224, 16), (240, 16), (160, 16), (224, 14)])
def test_vit_qkv_attention_fused(spi, zoo, gpu, img, patch, fold, monkeypatch):
    """The fused QKV projection + attention kernel on ViT (round 6: 256-row tiles for 129..256
    tokens, SPI_QKV_ATTN=2 -- S = 197 at 224/16, 226 at 240/16; 101 at 160/16 takes the 128-row
    tile; 257 at 224/14 falls back to the two launches) against SPI_QKV_ATTN=0 and the oracle,
    with and without the LayerNorm fold."""
    rng = np.random.default_rng(37 + img + patch)
    m = zoo.vit(image=img, patch=patch, layers=2, heads=4, dim=256, mlp_dim=512)
    x = image(rng, 2, img)
    ref = cpu_inference(m, [x])[0]
    monkeypatch.setenv("SPI_LN_FOLD", fold)
    monkeypatch.setenv("SPI_QKV_ATTN", "2")
    rep = spi.ModelReplica(m, 0, "fp16", max_batch=2, image_size=img)
    fused = hip_forward(spi, rep, [x], ref.shape)
    ins = [torch.from_numpy(np.ascontiguousarray(x)).cuda()]
    ops = rep.profile(ins, torch.empty(ref.shape, device="cuda"), torch.cuda.current_stream().cuda_stream)
    names = {o["name"] for o in ops}
    monkeypatch.setenv("SPI_QKV_ATTN", "0")
    plain = hip_forward(spi, spi.ModelReplica(m, 0, "fp16", max_batch=2, image_size=img), [x], ref.shape)
    S = (img // patch) ** 2 + 1
    d = normalized_max_error(fused, plain)
    e = normalized_max_error(fused, ref)
    print(f"vit qkv+attention fused S{S} fold{fold}: vs unfused {d:.3e} (identical: {np.array_equal(fused, plain)}), "
          f"vs oracle {e:.3e}, ops {sorted(n for n in names if 'att' in n)}")
    assert (f"qkv_attention_S{S}" in names) == (S <= 256)
    # the unfused QKV GEMM runs on gemm256 here (a different k order than the fused kernel's, so
    # some fp16 roundings of Q / K / V flip): 2.2e-4 measured at S = 197 with the fold
    assert e < 1e-3 and d < 5e-4, (e, d)


def test_affine_codelet_like_reference(spi, gpu):
    """x + 1.5 on {1,2,3} (tests/unit/core/unit_starpu_setup.cpp:2332-2433)."""
    rep = spi.ModelReplica(None, 0, "fp32", max_batch=3, family="affine", affine=(1.0, 1.5))
    x = torch.tensor([1.0, 2.0, 3.0], device="cuda")
    out = torch.zeros(3, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    params = spi.make_params([[3]], [torch.float32], models_gpu=[rep])
    bufs = [spi.make_variable_interface(x.data_ptr(), 12), spi.make_variable_interface(out.data_ptr(), 12)]
    with spi.worker_context(77, 0, stream.cuda_stream):
        args = spi.InferenceCodelet.hip_inference_func(bufs, params)
    stream.synchronize()
    assert out.cpu().tolist() == [2.5, 3.5, 4.5]
    assert args.device_id == 0 and args.worker_id == 77 and args.executed_on == 2
    assert args.codelet_start_ns > 0 and args.codelet_end_ns >= args.codelet_start_ns


GOLDEN_FIXTURES = ["resnet18_img64_b2", "resnet_bottleneck_1221_img64_b2", "bert_L2_S16_b2_masked",
                   "vit_img32_p16_L2_D128_b2"]


@pytest.mark.parametrize("name", GOLDEN_FIXTURES)
@pytest.mark.parametrize("prec", ["fp32", "fp16x3", "fp16"])
def test_hip_matches_committed_golden_fixtures(spi, gpu, name, prec):
    """HIP codelet vs the committed CPU-oracle fixtures (tests/golden/make_golden.py)."""
    import importlib
    import os
    import sys
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, golden)
    mk = importlib.import_module("make_golden")
    g = np.load(os.path.join(golden, "models.npz"))
    model, _ = mk.SMALL[name]()
    inputs = [g[f"{name}__in{i}"] for i in range(2) if f"{name}__in{i}" in g]
    ref = g[f"{name}__out"]
    kw = {"image_size": inputs[0].shape[-1]} if inputs[0].ndim == 4 else {"seq_len": 128}
    rep = spi.ModelReplica(model, 0, prec, max_batch=2, **kw)
    got = hip_forward(spi, rep, inputs, ref.shape)
    err = normalized_max_error(got, ref)
    # plain fp16 operands: the north_star 1e-3 bar on BERT (8.6e-4 measured); the tiny random
    # ResNets / ViT-D128 sit at their format floor (2.4e-3 / 1.1e-3), see TOL_RESNET_PLAIN_FP16
    tol = {"fp32": 1e-5, "fp16x3": 1e-5, "fp16": 1e-3 if name.startswith("bert") else TOL_RESNET_PLAIN_FP16}[prec]
    print(f"golden {name} {prec} err={err:.3e}")
    assert err < tol


@pytest.mark.parametrize("prec", ["fp16", "fp16x3", "fp16m"])
def test_resnet18_fused_stem_matches_unfused(spi, zoo, gpu, prec, monkeypatch):
    """The fused stem (one launch on the NCHW input) against the ingest + stem GEMM + max pool
    path (SPI_STEM_FUSED=0) on the same replica weights: the same numbers up to the
    accumulation order of the 147-term stem dot products."""
    rng = np.random.default_rng(5)
    m = zoo.resnet18(image=224)
    x = image(rng, 2, 224)
    ref = cpu_inference(m, [x])[0]
    fused = hip_forward(spi, spi.ModelReplica(m, 0, prec, max_batch=2), [x], ref.shape)
    monkeypatch.setenv("SPI_STEM_FUSED", "0")
    unfused = hip_forward(spi, spi.ModelReplica(m, 0, prec, max_batch=2), [x], ref.shape)
    d = normalized_max_error(fused, unfused)
    print(f"resnet18 {prec} fused vs unfused stem: {d:.3e}, vs oracle {normalized_max_error(fused, ref):.3e}")
    assert d < (1e-5 if prec == "fp16x3" else 1e-3)
    assert normalized_max_error(fused, ref) < resnet_tol(prec)


def test_resnet18_wide_image_unfused_stem(spi, zoo, gpu):
    """Images wider than 224 (stem output > 112 columns) take the ingest + stem GEMM + max pool path."""
    rng = np.random.default_rng(9)
    m = zoo.resnet18(image=240)
    x = image(rng, 1, 240)
    ref = cpu_inference(m, [x])[0]
    got = hip_forward(spi, spi.ModelReplica(m, 0, "fp16m", max_batch=1, image_size=240), [x], ref.shape)
    assert normalized_max_error(got, ref) < TOL_RESNET_PLAIN_FP16
