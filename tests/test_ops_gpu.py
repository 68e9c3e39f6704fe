"""Kernel-level parity: each HIP kernel (include/spi_ops.h) vs a plain fp32
PyTorch reference of the same op.

Tolerances are normalised max-abs error (max|got - ref| / max|ref|):
fp32 (exact fp32 MFMA FMA chains) 1e-5; fp16x3 (split fp16) 1e-5; fp16 (fp16
operands rounded from the fp32 reference inputs, fp32 accumulation) 5e-3.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle.cpu_codelet import normalized_max_error

pytestmark = pytest.mark.gpu

TOL = {"fp32": 1e-5, "fp16x3": 1e-5, "fp16": 5e-3}
PRECS = ["fp32", "fp16", "fp16x3"]


@pytest.fixture(scope="module")
def ops(spi, gpu):
    import importlib
    return importlib.import_module("starpu-inference-server_amd.ops")


def test_gemm_identity_asymmetric(ops):
    """A = I with an asymmetric B catches a transposed C write (guide 3)."""
    for prec in PRECS:
        n = 64
        A = torch.eye(n, device="cuda").to(ops.act_dtype(prec))
        B = np.arange(n * n, dtype=np.float32).reshape(n, n) % 17 - 8  # exact in fp16
        out = ops.gemm(prec, A, ops.pack_weight(prec, B), n)
        np.testing.assert_array_equal(out.cpu().numpy(), B.T)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("M,N,K", [(1, 1000, 512), (8, 1000, 2048), (100, 72, 96), (1024, 768, 3072),
                                   (392, 512, 4608), (3152, 3072, 1024), (6144, 1000, 256)])
@pytest.mark.parametrize("act", [None, "relu", "gelu"])
def test_gemm_bias_residual_act(ops, prec, M, N, K, act):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    dt = ops.act_dtype(prec)
    A_in = A.to(dt)
    ref = A_in.float() @ (W.half().float() if prec == "fp16" else W).T + b + R
    ref = {None: ref, "relu": F.relu(ref), "gelu": F.gelu(ref)}[act]
    out = ops.gemm(prec, A_in.cuda(), ops.pack_weight(prec, W), N, bias=b.cuda(), residual=R.cuda(), act=act)
    err = normalized_max_error(out.cpu().numpy(), ref.numpy())
    assert err < TOL[prec], f"{prec} {M}x{N}x{K} {act}: {err:.3e}"


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("B,H,cin,cout,k,stride", [(2, 224, 3, 64, 7, 2), (3, 56, 64, 64, 3, 1), (2, 56, 64, 128, 3, 2),
                                                   (2, 14, 256, 512, 1, 2), (4, 7, 512, 512, 3, 1),
                                                   (1, 9, 16, 24, 3, 1),
                                                   # halo-band convs (kConvHalo): partial last band,
                                                   # odd sizes, 3-row bands, split-K over channel blocks
                                                   (2, 14, 128, 128, 3, 1), (2, 13, 64, 64, 3, 1),
                                                   (2, 40, 64, 64, 3, 1), (1, 28, 128, 256, 3, 1)])
def test_conv2d_nhwc(ops, prec, B, H, cin, cout, k, stride):
    g = torch.Generator().manual_seed(B * 1000 + H + cin + cout)
    x = torch.rand(B, cin, H, H, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    b = torch.randn(cout, generator=g)
    pad = k // 2
    cin_pad = max(cin, 8 if prec == "fp16" else 4)
    dt = ops.act_dtype(prec)
    x_nhwc = torch.zeros(B, H, H, cin_pad)
    x_nhwc[..., :cin] = x.permute(0, 2, 3, 1)
    x_in = x_nhwc.to(dt)
    w_ref = w.half().float() if prec == "fp16" else w
    ref = F.relu(F.conv2d(x_in[..., :cin].float().permute(0, 3, 1, 2), w_ref, b, stride, pad)).permute(0, 2, 3, 1)
    wp = ops.pack_weight(prec, ops.conv_weight_matrix(w, cin_pad))
    out = ops.conv2d(prec, x_in.cuda(), wp, cout, k, k, stride, pad, bias=b.cuda(), act="relu")
    err = normalized_max_error(out.float().cpu().numpy(), ref.numpy())
    tol = TOL[prec] if prec != "fp16" else 2e-3
    assert err < tol, f"{prec} conv {B}x{H}x{cin}->{cout} k{k}s{stride}: {err:.3e}"


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
@pytest.mark.parametrize("B,S,heads,masked", [(2, 128, 12, False), (3, 80, 4, True), (2, 197, 16, False),
                                              (1, 5, 2, False), (2, 64, 2, True), (2, 197, 3, True),
                                              (8, 128, 12, True), (2, 224, 3, True), (1, 225, 2, True),
                                              (2, 129, 2, True), (1, 161, 2, False)])
def test_attention(ops, prec, B, S, heads, masked):
    g = torch.Generator().manual_seed(B * S + heads)
    D = heads * 64
    qkv = torch.randn(B * S, 3 * D, generator=g) * 1.5
    dt = ops.act_dtype(prec)
    qkv_in = qkv.to(dt)
    q, k, v = qkv_in.float().view(B, S, 3, heads, 64).permute(2, 0, 3, 1, 4)
    bias = torch.zeros(B, S)
    if masked:
        bias[-1, S // 2:] = torch.finfo(torch.float32).min
        bias[0, :3] = torch.finfo(torch.float32).min
    scores = q @ k.transpose(-1, -2) * 0.125 + bias[:, None, None, :]
    ref = (scores.softmax(-1) @ v).permute(0, 2, 1, 3).reshape(B * S, D)
    ctx = ops.attention(prec, qkv_in.cuda(), B, S, heads, mask_bias=bias.cuda() if masked else None)
    err = normalized_max_error(ctx.float().cpu().numpy(), ref.numpy())
    tol = 1e-5 if prec == "fp32" else 3e-3
    assert err < tol, f"{prec} attention B{B} S{S} H{heads}: {err:.3e}"


@pytest.mark.parametrize("S", [129, 197, 224])
def test_attention_whole_sequence_staging_matches_tiles(ops, S):
    """Round 6: for 128 < S <= 224 the fp16 kernel stages the whole K / V once (SPI_ATTN_WHOLE=2,
    default: one 16-wave workgroup per head; =1 two 8-wave ones); the per-tile staging (=0) runs the same arithmetic in the same order: bit-identical."""
    B, heads = 2, 3
    g = torch.Generator().manual_seed(S)
    qkv = (torch.randn(B * S, 3 * heads * 64, generator=g) * 1.5).half().cuda()
    bias = torch.zeros(B, S)
    bias[1, S - 7:] = torch.finfo(torch.float32).min
    outs = {}
    try:
        for whole in ("1", "2", "0"):
            os.environ["SPI_ATTN_WHOLE"] = whole
            ops.lib.spi_debug_gemm_reload_env()
            outs[whole] = ops.attention("fp16", qkv, B, S, heads, mask_bias=bias.cuda()).cpu()
    finally:
        os.environ.pop("SPI_ATTN_WHOLE", None)
        ops.lib.spi_debug_gemm_reload_env()
    assert torch.equal(outs["1"], outs["0"]) and torch.equal(outs["2"], outs["0"])


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
def test_attention_fully_masked_row(ops, prec):
    """A fully masked row is uniform over the keys (finfo.min bias, as HF BERT)."""
    B, S, heads = 1, 16, 1
    qkv = torch.randn(B * S, 3 * 64).to(ops.act_dtype(prec))
    bias = torch.full((B, S), torch.finfo(torch.float32).min)
    ctx = ops.attention(prec, qkv.cuda(), B, S, heads, mask_bias=bias.cuda())
    v = qkv[:, 128:].float()
    tol = 1e-5 if prec == "fp32" else 2e-3
    np.testing.assert_allclose(ctx.float().cpu().numpy(), v.mean(0, keepdim=True).expand(S, 64).numpy(), rtol=tol,
                               atol=tol)


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
@pytest.mark.parametrize("rows,D,eps", [(1024, 768, 1e-12), (394, 1024, 1e-6), (3, 64, 1e-5)])
def test_layernorm(ops, prec, rows, D, eps):
    g = torch.Generator().manual_seed(rows + D)
    x = torch.randn(rows, D, generator=g) * 3 + 1
    gamma = torch.randn(D, generator=g)
    beta = torch.randn(D, generator=g)
    ref = F.layer_norm(x, (D,), gamma, beta, eps)
    yf, yt = ops.layernorm(prec, x.cuda(), gamma.cuda(), beta.cuda(), eps)
    assert normalized_max_error(yf.cpu().numpy(), ref.numpy()) < 2e-6
    if prec == "fp16":
        assert normalized_max_error(yt.float().cpu().numpy(), ref.numpy()) < 1e-3


# ---- fp16x3 on split activations (precision 3, the layout the fp16x3 ResNet forward keeps in HBM) ----

@pytest.mark.parametrize("B,H,cin,cout,k,stride,res", [(3, 56, 64, 64, 3, 1, True), (2, 56, 64, 128, 3, 2, False),
                                                       (2, 28, 128, 128, 3, 1, True), (2, 14, 256, 512, 1, 2, False),
                                                       (4, 7, 512, 512, 3, 1, True), (1, 9, 32, 96, 3, 1, True),
                                                       (2, 14, 128, 128, 3, 1, True), (2, 13, 64, 64, 3, 1, True),
                                                       (2, 40, 64, 64, 3, 1, False), (1, 9, 32, 128, 3, 1, True)])
def test_conv2d_split_layout(ops, B, H, cin, cout, k, stride, res):
    """Split A / residual / output conv (the tap-walk kernel of every fp16x3 ResNet conv
    but the stem) vs an fp32 conv on the values the split layout holds."""
    g = torch.Generator().manual_seed(B * 100 + H + cin + cout + k)
    x = torch.randn(B, H, H, cin, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    b = torch.randn(cout, generator=g)
    pad = k // 2
    oh = (H + 2 * pad - k) // stride + 1
    r = torch.randn(B, oh, oh, cout, generator=g) if res else None
    xs = ops.to_split(x)
    x_val = ops.from_split(xs)  # the values the kernel sees (hi + lo)
    ref = F.conv2d(x_val.permute(0, 3, 1, 2), w, b, stride, pad).permute(0, 2, 3, 1)
    if res:
        ref = ref + ops.from_split(ops.to_split(r))
    ref = F.relu(ref)
    wp = ops.pack_weight("fp16x3s", ops.conv_weight_matrix(w, cin))
    out = ops.conv2d("fp16x3s", xs.cuda(), wp, cout, k, k, stride, pad, bias=b.cuda(), act="relu",
                     residual=ops.to_split(r).cuda() if res else None)
    err = normalized_max_error(ops.from_split(out.cpu()).numpy(), ref.numpy())
    assert err < 1e-5, f"split conv {B}x{H}x{cin}->{cout} k{k}s{stride}: {err:.3e}"


def conv_plan(ops, prec_id, B, H, cin, cout, k=3, stride=1, pad=1):
    import ctypes as C
    out = (C.c_int * 8)()
    assert ops.lib.spi_debug_conv_plan(prec_id, B, H, H, cin, cout, k, k, stride, pad, out) == 0
    return dict(zip(("bm", "bn", "stages", "splits", "halo", "win", "nw", "k_per_split"), list(out)))


@pytest.mark.parametrize("prec", ["fp16", "fp16x3s"])
@pytest.mark.parametrize("B,H,cin,cout,res", [(8, 28, 128, 128, True), (8, 14, 256, 256, True), (8, 7, 512, 512, False),
                                              (3, 5, 64, 64, True), (2, 13, 128, 64, False), (1, 3, 64, 128, True),
                                              (5, 9, 64, 64, True), (32, 7, 512, 512, True), (1, 28, 128, 128, False),
                                              # 128 x 64 tiles (136-row windows)
                                              (32, 14, 256, 256, True), (16, 28, 128, 128, False)])
def test_conv3x3_window_kind(ops, prec, B, H, cin, cout, res):
    """kConvTapW (round 4): the 3x3/s1 tap walk whose three kw taps share one DMA'd window of
    BM + 2 consecutive pixels, taps in the padding zeroed at fragment read -- every 64x64 and
    128x64 tap plan of such a conv (split-K slices of whole (kh, channel block) super-steps; ragged M, maps 3 to
    28 wide, several images per tile).  Checked against an fp32 conv and against the plain tap
    walk (SPI_GEMM_WIN=0) and with the 64-row tiles as two K groups of 4 waves (SPI_GEMM_WIN=2 /
    3, round 5: 8-wave workgroups reducing through LDS); halo kinds and the weight-resident
    64->64 conv off so every shape takes it."""
    import os
    g = torch.Generator().manual_seed(B * 7 + H * 3 + cin + cout)
    x = torch.randn(B, H, H, cin, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g)
    r = torch.randn(B, H, H, cout, generator=g) if res else None
    split = prec == "fp16x3s"
    if split:
        xin, rin = ops.to_split(x), (ops.to_split(r) if res else None)
        x_val = ops.from_split(xin)
        r_val = ops.from_split(rin) if res else None
        w_ref = w
    else:
        xin, rin = x.half(), (r.half() if res else None)
        x_val, r_val, w_ref = xin.float(), (rin.float() if res else None), w.half().float()
    ref = F.conv2d(x_val.permute(0, 3, 1, 2), w_ref, b, 1, 1).permute(0, 2, 3, 1)
    if res:
        ref = ref + r_val
    ref = F.relu(ref)
    wp = ops.pack_weight(prec, ops.conv_weight_matrix(w, cin))
    outs = {}
    try:
        os.environ["SPI_GEMM_HALO_CFG"] = "0"
        os.environ["SPI_CONV_WRES"] = "0"
        for win in ("1", "0", "2", "3"):
            os.environ["SPI_GEMM_WIN"] = win
            ops.lib.spi_debug_gemm_reload_env()
            pl = conv_plan(ops, 3 if split else 1, B, H, cin, cout)
            assert pl["win"] == min(1, int(win)) and pl["bm"] in (64, 128), pl
            if win != "0":
                tiles128 = -(-B * H * H // 128) * -(-cout // 64)  # 128 x 64 tiles (plan target 128)
                assert pl["bm"] == (128 if tiles128 >= 128 else 64), pl
                # K groups (round 5): 64-row tiles whose 9 Cin / k-step steps split into an
                # even number of 3-step super-steps
                ksteps = 9 * cin // (32 if split else 64)
                kg = win in ("2", "3") and pl["bm"] == 64 and ksteps % 6 == 0
                assert pl["nw"] == (8 if kg else 4), pl
                if kg:
                    assert (pl["k_per_split"] // (32 if split else 64)) % 6 == 0, pl
            out = ops.conv2d(prec, xin.cuda(), wp, cout, 3, 3, 1, 1, bias=b.cuda(), act="relu",
                             residual=rin.cuda() if res else None)
            torch.cuda.synchronize()
            outs[win] = (ops.from_split(out.cpu()) if split else out.float().cpu())
    finally:
        os.environ.pop("SPI_GEMM_HALO_CFG", None)
        os.environ.pop("SPI_CONV_WRES", None)
        os.environ.pop("SPI_GEMM_WIN", None)
        ops.lib.spi_debug_gemm_reload_env()
    tol = 1e-5 if split else 2e-3
    for win, o in outs.items():
        err = normalized_max_error(o.numpy(), ref.numpy())
        assert err < tol, f"{prec} 3x3 conv B{B} H{H} {cin}->{cout} window={win}: {err:.3e}"


@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (100, 96, 160), (392, 512, 4608), (1024, 768, 3072),
                                   (3152, 3072, 1024)])
def test_gemm_split_layout(ops, M, N, K):
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    As, Rs = ops.to_split(A), ops.to_split(R)
    ref = ops.from_split(As) @ W.T + b + ops.from_split(Rs)
    out = ops.gemm("fp16x3s", As.cuda(), ops.pack_weight("fp16x3s", W), N, bias=b.cuda(), residual=Rs.cuda(),
                   out=torch.empty(M, N, device="cuda"))
    err = normalized_max_error(ops.from_split(out.cpu()).numpy(), ref.numpy())
    assert err < 1e-5, f"split gemm {M}x{N}x{K}: {err:.3e}"


def test_split_layout_rejects_bad_shapes(ops):
    x = torch.zeros(1, 8, 8, 16, device="cuda")
    wp = ops.pack_weight("fp16x3s", np.zeros((32, 9 * 16), np.float32))
    with pytest.raises(ops.OpError):
        ops.conv2d("fp16x3s", x, wp, 32, 3, 3, 1, 1)  # Cin 16 < 32


@pytest.mark.parametrize("prec", PRECS + ["fp16x3s"])
@pytest.mark.parametrize("B,HW,C,N", [(8, 49, 512, 1000), (3, 4, 512, 1000), (2, 49, 2048, 1000), (5, 64, 96, 70)])
def test_avgpool_fc_fused(ops, prec, B, HW, C, N):
    """ResNet's avgpool + fc as one GEMM launch (GemmDesc::pool_rows): the column mean of each
    image's pixel rows of A . W^T, plus bias -- vs fp32 torch mean-then-linear."""
    if prec == "fp16x3s" and C % 32:
        pytest.skip("split layout needs C % 32 == 0")
    g = torch.Generator().manual_seed(B * HW + C)
    x = torch.rand(B, HW, C, generator=g)
    W = torch.randn(N, C, generator=g) / C ** 0.5
    b = torch.randn(N, generator=g)
    base = "fp16x3" if prec == "fp16x3s" else prec
    xin = ops.to_split(x) if prec == "fp16x3s" else x.to(ops.act_dtype(prec))
    ref = xin.float().mean(1) if prec in ("fp32", "fp16") else x.mean(1)
    ref = ref @ (W.half().float() if prec == "fp16" else W).T + b
    out = ops.avgpool_fc(prec, xin.cuda(), ops.pack_weight(base, W), N, bias=b.cuda())
    err = normalized_max_error(out.cpu().numpy(), ref.numpy())
    assert err < TOL[base], f"{prec} B{B} HW{HW} C{C} N{N}: {err:.3e}"


# ---- halo-band candidates (SPI_GEMM_HALO_CFG): aligned / stacked bands, 64 / 128 / 256-row tiles ----

@pytest.fixture
def halo_cfg(ops):
    import os

    def set_cfg(cfg):
        if cfg:
            os.environ["SPI_GEMM_HALO_CFG"] = cfg
        else:
            os.environ.pop("SPI_GEMM_HALO_CFG", None)
        ops.lib.spi_debug_gemm_reload_env()

    yield set_cfg
    set_cfg("")


@pytest.mark.parametrize("cfg", ["64,a", "64,s", "128,a", "128,s", "256,a", "256,s"])
@pytest.mark.parametrize("B,H,cin,cout", [(8, 7, 512, 512), (3, 7, 64, 64), (2, 14, 128, 128), (3, 28, 64, 128),
                                          (1, 56, 64, 64), (5, 9, 32, 64), (4, 13, 64, 64)])
def test_conv_halo_candidates_split_layout(ops, halo_cfg, cfg, B, H, cin, cout):
    """Every halo candidate (bands spanning images in the stacked mode, split-K over
    channel blocks, the 8-wave 256-row kind) against an fp32 conv on the split values."""
    g = torch.Generator().manual_seed(B * 131 + H + cin + cout)
    x = torch.randn(B, H, H, cin, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    b = torch.randn(cout, generator=g)
    r = torch.randn(B, H, H, cout, generator=g)
    xs = ops.to_split(x)
    ref = F.conv2d(ops.from_split(xs).permute(0, 3, 1, 2), w, b, 1, 1).permute(0, 2, 3, 1)
    ref = F.relu(ref + ops.from_split(ops.to_split(r)))
    wp = ops.pack_weight("fp16x3s", ops.conv_weight_matrix(w, cin))
    halo_cfg(cfg)
    out = ops.conv2d("fp16x3s", xs.cuda(), wp, cout, 3, 3, 1, 1, bias=b.cuda(), act="relu",
                     residual=ops.to_split(r).cuda())
    err = normalized_max_error(ops.from_split(out.cpu()).numpy(), ref.numpy())
    assert err < 1e-5, f"halo {cfg} conv {B}x{H}x{cin}->{cout}: {err:.3e}"


@pytest.mark.parametrize("cfg", ["128,s", "256,s", "256,a"])
@pytest.mark.parametrize("B,H,cin,cout", [(8, 7, 512, 512), (2, 14, 256, 256)])
def test_conv_halo_candidates_fp16(ops, halo_cfg, cfg, B, H, cin, cout):
    g = torch.Generator().manual_seed(B * 7 + H + cin)
    x = torch.rand(B, cin, H, H, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    x_in = x.permute(0, 2, 3, 1).contiguous().half()
    ref = F.relu(F.conv2d(x_in.float().permute(0, 3, 1, 2), w.half().float(), None, 1, 1)).permute(0, 2, 3, 1)
    wp = ops.pack_weight("fp16", ops.conv_weight_matrix(w, cin))
    halo_cfg(cfg)
    out = ops.conv2d("fp16", x_in.cuda(), wp, cout, 3, 3, 1, 1, act="relu")
    err = normalized_max_error(out.float().cpu().numpy(), ref.numpy())
    assert err < 2e-3, f"fp16 halo {cfg} conv {B}x{H}x{cin}->{cout}: {err:.3e}"


def stem_pool_ref(x, w, b):
    """torchvision's conv1 (BN folded into w / b) + relu + maxpool, fp32."""
    return F.max_pool2d(F.relu(F.conv2d(x, w, b, stride=2, padding=3)), 3, 2, 1).permute(0, 2, 3, 1)


@pytest.mark.parametrize("prec", ["fp16", "fp16m", "fp16x3s", "fp16x3"])
@pytest.mark.parametrize("B,H,W,rows", [(8, 224, 224, 0), (8, 224, 224, 2), (3, 64, 64, 0), (1, 65, 47, 0),
                                        (2, 33, 17, 2), (1, 9, 9, 0), (2, 223, 224, 1)])
def test_stem_pool_fused(ops, prec, B, H, W, rows):
    """Fused stem (NCHW fp32 image -> 7x7/s2 conv + bias + ReLU -> 3x3/s2 max pool, one launch)
    vs F.conv2d / relu / max_pool2d: odd sizes exercise the partial column blocks, the pool's
    edge windows and a last workgroup with fewer pooled rows than rows_per_block.  fp16m is the
    stem the fp16m model runs (fp16 image x hi + lo weights; ADVICE r05: the op test had covered
    the split-image kernel only)."""
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + W + rows)
    x = torch.rand(B, 3, H, W, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    b = torch.randn(64, generator=g) * 0.1
    if prec == "fp16":
        ref = stem_pool_ref(x.half().float(), w.half().float(), b)
    elif prec == "fp16m":  # the image rounded to fp16, the weights at ~22 bits
        ref = stem_pool_ref(x.half().double(), w.double(), b.double()).float()
    else:
        ref = stem_pool_ref(x.double(), w.double(), b.double()).float()
    out = ops.stem_pool(prec, x.cuda(), w, b.cuda(), rows_per_block=rows)
    torch.cuda.synchronize()
    got = ops.from_split(out.cpu()) if prec == "fp16x3s" else out.float().cpu()
    assert got.shape == ref.shape
    err = normalized_max_error(got.numpy(), ref.numpy())
    # fp16 / fp16m store fp16 (relative 2^-11); fp16x3s stores hi + lo (~2^-22)
    tol = 1e-5 if prec == "fp16x3s" else 1e-3
    assert err < tol, f"stem_pool {prec} {B}x{H}x{W}: {err:.3e}"


@pytest.fixture(params=["1", "0,1,3", "0,1,2"], ids=["bm256", "bm128", "bm128b2"])
def gemm256_everywhere(ops, request):
    """Every eligible fp16 GEMM on gemm256.hip, at tile height 256 (SPI_GEMM_256_MIN=1) or 128
    (the 128 x 256 tile's two-phase loop on three k-tile buffers, =0,1,3, or two, =0,1,2)."""
    import os
    os.environ["SPI_GEMM_256_MIN"] = request.param
    ops.lib.spi_debug_gemm_reload_env()
    yield request.param
    os.environ.pop("SPI_GEMM_256_MIN", None)
    ops.lib.spi_debug_gemm_reload_env()


@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (100, 256, 64), (300, 512, 128), (256, 768, 192), (1000, 1024, 640),
                                   (3152, 1024, 4096), (1024, 2304, 768), (129, 256, 320)])
@pytest.mark.parametrize("act,res,out_f32", [(None, None, True), ("gelu", None, False), ("relu", "f16", False),
                                             (None, "f32", True)])
def test_gemm256_tiles(ops, gemm256_everywhere, M, N, K, act, res, out_f32):
    """The 8-wave phased GEMM (gemm256.hip) at both tile heights: one k-tile (the peeled last
    tile only), 2 to 5 k-tiles (every tail of the 128-row loop), ragged M, bias / GELU / ReLU,
    fp16 and fp32 residuals, fp16 and fp32 outputs."""
    g = torch.Generator().manual_seed(M * 3 + N + K)
    A = torch.randn(M, K, generator=g).half()
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = None
    if res:
        R = torch.randn(M, N, generator=g)
        R = R.half() if res == "f16" else R
    ref = A.float() @ W.half().float().T + b
    if R is not None:
        ref = ref + R.float()
    if act == "gelu":
        ref = F.gelu(ref)
    elif act == "relu":
        ref = F.relu(ref)
    out = ops.gemm("fp16", A.cuda(), ops.pack_weight("fp16", W), N, bias=b.cuda(),
                   residual=None if R is None else R.cuda(), out_f32=out_f32, act=act)
    torch.cuda.synchronize()
    err = normalized_max_error(out.float().cpu().numpy(), ref.numpy())
    assert err < (1e-5 if out_f32 else 2e-3), f"gemm256 {M}x{N}x{K} {act} {res}: {err:.3e}"


@pytest.mark.parametrize("router", ["everywhere", "longk"])
@pytest.mark.parametrize("M,N,K", [(3152, 1024, 4096), (3152, 1024, 1024), (300, 512, 128)])
def test_gemm256_in_place_residual(ops, gemm256_everywhere, router, M, N, K):
    """C is the fp32 residual buffer itself (the transformer's residual stream, updated in place)
    and M is ragged: rows past M in the last tile row must not be stored (a duplicate store of row
    M - 1 races with the real one and can add the GEMM twice).  `longk` runs with the default
    routing (SPI_GEMM_256_LONGK: ViT-L's FFN2 / out-projection shapes)."""
    import os
    if router == "longk":
        os.environ.pop("SPI_GEMM_256_MIN", None)
        ops.lib.spi_debug_gemm_reload_env()
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).half()
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    ref = A.float() @ W.half().float().T + b + R
    Rd = R.cuda()
    for _ in range(3):  # the race shows up on some launches only
        Rd.copy_(R.cuda())
        ops.gemm("fp16", A.cuda(), ops.pack_weight("fp16", W), N, bias=b.cuda(), residual=Rd, out=Rd, out_f32=True)
        torch.cuda.synchronize()
        err = normalized_max_error(Rd.cpu().numpy(), ref.numpy())
        assert err < 1e-5, f"in-place gemm {M}x{N}x{K} ({router}): {err:.3e}"


@pytest.mark.parametrize("maxsplit", ["1", "2", "3", "0"])
@pytest.mark.parametrize("M,N,K,res", [(600, 512, 4096, "f32"), (3152, 1024, 2048, None), (257, 256, 3072, "f16")])
def test_gemm256_split_k(ops, gemm256_everywhere, maxsplit, M, N, K, res):
    """gemm256's split-K (opt-in, SPI_GEMM_256_LONGK's third field; grids under 128 workgroups:
    slices of >= 16 k-tiles, at most 4; the
    last slice to arrive sums the write-through slabs in slice order).  SPI_GEMM_MAXSPLIT caps
    the slices (0 = uncapped: 4 for 600x512x4096, 2 for 3152x1024x2048, 3 for 257x256x3072;
    a cap of 3 on the first gives a short last slice).  The sum order does not depend on
    arrival: two launches agree bit for bit."""
    import os
    os.environ["SPI_GEMM_256_LONGK"] = "48,1024,4"  # split-K is opt-in (third field: slices)
    os.environ["SPI_GEMM_MAXSPLIT"] = maxsplit
    ops.lib.spi_debug_gemm_reload_env()
    try:
        g = torch.Generator().manual_seed(M + 7 * N + K)
        A = torch.randn(M, K, generator=g).half()
        W = torch.randn(N, K, generator=g) / K ** 0.5
        b = torch.randn(N, generator=g)
        R = None if res is None else torch.randn(M, N, generator=g)
        if res == "f16":
            R = R.half()
        ref = A.float() @ W.half().float().T + b + (0 if R is None else R.float())
        Wp = ops.pack_weight("fp16", W)
        outs = [ops.gemm("fp16", A.cuda(), Wp, N, bias=b.cuda(), residual=None if R is None else R.cuda(),
                         out_f32=True) for _ in range(2)]
        torch.cuda.synchronize()
        err = normalized_max_error(outs[0].cpu().numpy(), ref.numpy())
        assert err < 1e-5, f"gemm256 split-K {M}x{N}x{K} (max {maxsplit}): {err:.3e}"
        assert torch.equal(outs[0], outs[1]), "split-K sums depend on arrival order"
    finally:
        os.environ.pop("SPI_GEMM_MAXSPLIT", None)
        os.environ.pop("SPI_GEMM_256_LONGK", None)
        ops.lib.spi_debug_gemm_reload_env()


def test_gemm256_unaligned_output(ops, gemm256_everywhere):
    """An output buffer off 16-byte alignment takes gemm256's per-element epilogue."""
    M, N, K = 300, 512, 128
    g = torch.Generator().manual_seed(11)
    A = torch.randn(M, K, generator=g).half()
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    ref = F.gelu(A.float() @ W.half().float().T + b)
    out = torch.empty(M * N + 1, device="cuda", dtype=torch.float16)[1:].view(M, N)
    ops.gemm("fp16", A.cuda(), ops.pack_weight("fp16", W), N, bias=b.cuda(), out=out, out_f32=False, act="gelu")
    torch.cuda.synchronize()
    assert normalized_max_error(out.float().cpu().numpy(), ref.numpy()) < 2e-3


@pytest.mark.parametrize("B,H", [(8, 56), (1, 56), (3, 16), (2, 13), (2, 40), (5, 28), (1, 61), (32, 56), (19, 56)])
@pytest.mark.parametrize("res,act,bias", [(True, "relu", True), (False, "relu", True), (True, None, True),
                                          (False, None, False)])
def test_conv3x3_c64_weight_resident(ops, B, H, res, act, bias):
    """The weight-resident 64 -> 64 3x3 conv (conv_wres.hip, ResNet layer 1): bands of 2 rows at
    56 wide, 8 at 16 wide, partial last bands (13, 61), ResNet-152's bs32 grid (896 bands) and an
    odd band count (19 x 28), with / without the residual and ReLU, against an fp32 conv of the
    fp16-rounded operands."""
    g = torch.Generator().manual_seed(B * 100 + H)
    x = torch.rand(B, H, H, 64, generator=g).half()
    w = torch.randn(64, 64, 3, 3, generator=g) * (2.0 / 576) ** 0.5
    b = torch.randn(64, generator=g) if bias else None
    r = torch.randn(B, H, H, 64, generator=g).half() if res else None
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.half().float(), b, 1, 1).permute(0, 2, 3, 1)
    if res:
        ref = ref + r.float()
    if act == "relu":
        ref = F.relu(ref)
    wp = ops.pack_weight("fp16", ops.conv_weight_matrix(w, 64))
    import os
    try:  # every eligible conv (the default keeps the kernel for grids under 128 row tiles)
        os.environ["SPI_CONV_WRES"] = "2"
        ops.lib.spi_debug_gemm_reload_env()
        out = ops.conv2d("fp16", x.cuda(), wp, 64, 3, 3, 1, 1, bias=b.cuda() if bias else None,
                         residual=r.cuda() if res else None, act=act)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("SPI_CONV_WRES", None)
        ops.lib.spi_debug_gemm_reload_env()
    err = normalized_max_error(out.float().cpu().numpy(), ref.numpy())
    assert err < 2e-3, f"wres conv B{B} H{H} res={res} act={act}: {err:.3e}"
