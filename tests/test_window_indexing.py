"""Host-side check of the kw-window tap walk's indexing (gemm.hip kConvTapW).

For a 3x3 / stride-1 / padding-1 conv the kernel reads, per (kh, channel block) of a 64-row
tile starting at output row m0, the 72 global pixels from m0 + (kh - 1) W - 1 on (rows outside
[0, M) as zeros), feeds tap kw of tile row r from window row r + kw, and zeroes taps outside the
image by a 9-bit per-row mask built from (oh, ow) the way the kernel builds it.  This restates
that indexing in numpy and compares it with a direct convolution, so the derivation is pinned
on the CPU (the GPU parity test is tests/test_ops_gpu.py::test_conv3x3_window_kind)."""
import numpy as np
import pytest


def window_conv(x, w, B, H, W):
    M, cin = x.shape
    cout = w.shape[0]
    out = np.zeros((M, cout))
    rows = np.arange(64)
    for m0 in range(0, M, 64):
        m = m0 + rows
        valid = m < M
        mm = np.where(valid, m, 0)
        img = mm // (H * W)
        rem = mm - img * H * W
        oh, ow = rem // W, rem % W
        cols = (ow > 0).astype(np.int64) | 2 | ((ow + 1 < W).astype(np.int64) << 2)
        mask = np.where(oh > 0, cols, 0) | (cols << 3) | np.where(oh + 1 < H, cols << 6, 0)
        mask = np.where(valid, mask, 0)
        acc = np.zeros((64, cout))
        for kh in range(3):
            pix = m0 + (kh - 1) * W - 1 + np.arange(72)
            win = np.where(((pix >= 0) & (pix < M))[:, None], x[np.clip(pix, 0, M - 1)], 0.0)
            for kw in range(3):
                ok = ((mask >> (kh * 3 + kw)) & 1) == 1
                acc += np.where(ok[:, None], win[rows + kw], 0.0) @ w[:, kh, kw].T
        out[m[valid]] = acc[valid]
    return out


def direct_conv(x, w, B, H, W):
    cin = x.shape[1]
    xp = np.zeros((B, H + 2, W + 2, cin))
    xp[:, 1:-1, 1:-1] = x.reshape(B, H, W, cin)
    out = np.zeros((B, H, W, w.shape[0]))
    for kh in range(3):
        for kw in range(3):
            out += np.einsum("bhwc,nc->bhwn", xp[:, kh:kh + H, kw:kw + W], w[:, kh, kw])
    return out.reshape(B * H * W, -1)


@pytest.mark.parametrize("B,H,W", [(2, 7, 7), (3, 14, 14), (1, 5, 9), (2, 13, 3), (8, 7, 7), (1, 3, 3), (2, 28, 28)])
def test_window_indexing_matches_direct_conv(B, H, W):
    rng = np.random.default_rng(B * 100 + H * 10 + W)
    x = rng.standard_normal((B * H * W, 4))
    w = rng.standard_normal((5, 3, 3, 4))
    np.testing.assert_allclose(window_conv(x, w, B, H, W), direct_conv(x, w, B, H, W), atol=1e-12)
