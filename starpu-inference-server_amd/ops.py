"""Op-level wrappers over include/spi_ops.h (kernel parity tests, micro-benchmarks).

Every call goes to libspi_hip.so; tensors are torch device tensors used as
plain HBM buffers (torch shares the process's HIP runtime, see _native.py).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as N
from ._native import lib

PREC = {"fp32": 0, "fp16": 1, "fp16x3": 2, "fp16x3s": 3}  # fp16x3s: split activation layout
ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2}


class OpError(RuntimeError):
    pass


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _check(rc):
    if rc != 0:
        raise OpError(N.last_error())


def act_dtype(prec: str) -> torch.dtype:
    return torch.float16 if prec == "fp16" else torch.float32


def to_split(x: torch.Tensor) -> torch.Tensor:
    """fp32 [..., C] (C % 32 == 0) -> the split layout (fp16x3s operands), stored in a
    float32 tensor of the same shape: per 32-channel block [32 hi fp16 | 32 lo fp16]."""
    x = x.float().contiguous()
    hi = x.half()
    lo = (x - hi.float()).half()
    blk = x.shape[-1] // 32
    s = torch.cat([hi.reshape(*x.shape[:-1], blk, 32), lo.reshape(*x.shape[:-1], blk, 32)], dim=-1)
    return s.contiguous().view(torch.float32).reshape(x.shape)


def from_split(s: torch.Tensor) -> torch.Tensor:
    """Inverse of to_split: hi + lo in fp32."""
    blk = s.shape[-1] // 32
    h = s.contiguous().view(torch.float16).reshape(*s.shape[:-1], blk, 64)
    return (h[..., :32].float() + h[..., 32:].float()).reshape(s.shape)


def pack_weight(prec: str, w: np.ndarray | torch.Tensor, device="cuda") -> torch.Tensor:
    """[N][K] fp32 -> packed device buffer (uint8 tensor)."""
    w = np.ascontiguousarray(np.asarray(w.cpu() if isinstance(w, torch.Tensor) else w, dtype=np.float32))
    n, k = w.shape
    npad, kpad = C.c_int32(), C.c_int32()
    nbytes = lib.spi_op_packed_bytes(PREC[prec], n, k, C.byref(npad), C.byref(kpad))
    host = np.empty(nbytes, dtype=np.uint8)
    _check(lib.spi_op_pack_weight(PREC[prec], w.ctypes.data, n, k, host.ctypes.data))
    return torch.from_numpy(host).to(device)


def conv_weight_matrix(w: torch.Tensor, cin_pad: int) -> np.ndarray:
    """torch conv weight [Cout][Cin][KH][KW] -> [Cout][KH*KW*cin_pad] (k = (kh*KW+kw)*cin_pad + c)."""
    cout, cin, kh, kw = w.shape
    m = torch.zeros(cout, kh, kw, cin_pad)
    m[..., :cin] = w.permute(0, 2, 3, 1)
    return m.reshape(cout, kh * kw * cin_pad).numpy()


def workspace(device="cuda") -> torch.Tensor:
    return torch.zeros(lib.spi_op_workspace_bytes(), dtype=torch.uint8, device=device)


def gemm(prec, A, W_packed, N_, bias=None, residual=None, out=None, out_f32=True, act=None, ws=None,
         stream=None, res_f32=None):
    M, K = A.shape
    if out is None:
        out = torch.empty(M, N_, device=A.device, dtype=torch.float32 if out_f32 else act_dtype(prec))
    split = prec == "fp16x3s"  # float32-storage tensors holding the split layout, not fp32 values
    if res_f32 is None:
        res_f32 = residual is not None and residual.dtype == torch.float32 and not split
    ws = workspace(A.device) if ws is None else ws
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    _check(lib.spi_op_gemm(PREC[prec], _ptr(A), M, K, A.stride(0), _ptr(W_packed), N_, _ptr(bias), _ptr(residual),
                           int(res_f32), residual.stride(0) if residual is not None else 0, _ptr(out),
                           int(out.dtype == torch.float32 and not split), out.stride(0), ACT[act], _ptr(ws), C.c_void_p(s)))
    return out


def conv2d(prec, x_nhwc, W_packed, cout, kh, kw, stride, pad, bias=None, residual=None, act=None, ws=None,
           stream=None, out=None):
    B, H, W_, cin = x_nhwc.shape
    oh, ow = (H + 2 * pad - kh) // stride + 1, (W_ + 2 * pad - kw) // stride + 1
    if out is None:
        out = torch.empty(B, oh, ow, cout, device=x_nhwc.device, dtype=x_nhwc.dtype)
    ws = workspace(x_nhwc.device) if ws is None else ws
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    _check(lib.spi_op_conv2d(PREC[prec], _ptr(x_nhwc), B, H, W_, cin, _ptr(W_packed), cout, kh, kw, stride, pad,
                             _ptr(bias), _ptr(residual), _ptr(out), ACT[act], _ptr(ws), C.c_void_p(s)))
    return out


def attention(prec, qkv, B, S, heads, mask_bias=None, scale=0.125, stream=None):
    D = heads * 64
    ctx = torch.empty(B * S, D, device=qkv.device, dtype=qkv.dtype)
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    _check(lib.spi_op_attention(PREC[prec], _ptr(qkv), _ptr(mask_bias), _ptr(ctx), B, S, heads, scale,
                                C.c_void_p(s)))
    return ctx


def layernorm(prec, x, gamma, beta, eps, stream=None):
    rows, D = x.shape
    yf = torch.empty_like(x)
    yt = torch.empty(rows, D, device=x.device, dtype=torch.float16) if prec == "fp16" else None
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    _check(lib.spi_op_layernorm(PREC[prec], _ptr(x), _ptr(gamma), _ptr(beta), _ptr(yf), _ptr(yt), rows, D, eps,
                                C.c_void_p(s)))
    return yf, yt


def avgpool_fc(prec, x, W_packed, N_, bias=None, act=None, ws=None, stream=None):
    """Fused global average pool + linear layer: x [B][HW][C] -> fp32 [B][N] (one launch)."""
    B, HW, Cc = x.shape
    out = torch.empty(B, N_, device=x.device, dtype=torch.float32)
    ws = workspace(x.device) if ws is None else ws
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    _check(lib.spi_op_avgpool_fc(PREC[prec], _ptr(x), B, HW, Cc, _ptr(W_packed), N_, _ptr(bias), _ptr(out), ACT[act],
                                 _ptr(ws), C.c_void_p(s)))
    return out


# fp16 operands / fp16 image x hi+lo weights (the model's fp16m stem) / hi+lo image x hi+lo weights, split out
# (fp16x3s) or fp16 out (fp16x3)
STEM_PREC = {"fp16": 1, "fp16m": 2, "fp16x3s": 3, "fp16x3": 4}


def stem_pool(prec, x_nchw, w_folded, bias, rows_per_block=0, stream=None):
    """Fused ResNet stem (7x7/s2 conv over 3 channels, 64 out, folded BN bias, ReLU, 3x3/s2 max pool)
    on the NCHW fp32 image, one launch.  Returns NHWC [B][PH][PW][64]: fp16, or for fp16x3s the split
    layout in a float32-storage tensor."""
    B, _, H, W_ = x_nchw.shape
    oh, ow = (H - 1) // 2 + 1, (W_ - 1) // 2 + 1
    ph, pw = (oh - 1) // 2 + 1, (ow - 1) // 2 + 1
    w = np.ascontiguousarray(np.asarray(w_folded.cpu() if isinstance(w_folded, torch.Tensor) else w_folded,
                                        dtype=np.float32))
    host = np.empty(lib.spi_op_stem_pool_bytes(), dtype=np.uint8)
    _check(lib.spi_op_stem_pool_pack(w.ctypes.data, host.ctypes.data))
    wp = torch.from_numpy(host).to(x_nchw.device)
    out = torch.empty(B, ph, pw, 64, device=x_nchw.device,
                      dtype=torch.float32 if prec == "fp16x3s" else torch.float16)
    s = torch.cuda.current_stream().cuda_stream if stream is None else stream
    _check(lib.spi_op_stem_pool(STEM_PREC[prec], _ptr(x_nchw), B, H, W_, _ptr(wp), _ptr(bias), _ptr(out),
                                rows_per_block, C.c_void_p(s)))
    return out
