/*
 * spi_ops.h — op-level C entry points of the MI355X kernels.
 *
 * Not part of the codelet boundary (that is spi_codelet.h): these expose the
 * individual HIP kernels the forward passes are built from, for kernel-level
 * parity tests against a plain fp32 reference and for micro-benchmarks.  All
 * pointers are device pointers unless marked host; every call only enqueues
 * on `stream`.  Return 0 on success, non-zero on invalid arguments / HIP error
 * (message in spi_last_error()).
 *
 * precision: 0 fp32, 1 fp16, 2 fp16x3 (fp32 activations split into hi/lo fp16
 * at fragment read), 3 fp16x3 on SPLIT activations: every activation operand
 * (A, residual, C) uses the split layout the fp16x3 ResNet forward keeps in
 * HBM -- per row, blocks of 32 elements stored as [32 hi fp16 | 32 lo fp16]
 * (128 bytes, the size of 32 fp32), hi = fp16(x), lo = fp16(x - hi).  It needs
 * K (GEMM) / Cin (conv) and N / Cout to be multiples of 32 and <= 31 filter taps.
 */
#ifndef SPI_OPS_H
#define SPI_OPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Packed weight layout for a [N][K] fp32 matrix: rows padded to Npad = 128k,
 * columns to Kpad = 64k; fp16 / fp32 elements, or for fp16x3 (2 and 3) per
 * 32-k block [32 hi fp16 | 32 lo fp16].  Returns the packed byte count; writes Npad/Kpad.
 * One exception to "zero padded": an fp16 [64][576] matrix (a 3x3 conv over 64 channels)
 * carries, in its padding rows 64..127, the weight-resident conv's LDS image of rows 0..63
 * (per tap t, row n, 16-byte slot s: chunk s ^ (n & 7) of row n's taps-t block), and
 * spi_op_conv2d routes such convs to that kernel, which reads those rows.  Packed weights
 * for spi_op_conv2d / spi_op_gemm must therefore come from spi_op_pack_weight, whole. */
size_t spi_op_packed_bytes(int32_t precision, int32_t N, int32_t K, int32_t* Npad, int32_t* Kpad);
/* Host-side packing: w_host fp32 [N][K] -> dst_host (spi_op_packed_bytes bytes). */
int spi_op_pack_weight(int32_t precision, const float* w_host, int32_t N, int32_t K, void* dst_host);

/* Bytes of device scratch a GEMM / conv call needs (zero line, split-K slabs
 * and tickets).  The scratch must be zero-filled once before first use. */
size_t spi_op_workspace_bytes(void);

/* C[M,N] = act(A[M,K] . W^T + bias + residual); act: 0 none, 1 relu, 2 gelu.
 * A: fp16 (precision fp16), fp32 (fp32 / fp16x3) or split (3), row stride lda
 * (elements).  residual: same element type as A unless res_f32; C: fp32 when
 * out_f32 (not with split). */
int spi_op_gemm(int32_t precision, const void* A, int32_t M, int32_t K, int32_t lda,
                const void* W_packed, int32_t N, const float* bias, const void* residual,
                int32_t res_f32, int32_t ldr, void* C, int32_t out_f32, int32_t ldc,
                int32_t act, void* workspace, void* stream);

/* NHWC conv as implicit GEMM: x [B][H][W][Cin] (Cin a power of two >= 8 for fp16,
 * >= 4 for fp32 / fp16x3, >= 32 for split), W packed from [Cout][KH][KW][Cin]
 * order, y [B][OH][OW][Cout]; residual (optional) shaped like y. */
int spi_op_conv2d(int32_t precision, const void* x, int32_t B, int32_t H, int32_t W,
                  int32_t Cin, const void* W_packed, int32_t Cout, int32_t KH, int32_t KW,
                  int32_t stride, int32_t pad, const float* bias, const void* residual,
                  void* y, int32_t act, void* workspace, void* stream);

/* Fused global average pool + linear layer (ResNet avgpool + fc in one launch):
 * x [B][HW][C] (fp32 / fp16 / split by precision, HW <= 64), W packed from the
 * [N][C] fc weight; y fp32 [B][N] = act(mean_hw(x) . W^T + bias). */
int spi_op_avgpool_fc(int32_t precision, const void* x, int32_t B, int32_t HW, int32_t C, const void* W_packed,
                      int32_t N, const float* bias, float* y, int32_t act, void* workspace, void* stream);

/* Fused ResNet stem: x NCHW fp32 [B][3][H][W] -> 7x7/s2/p3 conv (64 channels,
 * BN folded into w / bias) + ReLU -> 3x3/s2/p1 max pool -> y NHWC [B][PH][PW][64].
 * precision 1: fp16 image and weights, fp16 y; 2: the fp16m stem -- fp16 image x hi + lo fp16
 * weights, fp16 y; 3: hi + lo image x hi + lo weights (fp32-grade), y in the split layout (the
 * fp16x3 stem); 4: as 3 with fp16 y.  W_packed: spi_op_stem_pool_bytes()
 * of device memory filled from spi_op_stem_pool_pack(w_host fp32 [64][3][7][7]).
 * rows_per_block: 0 = default (2 pooled rows per 8-wave workgroup for maps wider than 64,
 * else 1 per 4 waves), 1 or 2 = that many per 4-wave workgroup.  W <= 224. */
size_t spi_op_stem_pool_bytes(void);
int spi_op_stem_pool_pack(const float* w_host, void* dst_host);
int spi_op_stem_pool(int32_t precision, const float* x, int32_t B, int32_t H, int32_t W,
                     const void* W_packed, const float* bias, void* y, int32_t rows_per_block, void* stream);

/* Multi-head attention over packed qkv [B*S][3*D] (fp16 or fp32), head_dim 64. */
int spi_op_attention(int32_t precision, const void* qkv, const float* mask_bias, void* ctx,
                     int32_t B, int32_t S, int32_t heads, float scale, void* stream);

/* Row LayerNorm: x fp32 [rows][D] -> yf fp32 and/or yt (fp16 when precision fp16). */
int spi_op_layernorm(int32_t precision, const float* x, const float* gamma, const float* beta,
                     float* yf, void* yt, int32_t rows, int32_t D, float eps, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SPI_OPS_H */
