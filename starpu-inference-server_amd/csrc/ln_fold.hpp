// LayerNorm folded across GEMMs: the device side (GemmDesc::ln_in_chunks / res_ln_chunks /
// ln_out).  A transformer block's LayerNorm never runs as its own launch:
// the GEMM that produces the pre-LN rows writes their per-64-column-chunk statistics, the
// GEMM that consumes the normalised rows folds the normalisation into its epilogue
// (LN(x) W^T = rstd (x W'^T - mean c1) + W beta, W' = W diag(gamma)), and a post-LN block's
// next residual add recomputes LN(x) element-wise from x and the same statistics.
#pragma once
#include "spi_kernels.hpp"

namespace spi {

// mean and rstd of row m from its `chunks` (mean, M2) partials over 64 columns each (Chan).
// Up to 16 chunks (D <= 1024: every BERT / ViT width) all loads go out before any use -- one
// memory latency per row; a loop of dependent loads per row had doubled the consuming GEMMs
// (round 4, tools/loaded_ops.py).  Callers compute a tile's rows once, into LDS (ln_tile_stats).
__device__ __forceinline__ void ln_row_stats(const float* stats, int m, int chunks, float eps, float& mean,
                                             float& rstd) {
  const float2* p = reinterpret_cast<const float2*>(stats) + (size_t)m * chunks;
  if (chunks <= 16) {
    float2 v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = c < chunks ? p[c] : float2{0.f, 0.f};
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += v[c].x;
    mean = s / (float)chunks;
    float m2 = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float dm = v[c].x - mean;
      m2 += c < chunks ? v[c].y + 64.f * dm * dm : 0.f;
    }
    rstd = rsqrtf(m2 / (64.f * (float)chunks) + eps);
    return;
  }
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += p[c].x;
  mean = s / (float)chunks;
  float m2 = 0.f;
  for (int c = 0; c < chunks; ++c) {
    const float2 v = p[c];
    const float dm = v.x - mean;
    m2 += v.y + 64.f * dm * dm;
  }
  rstd = rsqrtf(m2 / (64.f * (float)chunks) + eps);
}

// {mean, rstd} of a tile's `rows` rows (m0 on, clamped to M - 1) into `out`, one row per thread.
__device__ __forceinline__ void ln_tile_stats(const float* stats, int m0, int rows, int M, int chunks, float eps,
                                              float2* out, int tid, int nthreads) {
  for (int r = tid; r < rows; r += nthreads) {
    float mean, rstd;
    ln_row_stats(stats, min(m0 + r, M - 1), chunks, eps, mean, rstd);
    out[r] = float2{mean, rstd};
  }
}

// (mean, M2) of one row's 64-column chunk held as 8 values by each of 8 consecutive lanes
// (lane & 7 = the 8-column group inside the chunk); every lane gets the result.
__device__ __forceinline__ void ln_chunk_stats(const float (&y)[8], float& mean, float& m2) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s += y[e];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  mean = s * (1.f / 64.f);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) q += (y[e] - mean) * (y[e] - mean);
  q += __shfl_xor(q, 1, 64);
  q += __shfl_xor(q, 2, 64);
  q += __shfl_xor(q, 4, 64);
  m2 = q;
}

}  // namespace spi
