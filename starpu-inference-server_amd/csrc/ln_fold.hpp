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
__device__ __forceinline__ void ln_row_stats(const float* stats, int m, int chunks, float eps, float& mean,
                                             float& rstd) {
  const float2* p = reinterpret_cast<const float2*>(stats) + (size_t)m * chunks;
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
