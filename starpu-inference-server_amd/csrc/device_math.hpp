// Device math shared by the GEMM epilogues (gemm.hip, gemm256.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace spi {

// erf for the GELU epilogues (torch.nn.GELU(approximate='none') = x/2 (1 + erf(x/sqrt 2))).
// ocml's erff branches between a polynomial range and an exp range (~40 VALU per element
// under divergence); at 65536 GELUs per 256x256 tile that was 10 us of a 53 us ViT-L FFN1
// launch (3152 x 4096 x 1024).  This is the clamped odd rational x P(x^2) / Q(x^2)
// (degree 13 / 8, the minimax form of Eigen's fast erf): 12 FMAs and one reciprocal,
// max |error| 4.5e-7 over the real line in fp32 (checked against scipy's erf on 2e6
// points, tools/fast_erf_check.py), so GELU stays inside the fp32 parity bar (1e-5
// normalised) and far below an fp16 output ulp.
// Horner coefficients, highest power of x^2 first: erf(x) = x P(x^2) / Q(x^2) on |x| <= 4
constexpr float kErfP[7] = {-2.72614225801306e-10f, 2.77068142495902e-08f, -2.10102402082508e-06f,
                            -5.69250639462346e-05f, -7.34990630326855e-04f, -2.95459980854025e-03f,
                            -1.60960333262415e-02f};
constexpr float kErfQ[5] = {-1.45660718464996e-05f, -2.13374055278905e-04f, -1.68282697438203e-03f,
                            -7.37332916720468e-03f, -1.42647390514189e-02f};
constexpr float kErfClamp = 4.f;

__device__ __forceinline__ float fast_erf(float x) {
  x = __builtin_amdgcn_fmed3f(x, -kErfClamp, kErfClamp);
  const float x2 = x * x;
  float p = kErfP[0], q = kErfQ[0];
#pragma unroll
  for (int i = 1; i < 7; ++i) p = fmaf(p, x2, kErfP[i]);
#pragma unroll
  for (int i = 1; i < 5; ++i) q = fmaf(q, x2, kErfQ[i]);
  return x * p * __builtin_amdgcn_rcpf(q);
}

__device__ __forceinline__ float gelu(float v) { return 0.5f * v * (1.f + fast_erf(v * 0.70710678118654752f)); }

// Two GELUs for the fp16-operand 256x256 GEMM (gemm256.hip), on the packed fp32 VALU.
// Its epilogue has 128 GELUs per lane and no MFMA beside them, so the VALU count is the
// cost (the 13 / 8 form took 11 us of a 41 us ViT-L FFN1 launch).  A lower-order
// rational, x P(x^2) / Q(x^2) of degree 7 / 6 (Q(0) = 1, clamp 3.25; fitted by p-norm
// least squares, tools/fast_erf_check.py): 6 FMAs instead of 10, max |error| 2.5e-6 --
// GELU off by < 6e-6 absolute, 80x under an fp16 output's half-ulp at 1.
constexpr float kErfP16[4] = {7.601940945e-04f, 4.336920874e-02f, 1.531434375e-01f, 1.128384723e+00f};
constexpr float kErfQ16[4] = {9.377788357e-03f, 9.460845138e-02f, 4.691170607e-01f, 1.f};
constexpr float kErfClamp16 = 3.25f;

typedef float float2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2v gelu2(float2v v) {
  float2v x = v * 0.70710678118654752f;
  x.x = __builtin_amdgcn_fmed3f(x.x, -kErfClamp16, kErfClamp16);
  x.y = __builtin_amdgcn_fmed3f(x.y, -kErfClamp16, kErfClamp16);
  const float2v x2 = x * x;
  float2v p = kErfP16[0], q = kErfQ16[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) p = __builtin_elementwise_fma(p, x2, (float2v)kErfP16[i]);
#pragma unroll
  for (int i = 1; i < 4; ++i) q = __builtin_elementwise_fma(q, x2, (float2v)kErfQ16[i]);
  const float2v r = {__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  const float2v h = v * 0.5f;
  return __builtin_elementwise_fma(h, x * p * r, h);
}

}  // namespace spi
