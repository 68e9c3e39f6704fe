// HBM-bound kernels around the MFMA contractions (gfx950): layout ingest,
// pooling, LayerNorm, BERT embedding gather + LN, ViT patchify/assembly.
// All loads/stores are 16-byte vectors where the layout allows (G13).
#include "ln_fold.hpp"
#include "spi_kernels.hpp"

#include <algorithm>
#include <stdexcept>

namespace spi {
namespace {

template <typename T>
__device__ __forceinline__ T cvt(float v) { return static_cast<T>(v); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

int grid_for(size_t n, int block = 256, int cap = 8192) {
  return (int)std::max<size_t>(1, std::min<size_t>((n + block - 1) / block, cap));
}

// NCHW fp32 -> NHWC (T) with channel padding; one thread per pixel.
template <typename T>
__global__ void ingest_kernel(const float* __restrict__ x, T* __restrict__ y, int B,
                              int C, int H, int W, int cpad) {
  const size_t npix = (size_t)B * H * W;
  const size_t HW = (size_t)H * W;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < npix;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t b = i / HW, hw = i - b * HW;
    T* dst = y + i * cpad;
    for (int c = 0; c < cpad; ++c)
      dst[c] = c < C ? cvt<T>(x[(b * C + c) * HW + hw]) : cvt<T>(0.f);
  }
}

// Max pool on NHWC; one thread per (output pixel, 16-byte channel vector).
template <typename T>
__global__ void maxpool_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int H,
                               int W, int C, int OH, int OW, int k, int stride, int pad) {
  constexpr int VEC = 16 / (int)sizeof(T);
  const int CV = C / VEC;
  const size_t n = (size_t)B * OH * OW * CV;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    size_t r = i / CV;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    float m[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) m[e] = -INFINITY;
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * stride - pad + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * stride - pad + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(x + (((size_t)b * H + ih) * W + iw) * C + cv * VEC);
        const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
        for (int q = 0; q < VEC; ++q) m[q] = fmaxf(m[q], static_cast<float>(e[q]));
      }
    }
    T o[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) o[q] = cvt<T>(m[q]);
    *reinterpret_cast<uint4*>(y + i * VEC) = *reinterpret_cast<const uint4*>(o);
  }
}

// F16X3 split activations: per pixel, C/32 blocks of [32 hi | 32 lo] fp16.
// Channel group g (8 channels) has its hi vector at fp16 offset split_goff(g)
// and its lo vector 32 further on.
__device__ __forceinline__ int split_goff(int g) { return (g >> 2) * 64 + (g & 3) * 8; }

__device__ __forceinline__ void split_load8(const _Float16* p, float v[8]) {
  const uint4 h = *reinterpret_cast<const uint4*>(p);
  const uint4 l = *reinterpret_cast<const uint4*>(p + 32);
  const _Float16* hh = reinterpret_cast<const _Float16*>(&h);
  const _Float16* ll = reinterpret_cast<const _Float16*>(&l);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = static_cast<float>(hh[q]) + static_cast<float>(ll[q]);
}

__device__ __forceinline__ void split_store8(_Float16* p, const float v[8]) {
  _Float16 h[8], l[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    h[q] = static_cast<_Float16>(v[q]);
    l[q] = static_cast<_Float16>(v[q] - static_cast<float>(h[q]));
  }
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(h);
  *reinterpret_cast<uint4*>(p + 32) = *reinterpret_cast<const uint4*>(l);
}

// Max pool split -> split; one thread per (output pixel, 8-channel group).
__global__ void maxpool_split_kernel(const _Float16* __restrict__ x, _Float16* __restrict__ y, int B, int H,
                                     int W, int C, int OH, int OW, int k, int stride, int pad) {
  const int G = C / 8;
  const size_t n = (size_t)B * OH * OW * G;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int g = (int)(i % G);
    const size_t pix = i / G;
    const int ow = (int)(pix % OW);
    const size_t r = pix / OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    float m[8], v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) m[q] = -INFINITY;
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * stride - pad + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * stride - pad + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        split_load8(x + (((size_t)b * H + ih) * W + iw) * C * 2 + split_goff(g), v);
#pragma unroll
        for (int q = 0; q < 8; ++q) m[q] = fmaxf(m[q], v[q]);
      }
    }
    split_store8(y + pix * C * 2 + split_goff(g), m);
  }
}

// Average pool split -> fp32 [B, C]; one block per image, thread (p, g) sums
// pixels p, p+P, ... of channel group g, the P partial sums meet in LDS.
__global__ __launch_bounds__(256) void avgpool_split_kernel(const _Float16* __restrict__ x, float* __restrict__ y,
                                                            int HW, int C) {
  __shared__ float part[256 * 8];
  const int b = blockIdx.x, G = C / 8;
  const _Float16* img = x + (size_t)b * HW * C * 2;
  for (int g0 = 0; g0 < G; g0 += 256) {
    const int Gc = min(256, G - g0);
    const int P = 256 / Gc;
    const int p = threadIdx.x / Gc, g = g0 + threadIdx.x % Gc;
    float s[8] = {}, v[8];
    if (p < P)
      for (int px = p; px < HW; px += P) {
        split_load8(img + (size_t)px * C * 2 + split_goff(g), v);
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] += v[q];
      }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) part[threadIdx.x * 8 + q] = s[q];
    __syncthreads();
    if (threadIdx.x < Gc) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float t = 0.f;
        for (int pp = 0; pp < P; ++pp) t += part[(pp * Gc + threadIdx.x) * 8 + q];
        y[(size_t)b * C + (size_t)(g0 + threadIdx.x) * 8 + q] = t / (float)HW;
      }
    }
  }
}

// Global average pool: one block per image; thread (g, c) sums pixels g, g+G, ...
// of its 16-byte channel vector c, then the G partial sums meet in LDS.
template <typename T, typename TO = T>
__global__ __launch_bounds__(256) void avgpool_kernel(const T* __restrict__ x, TO* __restrict__ y,
                                                      int B, int HW, int C) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ float part[256 * VEC];
  const int b = blockIdx.x;
  const int CV = C / VEC;
  const T* img = x + (size_t)b * HW * C;
  if (CV <= 256) {
    const int G = 256 / CV;
    const int g = threadIdx.x / CV, cv = threadIdx.x % CV;
    float s[VEC] = {};
    if (g < G)
      for (int p = g; p < HW; p += G) {
        const uint4 v = *reinterpret_cast<const uint4*>(img + (size_t)p * C + cv * VEC);
        const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
        for (int q = 0; q < VEC; ++q) s[q] += static_cast<float>(e[q]);
      }
#pragma unroll
    for (int q = 0; q < VEC; ++q) part[threadIdx.x * VEC + q] = s[q];
    __syncthreads();
    if (threadIdx.x < CV) {
      TO o[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        float t = 0.f;
        for (int gg = 0; gg < G; ++gg) t += part[(gg * CV + threadIdx.x) * VEC + q];
        o[q] = cvt<TO>(t / (float)HW);
      }
#pragma unroll
      for (int h = 0; h < (int)sizeof(o) / 16; ++h)
        reinterpret_cast<uint4*>(y + (size_t)b * C + threadIdx.x * VEC)[h] = reinterpret_cast<const uint4*>(o)[h];
    }
  } else {
    for (int cv = threadIdx.x; cv < CV; cv += 256) {
      float s[VEC] = {};
      for (int p = 0; p < HW; ++p) {
        const uint4 v = *reinterpret_cast<const uint4*>(img + (size_t)p * C + cv * VEC);
        const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
        for (int q = 0; q < VEC; ++q) s[q] += static_cast<float>(e[q]);
      }
      TO o[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) o[q] = cvt<TO>(s[q] / (float)HW);
#pragma unroll
      for (int h = 0; h < (int)sizeof(o) / 16; ++h)
        reinterpret_cast<uint4*>(y + (size_t)b * C + cv * VEC)[h] = reinterpret_cast<const uint4*>(o)[h];
    }
  }
}

// One wave per row, D <= 64*16.  Two-pass mean/variance in fp32 registers.
template <typename T, int VPL>
__device__ __forceinline__ void ln_row(const float (&v)[VPL], int D, const float* g,
                                       const float* b, float eps, float* yf, T* yt,
                                       int lane) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) s += v[j];
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < D) {
      const float t = v[j] - mean;
      q += t * t;
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < D) {
      const float o = (v[j] - mean) * rstd * g[c] + b[c];
      if (yf) yf[c] = o;
      if (yt) yt[c] = cvt<T>(o);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* x, int ldx,
                                                        const float* g, const float* b,
                                                        float* yf, T* yt, int ldy,
                                                        int rows, int D, float eps) {
  constexpr int VPL = 16;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (size_t)row * ldx;
  float v[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? xr[c] : 0.f;
  }
  ln_row<T, VPL>(v, D, g, b, eps, yf ? yf + (size_t)row * ldy : nullptr,
                 yt ? yt + (size_t)row * ldy : nullptr, lane);
}

// LayerNorm of rows held in two fp16 planes (GemmDesc::res_planes: x = hi + lo, lo `plane`
// elements after hi) -- ViT's final class-token LayerNorm over the two-plane residual stream.
template <typename T>
__global__ __launch_bounds__(256) void layernorm_planes_kernel(const _Float16* xh, size_t plane, int ldx,
                                                               const float* g, const float* b, float* yf, T* yt,
                                                               int ldy, int rows, int D, float eps) {
  constexpr int VPL = 16;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const _Float16* xr = xh + (size_t)row * ldx;
  float v[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? static_cast<float>(xr[c]) + static_cast<float>(xr[c + plane]) : 0.f;
  }
  ln_row<T, VPL>(v, D, g, b, eps, yf ? yf + (size_t)row * ldy : nullptr, yt ? yt + (size_t)row * ldy : nullptr,
                 lane);
}

// The same for D = NV * 256 (BERT-base 768, ViT-L 1024): lane l holds NV groups of 4 columns
// (c = 4 (64 j + l)), read as 8-byte hi and lo vectors -- the vector form of layernorm_vec_kernel
// (round 6: the scalar planes kernel ran BERT's output LayerNorm in 10.3 us against 4.6 for the
// fp32 vector one).
template <typename T, int NV>
__global__ __launch_bounds__(256) void layernorm_planes_vec_kernel(const _Float16* __restrict__ xh, size_t plane,
                                                                   int ldx, const float* __restrict__ g,
                                                                   const float* __restrict__ b, float* yf, T* yt,
                                                                   int ldy, int rows, float eps) {
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = NV * 256;
  const half4* xr = reinterpret_cast<const half4*>(xh + (size_t)row * ldx);
  const half4* lr = reinterpret_cast<const half4*>(xh + (size_t)row * ldx + plane);
  half4 hv[NV], lv[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    hv[j] = xr[j * 64 + lane];
    lv[j] = lr[j * 64 + lane];
  }
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  float4 gg[NV], bb[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    gg[j] = g4[j * 64 + lane];
    bb[j] = b4[j * 64 + lane];
  }
  float v[NV][4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[j][e] = static_cast<float>(hv[j][e]) + static_cast<float>(lv[j][e]);
      s += v[j][e];
    }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) q += (v[j][e] - mean) * (v[j][e] - mean);
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c4 = j * 64 + lane;
    float4 o;
    o.x = (v[j][0] - mean) * rstd * gg[j].x + bb[j].x;
    o.y = (v[j][1] - mean) * rstd * gg[j].y + bb[j].y;
    o.z = (v[j][2] - mean) * rstd * gg[j].z + bb[j].z;
    o.w = (v[j][3] - mean) * rstd * gg[j].w + bb[j].w;
    if (yf) reinterpret_cast<float4*>(yf + (size_t)row * ldy)[c4] = o;
    if (yt) {
      if constexpr (sizeof(T) == 2) {
        half4 h;
        h[0] = static_cast<_Float16>(o.x);
        h[1] = static_cast<_Float16>(o.y);
        h[2] = static_cast<_Float16>(o.z);
        h[3] = static_cast<_Float16>(o.w);
        reinterpret_cast<half4*>(yt + (size_t)row * ldy)[c4] = h;
      } else {
        reinterpret_cast<float4*>(yt + (size_t)row * ldy)[c4] = o;
      }
    }
  }
}

// LayerNorm rows of D = NV * 256: one wave per row, every lane holds NV float4
// column groups (c = 4 * (64 j + lane)), so the row moves as 16-byte loads and
// stores (fp16 copies as 8-byte stores) -- a quarter of the scalar kernel's
// memory instructions; same two-pass fp32 statistics.
template <typename T, int NV>
__global__ __launch_bounds__(256) void layernorm_vec_kernel(const float* __restrict__ x, int ldx,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ b, float* yf, T* yt,
                                                            int ldy, int rows, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int D = NV * 256;
  const float4* xr = reinterpret_cast<const float4*>(x + (size_t)row * ldx);
  float4 v[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = xr[j * 64 + lane];
  // gamma / beta issued with the row, not after the two reductions: one memory round trip
  // fewer on the wave's dependent chain (the kernel is one such chain per row)
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  float4 gg[NV], bb[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    gg[j] = g4[j * 64 + lane];
    bb[j] = b4[j * 64 + lane];
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float a0 = v[j].x - mean, a1 = v[j].y - mean, a2 = v[j].z - mean, a3 = v[j].w - mean;
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c4 = j * 64 + lane;
    float4 o;
    o.x = (v[j].x - mean) * rstd * gg[j].x + bb[j].x;
    o.y = (v[j].y - mean) * rstd * gg[j].y + bb[j].y;
    o.z = (v[j].z - mean) * rstd * gg[j].z + bb[j].z;
    o.w = (v[j].w - mean) * rstd * gg[j].w + bb[j].w;
    if (yf) reinterpret_cast<float4*>(yf + (size_t)row * ldy)[c4] = o;
    if (yt) {
      if constexpr (sizeof(T) == 2) {
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
        half4 h;
        h[0] = static_cast<_Float16>(o.x);
        h[1] = static_cast<_Float16>(o.y);
        h[2] = static_cast<_Float16>(o.z);
        h[3] = static_cast<_Float16>(o.w);
        reinterpret_cast<half4*>(yt + (size_t)row * ldy)[c4] = h;
      } else {
        reinterpret_cast<float4*>(yt + (size_t)row * ldy)[c4] = o;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bert_embed_kernel(
    const int64_t* ids, const float* word, const float* pos, const float* type0,
    const float* g, const float* b, float* yf, T* yt, int B, int S, int D, int vocab,
    float eps, const int64_t* mask, float* mask_bias) {
  constexpr int VPL = 16;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B * S) return;
  if (mask && lane == 0) mask_bias[row] = mask[row] != 0 ? 0.f : -3.4028234663852886e38f;
  const int s = row % S;
  int64_t id = ids[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const float* w = word + (size_t)id * D;
  const float* p = pos + (size_t)s * D;
  float v[VPL];
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? (w[c] + type0[c]) + p[c] : 0.f;
  }
  ln_row<T, VPL>(v, D, g, b, eps, yf + (size_t)row * D, yt ? yt + (size_t)row * D : nullptr,
                 lane);
}

// The same for D = NV * 256 with 16-byte gathers: lane l holds NV groups of 4 columns
// (c = 4 (64 j + l)) -- a quarter of the scalar kernel's memory instructions (round 6: BERT-base's
// embedding ran 14.6 us in the loop trace, 1.7 % of C3).
template <typename T, int NV>
__global__ __launch_bounds__(256) void bert_embed_vec_kernel(const int64_t* ids, const float* __restrict__ word,
                                                             const float* __restrict__ pos,
                                                             const float* __restrict__ type0,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ b, float* yf, T* yt, int B,
                                                             int S, int vocab, float eps, const int64_t* mask,
                                                             float* mask_bias) {
  constexpr int D = NV * 256;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B * S) return;
  // the attention's additive key bias of this token, (1 - m) * finfo(f32).min (mask_bias_kernel's)
  if (mask && lane == 0) mask_bias[row] = mask[row] != 0 ? 0.f : -3.4028234663852886e38f;
  const int s = row % S;
  int64_t id = ids[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const float4* w4 = reinterpret_cast<const float4*>(word + (size_t)id * D);
  const float4* p4 = reinterpret_cast<const float4*>(pos + (size_t)s * D);
  const float4* t4 = reinterpret_cast<const float4*>(type0);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  float4 v[NV], gg[NV], bb[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c4 = j * 64 + lane;
    const float4 w = w4[c4], t = t4[c4], p = p4[c4];
    v[j] = float4{(w.x + t.x) + p.x, (w.y + t.y) + p.y, (w.z + t.z) + p.z, (w.w + t.w) + p.w};
    gg[j] = g4[c4];
    bb[j] = b4[c4];
  }
  float sm = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) sm += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  const float mean = wave_sum(sm) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float a0 = v[j].x - mean, a1 = v[j].y - mean, a2 = v[j].z - mean, a3 = v[j].w - mean;
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c4 = j * 64 + lane;
    float4 o;
    o.x = (v[j].x - mean) * rstd * gg[j].x + bb[j].x;
    o.y = (v[j].y - mean) * rstd * gg[j].y + bb[j].y;
    o.z = (v[j].z - mean) * rstd * gg[j].z + bb[j].z;
    o.w = (v[j].w - mean) * rstd * gg[j].w + bb[j].w;
    reinterpret_cast<float4*>(yf + (size_t)row * D)[c4] = o;
    if (yt) {
      if constexpr (sizeof(T) == 2) {
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
        half4 h;
        h[0] = static_cast<_Float16>(o.x);
        h[1] = static_cast<_Float16>(o.y);
        h[2] = static_cast<_Float16>(o.z);
        h[3] = static_cast<_Float16>(o.w);
        reinterpret_cast<half4*>(yt + (size_t)row * D)[c4] = h;
      } else {
        reinterpret_cast<float4*>(yt + (size_t)row * D)[c4] = o;
      }
    }
  }
}

__global__ void mask_bias_kernel(const int64_t* mask, float* bias, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    bias[i] = mask[i] != 0 ? 0.f : -3.4028234663852886e38f;  // (1 - m) * finfo(f32).min
}

// ViT patchify: row (b, ph, pw), column c*ps*ps + kh*ps + kw (conv weight flatten order).
template <typename T>
__global__ void patchify_kernel(const float* __restrict__ x, T* __restrict__ y, int B,
                                int C, int H, int W, int ps) {
  const int GH = H / ps, GW = W / ps;
  const int K = C * ps * ps;
  const size_t n = (size_t)B * GH * GW * K;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    const size_t row = i / K;
    const int pw = (int)(row % GW);
    const int ph = (int)((row / GW) % GH);
    const int b = (int)(row / ((size_t)GW * GH));
    const int c = k / (ps * ps);
    const int kh = (k / ps) % ps, kw = k % ps;
    y[i] = cvt<T>(x[(((size_t)b * C + c) * H + ph * ps + kh) * W + pw * ps + kw]);
  }
}

// Vector form (round 6; ps % 8 == 0, W % 4 == 0, 16-byte aligned x / y): one thread per 8
// consecutive kw of one (patch row, c, kh): two 16-byte loads, one 16-byte (fp16) or two (fp32)
// stores; consecutive threads write consecutive y chunks.  32-bit index math (host-checked).
template <typename T>
__global__ __launch_bounds__(256) void patchify_vec_kernel(const float* __restrict__ x, T* __restrict__ y, int C,
                                                           int H, int W, int ps, int GH, int GW, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const int segs = ps >> 3;
  const int seg = t % segs;
  int r = t / segs;
  const int kh = r % ps;
  r /= ps;
  const int c = r % C;
  const int row = r / C;  // (b, ph, pw)
  const int pw = row % GW, ph = (row / GW) % GH, b = row / (GW * GH);
  const float4* src =
      reinterpret_cast<const float4*>(x + ((size_t)(b * C + c) * H + ph * ps + kh) * W + pw * ps + seg * 8);
  const float4 v0 = src[0], v1 = src[1];
  T* dst = y + (size_t)row * (C * ps * ps) + (c * ps + kh) * ps + seg * 8;
  if constexpr (sizeof(T) == 2) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const h8 o = {(_Float16)v0.x, (_Float16)v0.y, (_Float16)v0.z, (_Float16)v0.w,
                  (_Float16)v1.x, (_Float16)v1.y, (_Float16)v1.z, (_Float16)v1.w};
    *reinterpret_cast<h8*>(dst) = o;
  } else {
    reinterpret_cast<float4*>(dst)[0] = v0;
    reinterpret_cast<float4*>(dst)[1] = v1;
  }
}

__global__ void vit_assemble_kernel(const float* __restrict__ patches,
                                    const float* __restrict__ cls,
                                    const float* __restrict__ pos, float* __restrict__ x,
                                    int B, int P, int D) {
  const size_t n = (size_t)B * (P + 1) * D;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    const size_t r = i / D;
    const int t = (int)(r % (P + 1));
    const int b = (int)(r / (P + 1));
    const float v = t == 0 ? cls[c] : patches[((size_t)b * P + (t - 1)) * D + c];
    x[i] = v + pos[(size_t)t * D + c];
  }
}

// ViT stream assembly into the two-plane residual stream (GemmDesc::res_planes) plus the rows'
// per-64-column chunk statistics (ln_fold.hpp) that the first layer's folded QKV GEMM reads: one
// thread per 8 columns of a row, 8 consecutive threads = one 64-column chunk (D % 64 == 0, so a
// chunk never straddles rows or 8-lane groups); 16-byte loads and stores.
__global__ __launch_bounds__(256) void vit_assemble_planes_kernel(const float* __restrict__ patches,
                                                                  const float* __restrict__ cls,
                                                                  const float* __restrict__ pos,
                                                                  _Float16* __restrict__ xh, size_t plane,
                                                                  float* __restrict__ stats, int B, int P, int D) {
  typedef _Float16 half8 __attribute__((ext_vector_type(8)));
  const int groups = D >> 3;
  const size_t n = (size_t)B * (P + 1) * groups;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  // every lane of an 8-lane group takes part in the chunk shuffles: past the end, repeat the last
  // group (n is a multiple of 8) and store nothing
  const size_t gi = gid < n ? gid : n - 1;
  const size_t r = gi / groups;
  const int c0 = (int)(gi - r * groups) * 8;
  const int t = (int)(r % (P + 1)), b = (int)(r / (P + 1));
  const float* src = t == 0 ? cls + c0 : patches + ((size_t)b * P + (t - 1)) * D + c0;
  const float* pp = pos + (size_t)t * D + c0;
  const float4 s0 = reinterpret_cast<const float4*>(src)[0], s1 = reinterpret_cast<const float4*>(src)[1];
  const float4 p0 = reinterpret_cast<const float4*>(pp)[0], p1 = reinterpret_cast<const float4*>(pp)[1];
  const float y[8] = {s0.x + p0.x, s0.y + p0.y, s0.z + p0.z, s0.w + p0.w,
                      s1.x + p1.x, s1.y + p1.y, s1.z + p1.z, s1.w + p1.w};
  float mean, m2;
  ln_chunk_stats(y, mean, m2);
  if (gid >= n) return;
  half8 hi, lo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    hi[e] = static_cast<_Float16>(y[e]);
    lo[e] = static_cast<_Float16>(y[e] - static_cast<float>(hi[e]));
  }
  _Float16* xr = xh + r * D + c0;
  *reinterpret_cast<half8*>(xr) = hi;
  *reinterpret_cast<half8*>(xr + plane) = lo;
  if (stats && (c0 & 63) == 0) reinterpret_cast<float2*>(stats)[r * (D >> 6) + (c0 >> 6)] = float2{mean, m2};
}

template <typename T>
__global__ void gather_rows_kernel(const float* __restrict__ x, T* __restrict__ y, int rows,
                                   int stride_rows, int D) {
  const size_t n = (size_t)rows * D;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / D, c = i - r * D;
    y[i] = cvt<T>(x[r * stride_rows * D + c]);
  }
}

__global__ void affine_kernel(const float* x, float* y, size_t n, float scale, float shift) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    y[i] = x[i] * scale + shift;
}

}  // namespace


void ingest_nchw(const float* x, void* y, int B, int C, int H, int W, int cpad, bool f16,
                 hipStream_t s) {
  const size_t n = (size_t)B * H * W;
  if (f16)
    SPI_LAUNCH((ingest_kernel<_Float16>), dim3(grid_for(n)), dim3(256), 0, s, x,
                       (_Float16*)y, B, C, H, W, cpad);
  else
    SPI_LAUNCH((ingest_kernel<float>), dim3(grid_for(n)), dim3(256), 0, s, x,
                       (float*)y, B, C, H, W, cpad);
}

void maxpool_nhwc(const void* x, void* y, int B, int H, int W, int C, int OH, int OW, int k,
                  int stride, int pad, bool f16, hipStream_t s) {
  const size_t n = (size_t)B * OH * OW * C / (f16 ? 8 : 4);
  if (f16)
    SPI_LAUNCH((maxpool_kernel<_Float16>), dim3(grid_for(n)), dim3(256), 0, s,
                       (const _Float16*)x, (_Float16*)y, B, H, W, C, OH, OW, k, stride, pad);
  else
    SPI_LAUNCH((maxpool_kernel<float>), dim3(grid_for(n)), dim3(256), 0, s,
                       (const float*)x, (float*)y, B, H, W, C, OH, OW, k, stride, pad);
}

void maxpool_nhwc_split(const void* x, void* y, int B, int H, int W, int C, int OH, int OW, int k, int stride,
                        int pad, hipStream_t s) {
  const size_t n = (size_t)B * OH * OW * (C / 8);
  SPI_LAUNCH(maxpool_split_kernel, dim3(grid_for(n)), dim3(256), 0, s, (const _Float16*)x, (_Float16*)y, B,
                     H, W, C, OH, OW, k, stride, pad);
}

void avgpool_nhwc_split(const void* x, float* y, int B, int HW, int C, hipStream_t s) {
  SPI_LAUNCH(avgpool_split_kernel, dim3(B), dim3(256), 0, s, (const _Float16*)x, y, HW, C);
}

void avgpool_nhwc(const void* x, void* y, int B, int HW, int C, bool f16, hipStream_t s, bool out_f32) {
  if (f16 && out_f32)
    SPI_LAUNCH((avgpool_kernel<_Float16, float>), dim3(B), dim3(256), 0, s, (const _Float16*)x,
                       (float*)y, B, HW, C);
  else if (f16)
    SPI_LAUNCH((avgpool_kernel<_Float16>), dim3(B), dim3(256), 0, s, (const _Float16*)x,
                       (_Float16*)y, B, HW, C);
  else
    SPI_LAUNCH((avgpool_kernel<float>), dim3(B), dim3(256), 0, s, (const float*)x,
                       (float*)y, B, HW, C);
}

void layernorm(const float* x, int ldx, const float* g, const float* b, float* yf, void* yt,
               int ldy, int rows, int D, float eps, bool f16, hipStream_t s) {
  const dim3 grid((rows + 3) / 4);
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool vec = D % 256 == 0 && (D == 768 || D == 1024) && ldx % 4 == 0 && ldy % 4 == 0 && al16(x) &&
                   al16(g) && al16(b) && (!yf || al16(yf)) && (!yt || ((reinterpret_cast<uintptr_t>(yt) & 7) == 0));
  if (vec) {
    if (D == 768 && f16)
      SPI_LAUNCH((layernorm_vec_kernel<_Float16, 3>), grid, dim3(256), 0, s, x, ldx, g, b, yf,
                         (_Float16*)yt, ldy, rows, eps);
    else if (D == 768)
      SPI_LAUNCH((layernorm_vec_kernel<float, 3>), grid, dim3(256), 0, s, x, ldx, g, b, yf, (float*)yt,
                         ldy, rows, eps);
    else if (f16)
      SPI_LAUNCH((layernorm_vec_kernel<_Float16, 4>), grid, dim3(256), 0, s, x, ldx, g, b, yf,
                         (_Float16*)yt, ldy, rows, eps);
    else
      SPI_LAUNCH((layernorm_vec_kernel<float, 4>), grid, dim3(256), 0, s, x, ldx, g, b, yf, (float*)yt,
                         ldy, rows, eps);
    return;
  }
  if (f16)
    SPI_LAUNCH((layernorm_kernel<_Float16>), grid, dim3(256), 0, s, x, ldx, g, b, yf,
                       (_Float16*)yt, ldy, rows, D, eps);
  else
    SPI_LAUNCH((layernorm_kernel<float>), grid, dim3(256), 0, s, x, ldx, g, b, yf,
                       (float*)yt, ldy, rows, D, eps);
}

void bert_embed(const int64_t* ids, const float* word, const float* pos, const float* type0,
                const float* g, const float* b, float* yf, void* yt, int B, int S, int D,
                int vocab, float eps, bool f16, hipStream_t s, const int64_t* mask, float* mask_bias) {
  const dim3 grid((B * S + 3) / 4);
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if ((D == 768 || D == 1024) && al16(word) && al16(pos) && al16(type0) && al16(g) && al16(b) && al16(yf) &&
      (!yt || (reinterpret_cast<uintptr_t>(yt) & (f16 ? 7 : 15)) == 0)) {
    if (D == 768 && f16)
      SPI_LAUNCH((bert_embed_vec_kernel<_Float16, 3>), grid, dim3(256), 0, s, ids, word, pos, type0, g, b, yf,
                 (_Float16*)yt, B, S, vocab, eps, mask, mask_bias);
    else if (D == 768)
      SPI_LAUNCH((bert_embed_vec_kernel<float, 3>), grid, dim3(256), 0, s, ids, word, pos, type0, g, b, yf,
                 (float*)yt, B, S, vocab, eps, mask, mask_bias);
    else if (f16)
      SPI_LAUNCH((bert_embed_vec_kernel<_Float16, 4>), grid, dim3(256), 0, s, ids, word, pos, type0, g, b, yf,
                 (_Float16*)yt, B, S, vocab, eps, mask, mask_bias);
    else
      SPI_LAUNCH((bert_embed_vec_kernel<float, 4>), grid, dim3(256), 0, s, ids, word, pos, type0, g, b, yf,
                 (float*)yt, B, S, vocab, eps, mask, mask_bias);
    return;
  }
  if (f16)
    SPI_LAUNCH((bert_embed_kernel<_Float16>), grid, dim3(256), 0, s, ids, word, pos,
                       type0, g, b, yf, (_Float16*)yt, B, S, D, vocab, eps, mask, mask_bias);
  else
    SPI_LAUNCH((bert_embed_kernel<float>), grid, dim3(256), 0, s, ids, word, pos,
                       type0, g, b, yf, (float*)yt, B, S, D, vocab, eps, mask, mask_bias);
}

void mask_to_bias(const int64_t* mask, float* bias, int n, hipStream_t s) {
  SPI_LAUNCH(mask_bias_kernel, dim3(grid_for(n)), dim3(256), 0, s, mask, bias, n);
}

void patchify(const float* x, void* y, int B, int C, int H, int W, int ps, bool f16,
              hipStream_t s) {
  const size_t n = (size_t)B * C * H * W;
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (ps % 8 == 0 && W % 4 == 0 && n / 8 < (size_t)INT32_MAX && n < (size_t)INT32_MAX && al16(x) && al16(y)) {
    const int GH = H / ps, GW = W / ps;
    const int nt = B * GH * GW * C * ps * (ps / 8);
    if (f16)
      SPI_LAUNCH((patchify_vec_kernel<_Float16>), dim3((nt + 255) / 256), dim3(256), 0, s, x, (_Float16*)y, C, H, W,
                 ps, GH, GW, nt);
    else
      SPI_LAUNCH((patchify_vec_kernel<float>), dim3((nt + 255) / 256), dim3(256), 0, s, x, (float*)y, C, H, W, ps, GH,
                 GW, nt);
    return;
  }
  if (f16)
    SPI_LAUNCH((patchify_kernel<_Float16>), dim3(grid_for(n)), dim3(256), 0, s, x,
                       (_Float16*)y, B, C, H, W, ps);
  else
    SPI_LAUNCH((patchify_kernel<float>), dim3(grid_for(n)), dim3(256), 0, s, x,
                       (float*)y, B, C, H, W, ps);
}

void vit_assemble(const float* patches, const float* cls, const float* pos, float* x, int B,
                  int P, int D, hipStream_t s) {
  const size_t n = (size_t)B * (P + 1) * D;
  SPI_LAUNCH(vit_assemble_kernel, dim3(grid_for(n)), dim3(256), 0, s, patches, cls,
                     pos, x, B, P, D);
}

void vit_assemble_planes(const float* patches, const float* cls, const float* pos, _Float16* xh, size_t plane,
                         float* stats, int B, int P, int D, hipStream_t s) {
  if (D % 64 || plane % 8) throw std::invalid_argument("vit_assemble_planes: D % 64 == 0, plane % 8 == 0");
  const size_t n = (size_t)B * (P + 1) * (D / 8);
  SPI_LAUNCH(vit_assemble_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, patches, cls, pos, xh,
             plane, stats, B, P, D);
}

void layernorm_planes(const _Float16* xh, size_t plane, int ldx, const float* g, const float* b, float* yf, void* yt,
                      int ldy, int rows, int D, float eps, bool f16, hipStream_t s) {
  if (D > 1024) throw std::invalid_argument("layernorm_planes: D <= 1024");
  const dim3 grid((rows + 3) / 4);
  const auto al = [](const void* q, uintptr_t a) { return (reinterpret_cast<uintptr_t>(q) & (a - 1)) == 0; };
  if ((D == 768 || D == 1024) && ldx % 4 == 0 && plane % 4 == 0 && ldy % 4 == 0 && al(xh, 8) && al(g, 16) &&
      al(b, 16) && (!yf || al(yf, 16)) && (!yt || al(yt, f16 ? 8 : 16))) {
    if (D == 768 && f16)
      SPI_LAUNCH((layernorm_planes_vec_kernel<_Float16, 3>), grid, dim3(256), 0, s, xh, plane, ldx, g, b, yf,
                 (_Float16*)yt, ldy, rows, eps);
    else if (D == 768)
      SPI_LAUNCH((layernorm_planes_vec_kernel<float, 3>), grid, dim3(256), 0, s, xh, plane, ldx, g, b, yf, (float*)yt,
                 ldy, rows, eps);
    else if (f16)
      SPI_LAUNCH((layernorm_planes_vec_kernel<_Float16, 4>), grid, dim3(256), 0, s, xh, plane, ldx, g, b, yf,
                 (_Float16*)yt, ldy, rows, eps);
    else
      SPI_LAUNCH((layernorm_planes_vec_kernel<float, 4>), grid, dim3(256), 0, s, xh, plane, ldx, g, b, yf, (float*)yt,
                 ldy, rows, eps);
    return;
  }
  if (f16)
    SPI_LAUNCH((layernorm_planes_kernel<_Float16>), grid, dim3(256), 0, s, xh, plane, ldx, g, b, yf, (_Float16*)yt,
               ldy, rows, D, eps);
  else
    SPI_LAUNCH((layernorm_planes_kernel<float>), grid, dim3(256), 0, s, xh, plane, ldx, g, b, yf, (float*)yt, ldy,
               rows, D, eps);
}

void gather_rows(const float* x, void* y, int rows, int stride_rows, int D, bool f16,
                 hipStream_t s) {
  const size_t n = (size_t)rows * D;
  if (f16)
    SPI_LAUNCH((gather_rows_kernel<_Float16>), dim3(grid_for(n)), dim3(256), 0, s, x,
                       (_Float16*)y, rows, stride_rows, D);
  else
    SPI_LAUNCH((gather_rows_kernel<float>), dim3(grid_for(n)), dim3(256), 0, s, x,
                       (float*)y, rows, stride_rows, D);
}

void affine(const float* x, float* y, size_t n, float scale, float shift, hipStream_t s) {
  SPI_LAUNCH(affine_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n, scale, shift);
}

}  // namespace spi
