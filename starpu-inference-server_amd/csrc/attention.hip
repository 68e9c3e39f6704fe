// Fused multi-head attention for BERT-base (S=128) and ViT-L/16 (S=197), gfx950.
//
// One workgroup = 4 waves = 64 query rows of one (batch, head); each wave owns
// 16 rows.  Per 64-key tile: K and V^T are staged in LDS (V transposed on the
// way in so that PV's B operand is K-contiguous), S = Q K^T on MFMA with the
// wave's Q fragment held in registers, online softmax in fp32 (row max / row
// sum with 16-lane xor shuffles: rows sit on 4*(lane>>4)+r, keys on lane&15),
// P goes through a wave-private LDS image to become the A operand of PV.
// Keys past S (ViT's 197 = 3*64 + 5) are masked to -inf, the BERT attention
// mask arrives as an additive fp32 bias ((1 - m) * finfo(f32).min, the value
// HF's BertModel adds).  head_dim is fixed at 64.
#include "spi_kernels.hpp"

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int HD = 64;
constexpr int QT = 64;
constexpr int KT = 64;

template <typename T>
__global__ __launch_bounds__(256) void attn_kernel(const T* __restrict__ qkv,
                                                   const float* __restrict__ mask_bias,
                                                   T* __restrict__ ctx, int S, int H,
                                                   float scale) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int LD = HD + EPC;   // K row stride
  constexpr int VLD = KT + EPC;  // V^T / P row stride
  __shared__ __attribute__((aligned(16))) T Ks[KT * LD];
  __shared__ __attribute__((aligned(16))) T Vt[HD * VLD];
  __shared__ __attribute__((aligned(16))) T Ps[4 * 16 * VLD];

  const int D = H * HD, ld = 3 * D;
  const int b = blockIdx.y / H, h = blockIdx.y % H;
  const int q0 = blockIdx.x * QT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const T* base = qkv + (size_t)b * S * ld;
  T* Pw = Ps + wave * 16 * VLD;

  const int qa = q0 + wave * 16 + fr;  // this lane's A-operand row
  half8 qf16[2];
  floatx4 qf32[4];
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qa < S) v = *reinterpret_cast<const half8*>(base + (size_t)qa * ld + h * HD + s * 32 + fq * 8);
      qf16[s] = v;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (qa < S) v = *reinterpret_cast<const floatx4*>(base + (size_t)qa * ld + h * HD + fq * 16 + s * 4);
      qf32[s] = v;
    }
  }

  float m_r[4], l_r[4];
  floatx4 o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m_r[r] = -INFINITY;
    l_r[r] = 0.f;
    o[r] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  // K / V tiles go through registers one tile ahead: tile t + 1's global loads are in
  // flight while tile t computes.  Raw barriers (LDS wait + s_barrier): a
  // __syncthreads() fence would also wait for those loads.
  constexpr int NCH = KT * HD / EPC / 256;  // 16-byte chunks of K (and of V) per thread per tile
  uint4 kreg[NCH], vreg[NCH];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * 256;
      const int key = c / (HD / EPC), dc = c % (HD / EPC);
      const int kk = k0 + key;
      kreg[i] = vreg[i] = make_uint4(0, 0, 0, 0);
      if (kk < S) {
        kreg[i] = *reinterpret_cast<const uint4*>(base + (size_t)kk * ld + D + h * HD + dc * EPC);
        vreg[i] = *reinterpret_cast<const uint4*>(base + (size_t)kk * ld + 2 * D + h * HD + dc * EPC);
      }
    }
  };
  fetch(0);
  for (int k0 = 0; k0 < S; k0 += KT) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the previous tile's Ks / Vt reads are done
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * 256;
      const int key = c / (HD / EPC), dc = c % (HD / EPC);
      *reinterpret_cast<uint4*>(Ks + key * LD + dc * EPC) = kreg[i];
      const T* ve = reinterpret_cast<const T*>(&vreg[i]);
#pragma unroll
      for (int e = 0; e < EPC; ++e) Vt[(dc * EPC + e) * VLD + key] = ve[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (k0 + KT < S) fetch(k0 + KT);

    floatx4 sacc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sacc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const half8 kf = *reinterpret_cast<const half8*>(Ks + (j * 16 + fr) * LD + s * 32 + fq * 8);
          sacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf16[s], kf, sacc[j], 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* kr = reinterpret_cast<const float*>(Ks) + (j * 16 + fr) * LD + fq * 16;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const floatx4 kv = *reinterpret_cast<const floatx4*>(kr + s4 * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sacc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf32[s4][e], kv[e], sacc[j], 0, 0, 0);
        }
      }
    }

    float bias[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = k0 + j * 16 + fr;
      bias[j] = key < S ? (mask_bias ? mask_bias[(size_t)b * S + key] : 0.f) : -INFINITY;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float sc[4];
      float tmax = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sc[j] = sacc[j][r] * scale + bias[j];
        tmax = fmaxf(tmax, sc[j]);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) tmax = fmaxf(tmax, __shfl_xor(tmax, off, 64));
      const float m_new = fmaxf(m_r[r], tmax);
      const float alpha = __expf(m_r[r] - m_new);
      float rs = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = __expf(sc[j] - m_new);
        rs += p;
        Pw[(fq * 4 + r) * VLD + j * 16 + fr] = static_cast<T>(p);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      l_r[r] = l_r[r] * alpha + rs;
      m_r[r] = m_new;
#pragma unroll
      for (int dblk = 0; dblk < 4; ++dblk) o[dblk][r] *= alpha;
    }
    // P is wave-private: its writes retired, the wave's own lanes read it back (no workgroup barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const half8 pf = *reinterpret_cast<const half8*>(Pw + fr * VLD + s * 32 + fq * 8);
#pragma unroll
        for (int dblk = 0; dblk < 4; ++dblk) {
          const half8 vf = *reinterpret_cast<const half8*>(Vt + (dblk * 16 + fr) * VLD + s * 32 + fq * 8);
          o[dblk] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, vf, o[dblk], 0, 0, 0);
        }
      }
    } else {
      const float* pr = reinterpret_cast<const float*>(Pw) + fr * VLD + fq * 16;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const floatx4 pv = *reinterpret_cast<const floatx4*>(pr + s4 * 4);
#pragma unroll
        for (int dblk = 0; dblk < 4; ++dblk) {
          const floatx4 vv = *reinterpret_cast<const floatx4*>(
              reinterpret_cast<const float*>(Vt) + (dblk * 16 + fr) * VLD + fq * 16 + s4 * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o[dblk] = __builtin_amdgcn_mfma_f32_16x16x4f32(pv[e], vv[e], o[dblk], 0, 0, 0);
        }
      }
    }
  }

#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + wave * 16 + fq * 4 + r;
    if (q >= S) continue;
    const float inv = 1.f / l_r[r];
#pragma unroll
    for (int dblk = 0; dblk < 4; ++dblk)
      ctx[((size_t)b * S + q) * D + h * HD + dblk * 16 + fr] = static_cast<T>(o[dblk][r] * inv);
  }
}

}  // namespace

void attention(const void* qkv, const float* mask_bias, void* ctx, int B, int S, int heads,
               int hd, float scale, bool f16, hipStream_t s) {
  if (hd != HD) return;  // validated at model build time
  const dim3 grid((S + QT - 1) / QT, B * heads);
  if (f16)
    hipLaunchKernelGGL((attn_kernel<_Float16>), grid, dim3(256), 0, s, (const _Float16*)qkv,
                       mask_bias, (_Float16*)ctx, S, heads, scale);
  else
    hipLaunchKernelGGL((attn_kernel<float>), grid, dim3(256), 0, s, (const float*)qkv,
                       mask_bias, (float*)ctx, S, heads, scale);
}

}  // namespace spi
