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

#include <cstdlib>

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

// fp16, swapped orientation (round 3): S^T = K Q^T puts the key on the MFMA row and the
// query on the lane (cdna_hip_programming.md §3, "An accumulator tile as the next MFMA's
// operand"), so
//   * a lane's softmax row is its own query: the row max / sum are the lane's 16 scores
//     plus two xor shuffles (lanes 16 and 32 apart) instead of four per row;
//   * P^T leaves the accumulators already shaped as the B operand of O^T = V^T P^T -- the
//     fp32 -> fp16 conversion only, no LDS round trip for P (the round-2 kernel wrote P
//     with 16 two-byte stores per lane per tile and read it back);
//   * V stays row-major in LDS (16-byte stores, no scalar transpose on the way in) and
//     V^T's A fragments come out of it by ds_read_b64_tr_b16 (T10): lane 4q + p of a
//     16-lane group addresses row q, columns 4p..4p+3 of a 4 x 16 block, lane i receives
//     column i.  The k order inside a 32-key step is the accumulator's: element j of
//     lane group g is key 16 (2 s + j / 4) + 4 g + j % 4, on both operands.
// O^T's accumulator holds 4 consecutive head dims of one query per lane: 8-byte stores.
// NW waves per workgroup = 16 NW query rows: 4 (BERT) or 8 (ViT's S = 197: the K / V tiles are
// staged once per 128 queries instead of per 64; 2 query tiles per head instead of 4).
// SK > 0 (round 6, S <= SK): the whole sequence's K and V are staged once (SK rows, zero past
// S) behind one barrier, and the key-tile loop runs with no barrier and no global load: ViT's
// four 64-key tiles no longer pay a load-latency + barrier round trip each.  NW = 16 with SK: one
// workgroup per (batch, head), so K / V are read once per head.
template <int NW, int SK>
__global__ __launch_bounds__(64 * NW) void attn_f16_swapped_kernel(const _Float16* __restrict__ qkv,
                                                               const float* __restrict__ mask_bias,
                                                               _Float16* __restrict__ ctx, int S, int H,
                                                               float scale) {
  typedef _Float16 half4 __attribute__((ext_vector_type(4)));
  typedef short short4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) short4v lds_s4;
  constexpr int LD = HD + 8;  // K / V row stride in elements (144 B: 16-byte rows, 8-byte tr reads)
  constexpr int KR = SK ? SK : KT;  // staged key rows
  __shared__ __attribute__((aligned(16))) _Float16 Ks[KR * LD];
  __shared__ __attribute__((aligned(16))) _Float16 Vs[KR * LD];

  const int D = H * HD, ld = 3 * D;
  const int b = blockIdx.y / H, h = blockIdx.y % H;
  constexpr int NT = 64 * NW;
  const int q0 = blockIdx.x * (16 * NW);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const _Float16* base = qkv + (size_t)b * S * ld;

  // Q^T as the B operand: lane (fq, fr) holds Q[query fr][head dims 32 s + 8 fq ..]
  const int qa = q0 + wave * 16 + fr;
  half8 qf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (qa < S) v = *reinterpret_cast<const half8*>(base + (size_t)qa * ld + h * HD + s * 32 + fq * 8);
    qf[s] = v;
  }
  float m_q = -INFINITY, l_q = 0.f;  // this lane's query
  floatx4 o[4];                      // o[dblk][r]: head dim 16 dblk + 4 fq + r of query fr
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = floatx4{0.f, 0.f, 0.f, 0.f};

  constexpr int NCH = KT * HD / 8 / NT > 0 ? KT * HD / 8 / NT : 1;  // 16-byte chunks of K (and V) per thread per tile
  uint4 kreg[NCH], vreg[NCH];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * NT;
      const int key = c / (HD / 8), dc = c % (HD / 8);
      const int kk = k0 + key;
      kreg[i] = vreg[i] = make_uint4(0, 0, 0, 0);
      if (kk < S) {
        kreg[i] = *reinterpret_cast<const uint4*>(base + (size_t)kk * ld + D + h * HD + dc * 8);
        vreg[i] = *reinterpret_cast<const uint4*>(base + (size_t)kk * ld + 2 * D + h * HD + dc * 8);
      }
    }
  };
  // tr-read addresses (byte offsets into Vs) of lane (fq, fr) for key half t of step s and
  // head-dim block dblk: row 32 s + 16 t + 4 fq + fr / 4, columns 16 dblk + 4 (fr % 4)
  const int tr_off = ((4 * fq + (fr >> 2)) * LD + 4 * (fr & 3)) * 2;
  const bool live = q0 + wave * 16 < S;  // wave-uniform
  if constexpr (SK > 0) {
    // the whole sequence: SK * 8 16-byte chunks of K and of V, rows past S zero (V's rows
    // past S meet P = 0 in the last 32-key step, so they must be finite)
    constexpr int NW_CH = (SK * (HD / 8) + NT - 1) / NT;
    uint4 kw[NW_CH], vw[NW_CH];
#pragma unroll
    for (int i = 0; i < NW_CH; ++i) {
      const int c = tid + i * NT;
      const int key = c / (HD / 8), dc = c % (HD / 8);
      kw[i] = vw[i] = make_uint4(0, 0, 0, 0);
      if (key < S) {
        kw[i] = *reinterpret_cast<const uint4*>(base + (size_t)key * ld + D + h * HD + dc * 8);
        vw[i] = *reinterpret_cast<const uint4*>(base + (size_t)key * ld + 2 * D + h * HD + dc * 8);
      }
    }
#pragma unroll
    for (int i = 0; i < NW_CH; ++i) {
      const int c = tid + i * NT;
      const int key = c / (HD / 8), dc = c % (HD / 8);
      if (key < SK) {
        *reinterpret_cast<uint4*>(Ks + key * LD + dc * 8) = kw[i];
        *reinterpret_cast<uint4*>(Vs + key * LD + dc * 8) = vw[i];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (!live) return;  // no barrier follows
  } else {
    fetch(0);
  }
  for (int k0 = 0; k0 < S; k0 += KT) {
    if constexpr (SK == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // the previous tile's reads are done
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int c = tid + i * NT;
        const int key = c / (HD / 8), dc = c % (HD / 8);
        *reinterpret_cast<uint4*>(Ks + key * LD + dc * 8) = kreg[i];
        *reinterpret_cast<uint4*>(Vs + key * LD + dc * 8) = vreg[i];
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (k0 + KT < S) fetch(k0 + KT);
    }

    // A wave whose 16 queries all lie past S (ViT's last query tile: 5 of 64 rows) only
    // stages; key blocks past S skip their MFMAs (their scores are -inf through the bias, so
    // their P is 0 either way).  Both conditions are wave-uniform (EXEC stays full for the
    // transposed reads).
    if (!live) continue;
    const int kleft = S - k0;
    const int kb = SK ? k0 : 0;  // the tile's first staged row
    // S^T: sacc[j][r] = score of key k0 + 16 j + 4 fq + r for query fr
    floatx4 sacc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sacc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (j * 16 < kleft) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const half8 kf = *reinterpret_cast<const half8*>(Ks + (kb + j * 16 + fr) * LD + s * 32 + fq * 8);
          sacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[s], sacc[j], 0, 0, 0);
        }
      }
    }
    float sc[4][4];
    float tmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + j * 16 + fq * 4 + r;
        const float bias = key < S ? (mask_bias ? mask_bias[(size_t)b * S + key] : 0.f) : -INFINITY;
        sc[j][r] = sacc[j][r] * scale + bias;
        tmax = fmaxf(tmax, sc[j][r]);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_q, tmax);
    const float alpha = __expf(m_q - m_new);
    float rs = 0.f;
    half8 pf[2];  // P^T as the B operand of step s: element 4 t + r = key 16 (2 s + t) + 4 fq + r
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(sc[j][r] - m_new);
        rs += p;
        pf[j >> 1][(j & 1) * 4 + r] = static_cast<_Float16>(p);
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l_q = l_q * alpha + rs;
    m_q = m_new;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] *= alpha;

    // O^T += V^T P^T
    __attribute__((address_space(3))) char* vb =
        (__attribute__((address_space(3))) char*)Vs + tr_off + kb * LD * 2;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s * 32 >= kleft) break;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const half4 lo = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vb + ((32 * s) * LD + 16 * d) * 2)));
        const half4 hi = __builtin_bit_cast(
            half4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vb + ((32 * s + 16) * LD + 16 * d) * 2)));
        const half8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf[s], o[d], 0, 0, 0);
      }
    }
  }

  if (qa < S) {
    const float inv = 1.f / l_q;
    _Float16* out = ctx + ((size_t)b * S + qa) * D + h * HD + fq * 4;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const half4 v = {static_cast<_Float16>(o[d][0] * inv), static_cast<_Float16>(o[d][1] * inv),
                       static_cast<_Float16>(o[d][2] * inv), static_cast<_Float16>(o[d][3] * inv)};
      *reinterpret_cast<half4*>(out + d * 16) = v;
    }
  }
}

}  // namespace

// SPI_ATTN_WHOLE (S in 129..224): 2 (default) one 16-wave workgroup per (batch, head), 1 two 8-wave
// workgroups per head, both staging the whole K / V once; 0 the per-tile staging.  ViT-L under the
// four streams: 2 +1.4 %, 1 +0.6 % over 0 (profiles/r06/attn_whole/)
static int g_attn_whole = -1;
static int attn_knobs_whole() {
  if (g_attn_whole < 0) {
    const char* e = std::getenv("SPI_ATTN_WHOLE");
    g_attn_whole = (e && *e) ? std::atoi(e) : 2;
  }
  return g_attn_whole;
}

void attention_reload_env() { g_attn_whole = -1; }

// fp16: the swapped orientation, 8-wave workgroups of 128 queries for S > 128 (ViT-L's 197),
// 4 waves of 64 queries otherwise; fp32: the round-2 orientation (the round-2 fp16 kernel
// and the forced 4 / 8-wave variants were removed in round 4).
void attention(const void* qkv, const float* mask_bias, void* ctx, int B, int S, int heads,
               int hd, float scale, bool f16, hipStream_t s) {
  if (hd != HD) return;  // validated at model build time
  const dim3 grid((S + QT - 1) / QT, B * heads);
#ifndef SPI_ATTN_S8_MIN  // variant builds: the 8-wave kernel from this sequence length on
#define SPI_ATTN_S8_MIN 129
#endif
  if (f16 && S >= SPI_ATTN_S8_MIN) {
    const dim3 g8((S + 127) / 128, B * heads);
    // whole-sequence staging up to 224 keys (64.5 KiB: two workgroups per CU), tiles beyond;
    // the 16-wave form stages K / V once per head instead of once per 128 queries
    const int whole = attn_knobs_whole();
    if (whole == 2 && S <= 224)  // one 16-wave workgroup per (batch, head): K / V staged once per head
      SPI_LAUNCH((attn_f16_swapped_kernel<16, 224>), dim3((S + 255) / 256, B * heads), dim3(1024), 0, s,
                 (const _Float16*)qkv, mask_bias, (_Float16*)ctx, S, heads, scale);
    else if (whole && S <= 224)
      SPI_LAUNCH((attn_f16_swapped_kernel<8, 224>), g8, dim3(512), 0, s, (const _Float16*)qkv, mask_bias,
                 (_Float16*)ctx, S, heads, scale);
    else
      SPI_LAUNCH((attn_f16_swapped_kernel<8, 0>), g8, dim3(512), 0, s, (const _Float16*)qkv, mask_bias,
                 (_Float16*)ctx, S, heads, scale);
  } else if (f16) {
    SPI_LAUNCH((attn_f16_swapped_kernel<4, 0>), grid, dim3(256), 0, s, (const _Float16*)qkv, mask_bias,
                       (_Float16*)ctx, S, heads, scale);
  } else {
    SPI_LAUNCH((attn_kernel<float>), grid, dim3(256), 0, s, (const float*)qkv,
                       mask_bias, (float*)ctx, S, heads, scale);
  }
}

}  // namespace spi
