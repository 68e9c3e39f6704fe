// Fused QKV projection + multi-head attention for sequences of at most 256 tokens (BERT-base at
// seq 128, ViT-L/16 at 197: north_star's "QKV-GEMM + softmax fused"), fp16, gfx950.
//
// One 8-wave workgroup per (sequence b, head h), QR = 128 or 256 token rows (S <= QR):
//   1. GEMM: the sequence's <= QR token rows (the fp16 copy of the layer input, or of the
//      pre-LayerNorm rows when the LayerNorm is folded -- ln_fold.hpp's consumer epilogue)
//      times the head's 192 packed QKV weight rows (q | k | v, 64 each), K = D.  Both operands
//      go HBM -> LDS by LDS-DMA (1 KiB pieces, (QR + 192) / 64 per wave per 64-deep k-step, the
//      XOR swizzle on the source address) through a 2-stage ring (QR 128: 80 KiB, two workgroups
//      per CU; QR 256: 112 KiB); waves 2 (rows) x 4 (columns), a QR/2 x 48 output block each,
//      v_mfma_f32_16x16x32_f16.
//   2. Epilogue: bias (+ the fold's rstd (acc - mean c1)) and the fp16 rounding the unfused
//      QKV GEMM applies, into LDS as Q / K / V [QR][72] (144-byte rows) over the ring.
//   3. Attention on the LDS-resident Q / K / V: attention.hip's swapped orientation (S^T = K Q^T,
//      the query on the lane, online softmax in fp32, P^T kept in registers as the B operand of
//      O^T = V^T P^T, V^T fragments by ds_read_b64_tr_b16), 16 queries per wave per pass (QR / 128
//      passes); every key of the sequence is already in LDS, so no K / V staging or barrier
//      between key tiles.
// Replaces the QKV GEMM launch, the Q / K / V round trip through HBM (B S 3 D fp16 written and
// read back) and the attention launch's own staging.  Same arithmetic as the unfused pair
// (fp16 Q / K / V, fp32 scores and softmax, fp16 P), DESIGN.md 3.7.
#include "ln_fold.hpp"
#include "spi_kernels.hpp"

#include <cstdlib>
#include <stdexcept>

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_s4;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int HD = 64;                      // head dim
constexpr int QC = 3 * HD;                  // q | k | v columns of one head
constexpr int LDQ = HD + 8;                 // Q / K / V row stride in elements (144 B)
// Geometry by token rows per workgroup QR (S <= QR): one 64-deep k-step of A is QR x 128 bytes,
// of W 192 x 128; 1 KiB LDS-DMA pieces per stage, per wave; Q / K / V over the ring after the
// k-loop, the rows' {mean, rstd} (fold) after them.
// HP heads per workgroup (round 6): 8 HP waves, the A rows staged once for the HP heads' W rows.
template <int QR, int HP = 1>
struct QkvGeo {
  static constexpr int A_BYTES = QR * 128;               // 16 / 32 KiB
  static constexpr int W_BYTES = QC * 128;               // one head's 192 W rows: 24 KiB
  static constexpr int STAGE = A_BYTES + HP * W_BYTES;   // 40 / 56 KiB (HP 2: 64 KiB)
  static constexpr int PIECES = (QR + HP * QC) / 8;      // 40 / 56 (HP 2: 64)
  static constexpr int PPW = PIECES / (8 * HP);          // 5 / 7 (HP 2: 4)
  static constexpr int HEAD_QKV = 3 * QR * LDQ * 2;      // one head's Q / K / V
  static constexpr int QKV_BYTES = HP * HEAD_QKV;
  static constexpr int STATS_OFF = QKV_BYTES;
  static constexpr int MI = QR / 32;                     // 16-row fragments per wave (2 wave rows)
  static_assert(PIECES % (8 * HP) == 0 && STATS_OFF + QR * 8 <= 2 * STAGE, "tile geometry");
};

struct QkvAttnArgs {
  const _Float16* A;  // [B S][lda] fp16 rows
  const _Float16* W;  // packed [Npad][ldw] fp16: rows 0..D-1 q, D..2D-1 k, 2D..3D-1 v
  const float* bias;  // [3 D]
  const float* ln_stats;  // fold: the A rows' chunk statistics ([B S][chunks][2]), else null
  const float* c1;        // fold: [3 D]
  const float* mask_bias; // [B S] additive key bias, or null
  _Float16* ctx;          // [B S][D]
  int lda, ldw, S, H, K, ln_chunks;
  float ln_eps, scale;
};

template <int N>
__device__ __forceinline__ void wait_vm_bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));  // vmcnt(N) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// STG ring stages: 3 (120 KiB, stage t + 2 in flight while t computes) or 2 (80 KiB: two
// workgroups fit a CU)
template <bool LNC, int STG, int QR, int HP = 1>
__global__ __launch_bounds__(512 * HP) void qkv_attn_kernel(const QkvAttnArgs g) {
  using Geo = QkvGeo<QR, HP>;
  constexpr int A_BYTES = Geo::A_BYTES, STAGE = Geo::STAGE, PPW = Geo::PPW, STATS_OFF = Geo::STATS_OFF;
  constexpr int MI = Geo::MI;
  __shared__ __attribute__((aligned(16))) char lds[STG * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave_g = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  // HP > 1: waves 8 hw .. 8 hw + 7 own head hw of the workgroup's HP (the loop below is the
  // one-head kernel's, on the head's W image and Q / K / V region); the A pieces are shared
  const int hw = wave_g >> 3, wave = wave_g & 7;
  const int hgroups = g.H / HP;
  const int b = blockIdx.x / hgroups, h0 = (blockIdx.x - b * hgroups) * HP, h = h0 + hw;
  const int S = g.S, D = g.H * HD;
  const size_t tok0 = (size_t)b * S;

  // LDS-DMA sources of this wave's PPW pieces (k-step 0): pieces 0 .. QR/8 - 1 the A rows, the
  // rest the W rows (tile column c -> packed row (c / 64) D + 64 h + c % 64)
  const char* src[PPW];
  int dst[PPW];
  {
    const int rl = lane >> 3, chunk = (lane & 7) ^ rl;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pc = wave_g * PPW + j;
      if (pc < QR / 8) {
        const int r = pc * 8 + rl;
        src[j] = reinterpret_cast<const char*>(g.A + (tok0 + min(r, S - 1)) * g.lda) + chunk * 16;
        dst[j] = pc * 1024;
      } else {
        const int cw = (pc - QR / 8) * 8 + rl;  // W image row: head cw / 192, column cw % 192
        const int c = cw % QC;
        const int wrow = (c >> 6) * D + (h0 + cw / QC) * HD + (c & 63);
        src[j] = reinterpret_cast<const char*>(g.W + (size_t)wrow * g.ldw) + chunk * 16;
        dst[j] = A_BYTES + (pc - QR / 8) * 1024;
      }
    }
  }
  auto stage = [&](int t) {
    char* buf = lds + (t % STG) * STAGE;
#pragma unroll
    for (int j = 0; j < PPW; ++j)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[j] + t * 128), (lds_ptr_t)(buf + dst[j]),
                                       16, 0, 0);
  };
  const int KT = g.K >> 6;
  // the fold's row statistics, once per row: the chunk loads go out first, the first two stages'
  // DMAs behind them, so waiting for the loads (vmcnt(2 PPW)) does not wait for the stages
  float2* const st = reinterpret_cast<float2*>(lds + STATS_OFF);
  [[maybe_unused]] float2 ch[16];
  if constexpr (LNC) {
    const float2* p = reinterpret_cast<const float2*>(g.ln_stats) + (tok0 + min(tid & (QR - 1), S - 1)) * g.ln_chunks;
#pragma unroll
    for (int c = 0; c < 16; ++c) ch[c] = p[min(c, g.ln_chunks - 1)];  // straight-line loads: counted vmcnt
#pragma unroll
    for (int c = 0; c < 16; ++c) ch[c] = c < g.ln_chunks ? ch[c] : float2{0.f, 0.f};
  }
  stage(0);
  if constexpr (STG == 3) stage(1);  // KT >= 2 (checked on the host): no branch, so the loads' wait stays counted
  [[maybe_unused]] float2 row_st = float2{0.f, 0.f};  // thread tid < 128: row tid's {mean, rstd}
  if constexpr (LNC) {
    {  // ln_row_stats' arithmetic (Chan) on the loaded partials; chunks <= 16 (D <= 1024); branch-free
      float sm = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) sm += ch[c].x;
      const float mean = sm / (float)g.ln_chunks;
      float m2 = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float dm = ch[c].x - mean;
        m2 += c < g.ln_chunks ? ch[c].y + 64.f * dm * dm : 0.f;
      }
      // kept in registers through the k-loop: an LDS store here, behind the stages' LDS-DMA into
      // the same array, would make hipcc drain them (vmcnt(0)) first
      row_st = float2{mean, rsqrtf(m2 / (64.f * (float)g.ln_chunks) + g.ln_eps)};
    }
  }

  const int wr = wave >> 2, wc = wave & 3;
  floatx4 acc[MI][3];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto rd = [&](const char* img, int row, int c) -> half8 {
    return *reinterpret_cast<const half8*>(img + row * 128 + ((c ^ (row & 7)) << 4));
  };
  for (int t = 0; t < KT; ++t) {
    // STG = 3: stage t landed (stage t + 1's pieces may stay in flight); every wave is past step
    // t - 1's reads, so the buffer of t + 2 (= that of t - 1) is free.  STG = 2: stage t landed,
    // then stage t + 1 goes into the buffer of t - 1.
    if (STG == 3 && t + 1 < KT)
      wait_vm_bar<PPW>();
    else
      wait_vm_bar<0>();
    if (t + STG - 1 < KT) stage(t + STG - 1);
    const char* buf = lds + (t % STG) * STAGE;
    half8 fa[2][MI], fb[2][3];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[kk][i] = rd(buf, (QR / 2) * wr + 16 * i + fr, kk * 4 + fq);
#pragma unroll
      for (int j = 0; j < 3; ++j) fb[kk][j] = rd(buf + A_BYTES + hw * Geo::W_BYTES, 48 * wc + 16 * j + fr, kk * 4 + fq);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // the ring's last reads are done: Q / K / V go over it
  if constexpr (LNC) {
    if (tid < QR) st[tid] = row_st;
    __syncthreads();
  }

  // epilogue: acc[i][j][v] is row (QR / 2) wr + 16 i + 4 fq + v, tile column 48 wc + 16 j + fr
  _Float16* const Qs = reinterpret_cast<_Float16*>(lds + hw * Geo::HEAD_QKV);
  _Float16* const Ks = Qs + QR * LDQ;
  _Float16* const Vs = Ks + QR * LDQ;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = 48 * wc + 16 * j + fr, part = c >> 6, d = c & 63;
    const int wrow = part * D + h * HD + d;
    const float bc = g.bias[wrow];
    [[maybe_unused]] float c1 = 0.f;
    if constexpr (LNC) c1 = g.c1[wrow];
    _Float16* const dstp = Qs + part * (QR * LDQ) + d;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int r = (QR / 2) * wr + 16 * i + 4 * fq + v;
        float y = acc[i][j][v];
        if constexpr (LNC) {
          const float2 s2 = st[r];
          y = s2.y * (y - s2.x * c1);
        }
        y += bc;
        dstp[r * LDQ] = r < S ? static_cast<_Float16>(y) : static_cast<_Float16>(0.f);
      }
  }
  __syncthreads();

  // attention: wave w owns queries 16 w .. 16 w + 15 of each 128-query pass (attention.hip's
  // swapped kernel, all keys in LDS)
  const int tr_off = ((4 * fq + (fr >> 2)) * LDQ + 4 * (fr & 3)) * 2;
  const float* mb = g.mask_bias ? g.mask_bias + tok0 : nullptr;
  for (int q0 = 16 * wave; q0 < S; q0 += 128) {  // wave-uniform; no barrier follows
    const int qa = q0 + fr;
    half8 qf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[s] = *reinterpret_cast<const half8*>(Qs + qa * LDQ + s * 32 + fq * 8);
    float m_q = -INFINITY, l_q = 0.f;
    floatx4 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < S; k0 += 64) {
      const int kleft = S - k0;
      floatx4 sacc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sacc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (j * 16 < kleft) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const half8 kf = *reinterpret_cast<const half8*>(Ks + (k0 + j * 16 + fr) * LDQ + s * 32 + fq * 8);
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
          const float bias = key < S ? (mb ? mb[key] : 0.f) : -INFINITY;
          sc[j][r] = sacc[j][r] * g.scale + bias;
          tmax = fmaxf(tmax, sc[j][r]);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float m_new = fmaxf(m_q, tmax);
      const float alpha = __expf(m_q - m_new);
      float rs = 0.f;
      half8 pf[2];
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
      __attribute__((address_space(3))) char* vb = (__attribute__((address_space(3))) char*)Vs + tr_off + k0 * LDQ * 2;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s * 32 >= kleft) break;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const half4 lo = __builtin_bit_cast(
              half4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vb + ((32 * s) * LDQ + 16 * d) * 2)));
          const half4 hi = __builtin_bit_cast(
              half4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(vb + ((32 * s + 16) * LDQ + 16 * d) * 2)));
          const half8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[d] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf[s], o[d], 0, 0, 0);
        }
      }
    }
    if (qa < S) {
      const float inv = 1.f / l_q;
      _Float16* out = g.ctx + (tok0 + qa) * D + h * HD + fq * 4;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const half4 v = {static_cast<_Float16>(o[d][0] * inv), static_cast<_Float16>(o[d][1] * inv),
                         static_cast<_Float16>(o[d][2] * inv), static_cast<_Float16>(o[d][3] * inv)};
        *reinterpret_cast<half4*>(out + d * 16) = v;
      }
    }
  }
}

}  // namespace

constexpr int kQkvMaxS = 256;

// SPI_QKV_HP=2: two heads per 16-wave workgroup for S <= 128 (the A rows staged once for both:
// 20 % fewer bytes per head into LDS; 128 KiB, one workgroup per CU).  Bit-identical, but BERT-base
// bs8 under the four streams 25.1k -> 24.2k (-3.7 %, profiles/r06/rejected/): a 16-wave, 128 KiB
// workgroup waits for a whole free CU, so the default stays one head per workgroup
static int g_qkv_hp = -1;
void qkv_attn_reload_env() { g_qkv_hp = -1; }
static int qkv_hp() {
  if (g_qkv_hp < 0) {
    const char* e = std::getenv("SPI_QKV_HP");
    g_qkv_hp = (e && *e && std::atoi(e) == 2) ? 2 : 1;
  }
  return g_qkv_hp;
}

bool qkv_attention_eligible(int S, int heads, int hd, int K, int kpad, int krep, int lda, int ldw) {
  return S >= 1 && S <= kQkvMaxS && hd == HD && heads >= 2 && K == heads * HD && kpad == K && krep == 1 && K % 64 == 0 &&
         lda % 8 == 0 && ldw % 8 == 0;
}

void qkv_attention(const void* A, int lda, const void* W, int ldw, const float* bias, const float* ln_stats,
                   const float* c1, int ln_chunks, float ln_eps, const float* mask_bias, void* ctx, int B, int S,
                   int heads, float scale, hipStream_t s) {
  if (S < 1 || S > kQkvMaxS) throw std::invalid_argument("qkv_attention: 1 <= S <= 256");
  if (heads * HD < 128) throw std::invalid_argument("qkv_attention: K = heads * 64 >= 128");
  if ((reinterpret_cast<uintptr_t>(A) & 15) || (reinterpret_cast<uintptr_t>(W) & 15) || lda % 8 || ldw % 8)
    throw std::invalid_argument("qkv_attention: 16-byte aligned A / W rows");
  if (ln_stats && (!c1 || ln_chunks < 1 || ln_chunks > 16))
    throw std::invalid_argument("qkv_attention: fold needs c1 and 1..16 chunks");
  QkvAttnArgs g;
  g.A = static_cast<const _Float16*>(A);
  g.W = static_cast<const _Float16*>(W);
  g.bias = bias;
  g.ln_stats = ln_stats;
  g.c1 = c1;
  g.mask_bias = mask_bias;
  g.ctx = static_cast<_Float16*>(ctx);
  g.lda = lda;
  g.ldw = ldw;
  g.S = S;
  g.H = heads;
  g.K = heads * HD;
  g.ln_chunks = ln_chunks;
  g.ln_eps = ln_eps;
  g.scale = scale;
  const dim3 grid(B * heads), blk(512);
  // two stages (QR 128: 80 KiB, two workgroups per CU): BERT-base bs8 four streams 24.7-24.8k
  // seq/s against 24.0k with three (120 KiB) and 23.3-23.4k unfused (profiles/r05/qkv_attn/);
  // sequences of 129..256 tokens (ViT at 197) take the 256-row tile (112 KiB)
  if (S <= 128 && heads % 2 == 0 && qkv_hp() == 2) {
    const dim3 grid2(B * heads / 2), blk2(1024);
    if (ln_stats)
      SPI_LAUNCH((qkv_attn_kernel<true, 2, 128, 2>), grid2, blk2, 0, s, g);
    else
      SPI_LAUNCH((qkv_attn_kernel<false, 2, 128, 2>), grid2, blk2, 0, s, g);
  } else if (S <= 128) {
    if (ln_stats)
      SPI_LAUNCH((qkv_attn_kernel<true, 2, 128>), grid, blk, 0, s, g);
    else
      SPI_LAUNCH((qkv_attn_kernel<false, 2, 128>), grid, blk, 0, s, g);
  } else {
    if (ln_stats)
      SPI_LAUNCH((qkv_attn_kernel<true, 2, 256>), grid, blk, 0, s, g);
    else
      SPI_LAUNCH((qkv_attn_kernel<false, 2, 256>), grid, blk, 0, s, g);
  }
}

}  // namespace spi
