// MFMA GEMM and conv-as-implicit-GEMM for gfx950 (CDNA4).
//
// One kernel body serves every dense contraction of the three model families:
//   * ResNet conv + folded BN (+ residual) (+ ReLU)      -- implicit GEMM over NHWC
//   * ResNet FC, BERT/ViT QKV / out-proj / FFN (+GELU) (+residual) -- dense GEMM
// Operands are K-contiguous on both sides (activations [M][K], weights packed
// [Npad][Kpad]), so each lane's MFMA fragment is one 16-byte chunk.
//
// Precision modes (template MODE):
//   F16   v_mfma_f32_16x16x32_f16; lane l holds A[row l&15][k 8(l>>4)..+7].
//   F32   v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain); lane l feeds k index
//         (l>>4) of step s with element 8(l>>4)+s of its 32-byte chunk (the k
//         order is permuted identically on A and B, so the sum is unchanged).
//   F16X3 split fp16: fp32 activations are split on the way into LDS as
//         a = a_hi + a_lo (two fp16), weights are stored as two fp16 planes,
//         and each fragment issues hi*hi + hi*lo + lo*hi (the lo*lo term is
//         below fp32 rounding): fp32-grade results at the fp16 MFMA rate.
// Accumulators follow the gfx950 C/D map: col = lane&15, row = 4(lane>>4)+r.
//
// Tiles are staged global -> registers -> LDS (double-buffered, one barrier per
// 32-deep K step, next tile's loads issued before the current tile's MFMAs).
// Small-M layers are split along K; the workgroups of a tile publish fp32
// slabs and the last one to arrive (agent-scope release -> ticket -> acquire,
// cdna_hip_programming.md G16 / "In-launch split-K reduction") sums them and
// runs the epilogue, so no separate reduce launch is needed.
#include "spi_kernels.hpp"

#include <algorithm>
#include <cstdio>

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;

struct KArgs {
  GemmDesc d;
  GemmPtrs p;
  int k_per_split;
  int tiles_m;
  int cin_shift;
};

template <int MODE>
struct Traits;
template <>
struct Traits<(int)Prec::F16> {
  using A = _Float16;   // A element in HBM
  using L = _Float16;   // LDS / MFMA operand element
  using Out = _Float16; // default C / residual element
  static constexpr int KC = 8, PLANES = 1, AV = 1;  // k per chunk, weight planes, uint4 per A chunk
};
template <>
struct Traits<(int)Prec::F32> {
  using A = float;
  using L = float;
  using Out = float;
  static constexpr int KC = 4, PLANES = 1, AV = 1;
};
template <>
struct Traits<(int)Prec::F16X3> {
  using A = float;
  using L = _Float16;
  using Out = float;
  static constexpr int KC = 8, PLANES = 2, AV = 2;
};

__device__ __forceinline__ float apply_act(float v, Act act) {
  if (act == Act::Relu) return v > 0.f ? v : 0.f;
  if (act == Act::Gelu) return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  return v;
}

template <int MODE>
__device__ __forceinline__ void epilogue_store(const KArgs& a, int m, int n, float v) {
  using Out = typename Traits<MODE>::Out;
  const GemmDesc& d = a.d;
  if (a.p.bias) v += a.p.bias[n];
  if (a.p.res) {
    const size_t idx = (size_t)m * d.ldr + n;
    v += d.res_f32 ? static_cast<const float*>(a.p.res)[idx]
                   : static_cast<float>(static_cast<const Out*>(a.p.res)[idx]);
  }
  v = apply_act(v, d.act);
  if (d.out_f32)
    static_cast<float*>(a.p.C)[(size_t)m * d.ldc + n] = v;
  else
    static_cast<Out*>(a.p.C)[(size_t)m * d.ldc + n] = static_cast<Out>(v);
}

__device__ __forceinline__ void split8(const uint4& x0, const uint4& x1, uint4& hi, uint4& lo) {
  const float* f0 = reinterpret_cast<const float*>(&x0);
  const float* f1 = reinterpret_cast<const float*>(&x1);
  half8 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 a = static_cast<_Float16>(f0[e]);
    const _Float16 b = static_cast<_Float16>(f1[e]);
    h[e] = a;
    h[e + 4] = b;
    l[e] = static_cast<_Float16>(f0[e] - static_cast<float>(a));
    l[e + 4] = static_cast<_Float16>(f1[e] - static_cast<float>(b));
  }
  hi = *reinterpret_cast<uint4*>(&h);
  lo = *reinterpret_cast<uint4*>(&l);
}

template <int MODE, int BM, int BN, bool CONV>
__global__ __launch_bounds__(256) void gemm_kernel(KArgs a) {
  using TR = Traits<MODE>;
  using AT = typename TR::A;
  using LT = typename TR::L;
  constexpr int KC = TR::KC;
  constexpr int CPR = BK / KC;                 // chunks per tile row
  constexpr int LPAD = 16 / (int)sizeof(LT);   // 16-byte row pad
  constexpr int LD = BK + LPAD;                // LDS row stride (elements)
  constexpr int A_PER_T = BM * CPR / 256;
  constexpr int B_PER_T = BN * CPR / 256;
  static_assert(A_PER_T >= 1 && B_PER_T >= 1, "tile too small");
  constexpr int PL = TR::PLANES;
  constexpr int PLANE = (BM + BN) * LD;        // one precision plane of one buffer
  constexpr int BUF = PL * PLANE;
  __shared__ __attribute__((aligned(16))) LT lds[2 * BUF];
  __shared__ int s_last;

  const GemmDesc& d = a.d;
  const int tid = threadIdx.x;
  const int tile = blockIdx.x;
  const int tm = tile % a.tiles_m;
  const int tn = tile / a.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * a.k_per_split;
  const int kend = min(d.Kpad, kbeg + a.k_per_split);
  const int ntiles = (kend - kbeg) / BK;

  const AT* __restrict__ Ap = static_cast<const AT*>(a.p.A);
  const LT* __restrict__ Wp = static_cast<const LT*>(a.p.W);

  int a_row[A_PER_T], a_kc[A_PER_T], a_ih0[A_PER_T], a_iw0[A_PER_T];
  bool a_ok[A_PER_T];
  size_t a_base[A_PER_T];
#pragma unroll
  for (int t = 0; t < A_PER_T; ++t) {
    const int c = tid + t * 256;
    a_row[t] = c / CPR;
    a_kc[t] = c % CPR;
    const int m = m0 + a_row[t];
    a_ok[t] = m < d.M;
    if constexpr (CONV) {
      const int ohw = d.OH * d.OW;
      const int mm = a_ok[t] ? m : 0;
      const int img = mm / ohw;
      const int rem = mm - img * ohw;
      const int oh = rem / d.OW;
      const int ow = rem - oh * d.OW;
      a_ih0[t] = oh * d.stride - d.pad;
      a_iw0[t] = ow * d.stride - d.pad;
      a_base[t] = (size_t)img * d.H * d.W * d.Cin;
    } else {
      a_ih0[t] = a_iw0[t] = 0;
      a_base[t] = (size_t)(a_ok[t] ? m : 0) * d.lda;
    }
  }

  uint4 ra[A_PER_T][TR::AV], rb[B_PER_T][PL];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t) {
      const int k = k0 + a_kc[t] * KC;
#pragma unroll
      for (int v = 0; v < TR::AV; ++v) ra[t][v] = make_uint4(0, 0, 0, 0);
      if (a_ok[t] && k < d.K) {
        const AT* src = nullptr;
        if constexpr (CONV) {
          const int cell = k >> a.cin_shift;
          const int c = k & (d.Cin - 1);
          const int kh = cell / d.KW;
          const int kw = cell - kh * d.KW;
          const int ih = a_ih0[t] + kh, iw = a_iw0[t] + kw;
          if ((unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W)
            src = Ap + a_base[t] + ((size_t)(ih * d.W + iw) << a.cin_shift) + c;
        } else {
          src = Ap + a_base[t] + k;
        }
        if (src) {
#pragma unroll
          for (int v = 0; v < TR::AV; ++v) ra[t][v] = reinterpret_cast<const uint4*>(src)[v];
        }
      }
    }
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int c = tid + t * 256;
      const int row = c / CPR, kc = c % CPR;
      const LT* src = Wp + (size_t)(n0 + row) * d.Kpad + k0 + kc * KC;
#pragma unroll
      for (int p = 0; p < PL; ++p) rb[t][p] = *reinterpret_cast<const uint4*>(src + (size_t)p * d.wplane);
    }
  };
  auto store_tile = [&](int buf) {
    LT* base = lds + buf * BUF;
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t) {
      LT* dst = base + a_row[t] * LD + a_kc[t] * KC;
      if constexpr (MODE == (int)Prec::F16X3) {
        uint4 hi, lo;
        split8(ra[t][0], ra[t][1], hi, lo);
        *reinterpret_cast<uint4*>(dst) = hi;
        *reinterpret_cast<uint4*>(dst + PLANE) = lo;
      } else {
        *reinterpret_cast<uint4*>(dst) = ra[t][0];
      }
    }
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int c = tid + t * 256;
      const int row = c / CPR, kc = c % CPR;
      LT* dst = base + (BM + row) * LD + kc * KC;
#pragma unroll
      for (int p = 0; p < PL; ++p) *reinterpret_cast<uint4*>(dst + p * PLANE) = rb[t][p];
    }
  };

  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TI = WTM / 16, TJ = WTN / 16;
  const int fr = lane & 15, fq = lane >> 4;
  floatx4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (ntiles > 0) {
    load_tile(kbeg);
    store_tile(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load_tile(kbeg + (t + 1) * BK);
    const LT* As = lds + cur * BUF;
    const LT* Bs = As + BM * LD;
    if constexpr (MODE == (int)Prec::F16) {
      half8 af[TI], bf[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        af[i] = *reinterpret_cast<const half8*>(As + (wm * WTM + i * 16 + fr) * LD + fq * 8);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        bf[j] = *reinterpret_cast<const half8*>(Bs + (wn * WTN + j * 16 + fr) * LD + fq * 8);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    } else if constexpr (MODE == (int)Prec::F16X3) {
      half8 ah[TI], al[TI], bh[TJ], bl[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const LT* s = As + (wm * WTM + i * 16 + fr) * LD + fq * 8;
        ah[i] = *reinterpret_cast<const half8*>(s);
        al[i] = *reinterpret_cast<const half8*>(s + PLANE);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const LT* s = Bs + (wn * WTN + j * 16 + fr) * LD + fq * 8;
        bh[j] = *reinterpret_cast<const half8*>(s);
        bl[j] = *reinterpret_cast<const half8*>(s + PLANE);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    } else {
      floatx4 a0[TI], a1[TI], b0[TJ], b1[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const float* src = reinterpret_cast<const float*>(As) + (wm * WTM + i * 16 + fr) * LD + fq * 8;
        a0[i] = *reinterpret_cast<const floatx4*>(src);
        a1[i] = *reinterpret_cast<const floatx4*>(src + 4);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const float* src = reinterpret_cast<const float*>(Bs) + (wn * WTN + j * 16 + fr) * LD + fq * 8;
        b0[j] = *reinterpret_cast<const floatx4*>(src);
        b1[j] = *reinterpret_cast<const floatx4*>(src + 4);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[i][s], b0[j][s], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[i][s], b1[j][s], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (gridDim.y == 1) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
          const int n = n0 + wn * WTN + j * 16 + fr;
          if (m < d.M && n < d.N) epilogue_store<MODE>(a, m, n, acc[i][j][r]);
        }
    return;
  }

  // ---- split-K: publish this slice's slab, the last arriver reduces -------
  // Slabs are written in fragment order (thread tid's accumulator (i, j) is 16
  // contiguous bytes at ((i*TJ + j)*256 + tid)*16), write-through (sc1) so no
  // release fence is needed; the ticket is a relaxed agent-scope atomic; the
  // reducer reads every slab with sc1 loads (cdna_hip_programming.md, "In-launch
  // split-K reduction", sc1 variant).  Same thread <-> (m, n) map as above.
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int splits = gridDim.y;
  constexpr int SLAB = BM * BN;
  float* tile_slabs = a.p.partial + (size_t)tile * splits * SLAB;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(tile_slabs, (short)0, splits * SLAB * 4, 0x00020000);
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int off = (blockIdx.y * SLAB + ((i * TJ + j) * 256 + tid) * 4) * 4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, off, 0, 16);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int ticket = __hip_atomic_fetch_add(a.p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = ticket == splits - 1;
    if (s_last) __hip_atomic_store(a.p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      floatx4 sum = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int z = 0; z < splits; ++z) {
        const int off = (z * SLAB + ((i * TJ + j) * 256 + tid) * 4) * 4;
        sum += __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
        const int n = n0 + wn * WTN + j * 16 + fr;
        if (m < d.M && n < d.N) epilogue_store<MODE>(a, m, n, sum[r]);
      }
    }
}

struct Plan {
  int bm, bn, splits, k_per_split;
};

Plan choose_plan(const GemmDesc& d) {
  constexpr int kTarget = 256;  // CUs
  static const int cfg[3][2] = {{128, 128}, {128, 64}, {64, 64}};
  Plan pl{64, 64, 1, d.Kpad};
  for (auto& c : cfg) {
    if (c[1] == 128 && d.N <= 64) continue;
    const int tiles = ((d.M + c[0] - 1) / c[0]) * ((d.N + c[1] - 1) / c[1]);
    if (tiles >= kTarget) {
      pl.bm = c[0];
      pl.bn = c[1];
      return pl;
    }
  }
  const int tiles = ((d.M + 63) / 64) * ((d.N + 63) / 64);
  const int ktiles = d.Kpad / BK;
  int splits = 1;
  if (tiles < kTarget / 2 && ktiles >= 8) splits = std::max(1, std::min(ktiles / 4, (2 * kTarget + tiles - 1) / tiles));
  const int kt_per = (ktiles + splits - 1) / splits;
  pl.k_per_split = kt_per * BK;
  pl.splits = (ktiles + kt_per - 1) / kt_per;
  return pl;
}

int ilog2(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

template <int MODE, int BM, int BN>
void launch_tile(const KArgs& a, dim3 grid, hipStream_t s) {
  if (a.d.conv)
    hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_kernel<MODE, BM, BN, false>), grid, dim3(256), 0, s, a);
}

template <int MODE>
void launch(const GemmDesc& d, const GemmPtrs& p, hipStream_t s) {
  const Plan pl = choose_plan(d);
  KArgs a{d, p, pl.k_per_split, (d.M + pl.bm - 1) / pl.bm, d.conv ? ilog2(d.Cin) : 0};
  const int tiles_n = (d.N + pl.bn - 1) / pl.bn;
  const dim3 grid(a.tiles_m * tiles_n, pl.splits);
  if (pl.bm == 128 && pl.bn == 128)
    launch_tile<MODE, 128, 128>(a, grid, s);
  else if (pl.bm == 128)
    launch_tile<MODE, 128, 64>(a, grid, s);
  else
    launch_tile<MODE, 64, 64>(a, grid, s);
}

}  // namespace

size_t gemm_partial_floats(const GemmDesc& d) {
  const Plan pl = choose_plan(d);
  if (pl.splits <= 1) return 0;
  const size_t tiles = (size_t)((d.M + pl.bm - 1) / pl.bm) * ((d.N + pl.bn - 1) / pl.bn);
  return tiles * pl.splits * pl.bm * pl.bn;
}

size_t gemm_counter_slots(const GemmDesc& d) {
  const Plan pl = choose_plan(d);
  if (pl.splits <= 1) return 0;
  return (size_t)((d.M + pl.bm - 1) / pl.bm) * ((d.N + pl.bn - 1) / pl.bn);
}

void gemm(const GemmDesc& d, const GemmPtrs& p, Prec prec, hipStream_t s) {
  switch (prec) {
    case Prec::F16:
      launch<(int)Prec::F16>(d, p, s);
      break;
    case Prec::F32:
      launch<(int)Prec::F32>(d, p, s);
      break;
    case Prec::F16X3:
      launch<(int)Prec::F16X3>(d, p, s);
      break;
  }
}

}  // namespace spi
