// MFMA GEMM and conv-as-implicit-GEMM for gfx950 (CDNA4).
//
// One kernel body serves every dense contraction of the three model families:
//   * ResNet conv + folded BN (+ residual) (+ ReLU)      -- implicit GEMM over NHWC
//   * ResNet FC, BERT/ViT QKV / out-proj / FFN (+GELU) (+residual) -- dense GEMM
// Operands are K-contiguous on both sides (activations [M][K], weights packed
// [Npad][Kpad]), so each lane's MFMA fragment is one 16-byte chunk:
//   f16: v_mfma_f32_16x16x32_f16 -- lane l holds A[row l&15][k 8(l>>4)..+7]
//   f32: v_mfma_f32_16x16x4_f32  -- exact fp32 FMA chain; lane l feeds k index
//        (l>>4) of step s with element 8(l>>4)+s of its 32-byte chunk (the
//        k order is permuted identically on A and B, so the sum is unchanged).
// Accumulators follow the gfx950 C/D map: col = lane&15, row = 4(lane>>4)+r.
//
// Tiles are staged global -> registers -> LDS (double-buffered, one barrier per
// 32-deep K step, next tile's loads issued before the current tile's MFMAs).
// Small-M layers (ResNet layer4 at M = 49*B) are split along K into fp32
// partial slabs reduced by a second kernel that applies the epilogue.
#include "spi_kernels.hpp"

#include <algorithm>
#include <cstdio>

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct KArgs {
  GemmDesc d;
  GemmPtrs p;
  int k_per_split;
  int tiles_m;
  int cin_shift;
};

__device__ __forceinline__ float apply_act(float v, Act act) {
  if (act == Act::Relu) return v > 0.f ? v : 0.f;
  if (act == Act::Gelu) return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  return v;
}

template <typename T>
__device__ __forceinline__ float load_res(const void* res, bool res_f32, size_t idx) {
  if (res_f32) return static_cast<const float*>(res)[idx];
  return static_cast<float>(static_cast<const T*>(res)[idx]);
}

template <typename T>
__device__ __forceinline__ void epilogue_store(const KArgs& a, int m, int n, float v) {
  const GemmDesc& d = a.d;
  if (a.p.bias) v += a.p.bias[n];
  if (a.p.res) v += load_res<T>(a.p.res, d.res_f32, (size_t)m * d.ldr + n);
  v = apply_act(v, d.act);
  if (d.out_f32)
    static_cast<float*>(a.p.C)[(size_t)m * d.ldc + n] = v;
  else
    static_cast<T*>(a.p.C)[(size_t)m * d.ldc + n] = static_cast<T>(v);
}

template <typename T, int BM, int BN, bool CONV>
__global__ __launch_bounds__(256) void gemm_kernel(KArgs a) {
  constexpr int BK = 32;
  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-byte chunk
  constexpr int CPR = BK / EPC;             // chunks per tile row
  constexpr int LDS_LD = BK + EPC;          // padded row (elements)
  constexpr int A_PER_T = BM * CPR / 256;
  constexpr int B_PER_T = BN * CPR / 256;
  static_assert(A_PER_T >= 1 && B_PER_T >= 1, "tile too small");
  constexpr int BUF = (BM + BN) * LDS_LD;
  __shared__ __attribute__((aligned(16))) T lds[2 * BUF];

  const GemmDesc& d = a.d;
  const int tid = threadIdx.x;
  const int tm = blockIdx.x % a.tiles_m;
  const int tn = blockIdx.x / a.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * a.k_per_split;
  const int kend = min(d.Kpad, kbeg + a.k_per_split);
  const int ntiles = (kend - kbeg) / BK;

  const T* __restrict__ Ap = static_cast<const T*>(a.p.A);
  const T* __restrict__ Wp = static_cast<const T*>(a.p.W);

  // Per-thread A row bookkeeping (fixed across the K loop).
  int a_row[A_PER_T], a_kc[A_PER_T];
  bool a_ok[A_PER_T];
  int a_ih0[A_PER_T], a_iw0[A_PER_T];
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

  uint4 ra[A_PER_T], rb[B_PER_T];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t) {
      const int k = k0 + a_kc[t] * EPC;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_ok[t] && k < d.K) {
        if constexpr (CONV) {
          const int cell = k >> a.cin_shift;
          const int c = k & (d.Cin - 1);
          const int kh = cell / d.KW;
          const int kw = cell - kh * d.KW;
          const int ih = a_ih0[t] + kh, iw = a_iw0[t] + kw;
          if ((unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W)
            v = *reinterpret_cast<const uint4*>(
                Ap + a_base[t] + ((size_t)(ih * d.W + iw) << a.cin_shift) + c);
        } else {
          v = *reinterpret_cast<const uint4*>(Ap + a_base[t] + k);
        }
      }
      ra[t] = v;
    }
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int c = tid + t * 256;
      const int row = c / CPR, kc = c % CPR;
      rb[t] = *reinterpret_cast<const uint4*>(Wp + (size_t)(n0 + row) * d.Kpad + k0 + kc * EPC);
    }
  };
  auto store_tile = [&](int buf) {
    T* As = lds + buf * BUF;
    T* Bs = As + BM * LDS_LD;
#pragma unroll
    for (int t = 0; t < A_PER_T; ++t)
      *reinterpret_cast<uint4*>(As + a_row[t] * LDS_LD + a_kc[t] * EPC) = ra[t];
#pragma unroll
    for (int t = 0; t < B_PER_T; ++t) {
      const int c = tid + t * 256;
      const int row = c / CPR, kc = c % CPR;
      *reinterpret_cast<uint4*>(Bs + row * LDS_LD + kc * EPC) = rb[t];
    }
  };

  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TI = WTM / 16, TJ = WTN / 16;
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
    const T* As = lds + cur * BUF;
    const T* Bs = As + BM * LDS_LD;
    const int fr = lane & 15, fq = lane >> 4;
    if constexpr (sizeof(T) == 2) {
      half8 af[TI], bf[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        af[i] = *reinterpret_cast<const half8*>(As + (wm * WTM + i * 16 + fr) * LDS_LD + fq * 8);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        bf[j] = *reinterpret_cast<const half8*>(Bs + (wn * WTN + j * 16 + fr) * LDS_LD + fq * 8);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    } else {
      floatx4 a0[TI], a1[TI], b0[TJ], b1[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const float* src = reinterpret_cast<const float*>(As) + (wm * WTM + i * 16 + fr) * LDS_LD + fq * 8;
        a0[i] = *reinterpret_cast<const floatx4*>(src);
        a1[i] = *reinterpret_cast<const floatx4*>(src + 4);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const float* src = reinterpret_cast<const float*>(Bs) + (wn * WTN + j * 16 + fr) * LDS_LD + fq * 8;
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

  const bool split = gridDim.y > 1;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
        const int n = n0 + wn * WTN + j * 16 + fr;
        if (m < d.M && n < d.N) {
          if (split)
            a.p.partial[((size_t)blockIdx.y * d.M + m) * d.N + n] = acc[i][j][r];
          else
            epilogue_store<T>(a, m, n, acc[i][j][r]);
        }
      }
}

template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(KArgs a, int splits) {
  const size_t MN = (size_t)a.d.M * a.d.N;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < MN;
       idx += (size_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += a.p.partial[z * MN + idx];
    const int m = (int)(idx / a.d.N), n = (int)(idx % a.d.N);
    epilogue_store<T>(a, m, n, v);
  }
}

struct Plan {
  int bm, bn, splits, k_per_split;
};

Plan choose_plan(const GemmDesc& d) {
  Plan pl{};
  const int t128 = ((d.M + 127) / 128) * ((d.N + 127) / 128);
  if (t128 >= 240) {
    pl.bm = pl.bn = 128;
    pl.splits = 1;
    pl.k_per_split = d.Kpad;
    return pl;
  }
  pl.bm = pl.bn = 64;
  const int tiles = ((d.M + 63) / 64) * ((d.N + 63) / 64);
  const int ktiles = d.Kpad / 32;
  int splits = 1;
  if (tiles < 160 && ktiles >= 8) {
    splits = std::min(ktiles / 4, (512 + tiles - 1) / tiles);
    splits = std::max(splits, 1);
  }
  const int kt_per = (ktiles + splits - 1) / splits;
  pl.k_per_split = kt_per * 32;
  pl.splits = (ktiles + kt_per - 1) / kt_per;
  return pl;
}

int ilog2(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

template <typename T>
void launch(const GemmDesc& d, const GemmPtrs& p, hipStream_t s) {
  const Plan pl = choose_plan(d);
  KArgs a{d, p, pl.k_per_split, (d.M + pl.bm - 1) / pl.bm, d.conv ? ilog2(d.Cin) : 0};
  const int tiles_n = (d.N + pl.bn - 1) / pl.bn;
  dim3 grid(a.tiles_m * tiles_n, pl.splits);
  if (pl.bm == 128) {
    if (d.conv)
      hipLaunchKernelGGL((gemm_kernel<T, 128, 128, true>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_kernel<T, 128, 128, false>), grid, dim3(256), 0, s, a);
  } else {
    if (d.conv)
      hipLaunchKernelGGL((gemm_kernel<T, 64, 64, true>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_kernel<T, 64, 64, false>), grid, dim3(256), 0, s, a);
  }
  if (pl.splits > 1) {
    const size_t MN = (size_t)d.M * d.N;
    const int blocks = (int)std::min<size_t>((MN + 255) / 256, 2048);
    hipLaunchKernelGGL((splitk_reduce_kernel<T>), dim3(blocks), dim3(256), 0, s, a, pl.splits);
  }
}

}  // namespace

size_t gemm_partial_floats(const GemmDesc& d, bool /*f16*/) {
  const Plan pl = choose_plan(d);
  return pl.splits > 1 ? (size_t)pl.splits * d.M * d.N : 0;
}

void gemm(const GemmDesc& d, const GemmPtrs& p, bool f16, hipStream_t s) {
  if (f16)
    launch<_Float16>(d, p, s);
  else
    launch<float>(d, p, s);
}

}  // namespace spi
