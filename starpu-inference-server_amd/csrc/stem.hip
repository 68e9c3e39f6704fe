// Fused ResNet stem for gfx950: the task's NCHW fp32 image -> 7x7/s2/p3 conv +
// folded BN + ReLU -> 3x3/s2/p1 max pool -> the first stage's NHWC activation,
// in one launch (torchvision's conv1 / bn1 / relu / maxpool; SURVEY.md A14 "cast
// fused into the first kernel").  It replaces three launches of the generic path
// (ingest_nchw, the stem as an implicit GEMM over a padded NHWC copy, max pool):
// the 6.4 MB NHWC copy and the 12.8 MB (bs8, fp16) stem output never reach HBM.
//
// Workgroup = PR pooled rows of one image = R = 2 PR + 1 stem rows (the pool's
// row above is recomputed, (2 PR + 1) / 2 PR).  4 waves; wave w owns output
// channels [16 w, 16 w + 16) (its weights stay in registers for the launch:
// [hi | lo][64][24][8] fp16, 48 VGPRs split, 24 plain).
//
// Contraction order: k = (c, kh, kw) with kw padded to 8 -- 24 groups of 8
// (21 real, 3 zero), 6 k-steps of v_mfma_f32_16x16x32_f16.  A lane's fragment
// is 8 horizontally adjacent input pixels of one (channel, input row):
// columns 2 ow - 3 .. 2 ow + 4 (the kw = 7 weight is zero).  The workgroup's
// input rows are converted once into LDS planes (fp16 hi and, split modes,
// lo = fp16(x - hi)) indexed by column + 3, so the fragment is dwords
// [ow, ow + 4) of its plane.
//
// Phase-interleaved fragments: M-fragment `ph` of a 64-pixel group holds
// pixels ow = 64 grp + 4 i + ph (i = fragment row 0..15).  Its lane window,
// dwords [4 i + ph, 4 i + ph + 4), lies inside the two 16-byte-aligned blocks
// [4 i, 4 i + 8): two ds_read_b128 serve the four phase fragments, each one a
// compile-time selection of 4 of those 8 dwords (a plain per-pixel mapping
// would need 4-byte-aligned ds_read2_b32 at half the LDS rate, once per
// fragment).  Planes are 512 bytes apart, so the lane groups of a b128 read
// hit distinct banks.
//
// Epilogue in registers: with that mapping a lane holds 16 consecutive stem
// columns (64 grp + 16 (lane >> 4) + 4 v + ph) of one channel for every stem
// row; the vertical max is per lane, the horizontal max needs the column to the
// left from lane - 16 (ds_bpermute), and for the first lane group from the
// previous group (carried).  ReLU outputs are >= 0, so invalid pixels (outside
// the map) enter the max as 0; fragment rows past the map read finite LDS bytes
// and are discarded (MFMA rows are independent).  max commutes with the monotone
// fp16 rounding, so pooling the fp32 values and rounding once is what pooling
// the rounded stem outputs gives.
#include "spi_kernels.hpp"

#include <cstdlib>
#include <stdexcept>
#include <type_traits>

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));

constexpr int kCout = 64;
constexpr int kGroups = 24;  // (c, kh) groups of 8 kw values: 21 real + 3 zero
constexpr int kSteps = kGroups / 4;

template <int PR>
struct Geom {
  static constexpr int R = 2 * PR + 1;  // stem rows per workgroup
  static constexpr int NR = 2 * R + 5;  // input rows per workgroup
  static constexpr int WP = 256;        // plane width (fp16): columns -3 .. 2 kStemPoolMaxOW + 4, 512 B
  static constexpr int NPL = 3 * NR;    // planes (channel, input row)
  // one plane image in dwords, + slack: the last group's rows past the map read up to
  // 32 dwords beyond the last plane
  static constexpr int PD = NPL * WP / 2 + 32;
};
static_assert(2 * kStemPoolMaxOW + 5 < Geom<1>::WP, "plane covers the valid windows");

// phase PH_'s fragment from an 8-dword block pair: dwords (PH_ & 2) .. (PH_ & 2) + 3
template <int PH_>
__device__ __forceinline__ half8 window(const u32x8& b) {
  if constexpr (PH_ & 2)
    return __builtin_bit_cast(half8, __builtin_shufflevector(b, b, 2, 3, 4, 5));
  else
    return __builtin_bit_cast(half8, __builtin_shufflevector(b, b, 0, 1, 2, 3));
}

// OUT 0: fp16 NHWC [B][PH][PW][64]; 1: split NHWC (per pixel [32 hi | 32 lo] x 2).
// LOM 0: fp16 image x fp16 weights (one MFMA per fragment pair); 1: fp16 image x hi + lo weights
// (two: fp16m, round 5 -- the image's own fp16 rounding costs C2 0.03e-3 of parity margin,
// tools/prec_emulate.py, and its lo planes + third MFMA a third of the launch); 2: split image x
// split weights (three: fp16x3, fp32-grade).
template <int PR, int NW, int LOM, int OUT>
__global__ __launch_bounds__(64 * NW) void stem_pool_kernel(const float* __restrict__ x, const _Float16* __restrict__ w,
                                                            const float* __restrict__ bias, void* __restrict__ y, int H,
                                                            int W, int OH, int OW, int PH, int PW, int diag) {
  using G = Geom<PR>;
  constexpr int R = G::R, NR = G::NR, WP = G::WP, NPL = G::NPL, PD = G::PD, NT = 64 * NW;
  static_assert(NW == 4 || NW == 8, "4 waves (one per 16 channels), or 8 (x 2 pixel groups)");
  static_assert(NW == 4 || kStemPoolMaxOW <= 128, "8 waves: one 64-pixel group per wave");
  constexpr bool LO = LOM == 2;   // lo image planes
  constexpr bool WLO = LOM >= 1;  // lo weights
  // images: [copy 0 hi | copy 1 hi | copy 0 lo | copy 1 lo], copy 1 = copy 0 shifted one dword
  __shared__ __attribute__((aligned(16))) unsigned lds[(LO ? 4 : 2) * PD];
  __shared__ float xch[NW == 8 ? 2 * PR * kCout : 1];  // 8 waves: group 0's last column per pooled row
  const int b = blockIdx.y;
  const int pr0 = blockIdx.x * PR;
  const int sr0 = 2 * pr0 - 1;  // first stem row (the pool's padding row for pr0 = 0)
  const int ir0 = 2 * sr0 - 3;  // first input row
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int n = (wave & 3) * 16 + fr;

  // weights first: L2-resident, their latency overlaps the plane fill
  half8 wh[kSteps], wl[kSteps];
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    const _Float16* src = w + ((size_t)n * kGroups + 4 * s + fq) * 8;
    wh[s] = *reinterpret_cast<const half8*>(src);
    if constexpr (WLO) wl[s] = *reinterpret_cast<const half8*>(src + kCout * kGroups * 8);
  }
  const float bn = bias[n];
  if (diag == 3) return;  // diagnostic (SPI_STEM_DIAG): empty launch

  // planes: (c, input row ir0 + r) at lds[(c * NR + r) * WP + col + 3]; zero outside
  // the image.  Unrolled: every thread's loads are in flight before the first LDS
  // store (a rolled loop waits out one memory latency per iteration).
  const float* xb = x + (size_t)b * 3 * H * W;
  constexpr int HALF = WP / 2, ITER = (NPL * HALF + NT - 1) / NT;
  float v[ITER][2];
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int e = tid + it * NT;
    const int p = e / HALF, i = (e - p * HALF) * 2;
    const int c = p / NR, r = ir0 + (p - c * NR);
    v[it][0] = v[it][1] = 0.f;
    if (e < NPL * HALF && r >= 0 && r < H && diag != 1) {
      const float* row = xb + ((size_t)c * H + r) * W;
      const int c0 = i - 3;
      if (c0 >= 0 && c0 < W) v[it][0] = row[c0];
      if (c0 + 1 >= 0 && c0 + 1 < W) v[it][1] = row[c0 + 1];
    }
  }
  unsigned* ldw = lds;
  auto pack2 = [](_Float16 a, _Float16 b) {
    return __builtin_bit_cast(unsigned short, a) | (unsigned)__builtin_bit_cast(unsigned short, b) << 16;
  };
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int e = tid + it * NT;
    if (e >= NPL * HALF) continue;
    const _Float16 h0 = static_cast<_Float16>(v[it][0]), h1 = static_cast<_Float16>(v[it][1]);
    const unsigned hw = pack2(h0, h1);
    ldw[e] = hw;
    if (e) ldw[PD + e - 1] = hw;
    if constexpr (LO) {
      const unsigned lw = pack2(static_cast<_Float16>(v[it][0] - static_cast<float>(h0)),
                                static_cast<_Float16>(v[it][1] - static_cast<float>(h1)));
      ldw[2 * PD + e] = lw;
      if (e) ldw[3 * PD + e - 1] = lw;
    }
  }
  if (tid < 33) {  // the slack after the last plane: finite bytes for the discarded rows
#pragma unroll
    for (int c = 0; c < (LO ? 4 : 2); ++c) {
      if (c & 1)
        ldw[c * PD + NPL * HALF - 1 + tid] = 0u;  // copy 1: its last dword is copy 0's first slack dword
      else if (tid < 32)
        ldw[c * PD + NPL * HALF + tid] = 0u;
    }
  }
  __syncthreads();

  // per k-step plane (dword offset) of this lane's group (c, kh); zero groups read plane 0
  int goff[kSteps];
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    const int g = 4 * s + fq;
    const int c = g < 21 ? g / 7 : 0, kh = g < 21 ? g - 7 * (g / 7) : 0;
    goff[s] = (c * NR + kh) * HALF;
  }

  const int NG = diag == 2 ? 0 : (OW + 63) >> 6;  // diagnostic 2: fill only
  // Stem rows of one 64-pixel group, folded as they complete (bias + ReLU, invalid
  // pixels as 0) into the vertical max of each pooled row; lane column t = 4 v + ph
  // is stem column 64 grp + 16 fq + t.
  auto compute = [&](int grp, float (&vm)[PR][16]) {
    const int blk = grp * 64 + 4 * fr;  // dword of this lane's first block
    const int o0 = grp * 64 + 16 * fq;
    float bt[16];  // bias per lane column; -inf past the map, so ReLU sends those to 0
#pragma unroll
    for (int t = 0; t < 16; ++t) bt[t] = o0 + t < OW ? bn : -__builtin_inff();
#pragma unroll
    for (int p = 0; p < PR; ++p)
#pragma unroll
      for (int t = 0; t < 16; ++t) vm[p][t] = 0.f;
    floatx4 acc[4];
    // (stem row, k-step) steps, software-pipelined: step t + 1's blocks are read
    // before step t's twelve (split) / four MFMAs are issued.  A step reads dwords
    // [4 i, 4 i + 8) of copy 0 and of copy 1 (copy 0 shifted one dword) as 8-dword
    // vectors (two ds_read_b128 each, consecutive registers): phase 0 / 2 windows are
    // dwords 0-3 / 2-5 of copy 0, phase 1 / 3 the same of copy 1 -- even-aligned
    // register sub-ranges, so no window needs a register move.
    constexpr int T = kSteps * R;
    constexpr int NB = LO ? 4 : 2;
    u32x8 blk_[2][NB];
    auto load = [&](int t, u32x8(&dst)[NB]) {
      const int r = t / kSteps, s = t - r * kSteps;
      const unsigned* src = ldw + goff[s] + r * WP + blk;
#pragma unroll
      for (int c = 0; c < NB; ++c) dst[c] = *reinterpret_cast<const u32x8*>(src + c * PD);
    };
    load(0, blk_[0]);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int r = t / kSteps, s = t - r * kSteps;
      if (s == 0)
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) acc[ph] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (t + 1 < T) load(t + 1, blk_[(t + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const u32x8(&bb)[NB] = blk_[t & 1];
      auto mma = [&](auto phc) {
        constexpr int P = decltype(phc)::value;
        const half8 ah = window<P>(bb[P & 1]);
        if constexpr (LO) {
          const half8 al = window<P>(bb[2 + (P & 1)]);
          acc[P] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, wh[s], acc[P], 0, 0, 0);
        }
        if constexpr (WLO) acc[P] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wl[s], acc[P], 0, 0, 0);
        acc[P] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wh[s], acc[P], 0, 0, 0);
      };
      mma(std::integral_constant<int, 0>{});
      mma(std::integral_constant<int, 1>{});
      mma(std::integral_constant<int, 2>{});
      mma(std::integral_constant<int, 3>{});
      __builtin_amdgcn_sched_barrier(0);
      // row r complete: fold it into the pooled rows it belongs to (rows outside the
      // map skipped -- a wave-uniform test; columns past the map carry a -inf bias)
      if (s == kSteps - 1 && sr0 + r >= 0 && sr0 + r < OH) {
#pragma unroll
        for (int vv = 0; vv < 4; ++vv)
#pragma unroll
          for (int ph = 0; ph < 4; ++ph) {
            const int tt = 4 * vv + ph;
            const float u = acc[ph][vv] + bt[tt];
#pragma unroll
            for (int p = 0; p < PR; ++p)
              if (r >= 2 * p && r <= 2 * p + 2) vm[p][tt] = __builtin_fmaxf(__builtin_fmaxf(vm[p][tt], u), 0.f);
          }
      }
    }
  };
  // horizontal: pooled columns o0 / 2 + q, q = 0..7 (stem columns o0 + 2q - 1 .. o0 + 2q + 1);
  // column o0 - 1 from lane - 16, or for the first lane group `first` (the previous group's last)
  auto store = [&](int grp, const float (&vm)[PR][16], const float (&first)[PR]) {
    const int o0 = grp * 64 + 16 * fq;
#pragma unroll
    for (int p = 0; p < PR; ++p) {
      float left = __shfl_up(vm[p][15], 16, 64);
      if (fq == 0) left = first[p];
      const int pr = pr0 + p;
      if (pr >= PH) continue;
      const size_t m0 = ((size_t)b * PH + pr) * PW;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float l = q ? vm[p][2 * q - 1] : left;
        const float val = fmaxf(l, fmaxf(vm[p][2 * q], vm[p][2 * q + 1]));
        const int pc = o0 / 2 + q;
        if (pc >= PW) continue;
        const _Float16 hi = static_cast<_Float16>(val);
        if constexpr (OUT == 0) {
          static_cast<_Float16*>(y)[(m0 + pc) * kCout + n] = hi;
        } else {
          _Float16* o = static_cast<_Float16*>(y) + (m0 + pc) * kCout * 2 + (n >> 5) * 64 + (n & 31);
          o[0] = hi;
          o[32] = static_cast<_Float16>(val - static_cast<float>(hi));
        }
      }
    }
  };
  float vm[PR][16];
  if constexpr (NW == 4) {  // one wave walks every group, carrying the boundary column
    float carry[PR];
#pragma unroll
    for (int p = 0; p < PR; ++p) carry[p] = 0.f;
    for (int grp = 0; grp < NG; ++grp) {
      compute(grp, vm);
      store(grp, vm, carry);
#pragma unroll
      for (int p = 0; p < PR; ++p) carry[p] = __shfl(vm[p][15], 48 + fr, 64);
    }
  } else {  // waves 0-3 group 0, waves 4-7 group 1; group 0's last column through LDS
    const int grp = wave >> 2;
    const bool active = grp < NG;
    if (active) {
      compute(grp, vm);
      if (grp == 0 && fq == 3)
#pragma unroll
        for (int p = 0; p < PR; ++p) xch[p * kCout + n] = vm[p][15];
    }
    __syncthreads();
    if (active) {
      float first[PR];
#pragma unroll
      for (int p = 0; p < PR; ++p) first[p] = grp ? xch[p * kCout + n] : 0.f;
      store(grp, vm, first);
    }
  }
}

template <int PR, int NW>
void launch_pr(const float* x, const _Float16* w, const float* bias, void* y, int B, int H, int W, int OH, int OW,
               int PH, int PW, int lo, bool split, hipStream_t s) {
  // diagnostic builds only (-DSPI_STEM_DIAG=1: no image loads, 2: fill only, 3: empty)
#ifdef SPI_STEM_DIAG
  constexpr int diag = SPI_STEM_DIAG;
#else
  constexpr int diag = 0;
#endif
  const dim3 grid((PH + PR - 1) / PR, B), block(64 * NW);
  if (split)
    SPI_LAUNCH((stem_pool_kernel<PR, NW, 2, 1>), grid, block, 0, s, x, w, bias, y, H, W, OH, OW, PH, PW, diag);
  else if (lo == 2)
    SPI_LAUNCH((stem_pool_kernel<PR, NW, 2, 0>), grid, block, 0, s, x, w, bias, y, H, W, OH, OW, PH, PW, diag);
  else if (lo == 1)
    SPI_LAUNCH((stem_pool_kernel<PR, NW, 1, 0>), grid, block, 0, s, x, w, bias, y, H, W, OH, OW, PH, PW, diag);
  else
    SPI_LAUNCH((stem_pool_kernel<PR, NW, 0, 0>), grid, block, 0, s, x, w, bias, y, H, W, OH, OW, PH, PW, diag);
}

}  // namespace

void stem_pool_pack(const float* w, _Float16* dst) {
  // dst: [hi | lo][64][24][8]; w: folded [64][3][7][7] fp32
  for (int n = 0; n < kCout; ++n)
    for (int g = 0; g < kGroups; ++g)
      for (int kw = 0; kw < 8; ++kw) {
        const float v = (g < 21 && kw < 7) ? w[((size_t)n * 3 + g / 7) * 49 + (g % 7) * 7 + kw] : 0.f;
        const _Float16 hi = static_cast<_Float16>(v);
        const size_t i = ((size_t)n * kGroups + g) * 8 + kw;
        dst[i] = hi;
        dst[i + (size_t)kCout * kGroups * 8] = static_cast<_Float16>(v - static_cast<float>(hi));
      }
}

void stem_pool(const float* x, const void* w, const float* bias, void* y, int B, int H, int W, int lo, bool split,
               int pr, hipStream_t s) {
  const int OH = (H + 6 - 7) / 2 + 1, OW = (W + 6 - 7) / 2 + 1;
  const int PH = (OH + 2 - 3) / 2 + 1, PW = (OW + 2 - 3) / 2 + 1;
  if (OW > kStemPoolMaxOW || OH < 1 || OW < 1 || B < 1) throw std::runtime_error("stem_pool: unsupported image size");
  if (split && lo != 2) throw std::runtime_error("stem_pool: split output needs the split image and weights");
  if (lo < 0 || lo > 2) throw std::runtime_error("stem_pool: lo is 0, 1 or 2");
  const _Float16* wp = static_cast<const _Float16*>(w);
  // pr: 1 / 2 pooled rows per 4-wave workgroup; 0 (default): two rows per 8-wave
  // workgroup (one 64-pixel group per wave) when the map has two groups, else 1 x 4 waves
  if (pr == 2)
    launch_pr<2, 4>(x, wp, bias, y, B, H, W, OH, OW, PH, PW, lo, split, s);
  else if (pr == 1 || OW <= 64)
    launch_pr<1, 4>(x, wp, bias, y, B, H, W, OH, OW, PH, PW, lo, split, s);
  else
    launch_pr<2, 8>(x, wp, bias, y, B, H, W, OH, OW, PH, PW, lo, split, s);
}

}  // namespace spi
