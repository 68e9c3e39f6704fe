// Weight-resident 3x3 conv for 64 -> 64 channels (gfx950): ResNet layer-1 3x3 convs
// (ResNet-18 BasicBlocks, ResNet-152 bottleneck conv2), NHWC fp16, stride 1, pad 1,
// folded BN bias, optional residual, optional ReLU.
//
// Why a kernel of its own.  The implicit-GEMM conv (gemm.hip) stages every
// (tap, channel) k-step of A and W through an LDS ring: per 128 x 64 tile it
// moves 9 x 16 KiB of A and 9 x 8 KiB of W into the CU, and one CU takes in
// ~70-90 GB/s by LDS-DMA (MI355X_MICROARCH.md, "gather into LDS", "ring-gemm"), so
// the tile is ingest-bound at ~5x its MFMA time.  For 64 -> 64 channels the whole
// folded weight tensor is 9 x 64 x 64 fp16 = 72 KiB: it fits in LDS beside two
// halo buffers.  Here a workgroup
//   * DMAs the 72 KiB of weights ONCE (per-tap images in the ring's swizzled
//     [row][128 B] layout, chunk c of row n at slot c ^ (n & 7)),
//   * walks `bpw` bands of `th` whole output rows (the kConvHalo band: th rows x
//     W pixels as tile rows 0..127), DMAing each band's (th + 2) x (W + 2) input
//     pixels once into one of two halo buffers -- band j + 1's halo is issued
//     before band j computes, so it lands behind 144 MFMAs per wave,
//   * computes all 9 taps x 64 channels from LDS with no global access in the
//     k-loop (A fragments at halo pixel offset kh * (W + 2) + kw, B fragments
//     from the resident tap image),
//   * runs the epilogue through LDS (the band's own halo buffer, free by then):
//     fp32 tile parked with the 16-column XOR swizzle, then 16-byte bias +
//     residual + ReLU + fp16 row vectors.
// Per band it takes in (th + 2)(W + 2) x 128 B (29.7 KiB at W = 56) for
// 2 x 112 x 64 x 576 FLOP: ~320 FLOP per byte, MFMA-bound per CU.
#include "spi_kernels.hpp"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kRowB = 128;                  // 64 fp16 channels = one pixel row / one W row per tap
constexpr int kWImg = 64 * kRowB;           // one tap's [64 cout][64 cin] image: 8 KiB
constexpr int kWBytes = 9 * kWImg;          // 72 KiB resident weights
constexpr int kHaloPix = 256;               // halo buffer capacity in pixels
constexpr int kHBuf = kHaloPix * kRowB;     // 32 KiB (also the 128 x 64 fp32 epilogue tile)
constexpr int kLds = kWBytes + 2 * kHBuf;   // 136 KiB: one workgroup per CU
constexpr int BM = 128, BN = 64, NT = 256;  // tile rows (pixels of a band), columns, threads
constexpr int kWPieces = kWBytes / 1024 / 4;   // 18 weight DMA pieces per wave
constexpr int kHPieces = kHBuf / 1024 / 4;     // 8 halo DMA pieces per wave

struct WresArgs {
  const _Float16* x;    // [B][H][W][64]
  const char* w;        // packed [128][576] fp16 (pack_conv: k = tap * 64 + c), bias folded separately
  const float* bias;    // [64]
  const _Float16* res;  // [B][H][W][64] or nullptr
  _Float16* y;          // [B][H][W][64]
  const char* zeros;    // >= 16 zero bytes
  int H, W;             // input = output size
  int th;               // output rows per band
  int bands_per_img, bands, bpw;
  int relu;
};

__device__ __forceinline__ u32x4 rd_chunk(const char* img, int row, int c) {
  return *reinterpret_cast<const u32x4*>(img + row * kRowB + ((c ^ (row & 7)) << 4));
}

template <int N>
__device__ __forceinline__ void dma_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(NT, 1) void conv3x3_c64_wres(WresArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b_first = blockIdx.x * a.bpw;
  const int nb = min(a.bpw, a.bands - b_first);
  if (nb <= 0) return;  // uniform per workgroup
  const int Wp = a.W + 2;
  const int hp = (a.th + 2) * Wp;

  // ---- resident weights: 72 pieces of 1 KiB (8 rows x 128 B of one tap), 18 per wave
#pragma unroll
  for (int i = 0; i < kWPieces; ++i) {
    const int q = wave * kWPieces + i;
    const int tap = q >> 3, n = ((q & 7) << 3) + (lane >> 3), c = (lane & 7) ^ (n & 7);
    const char* src = a.w + (size_t)n * (9 * kRowB) + tap * kRowB + c * 16;
    __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(lds + q * 1024), 16, 0, 0);
  }

  // ---- halo bookkeeping, band-independent: piece i of this wave fills pixels
  // p = (wave * 8 + i) * 8 + lane / 8, slot lane % 8 <- chunk slot ^ (p & 7)
  int h_hy[kHPieces], h_off[kHPieces];
  bool h_ok[kHPieces];
#pragma unroll
  for (int i = 0; i < kHPieces; ++i) {
    const int p = ((wave * kHPieces + i) << 3) + (lane >> 3);
    const int c = (lane & 7) ^ (p & 7);
    const int hy = p / Wp, hx = p - hy * Wp;
    h_hy[i] = hy;
    h_ok[i] = p < hp && (unsigned)(hx - 1) < (unsigned)a.W;
    h_off[i] = ((hy - 1) * a.W + (hx - 1)) * 64 + c * 8;  // elements from the band's (oy0, 0) pixel
  }
  auto issue_halo = [&](int band, int buf) {
    const int img = band / a.bands_per_img, oy0 = (band - img * a.bands_per_img) * a.th;
    const _Float16* base = a.x + ((size_t)img * a.H + oy0) * a.W * 64;
    char* dst = lds + kWBytes + buf * kHBuf;
#pragma unroll
    for (int i = 0; i < kHPieces; ++i) {
      const int iy = oy0 - 1 + h_hy[i];
      const bool ok = h_ok[i] && (unsigned)iy < (unsigned)a.H;
      const char* src = ok ? reinterpret_cast<const char*>(base + h_off[i]) : a.zeros;
      __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(dst + (wave * kHPieces + i) * 1024), 16, 0, 0);
    }
  };

  // ---- fragment rows: wave (wm, wn) owns tile rows wm * 64 .. + 63 (TI = 4 blocks)
  // x columns wn * 32 .. + 31 (TJ = 2); tile row r = output pixel (ty, tx) of the band
  const int fr = lane & 15, fq = lane >> 4, wm = wave >> 1, wn = wave & 1;
  int h_row[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wm * 64 + i * 16 + fr;
    const int ty = r / a.W, tx = r - ty * a.W;
    h_row[i] = ty < a.th ? ty * Wp + tx : 0;  // rows past the band read pixel 0, never stored
  }

  issue_halo(b_first, 0);
  for (int j = 0; j < nb; ++j) {
    const int band = b_first + j;
    const bool next = j + 1 < nb;
    if (next) issue_halo(band + 1, (j + 1) & 1);  // the buffer band j - 1 used (its epilogue ended in a barrier)
    if (next)
      dma_wait_barrier<kHPieces>();  // everything but the next halo has landed
    else
      dma_wait_barrier<0>();
    const char* Hs = lds + kWBytes + (j & 1) * kHBuf;

    floatx4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = (tap / 3) * Wp + tap % 3;
      const char* Ws = lds + tap * kWImg;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        half8 af[4], bf[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = __builtin_bit_cast(half8, rd_chunk(Hs, h_row[i] + toff, kk * 4 + fq));
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          bf[jj] = __builtin_bit_cast(half8, rd_chunk(Ws, wn * 32 + jj * 16 + fr, kk * 4 + fq));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[jj], acc[i][jj], 0, 0, 0);
      }
    }

    // ---- epilogue through this band's halo buffer (every wave is done reading it)
    lds_barrier();
    float* T = reinterpret_cast<float*>(lds + kWBytes + (j & 1) * kHBuf);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * 64 + i * 16 + fq * 4 + r;
          const int col = (wn * 32 + jj * 16 + fr) ^ (fq << 4);  // (row >> 2) & 3 == fq
          T[row * BN + col] = acc[i][jj][r];
        }
    lds_barrier();
    {
      constexpr int G = BN / 8, RSTEP = NT / G, ITEMS = BM / RSTEP;  // 8 column groups, 32 rows apart, 4 rows
      const int cg = tid % G, r0 = tid / G, nb8 = cg * 8;
      const int img = band / a.bands_per_img, oy0 = (band - img * a.bands_per_img) * a.th;
      float bv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = a.bias[nb8 + e];
      int m[ITEMS];
      float yv[ITEMS][8];
#pragma unroll
      for (int it = 0; it < ITEMS; ++it) {
        const int row = r0 + it * RSTEP;
        const int ty = row / a.W, tx = row - ty * a.W;
        m[it] = (ty < a.th && oy0 + ty < a.H) ? ((img * a.H + oy0 + ty) * a.W + tx) : -1;
        const int mm = m[it] < 0 ? 0 : m[it];  // skipped rows load row 0 (always valid)
        if (a.res) {
          const half8 rv = *reinterpret_cast<const half8*>(a.res + (size_t)mm * 64 + nb8);
#pragma unroll
          for (int e = 0; e < 8; ++e) yv[it][e] = static_cast<float>(rv[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) yv[it][e] = 0.f;
        }
      }
#pragma unroll
      for (int it = 0; it < ITEMS; ++it) {
        const int row = r0 + it * RSTEP;
        const float* src = T + row * BN + (nb8 ^ (((row >> 2) & 3) << 4));
        const floatx4 x0 = *reinterpret_cast<const floatx4*>(src);
        const floatx4 x1 = *reinterpret_cast<const floatx4*>(src + 4);
        half8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = (e < 4 ? x0[e] : x1[e - 4]) + bv[e] + yv[it][e];
          if (a.relu) v = v > 0.f ? v : 0.f;
          h[e] = static_cast<_Float16>(v);
        }
        if (m[it] >= 0) *reinterpret_cast<half8*>(a.y + (size_t)m[it] * 64 + nb8) = h;
      }
    }
    lds_barrier();  // the tile is read before the next band's halo DMA reuses this buffer
  }
}

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoi(e) : dflt;
}

}  // namespace

// Output rows per band: as many as fill the 128-row tile while the halo fits 256 pixels.
static int wres_rows(int H, int W) {
  int th = std::min(H, BM / std::max(1, W));
  while (th > 0 && (th + 2) * (W + 2) > kHaloPix) --th;
  return th;
}

bool conv_wres_eligible(const GemmDesc& d, Prec prec, const GemmPtrs& p) {
  static const int on = env_int("SPI_CONV_WRES", 1);
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return on && prec == Prec::F16 && d.conv && d.KH == 3 && d.KW == 3 && d.stride == 1 && d.pad == 1 &&
         d.Cin == 64 && d.N == 64 && d.K == 576 && d.Kpad == 576 && d.krep == 1 && d.OH == d.H && d.OW == d.W &&
         !d.a_split && !d.out_split && !d.out_f32 && !d.res_f32 && !d.pool_rows && d.ldc == 64 &&
         (!p.res || d.ldr == 64) && d.act != Act::Gelu && wres_rows(d.H, d.W) >= 1 && al16(p.A) && al16(p.W) &&
         al16(p.C) && (!p.res || al16(p.res)) && p.zeros;
}

void conv_wres(const GemmDesc& d, const GemmPtrs& p, hipStream_t s) {
  WresArgs a{};
  a.x = static_cast<const _Float16*>(p.A);
  a.w = static_cast<const char*>(p.W);
  a.bias = p.bias;
  a.res = static_cast<const _Float16*>(p.res);
  a.y = static_cast<_Float16*>(p.C);
  a.zeros = static_cast<const char*>(p.zeros);
  a.H = d.H;
  a.W = d.W;
  a.th = wres_rows(d.H, d.W);
  if (a.th < 1) throw std::invalid_argument("conv_wres: map too wide for the halo buffer");
  a.bands_per_img = (d.H + a.th - 1) / a.th;
  const int imgs = d.M / (d.OH * d.OW);
  a.bands = imgs * a.bands_per_img;
  a.relu = d.act == Act::Relu;
  // bands per workgroup (SPI_CONV_WRES_BPW): 1 keeps the most workgroups in flight (the weights
  // are re-read from L2 per band), more amortise the 72 KiB weight fill over several bands
  static const int bpw_env = env_int("SPI_CONV_WRES_BPW", 0);
  int bpw = bpw_env > 0 ? bpw_env : (a.bands >= 512 ? 2 : 1);
  a.bpw = std::max(1, bpw);
  const int grid = (a.bands + a.bpw - 1) / a.bpw;
  hipLaunchKernelGGL(conv3x3_c64_wres, dim3(grid), dim3(NT), 0, s, a);
}

}  // namespace spi
