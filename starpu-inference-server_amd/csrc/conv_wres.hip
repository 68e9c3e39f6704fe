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
//   * owns one band of `th` whole output rows (the kConvHalo band: th rows x
//     W pixels as tile rows 0..127), DMAing its (th + 2) x (W + 2) input pixels
//     once into the halo buffer, ahead of the weights, tap by tap,
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
#include <type_traits>

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
// LDS: the halo buffer + the resident weights -- 104 KiB, so a 48 KiB workgroup of
// another worker stream's kernel still fits beside it on the CU.  (Several bands per
// workgroup -- one halo buffer reused, or two double-buffered -- measured -1 % / -5 % at
// four streams and were removed in round 4)
constexpr int kLds = kHBuf + kWBytes;
constexpr int BM = 128, BN = 64, NT = 256;  // tile rows (pixels of a band), columns, threads
constexpr int kWPieces = kWBytes / 1024 / 4;   // 18 weight DMA pieces per wave
constexpr int kHPieces = kHBuf / 1024 / 4;     // 8 halo DMA pieces per wave

struct WresArgs {
  const _Float16* x;    // [B][H][W][64]
  const char* w;        // packed [128][576] fp16: rows 0..63 the matrix, rows 64..127 the LDS image
  const float* bias;    // [64] (the zero line when the conv has none)
  const _Float16* res;  // [B][H][W][64] or nullptr
  _Float16* y;          // [B][H][W][64]
  const char* zeros;    // >= 256 zero bytes
  int H, W;             // input = output size
  int th;               // output rows per band
  int bands_per_img, bands;
};

__device__ __forceinline__ u32x4 rd_chunk(const char* img, int row, int c) {
  return *reinterpret_cast<const u32x4*>(img + row * kRowB + ((c ^ (row & 7)) << 4));
}

template <int N>
__device__ __forceinline__ void dma_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One 1-KiB LDS-DMA piece (lane l's 16 bytes from `src` to dst + 16 l), issued in
// inline asm so hipcc does not track it: with the builtin, hipcc cannot tell the
// pending DMA from the LDS the next ds_reads touch and drains every DMA
// (s_waitcnt vmcnt(0)) before them, which would serialise the next band's halo with
// this band's k-loop.  The caller counts these with dma_wait_barrier<N>
// (cdna_hip_programming.md 5.7, the M0-saving LDS-DMA recipe).
__device__ __forceinline__ void glds16(const void* src, const char* dst) {
  const lds_ptr_t lp = (lds_ptr_t)(const_cast<char*>(dst));
  const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lp);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(m0v)
               : "memory");
}

// Diagnostic build (-DSPI_WRES_STAMPS): per-workgroup s_memtime stamps of the phases of
// its first two bands (tools/wres_stamps.py); no output value depends on them.
#ifdef SPI_WRES_STAMPS
__device__ unsigned long long g_wres_stamps[4096 * 10];
#define WRES_STAMP(k)                                                                   \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    if (tid == 0 && blockIdx.x < 4096) g_wres_stamps[blockIdx.x * 10 + (k)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
#else
#define WRES_STAMP(k) \
  do {                \
  } while (0)
#endif

template <int T, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (T < N) {
    f(std::integral_constant<int, T>{});
    static_for<T + 1, N>(f);
  }
}

// LDS map: the halo buffer at 0, the resident weights from kHBuf.
template <bool HAS_RES, bool RELU>
__global__ __launch_bounds__(NT, 1) void conv3x3_c64_wres(WresArgs a) {
  constexpr int kW0 = kHBuf;
  __shared__ __attribute__((aligned(16))) char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware band order: the hardware deals consecutive workgroups round-robin to the 8
  // XCDs; remapped, each XCD walks a contiguous run of bands, so the two input rows that
  // neighbouring bands share are fetched into one L2 once (bijective remap,
  // cdna_hip_programming.md T1)
  int wg = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = wg & 7, l = wg >> 3;
    if (nwg >= 16) wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
  }
  const int band = wg;
  if (band >= a.bands) return;  // uniform per workgroup
  const int Wp = a.W + 2;
  const int hp = (a.th + 2) * Wp;
#ifdef SPI_WRES_STAMPS
  if (tid == 0 && blockIdx.x < 4096) g_wres_stamps[blockIdx.x * 10 + 9] = __builtin_amdgcn_s_memrealtime();
#endif
  WRES_STAMP(0);

  // ---- resident weights: the packed matrix's padding rows hold the LDS image (pack.hpp:
  // pack_matrix_into), 72 contiguous pieces of 1 KiB, 18 per wave, issued after the band's
  // halo, two pieces per tap per wave in tap order: each tap starts as soon as its pieces
  // have landed.
  const char* wimg = a.w + (size_t)64 * (9 * kRowB);
  auto issue_w = [&] {
#pragma unroll
    for (int i = 0; i < kWPieces; ++i) {
      const int q = i * 4 + wave;  // tap t is pieces 8 t .. 8 t + 7
      glds16(wimg + q * 1024 + lane * 16, lds + kW0 + q * 1024);
    }
  };

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
  auto issue_halo = [&] {
    const int img = band / a.bands_per_img, oy0 = (band - img * a.bands_per_img) * a.th;
    const _Float16* base = a.x + ((size_t)img * a.H + oy0) * a.W * 64;
    char* dst = lds;
#pragma unroll
    for (int i = 0; i < kHPieces; ++i) {
      const int iy = oy0 - 1 + h_hy[i];
      const bool ok = h_ok[i] && (unsigned)iy < (unsigned)a.H;
      const char* src = ok ? reinterpret_cast<const char*>(base + h_off[i]) : a.zeros;
      glds16(src, dst + (wave * kHPieces + i) * 1024);
    }
  };

  // ---- fragment addresses, band-independent.  Wave (wm, wn) owns tile rows wm * 64 .. + 63
  // (TI = 4 blocks) x columns wn * 32 .. + 31 (TJ = 2); tile row r = output pixel (ty, tx) of
  // the band.  k-chunk t = (tap, kk): 32 channels kk * 32 .. of tap t / 2; the lane reads 16-byte
  // chunk kk * 4 + fq.  A: halo pixel of the row at tap (kh, kw), swizzled slot; B: tap image row.
  const int fr = lane & 15, fq = lane >> 4, wm = wave >> 1, wn = wave & 1;
  int aoff[9][2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wm * 64 + i * 16 + fr;
    const int ty = r / a.W, tx = r - ty * a.W;
    const int p0 = ty < a.th ? ty * Wp + tx : 0;  // rows past the band read pixel 0, never stored
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int p = p0 + (tap / 3) * Wp + tap % 3;
        aoff[tap][kk][i] = p * kRowB + (((kk * 4 + fq) ^ (p & 7)) << 4);
      }
  }
  int boff[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int n = wn * 32 + jj * 16 + fr;
      boff[kk][jj] = kW0 + n * kRowB + (((kk * 4 + fq) ^ (n & 7)) << 4);
    }

  // Epilogue bookkeeping, band-independent: thread -> 8-column group e_nb8, tile rows
  // e_r0 + it * 32; e_rel = pixel offset of the row inside the band, e_ty its output row
  // (>= th: a padding row, never stored).  The bias is read as two 16-byte loads (a.bias is
  // never null: the host points it at the zero line) -- per-element guarded loads had made
  // hipcc wait on eight dependent L2 round trips per band.
  constexpr int E_G = BN / 8, E_RSTEP = NT / E_G, E_ITEMS = BM / E_RSTEP;  // 8 groups, rows 32 apart, 4 rows
  const int e_nb8 = (tid % E_G) * 8, e_r0 = tid / E_G;
  int e_rel[E_ITEMS], e_ty[E_ITEMS];
#pragma unroll
  for (int it = 0; it < E_ITEMS; ++it) {
    const int row = e_r0 + it * E_RSTEP;
    const int ty = row / a.W, tx = row - ty * a.W;
    e_ty[it] = ty < a.th ? ty : 1 << 30;
    e_rel[it] = ty * a.W + tx;
  }

  // The band (every fragment read is a VGPR address plus an immediate).  The k-loop keeps
  // chunk t + 1's six fragment reads in flight behind chunk t's eight MFMAs (sched_barrier
  // pins the order; the compiler's counted lgkmcnt then waits only for chunk t).
  issue_halo();
  issue_w();
  {
    [[maybe_unused]] constexpr int sk = 1;
    dma_wait_barrier<2 * 8>();  // the halo and tap 0 have landed
    WRES_STAMP(sk);
    const char* Hs = lds;

    floatx4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = floatx4{0.f, 0.f, 0.f, 0.f};
    half8 fa[2][4], fb[2][2];
    auto load = [&](int t, int s) {
      const int tap = t >> 1, kk = t & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[s][i] = *reinterpret_cast<const half8*>(Hs + aoff[tap][kk][i]);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        fb[s][jj] = *reinterpret_cast<const half8*>(lds + boff[kk][jj] + tap * kWImg);
    };
    load(0, 0);
    static_for<0, 18>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t + 1 < 18) {
        // tap (t + 1) / 2's weight pieces land while the taps before it compute
        if constexpr ((t + 1) % 2 == 0) {
          constexpr int T = (t + 1) / 2;  // the tap that starts here
          dma_wait_barrier<2 * (8 - T)>();
        }
        load(t + 1, (t + 1) & 1);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t & 1][i], fb[t & 1][jj], acc[i][jj], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    WRES_STAMP(sk + 1);

    // ---- epilogue through this band's halo buffer (every wave is done reading it).  The
    // residual rows go out first (clamped rows: always-valid addresses, no branch), so their
    // latency hides behind the park; HAS_RES / RELU are template parameters -- a runtime
    // `if (res)` per row had made hipcc branch around each load and wait vmcnt(0) per row.
    const int img = band / a.bands_per_img, oy0 = (band - img * a.bands_per_img) * a.th;
    const int rows_left = a.H - oy0;  // output rows of this band inside the image
    const size_t mbase = ((size_t)img * a.H + oy0) * a.W;
    // the bias here rather than once per workgroup: a load pending across the k-loop makes
    // hipcc drain every vector-memory operation (vmcnt(0)) before the loop's first ds_read
    const floatx4 b0 = *reinterpret_cast<const floatx4*>(a.bias + e_nb8);
    const floatx4 b1 = *reinterpret_cast<const floatx4*>(a.bias + e_nb8 + 4);
    half8 rv[E_ITEMS];
    if constexpr (HAS_RES) {
#pragma unroll
      for (int it = 0; it < E_ITEMS; ++it) {
        const size_t mm = mbase + (e_ty[it] < rows_left ? e_rel[it] : 0);
        rv[it] = *reinterpret_cast<const half8*>(a.res + mm * 64 + e_nb8);
      }
    }
    lds_barrier();
#ifdef SPI_WRES_STAMPS_EPI
    if (sk == 1) WRES_STAMP(4);
#endif
    float* T = reinterpret_cast<float*>(lds);
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
#ifdef SPI_WRES_STAMPS_EPI
    if (sk == 1) WRES_STAMP(5);
#endif
    lds_barrier();
#ifdef SPI_WRES_STAMPS_EPI
    if (sk == 1) WRES_STAMP(6);
#endif
    half8 hv[E_ITEMS];
#pragma unroll
    for (int it = 0; it < E_ITEMS; ++it) {
      const int row = e_r0 + it * E_RSTEP;
      const float* src = T + row * BN + (e_nb8 ^ (((row >> 2) & 3) << 4));
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(src);
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(src + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = (e < 4 ? x0[e] + b0[e] : x1[e - 4] + b1[e - 4]);
        if constexpr (HAS_RES) v += static_cast<float>(rv[it][e]);
        if constexpr (RELU) v = v > 0.f ? v : 0.f;
        hv[it][e] = static_cast<_Float16>(v);
      }
    }
#pragma unroll
    for (int it = 0; it < E_ITEMS; ++it) {
#if defined(SPI_WRES_DIAG) && SPI_WRES_DIAG == 1  // diagnostic: no output stores (values kept live)
      asm volatile("" ::"v"(hv[it]));
#else
      if (e_ty[it] < rows_left) *reinterpret_cast<half8*>(a.y + (mbase + e_rel[it]) * 64 + e_nb8) = hv[it];
#endif
    }
    WRES_STAMP(sk + 2);
  }
  WRES_STAMP(7);
#ifdef SPI_WRES_STAMPS
  if (tid == 0 && blockIdx.x < 4096) g_wres_stamps[blockIdx.x * 10 + 8] = __builtin_amdgcn_s_memrealtime();
#endif
}

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoi(e) : dflt;
}

// SPI_CONV_WRES=0: never route here; 1 (default): only grids the implicit GEMM cannot fill,
// fewer than kWresMaxTiles 128-row tiles; 2: every eligible conv (the round-3..4 rule).  Round 5,
// under the four worker streams: since the kw-window kind (round 4) the implicit
// GEMM beats this kernel at ResNet-18 bs8 (+1.9 % fp16m, +2.2 % fp16) and ResNet-152 bs32 (+2.4 %),
// ties at ResNet-152 bs8, and loses at ResNet-18 bs1 (-3.9 %).  Read once;
// conv_wres_reload_env() (spi_debug_gemm_reload_env) re-reads it.
int& wres_on() {
  static int on = env_int("SPI_CONV_WRES", 1);
  return on;
}

}  // namespace

void conv_wres_reload_env() { wres_on() = env_int("SPI_CONV_WRES", 1); }

#ifdef SPI_WRES_STAMPS
extern "C" int spi_debug_wres_stamps(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wres_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif

// Output rows per band: as many as fill the 128-row tile while the halo fits 256 pixels.
static int wres_rows(int H, int W) {
  int th = std::min(H, BM / std::max(1, W));
  while (th > 0 && (th + 2) * (W + 2) > kHaloPix) --th;
  return th;
}

constexpr int kWresMaxTiles = 128;  // the general kernel's plan target

bool conv_wres_eligible(const GemmDesc& d, Prec prec, const GemmPtrs& p) {
  const int on = wres_on();
  if (on == 1 && (d.M + 127) / 128 >= kWresMaxTiles) return false;  // a full 128 x 64 window grid
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return on && prec == Prec::F16 && d.conv && d.KH == 3 && d.KW == 3 && d.stride == 1 && d.pad == 1 &&
         d.Cin == 64 && d.N == 64 && d.K == 576 && d.Kpad == 576 && d.krep == 1 && d.OH == d.H && d.OW == d.W &&
         !d.a_split && !d.out_split && !d.out_f32 && !d.res_f32 && !d.pool_rows && d.ldc == 64 &&
         (!p.res || d.ldr == 64) && d.act != Act::Gelu && wres_rows(d.H, d.W) >= 1 && al16(p.A) && al16(p.W) &&
         al16(p.C) && (!p.res || al16(p.res)) && (!p.bias || al16(p.bias)) && p.zeros && d.w_image;
}

void conv_wres(const GemmDesc& d, const GemmPtrs& p, hipStream_t s) {
  WresArgs a{};
  a.x = static_cast<const _Float16*>(p.A);
  a.w = static_cast<const char*>(p.W);
  a.bias = p.bias ? p.bias : static_cast<const float*>(p.zeros);  // the zero line: 64 floats
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
  const bool relu = d.act == Act::Relu;
  const dim3 grid(a.bands);
  if (a.res && relu)
    SPI_LAUNCH((conv3x3_c64_wres<true, true>), grid, dim3(NT), 0, s, a);
  else if (a.res)
    SPI_LAUNCH((conv3x3_c64_wres<true, false>), grid, dim3(NT), 0, s, a);
  else if (relu)
    SPI_LAUNCH((conv3x3_c64_wres<false, true>), grid, dim3(NT), 0, s, a);
  else
    SPI_LAUNCH((conv3x3_c64_wres<false, false>), grid, dim3(NT), 0, s, a);
}

}  // namespace spi
