// 256x256-tile fp16 GEMM for the large dense contractions (ViT-L QKV / FFN1 at
// bs16, any dense F16 GEMM with >= SPI_GEMM_256_MIN output tiles of 256^2):
//   C[M,N] = act(A[M,K] . W[N,K]^T + bias + residual), A fp16 row-major (lda),
//   W packed [Npad][Kpad] fp16 (K contiguous), C fp16 or fp32.
//
// Why a second kernel: the general kernel (gemm.hip) is a 2-barrier-per-k-step
// loop whose LDS-DMA for step t + 1 is waited with vmcnt(0) at the top of step
// t + 1, so every k-step exposes the DMA latency behind only one step of MFMAs
// (ViT-L FFN1 at 527 TF/s, hipBLASLt 858).  Here one 8-wave workgroup owns a
// 256x256 tile (wave (wr, wc) in 2 x 4: rows 128 wr.., columns 64 wc..; 128 fp32
// accumulators per lane) and every 64-deep k-tile runs as 4 phases of 16 MFMAs
// (one 64x32 quadrant of the wave's 128x64 output each).  The k-tile is staged
// as 4 quarters of 16 KiB, in the order the phases first read them:
//   Q0 = A rows {0..63, 128..191}   (phase 0: every wave's A rows of quadrant row 0)
//   Q1 = B rows {64 c .. 64 c + 31} (phase 0: quadrant column 0)
//   Q2 = B rows {64 c + 32 .. 64 c + 63} (phase 1)
//   Q3 = A rows {64..127, 192..255} (phase 2; phase 3 reuses registers)
// and phase p of k-tile t stages quarter p of k-tile t + 1 into the other of two
// 64 KiB buffers (2 LDS-DMA pieces of 1 KiB per wave).  So each quarter is in
// flight for three to four phases, and the wait before a phase's reads is a
// counted vmcnt(4) (the two quarters issued since stay in flight) + one raw
// s_barrier -- never vmcnt(0) inside the loop (cdna_hip_programming.md §5, "The
// 256^2 8-phase template" and "Pipelining across barriers": counted vmcnt, raw
// barrier, one LDS object).  WAR: quarter q of a buffer is restaged >= 3
// barriers after its last read.  LDS images are the general kernel's: 128-byte
// rows, 16-byte chunk c of row r at slot c ^ (r & 7), swizzle applied on the
// DMA source address (rule 21), conflict-free ds_read_b128 fragment reads.
#include "device_math.hpp"
#include "ln_fold.hpp"
#include "spi_kernels.hpp"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct G256Args {
  const _Float16* A;
  const _Float16* W;
  const float* bias;
  const void* res;
  void* C;
  int lda, ldw, ldr, ldc;
  int M, N, K;
  int tiles_m, tiles_n;
  int act;  // Act
  int res_f32, out_f32;
  int vec_ok;  // C / residual rows and pointers allow 16-byte vectors (LDS-staged epilogue)
  // LayerNorm fold (GemmDesc::ln_in_chunks / ln_out, ln_fold.hpp): consumer statistics of the
  // A rows + c1; producer statistics + fp16 copy of the output
  int ln_in_chunks, ln_out, ld16;
  float ln_in_eps;
  const float* ln_in_stats;
  const float* ln_c1;
  float* ln_out_stats;
  _Float16* c16;
  // split-K (gemm256_splits): `splits` slices of `ktp` k-tiles; fp32 slabs [tile][slice][256 x 256]
  // in fragment order and two counter words per tile (arrival ticket, published slabs)
  int splits, ktp;
  float* partial;
  int* counters;
  // tile order inside a slice: 0 row blocks fastest (consecutive tiles share a W panel), 1 column
  // tiles fastest (consecutive tiles share an A row block; SPI_GEMM_256_ORDER)
  int n_fast;
  size_t plane;  // RES = 3: residual and output in two fp16 planes, lo `plane` elements after hi
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kMaxSplits = 4;     // split-K slices (gemm256_splits)
constexpr int kMinSliceKt = 16;   // k-tiles per slice at least (ViT-L out-proj, K = 1024, 2 x 8: 52.9 us b2b vs 40.2 unsplit)
// diagnostic build -DSPI_G256_EPI_CALLS: leave the epilogue instances to the inliner (A/B)
#ifdef SPI_G256_EPI_CALLS
#define SPI_G256_EPI_INLINE
#else
#define SPI_G256_EPI_INLINE __attribute__((always_inline))
#endif

// Tile geometry by tile height BM (256: the 256 x 256 tile; 128: the 128 x 256 tile, round 5).
//   A k-tile is BM A rows + 256 B rows of 128 bytes: 64 KiB / 48 KiB.
//   BM = 256: two buffers, staged in 4 quarters of 16 KiB (below); BM = 128: three buffers
//   (144 KiB), staged in 3 thirds of 16 KiB -- T0 = the 128 A rows, T1 / T2 = the B rows of
//   n-half 0 / 1 -- one k-tile runs as 2 phases of 16 MFMAs (a wave owns 64 x 64: phase 0
//   reads A + B n-half 0, phase 1 B n-half 1), and the third k-tile ahead is in flight.
template <int BM, int NBUF>
struct G256Geo {
  static_assert(NBUF == 2 || (BM == 128 && NBUF == 3), "two k-tile buffers, three for 128-row tiles");
  static constexpr int kBufBytes = BM * 128 + 256 * 128;
  static constexpr int kBOff = BM * 128;
  static constexpr int kNBuf = NBUF;
  static constexpr int kNQ = BM == 256 ? 4 : 3;  // staging pieces of 16 KiB per k-tile
  static constexpr int kMA = BM / 32;             // 16-row fragments per wave (wave tile BM/2 x 64)
  static constexpr int kLds = kNBuf * kBufBytes;
  // the epilogue parks the tile in rounds of kRoundRows x 256 fp32: one wave row's rows per round,
  // or (128-row tile, three buffers) both wave rows at once
  static constexpr int kRoundRows = (BM == 128 && NBUF == 3) ? 128 : BM / 2;
  static_assert(kLds >= kRoundRows * 256 * 4, "an epilogue round parks kRoundRows x 256 fp32");
};

// 8-row piece base (tile row) of piece pc (0..15) of staging piece q
template <int BM>
__device__ __forceinline__ int quarter_row(int q, int pc) {
  if constexpr (BM == 128) {
    switch (q) {
      case 0: return pc * 8;                           // A rows 0..127
      case 1: return 64 * (pc >> 2) + (pc & 3) * 8;    // B n-half 0
      default: return 64 * (pc >> 2) + 32 + (pc & 3) * 8;  // B n-half 1
    }
  }
  switch (q) {
    case 0: return pc < 8 ? pc * 8 : 128 + (pc - 8) * 8;
    case 1: return 64 * (pc >> 2) + (pc & 3) * 8;
    case 2: return 64 * (pc >> 2) + 32 + (pc & 3) * 8;
    default: return pc < 8 ? 64 + pc * 8 : 192 + (pc - 8) * 8;
  }
}
template <int BM>
__device__ __forceinline__ constexpr bool quarter_is_a(int q) {
  return BM == 128 ? q == 0 : (q == 0 || q == 3);
}

// RES: 0 no residual, 1 fp16 residual, 2 fp32 residual, 3 residual and output in two fp16 planes
// (GemmDesc::res_planes / out_planes; a template parameter: the epilogue walk stays branch-free).
// wait until at most N of this wave's LDS-DMA instructions are outstanding and its LDS
// reads are done, then a workgroup barrier
// (the s_waitcnt builtin, not inline asm: hipcc's waitcnt pass then knows the fragment
// reads are done and does not add an lgkmcnt(0) in front of the next MFMAs, which would
// wait for the reads issued after this barrier too)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));  // vmcnt(N) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// wait until at most N of this wave's LDS-DMA instructions are outstanding (LDS reads
// stay in flight), then a workgroup barrier
template <int N>
__device__ __forceinline__ void vm_wait_nolgkm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));  // vmcnt(N) only
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Diagnostic build -DSPI_G256_TIMELINE (tools/g256_timeline.py): per workgroup, s_memrealtime at
// entry, after the prologue's first wait, after the k-loop and at exit, plus HW_ID / XCC_ID.
#ifdef SPI_G256_TIMELINE
__device__ unsigned long long g_g256_tl[8192 * 6];
#define G256_RT(x) x = __builtin_amdgcn_s_memrealtime()
#else
#define G256_RT(x)
#endif

// Ping-pong wave rows (the lock-step two-tile-ahead variant measured C5 -2.3 % and was removed, round 4)
template <int RES, int BM, int NBUF>
__global__ __launch_bounds__(512) void gemm256_kernel(const G256Args g) {
  using Geo = G256Geo<BM, NBUF>;
  constexpr int kBufBytes = Geo::kBufBytes, kBOff = Geo::kBOff, kNQ = Geo::kNQ, kMA = Geo::kMA;
  // ONE LDS object: with a second __shared__ variable beside the k-tile buffers hipcc's waitcnt
  // pass could no longer tell the LDS-DMA destinations from the fragment reads and put a
  // vmcnt(0) in front of every phase's reads (ViT-L FFN1 / QKV +15 %, round 4)
  // and exactly the k-tile buffers: 2 KiB more (the LayerNorm statistics, round 4) made
  // every launch 2-5 % slower (tools/ab_gemm.py, -DSPI_G256_LDS128 against it).  The split-K
  // ticket lives in buffer 0 once the k-loop's last reads are done; the statistics in registers.
  __shared__ __attribute__((aligned(16))) char lds[Geo::kLds];
  int* const s_ticket = reinterpret_cast<int*>(lds);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  [[maybe_unused]] unsigned long long tl0 = 0, tl1 = 0, tl2 = 0;
  G256_RT(tl0);
  // every return of the kernel goes through exit_stamp()
  auto exit_stamp = [&]() {
#ifdef SPI_G256_TIMELINE
    unsigned long long tl3;
    G256_RT(tl3);
    if (tid == 0 && blockIdx.x < 8192) {
      unsigned long long* o = g_g256_tl + (size_t)blockIdx.x * 6;
      o[0] = tl0;
      o[1] = tl1;
      o[2] = tl2;
      o[3] = tl3;
      o[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      o[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
#endif
  };
  const int fr = lane & 15, fq = lane >> 4;

  // XCD-aware bijective remap: the workgroups one XCD receives get consecutive ids (slice-major:
  // neighbours share a k-range of the same W panel)
  const int tiles = g.tiles_m * g.tiles_n, nwg = tiles * g.splits, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int slice = wgid / tiles, tile = wgid - slice * tiles;
  const int tm = g.n_fast ? tile / g.tiles_n : tile % g.tiles_m;
  const int tn = g.n_fast ? tile - tm * g.tiles_n : tile / g.tiles_m;
  const int m0 = tm * BM, n0 = tn * 256;
  const int kt0 = slice * g.ktp;
  const int KT = min(g.ktp, (g.K >> 6) - kt0);

  // per-lane DMA sources of each staging piece's two 1 KiB parts (k-tile 0); advance 128 B per k-tile
  const char* src[kNQ][2];
  int dsto[kNQ][2];
  {
    const int rl = lane >> 3, chunk = (lane & 7) ^ rl;  // row within the 8-row piece, swizzled chunk
#pragma unroll
    for (int q = 0; q < kNQ; ++q)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int base = quarter_row<BM>(q, wave * 2 + j);
        const int r = base + rl;
        if (quarter_is_a<BM>(q)) {
          const int m = min(m0 + r, g.M - 1);  // rows past M: a valid row, never stored
          src[q][j] = reinterpret_cast<const char*>(g.A + (size_t)m * g.lda + kt0 * 64) + chunk * 16;
          dsto[q][j] = base * 128;
        } else {
          src[q][j] = reinterpret_cast<const char*>(g.W + (size_t)(n0 + r) * g.ldw + kt0 * 64) + chunk * 16;
          dsto[q][j] = kBOff + base * 128;
        }
      }
  }
  auto bufof = [&](int kt) -> char* {
    if constexpr (Geo::kNBuf == 2)
      return lds + (kt & 1) * kBufBytes;
    else
      return lds + (kt % 3) * kBufBytes;
  };
  auto stage = [&](int q, int kt) {
    char* buf = bufof(kt);
    const int kofs = kt * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[q][j] + kofs),
                                       (lds_ptr_t)(buf + dsto[q][j]), 16, 0, 0);
  };

  // LNC (the LayerNorm consumer fold, RES = 0, ln_in_chunks > 0): the tile rows' {mean, rstd}.
  // Four lanes share a row: lane q of the four loads its 4 of the row's 16 chunk partials (two
  // 16-byte loads, ln_load) and the four combine them (ln_combine: Chan's formula over two
  // xor-shuffle rounds).  Each thread loading its row's 16 partials (round 4) had kept 32 more
  // registers live beside the 128 accumulators and spilled.  Where the loads go (round 6,
  // profiles/r06/ln_stats/): 256-row tiles at the epilogue's start -- in the last k-tile, to hide
  // the round trip, they spilled more (148 bytes per lane against 84) and measured slower (ViT-L
  // FFN1 35.2 vs 33.1 us back to back, C5 6.77k vs 6.99k); 128-row tiles (64 accumulators) under
  // the last k-tile's MFMAs (BERT-base's FFN1: C3 +0.8 % against the epilogue start).
  // Round h, half-wave lane l = tid & 31: row m0 + kRoundRows h + (tid >> 5) + 16 (l >> 2) -- the
  // epilogue walk's pass l >> 2 -- chunks 4 (l & 3) .. + 3.
  constexpr int kLnRounds = BM / Geo::kRoundRows;
  [[maybe_unused]] floatx4 ln_ch[RES == 0 ? kLnRounds : 1][2];
  [[maybe_unused]] float2 ln_st[RES == 0 ? kLnRounds : 1];
  [[maybe_unused]] const bool lnc = RES == 0 && g.ln_in_chunks > 0;
  auto ln_load = [&] {
    if constexpr (RES == 0) {
      if (lnc) {
        const int q = tid & 3, pass = (tid & 31) >> 2;
        // chunks past ln_in_chunks (D < 1024) re-read the row's last pair and are masked in ln_combine
        const int c0 = min(4 * q, g.ln_in_chunks - 2), c1 = min(4 * q + 2, g.ln_in_chunks - 2);
#pragma unroll
        for (int h = 0; h < kLnRounds; ++h) {
          const int m = min(m0 + Geo::kRoundRows * h + (tid >> 5) + 16 * pass, g.M - 1);
          const float* p = g.ln_in_stats + (size_t)m * g.ln_in_chunks * 2;
          ln_ch[h][0] = *reinterpret_cast<const floatx4*>(p + 2 * c0);
          ln_ch[h][1] = *reinterpret_cast<const floatx4*>(p + 2 * c1);
        }
      }
    }
  };
  auto ln_combine = [&] {
    if constexpr (RES == 0) {
      if (lnc) {
        const int q = tid & 3;
        const float k = (float)g.ln_in_chunks;
#pragma unroll
        for (int h = 0; h < kLnRounds; ++h) {
          // this lane's chunks 4 q + j: (mean, M2) = ln_ch[h][j / 2] components 2 (j & 1), + 1
          float mc[4], m2c[4];
          bool ok[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const floatx4 v = ln_ch[h][j >> 1];
            mc[j] = (j & 1) ? v[2] : v[0];
            m2c[j] = (j & 1) ? v[3] : v[1];
            ok[j] = 4 * q + j < g.ln_in_chunks;
          }
          float sm = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) sm += ok[j] ? mc[j] : 0.f;
          sm += __shfl_xor(sm, 1, 64);
          sm += __shfl_xor(sm, 2, 64);
          const float mean = sm / k;
          float m2 = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float dm = mc[j] - mean;
            m2 += ok[j] ? m2c[j] + 64.f * dm * dm : 0.f;
          }
          m2 += __shfl_xor(m2, 1, 64);
          m2 += __shfl_xor(m2, 2, 64);
          ln_st[h] = float2{mean, rsqrtf(m2 / (64.f * k) + g.ln_in_eps)};
        }
      }
    }
  };

  floatx4 acc[kMA][4];
#pragma unroll
  for (int a = 0; a < kMA; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 fa[kMA / 4][2][4];  // [m half][kk][i]
  half8 fb[2][2][2];        // [n half][kk][j]

  auto rd = [&](const char* img, int row, int c) -> half8 {
    return *reinterpret_cast<const half8*>(img + row * 128 + ((c ^ (row & 7)) << 4));
  };
  auto read_a = [&](const char* buf, int mq) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[mq][kk][i] = rd(buf, (BM / 2) * wr + 64 * mq + 16 * i + fr, kk * 4 + fq);
  };
  auto read_b = [&](const char* buf, int nq) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[nq][kk][j] = rd(buf + kBOff, 64 * wc + 32 * nq + 16 * j + fr, kk * 4 + fq);
  };
  auto mma = [&](int mq, int nq) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq * 4 + i][nq * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[mq][kk][i], fb[nq][kk][j], acc[mq * 4 + i][nq * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (BM == 256) {
    // Ping-pong (cdna_hip_programming.md §5, the 256² 8-phase template): every phase is
    //   [reads of its fragments, one quarter's LDS-DMA, counted vmcnt] B_a [MFMAs] B_b
    // and wave row 1 runs one barrier behind wave row 0 (an extra s_barrier up front, one
    // at the end for row 0), so between any two barriers one wave of each SIMD issues MFMAs
    // while the other one reads LDS / issues DMA: the MFMA pipe never waits for a read.
    // Reads: phase 0 A_m0 + B_n0 (Q0, Q1), 1 B_n1 (Q2), 2 A_m1 (Q3), 3 none.  Quarters
    // go out in one sequence s = 4 k + q, quarter s in global phase s - 6 (Q2 / Q3 of tile
    // t + 1 in phases 0 / 1 of tile t, Q0 / Q1 of tile t + 2 in phases 2 / 3): a region is
    // restaged >= 2 phases after its last read (WAR with the one-barrier skew), and a
    // quarter has ~4 phases to land.  The wait for phase P's quarter sits before B_a of
    // phase P - 1, so both wave rows have retired it a barrier before either reads it.
    // vmcnt after this phase's DMA, tile t with R = min(KT - 1 - t, 2) tiles after it:
    //   phase 0: R >= 1 8, R = 0 2;  phase 1: 8 / 0;  phase 3: R = 2 8, R = 1 4, R = 0 -.
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (q < 4 * KT) stage(q & 3, q >> 2);
    if (KT > 1)
      vm_wait_nolgkm<8>();
    else
      vm_wait_nolgkm<4>();
    if (wr == 1) bar();  // the skew
    G256_RT(tl1);
    auto ktile = [&](int kt, auto rem_c) {
      constexpr int R = decltype(rem_c)::value;
      const char* buf = bufof(kt);
      // phase 0
      read_a(buf, 0);
      read_b(buf, 0);
      if constexpr (R >= 1) stage(2, kt + 1);
      vm_wait_nolgkm<R >= 1 ? 8 : 2>();
      mma(0, 0);
      bar();
      // phase 1
      read_b(buf, 1);
      if constexpr (R >= 1) stage(3, kt + 1);
      vm_wait_nolgkm<R >= 1 ? 8 : 0>();
      mma(0, 1);
      bar();
      // phase 2
      read_a(buf, 1);
      if constexpr (R >= 2) stage(0, kt + 2);
      bar();
      mma(1, 0);
      bar();
      // phase 3
      if constexpr (R >= 2) stage(1, kt + 2);
      if constexpr (R >= 1)
        vm_wait_nolgkm<R >= 2 ? 8 : 4>();
      else
        bar();
      mma(1, 1);
      bar();
    };
    for (int kt = 0; kt < KT - 2; ++kt) ktile(kt, std::integral_constant<int, 2>{});
    if (KT > 1) ktile(KT - 2, std::integral_constant<int, 1>{});
    ktile(KT - 1, std::integral_constant<int, 0>{});
    if (wr == 0) bar();  // the skew, closed
  } else if constexpr (NBUF == 3) {
    // 128 x 256: the same ping-pong of the two wave rows, 2 phases per k-tile, three buffers.
    //   phase 0: reads A + B n-half 0 (T0, T1), stages T0 + T1 of tile t + 2, MFMAs (0, 0)
    //   phase 1: reads B n-half 1 (T2),        stages T2 of tile t + 2,      MFMAs (0, 1)
    // Tile t + 2 goes into the buffer of tile t - 1, whose thirds wave row 0 read two phases
    // earlier -- wave row 1 runs one barrier behind, so a region is restaged only after both
    // rows' reads of it are done (round 6: the first schedule restaged one phase after row 0's
    // read, racing row 1's).  The thirds go out in one sequence T0(0) T1(0) T2(0)
    // T0(1) ... (the prologue issues tiles 0 and 1), each has ~4 phases to land.
    // With R = KT - 1 - t tiles after tile t, the waits after each phase's DMA:
    //   phase 0 (T2(t) must have landed):      2 (3 [R >= 1] + 2 [R >= 2]) pieces younger
    //   phase 1 (T0, T1(t + 1) must have):     2 (1 + 3 [R >= 2]); R = 0: none
    const int npro = min(6, 3 * KT);
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (q < npro) stage(q % 3, q / 3);
    if (KT >= 2)
      vm_wait_nolgkm<8>();
    else
      vm_wait_nolgkm<2>();
    if (wr == 1) bar();  // the skew
    G256_RT(tl1);
    auto ktile = [&](int kt, auto rem_c) {
      constexpr int R = decltype(rem_c)::value;
      const char* buf = bufof(kt);
      // phase 0
      read_a(buf, 0);
      read_b(buf, 0);
      if constexpr (R >= 2) {
        stage(0, kt + 2);
        stage(1, kt + 2);
      }
      vm_wait_nolgkm<2 * ((R >= 1 ? 3 : 0) + (R >= 2 ? 2 : 0))>();
      mma(0, 0);
      bar();
      // phase 1
      read_b(buf, 1);
      if constexpr (R == 0) ln_load();  // (128-row tiles: under the last k-tile's MFMAs)
      if constexpr (R >= 2) stage(2, kt + 2);
      if constexpr (R >= 1)
        vm_wait_nolgkm<2 * (1 + (R >= 2 ? 3 : 0))>();
      else
        bar();
      mma(0, 1);
      bar();
    };
    for (int kt = 0; kt < KT - 2; ++kt) ktile(kt, std::integral_constant<int, 2>{});
    if (KT > 1) ktile(KT - 2, std::integral_constant<int, 1>{});
    ktile(KT - 1, std::integral_constant<int, 0>{});
    if (wr == 0) bar();  // the skew, closed
  } else {
    // 128 x 256 on two buffers (96 KiB: room for another kernel's 64 KiB workgroup on the CU).
    //   phase 0: reads T0, T1, stages T0 + T1 of tile t + 1 (that buffer's T0 / T1: read by row 0 in
    //            tile t - 1's phase 0, two phases earlier)
    //   phase 1: reads T2,     stages T2 of tile t + 1 (read in tile t - 1's phase 1)
    // so a region is restaged only after both wave rows' reads (the one-barrier skew; round 6, as
    // above), and a third has ~2 phases to land; waits (R = KT - 1 - t):
    //   phase 0 (T2(t)):         4 [R >= 1] pieces younger
    //   phase 1 (T0, T1(t + 1)): 2; R = 0: none
    const int npro = min(3, 3 * KT);
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q < npro) stage(q, 0);
    vm_wait_nolgkm<2>();
    if (wr == 1) bar();  // the skew
    G256_RT(tl1);
    auto ktile = [&](int kt, auto rem_c) {
      constexpr int R = decltype(rem_c)::value;
      const char* buf = bufof(kt);
      read_a(buf, 0);
      read_b(buf, 0);
      if constexpr (R >= 1) {
        stage(0, kt + 1);
        stage(1, kt + 1);
      }
      vm_wait_nolgkm<R >= 1 ? 4 : 0>();
      mma(0, 0);
      bar();
      read_b(buf, 1);
      if constexpr (R == 0) ln_load();  // (128-row tiles: under the last k-tile's MFMAs)
      if constexpr (R >= 1) stage(2, kt + 1);
      if constexpr (R >= 1)
        vm_wait_nolgkm<2>();
      else
        bar();
      mma(0, 1);
      bar();
    };
    for (int kt = 0; kt < KT - 1; ++kt) ktile(kt, std::integral_constant<int, 1>{});
    ktile(KT - 1, std::integral_constant<int, 0>{});
    if (wr == 0) bar();  // the skew, closed
  }

  G256_RT(tl2);
  if (g.splits > 1) {
    // Split-K hand-off, gemm.hip's protocol (tickets first; slices that are not last publish
    // their partial write-through (sc1) in fragment order -- thread tid's accumulator (a, b) is
    // 16 contiguous bytes at ((a * 4 + b) * 512 + tid) * 16 -- drain, and count it in the second
    // word; the last arriver polls the count, resets both words and reads the slabs with sc1
    // loads).  Partials are summed in slice order whichever slice arrives last (((p0 + p1) + p2)
    // + p3, the own partial from registers, slots past `splits` read as 0 through the buffer
    // range): results do not depend on arrival order.
    constexpr int SLAB = BM * 256;
    int* words = g.counters + 2 * tile;
    float* slabs = g.partial + (size_t)tile * g.splits * SLAB;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(slabs, (short)0, g.splits * SLAB * 4, 0x00020000);
    if (tid == 0) *s_ticket = __hip_atomic_fetch_add(words, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*s_ticket < g.splits - 1) {
#pragma unroll
      for (int a = 0; a < kMA; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a][b]), rs,
                                                 (slice * SLAB + ((a * 4 + b) * 512 + tid) * 4) * 4, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid == 0) __hip_atomic_fetch_add(words + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      exit_stamp();
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(words + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g.splits - 1)
        __builtin_amdgcn_s_sleep(1);
      __hip_atomic_store(words, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(words + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < kMA; ++a) {
      floatx4 v[kMaxSplits][4];
#pragma unroll
      for (int z = 0; z < kMaxSplits; ++z)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          v[z][b] = __builtin_bit_cast(
              floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, (z * SLAB + ((a * 4 + b) * 512 + tid) * 4) * 4, 0, 16));
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        floatx4 sum = slice == 0 ? acc[a][b] : v[0][b];
#pragma unroll
        for (int z = 1; z < kMaxSplits; ++z) sum += slice == z ? acc[a][b] : v[z][b];
        acc[a][b] = sum;
      }
    }
  }

  // Epilogue through LDS (the k-loop's buffers are free): per-element stores from the
  // fragment layout (2-4 bytes, 128 per lane) made the tail store-issue-bound -- as
  // long as the k-loop itself (cdna_hip_programming.md T21).  Two rounds, one per
  // wave row wr: its four waves park their 128 x 64 fp32 accumulators as a
  // [128][256] fp32 half-tile (16-column blocks XOR-swizzled by (row >> 2) & 3, so
  // a fragment's ds_write_b32 rows 4 apart hit different banks), then all 512
  // threads walk it in 8-column row vectors: bias, residual, activation, 16- or
  // 32-byte stores.  Unaligned strides / pointers take the per-element path.
  const Act act = static_cast<Act>(g.act);
  auto finish = [&](float y) {
    if (act == Act::Relu) return y > 0.f ? y : 0.f;
    if (act == Act::Gelu) return gelu(y);
    return y;
  };
  if (!g.vec_ok) {
    float bv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) bv[b] = g.bias ? g.bias[n0 + 64 * wc + 16 * b + fr] : 0.f;
#pragma unroll
    for (int a = 0; a < kMA; ++a)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = m0 + (BM / 2) * wr + 16 * a + 4 * fq + v;
        if (m >= g.M) continue;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int n = n0 + 64 * wc + 16 * b + fr;
          float y = acc[a][b][v] + bv[b];
          if (g.res) {  // residual before the activation, as the general kernel (conv + BN + x -> ReLU)
            const size_t ri = (size_t)m * g.ldr + n;
            const _Float16* rh = static_cast<const _Float16*>(g.res);
            y += RES == 3 ? static_cast<float>(rh[ri]) + static_cast<float>(rh[ri + g.plane])
                 : g.res_f32 ? static_cast<const float*>(g.res)[ri]
                             : static_cast<float>(rh[ri]);
          }
          y = finish(y);
          const size_t ci = (size_t)m * g.ldc + n;
          if constexpr (RES == 3) {
            _Float16* ch = static_cast<_Float16*>(g.C);
            ch[ci] = static_cast<_Float16>(y);
            ch[ci + g.plane] = static_cast<_Float16>(y - static_cast<float>(ch[ci]));
          } else if (g.out_f32)
            static_cast<float*>(g.C)[ci] = y;
          else
            static_cast<_Float16*>(g.C)[ci] = static_cast<_Float16>(y);
        }
      }
    exit_stamp();
    return;
  }
  // The walk is branch-free per row: the residual kind (none / fp16 / fp32) is a template
  // parameter and rows past M load a clamped, valid row; in the last tile row (GUARD) their
  // stores are skipped -- never store the duplicates: with C the residual buffer (in place,
  // ViT's residual stream) a duplicate raced with the real row (fixed in round 3).  A runtime
  // `if (res)` or a guarded bias load per element had hipcc branch around each load and wait
  // vmcnt(0) per row (the weight-resident conv measured that as 40 % of its epilogue).  Each
  // thread's 8 residual rows of a round are loaded before the round's park, so their latency
  // hides behind it.
  float* T = reinterpret_cast<float*>(lds);
  const int cg = tid & 31, r0 = tid >> 5;  // 8-column group, first row of this thread
  const int nb = n0 + 8 * cg;
  float bias8[8];
  if (g.bias) {
    const floatx4 b0 = *reinterpret_cast<const floatx4*>(g.bias + nb);
    const floatx4 b1 = *reinterpret_cast<const floatx4*>(g.bias + nb + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bias8[e] = b0[e];
      bias8[e + 4] = b1[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) bias8[e] = 0.f;
  }
  // activation and output format are dispatched once, outside the rounds (always_inline: left
  // to itself hipcc outlined the 12 instances as calls, spilling the accumulators -- 944 bytes of
  // scratch per thread -- around each)
  // LNC (compile-time: a launch without the fold carries none of its registers -- as a runtime
  // branch it cost every gemm256 launch 2-5 %): the consumer side of the LayerNorm fold.  The
  // walk's row of pass p in round h is m0 + 128 h + r0 + 16 p, shared by the 32 lanes of this
  // thread's half-wave; lane cg computes {mean, rstd} of pass cg & 7's row in both rounds (all
  // chunk loads in flight) and the walk takes them from lane (lane & 32) | p.
  // LNO (compile-time too): the producer side (chunk statistics + the fp16 copy of every row).
  auto epi = [&](auto act_c, auto f32_c, auto guard_c, auto lnc_c, auto lno_c) SPI_G256_EPI_INLINE {
    constexpr int ACT = decltype(act_c)::value;
    constexpr bool OUTF32 = decltype(f32_c)::value;
    constexpr bool GUARD = decltype(guard_c)::value;  // the tile crosses M
    constexpr bool LNC = decltype(lnc_c)::value;
    constexpr bool LNO = decltype(lno_c)::value;
    constexpr int kRR = Geo::kRoundRows, kRounds = BM / kRR, kPasses = kRR / 16;  // rounds of the LDS-parked tile
    [[maybe_unused]] float c18[8];
    if constexpr (LNC) {  // the rows' {mean, rstd} (ln_st)
      static_assert(kRounds == kLnRounds, "epilogue rounds");
      if constexpr (BM == 256) ln_load();  // (128-row tiles loaded them in the last k-tile)
      ln_combine();
      const floatx4 c0 = *reinterpret_cast<const floatx4*>(g.ln_c1 + nb);
      const floatx4 c1 = *reinterpret_cast<const floatx4*>(g.ln_c1 + nb + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        c18[e] = c0[e];
        c18[e + 4] = c1[e];
      }
    }
#pragma unroll
    for (int h = 0; h < kRounds; ++h) {
      // residual rows: a ring of four rows per thread, the first four loaded before the park
      // (all eight at once would spill next to the accumulators the other wave row still holds)
      constexpr int PRE = 4;
      half8 rvh[RES == 1 || RES == 3 ? PRE : 1];
      half8 rvl[RES == 3 ? PRE : 1];  // the lo plane's rows (RES = 3)
      floatx4 rvf[RES == 2 ? PRE : 1][2];
      auto res_row = [&](int pass) -> size_t {
        const int m = min(m0 + kRR * h + r0 + 16 * pass, g.M - 1);
        return (size_t)m * g.ldr + nb;
      };
      if constexpr (RES == 1 || RES == 3) {
#pragma unroll
        for (int pass = 0; pass < PRE; ++pass) {
          rvh[pass] = *reinterpret_cast<const half8*>(static_cast<const _Float16*>(g.res) + res_row(pass));
          if constexpr (RES == 3)
            rvl[pass] = *reinterpret_cast<const half8*>(static_cast<const _Float16*>(g.res) + res_row(pass) + g.plane);
        }
      }
      if constexpr (RES == 2) {
#pragma unroll
        for (int pass = 0; pass < PRE; ++pass) {
          const float* rp = static_cast<const float*>(g.res) + res_row(pass);
          rvf[pass][0] = *reinterpret_cast<const floatx4*>(rp);
          rvf[pass][1] = *reinterpret_cast<const floatx4*>(rp + 4);
        }
      }
      __syncthreads();  // the k-loop's last reads / the previous round's walk are done
      // BM = 256: wave row h owns the round's 128 rows; BM = 128: both wave rows park at once
      if (kRR == BM || wr == h) {
#pragma unroll
        for (int a = 0; a < kMA; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int row = (kRR == BM ? (BM / 2) * wr : 0) + 16 * a + 4 * fq + v;
              const int col = (64 * wc + 16 * b + fr) ^ (((row >> 2) & 3) << 4);
              T[row * 256 + col] = acc[a][b][v];
            }
      }
      __syncthreads();
      {
#pragma unroll
        for (int pass = 0; pass < kPasses; ++pass) {
          const int row = r0 + 16 * pass;
          const int m = m0 + kRR * h + row;
          const float* src = T + row * 256 + ((8 * cg) ^ (((row >> 2) & 3) << 4));
          const floatx4 x0 = *reinterpret_cast<const floatx4*>(src);
          const floatx4 x1 = *reinterpret_cast<const floatx4*>(src + 4);
          // residual rows through a ring of PRE slots: slot pass % PRE is consumed here and
          // refilled with row pass + PRE, so every load has PRE passes to land (round 5: the
          // passes past PRE had loaded their rows in the walk, latency exposed -- ViT-L
          // out-proj / FFN2 epilogues 10.3-10.5 us, tools/g256_timeline.py)
          float r[8] = {};
          if constexpr (RES == 1) {
            const half8 q = rvh[pass % PRE];
            if (pass + PRE < kPasses)
              rvh[pass % PRE] = *reinterpret_cast<const half8*>(static_cast<const _Float16*>(g.res) +
                                                               res_row(pass + PRE));
#pragma unroll
            for (int e = 0; e < 8; ++e) r[e] = static_cast<float>(q[e]);
          }
          if constexpr (RES == 3) {
            const half8 qh = rvh[pass % PRE], ql = rvl[pass % PRE];
            if (pass + PRE < kPasses) {
              const _Float16* rp = static_cast<const _Float16*>(g.res) + res_row(pass + PRE);
              rvh[pass % PRE] = *reinterpret_cast<const half8*>(rp);
              rvl[pass % PRE] = *reinterpret_cast<const half8*>(rp + g.plane);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) r[e] = static_cast<float>(qh[e]) + static_cast<float>(ql[e]);
          }
          if constexpr (RES == 2) {
            const floatx4 q0 = rvf[pass % PRE][0], q1 = rvf[pass % PRE][1];
            if (pass + PRE < kPasses) {
              const float* rp = static_cast<const float*>(g.res) + res_row(pass + PRE);
              rvf[pass % PRE][0] = *reinterpret_cast<const floatx4*>(rp);
              rvf[pass % PRE][1] = *reinterpret_cast<const floatx4*>(rp + 4);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              r[e] = q0[e];
              r[e + 4] = q1[e];
            }
          }
          float y[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] = e < 4 ? x0[e] : x1[e - 4];
          if constexpr (LNC) {  // LayerNorm of the A rows folded in: rstd (acc - mean c1)
            const int src = (lane & 32) | (pass << 2);  // a lane of the four that combined this pass's row
            const float mean = __shfl(ln_st[h].x, src, 64), rstd = __shfl(ln_st[h].y, src, 64);
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = rstd * (y[e] - mean * c18[e]);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            y[e] += bias8[e] + r[e];
            if constexpr (ACT == (int)Act::Relu) y[e] = y[e] > 0.f ? y[e] : 0.f;
          }
          if constexpr (ACT == (int)Act::Gelu) {
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const float2v g2 = gelu2(float2v{y[e], y[e + 1]});
              y[e] = g2.x;
              y[e + 1] = g2.y;
            }
          }
          // Rows past M exist only in tiles that cross M (GUARD, the last tile row): their stores
          // are skipped.  (Storing them as duplicates of row M - 1, as full tiles' branch-free walk
          // could, races with the real row M - 1 when C is the residual buffer itself -- the
          // transformer's in-place residual stream: a duplicate that reads the residual after the
          // real row's store adds the GEMM twice.)
          if constexpr (LNO) {  // producer: chunk statistics (all lanes shuffle) + the fp16 copy
            float mean, m2;
            ln_chunk_stats(y, mean, m2);
            if (m < g.M) {
              if ((cg & 7) == 0)
                reinterpret_cast<float2*>(g.ln_out_stats)[(size_t)m * (g.N >> 6) + (nb >> 6)] = float2{mean, m2};
              if constexpr (RES != 3) {  // (two planes: the hi plane is the copy)
                half8 hq;
#pragma unroll
                for (int e = 0; e < 8; ++e) hq[e] = static_cast<_Float16>(y[e]);
                *reinterpret_cast<half8*>(g.c16 + (size_t)m * g.ld16 + nb) = hq;
              }
            }
          }
          if constexpr (GUARD) {
            if (m >= g.M) continue;
          }
          const size_t ci = (size_t)m * g.ldc + nb;
          if constexpr (RES == 3) {
            half8 oh, ol;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              oh[e] = static_cast<_Float16>(y[e]);
              ol[e] = static_cast<_Float16>(y[e] - static_cast<float>(oh[e]));
            }
            *reinterpret_cast<half8*>(static_cast<_Float16*>(g.C) + ci) = oh;
            *reinterpret_cast<half8*>(static_cast<_Float16*>(g.C) + ci + g.plane) = ol;
          } else if constexpr (OUTF32) {
            *reinterpret_cast<floatx4*>(static_cast<float*>(g.C) + ci) = floatx4{y[0], y[1], y[2], y[3]};
            *reinterpret_cast<floatx4*>(static_cast<float*>(g.C) + ci + 4) = floatx4{y[4], y[5], y[6], y[7]};
          } else {
            half8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = static_cast<_Float16>(y[e]);
            *reinterpret_cast<half8*>(static_cast<_Float16*>(g.C) + ci) = o;
          }
        }
      }
    }
};
  auto by_guard = [&](auto act_c, auto f32_c, auto lnc_c, auto lno_c) SPI_G256_EPI_INLINE {
    if (m0 + BM <= g.M)  // workgroup-uniform: only the last tile row takes the guarded walk
      epi(act_c, f32_c, std::false_type{}, lnc_c, lno_c);
    else
      epi(act_c, f32_c, std::true_type{}, lnc_c, lno_c);
  };
  auto by_act = [&](auto f32_c, auto lnc_c, auto lno_c) SPI_G256_EPI_INLINE {
    if constexpr (RES >= 2) {
      // fp32 / two-plane residual streams (the transformer out-proj / FFN2) carry no activation:
      // the host routes such descs elsewhere, and their instances would only add register pressure
      // (round 6: RES = 3 spilled 100 bytes per lane with ReLU / GELU instances, 0 without)
      by_guard(std::integral_constant<int, (int)Act::None>{}, f32_c, lnc_c, lno_c);
      return;
    }
    if (act == Act::Gelu)
      by_guard(std::integral_constant<int, (int)Act::Gelu>{}, f32_c, lnc_c, lno_c);
    else if (act == Act::Relu)
      by_guard(std::integral_constant<int, (int)Act::Relu>{}, f32_c, lnc_c, lno_c);
    else
      by_guard(std::integral_constant<int, (int)Act::None>{}, f32_c, lnc_c, lno_c);
  };
  using F = std::false_type;
  using T1 = std::true_type;
  // the consumer fold exists for fp16 outputs without a residual (the QKV / FFN1 GEMMs), the
  // producer for fp32 outputs over an fp32 residual (ViT's out-proj / FFN2); checked on the host
  if constexpr (RES == 0) {
    if (g.ln_in_chunks > 0) {
      by_act(F{}, T1{}, F{});
      exit_stamp();
      return;
    }
  }
  if constexpr (RES == 2 || RES == 3) {  // (RES = 3: planes out, whatever OUTF32 says)
    if (g.ln_out) {
      by_act(T1{}, F{}, T1{});
      exit_stamp();
      return;
    }
  }
  if constexpr (RES == 3) {
    by_act(F{}, F{}, F{});
    exit_stamp();
    return;
  }
  if (g.out_f32)
    by_act(T1{}, F{}, F{});
  else
    by_act(F{}, F{}, F{});
  exit_stamp();
}

}  // namespace

void gemm256_reload_env() {}

#ifdef SPI_G256_TIMELINE
extern "C" int spi_debug_g256_timeline(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_g256_tl), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif

int gemm256_splits(const GemmDesc& d, int target, int max_split, int bm) {
  const int tiles = (d.M + bm - 1) / bm * (d.N / 256), kt = d.K / 64;
  if (tiles >= target || max_split == 1) return 1;
  int s = std::min({(target + tiles - 1) / tiles, kt / kMinSliceKt, kMaxSplits});
  if (max_split > 0) s = std::min(s, max_split);
  if (s <= 1) return 1;
  const int ktp = (kt + s - 1) / s;
  return (kt + ktp - 1) / ktp;
}

bool gemm256_eligible(const GemmDesc& d, Prec prec, int min_tiles, int bm) {
  if (min_tiles <= 0 || prec != Prec::F16 || d.conv || d.krep != 1 || d.a_split || d.out_split || d.pool_rows ||
      d.out_f16)
    return false;
  if (d.res_planes != d.out_planes) return false;  // two planes: residual and output together (RES = 3)
  if ((d.res_f32 || d.res_planes) && d.act != Act::None) return false;  // RES >= 2: no activation instances
  if (d.N % 256 || d.K % 64 || d.Kpad != d.K || d.lda % 8 || d.M < 1) return false;
  // no post-LN residual epilogue here (BERT's out-proj / FFN2 under the LayerNorm fold keep the
  // general kernel at every size; gemm256() rejects them)
  if (d.res_ln_chunks > 0) return false;
  return (d.M + bm - 1) / bm * (d.N / 256) >= min_tiles;
}

void gemm256(const GemmDesc& d, const GemmPtrs& p, int splits, hipStream_t s, int bm, int nbuf, int n_fast) {
  if (d.N % 256 || d.K % 64 || d.Kpad != d.K) throw std::invalid_argument("gemm256: N % 256, K % 64, Kpad == K");
  if (bm != 256 && bm != 128) throw std::invalid_argument("gemm256: 256- or 128-row tiles");
  if (splits < 1 || splits > kMaxSplits || (splits > 1 && (!p.partial || !p.counters)))
    throw std::invalid_argument("gemm256: 1..4 split-K slices, with slabs and counters");
  G256Args g;
  g.A = static_cast<const _Float16*>(p.A);
  g.W = static_cast<const _Float16*>(p.W);
  g.bias = p.bias;
  g.res = p.res;
  g.C = p.C;
  g.lda = d.lda;
  g.ldw = d.Kpad;
  g.ldr = d.ldr;
  g.ldc = d.ldc;
  g.M = d.M;
  g.N = d.N;
  g.K = d.K;
  g.tiles_m = (d.M + bm - 1) / bm;
  g.tiles_n = d.N / 256;
  g.act = static_cast<int>(d.act);
  g.res_f32 = d.res_f32;
  g.out_f32 = d.out_f32;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  g.vec_ok = d.ldc % 8 == 0 && al16(p.C) && (!p.res || (d.ldr % 8 == 0 && al16(p.res))) && (!p.bias || al16(p.bias))
                 ? 1 : 0;
  g.ln_in_chunks = d.ln_in_chunks;
  g.ln_in_eps = d.ln_in_eps;
  g.ln_out = d.ln_out ? 1 : 0;
  g.ld16 = d.ld16;
  g.ln_in_stats = p.ln.in_stats;
  g.ln_c1 = p.ln.c1;
  g.ln_out_stats = p.ln.out_stats;
  g.c16 = p.ln.c16;
  if ((d.ln_in_chunks > 0 || d.ln_out) && !g.vec_ok)
    throw std::invalid_argument("gemm256: the LayerNorm fold needs the vector epilogue");
  if (d.ln_in_chunks > 0 && (p.res || d.out_f32))
    throw std::invalid_argument("gemm256: the LayerNorm consumer fold is for fp16 outputs without a residual");
  const bool planes = d.res_planes || d.out_planes;
  if (planes && (!d.res_planes || !d.out_planes || !p.res || d.out_f32 || d.plane % 8))
    throw std::invalid_argument("gemm256: two planes for the residual and the output together");
  if (d.ln_out && (!p.res || !((d.res_f32 && d.out_f32) || planes)))
    throw std::invalid_argument("gemm256: the LayerNorm producer fold is for fp32 or two-plane outputs over the same residual");
  if (d.res_ln_chunks > 0) throw std::invalid_argument("gemm256: no residual LayerNorm (post-LN) epilogue");
  const int kt = d.K / 64;
  g.ktp = (kt + splits - 1) / splits;
  g.splits = (kt + g.ktp - 1) / g.ktp;
  if (g.splits != splits) throw std::invalid_argument("gemm256: splits must leave no empty slice");
  g.partial = p.partial;
  g.counters = p.counters;
  g.n_fast = n_fast ? 1 : 0;
  g.plane = d.plane;
  const int res = planes ? 3 : !p.res ? 0 : d.res_f32 ? 2 : 1;
  if (res >= 2 && d.act != Act::None)
    throw std::invalid_argument("gemm256: no activation over an fp32 / two-plane residual");
  const dim3 grid(g.tiles_m * g.tiles_n * g.splits), blk(512);
  if (bm == 256) {
    if (res == 0)
      SPI_LAUNCH((gemm256_kernel<0, 256, 2>), grid, blk, 0, s, g);
    else if (res == 1)
      SPI_LAUNCH((gemm256_kernel<1, 256, 2>), grid, blk, 0, s, g);
    else if (res == 2)
      SPI_LAUNCH((gemm256_kernel<2, 256, 2>), grid, blk, 0, s, g);
    else
      SPI_LAUNCH((gemm256_kernel<3, 256, 2>), grid, blk, 0, s, g);
  } else if (nbuf == 3) {
    if (res == 0)
      SPI_LAUNCH((gemm256_kernel<0, 128, 3>), grid, blk, 0, s, g);
    else if (res == 1)
      SPI_LAUNCH((gemm256_kernel<1, 128, 3>), grid, blk, 0, s, g);
    else if (res == 2)
      SPI_LAUNCH((gemm256_kernel<2, 128, 3>), grid, blk, 0, s, g);
    else
      SPI_LAUNCH((gemm256_kernel<3, 128, 3>), grid, blk, 0, s, g);
  } else {
    if (res == 0)
      SPI_LAUNCH((gemm256_kernel<0, 128, 2>), grid, blk, 0, s, g);
    else if (res == 1)
      SPI_LAUNCH((gemm256_kernel<1, 128, 2>), grid, blk, 0, s, g);
    else if (res == 2)
      SPI_LAUNCH((gemm256_kernel<2, 128, 2>), grid, blk, 0, s, g);
    else
      SPI_LAUNCH((gemm256_kernel<3, 128, 2>), grid, blk, 0, s, g);
  }
}

}  // namespace spi
