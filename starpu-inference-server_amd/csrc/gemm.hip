// MFMA GEMM and conv-as-implicit-GEMM for gfx950 (CDNA4).
//
// One kernel body serves every dense contraction of the three model families:
//   * ResNet conv + folded BN (+ residual) (+ ReLU)      -- implicit GEMM over NHWC
//   * ResNet FC, BERT/ViT QKV / out-proj / FFN (+GELU) (+residual) -- dense GEMM
//
// Staging.  Every k-step moves 128 bytes of each A row and each W row:
//   F16   64 fp16 k-values (2 x v_mfma_f32_16x16x32_f16 per fragment pair)
//   F32   32 fp32 k-values (8 x v_mfma_f32_16x16x4_f32; lane l feeds k index
//         (l>>4) of step s with element 8(l>>4)+s of its 32 bytes -- the same
//         permutation on A and B, so the sum is unchanged; exact fp32 FMA chain)
//   F16X3 32 fp32 A values + W row = 32 hi fp16 | 32 lo fp16 (interleaved
//         packing); A is split into hi/lo at fragment-read time; each fragment
//         pair issues lo*hi + hi*lo + hi*hi (fp32-grade at the fp16 rate).
// The tile images are filled with global_load_lds_dwordx4 (LDS-DMA, 1 KiB per
// wave instruction, lane-linear): image row r, 16-byte slot s holds global chunk
// s ^ (r & 7) -- the XOR swizzle is applied on the SOURCE address and undone on
// the ds_read_b128 (cdna_hip_programming.md rule 21), which makes the fp16
// fragment reads bank-conflict free.  Chunks outside the image (conv padding,
// rows past M, k past K) are read from a zeroed line, so the DMA never needs a
// predicate.  STAGES-deep ring: step t+STAGES-1 is issued right after the
// barrier that publishes step t, waits are counted vmcnt + s_barrier in one
// asm statement (no __syncthreads(): its vmcnt(0) would drain the prefetch).
//
// Small-M layers are split along K; the workgroups of a tile publish fp32 slabs
// write-through (sc1) and the last to arrive (relaxed agent-scope ticket) sums
// them with sc1 loads and runs the epilogue -- no second launch, no cache-wide
// fences (cdna_hip_programming.md, "In-launch split-K reduction").
#include "device_math.hpp"
#include "ln_fold.hpp"
#include "spi_kernels.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <stdexcept>

namespace spi {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;


// Diagnostic build only (-DSPI_GEMM_STAMPS): per-block s_memtime phase totals.
#ifdef SPI_GEMM_STAMPS
__device__ unsigned long long g_gemm_stamps[65536 * 8];
#define SPI_STAMP(v)                                                                         \
  do {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");               \
    __builtin_amdgcn_sched_barrier(0);                                                       \
  } while (0)
#else
#define SPI_STAMP(v) \
  do {               \
  } while (0)
#endif
// Diagnostic build only (-DSPI_GEMM_TIMELINE): four s_memrealtime stamps per
// workgroup (entry, k-loop start, k-loop end, exit; 100 MHz) and the hardware
// ids (HW_ID: CU / SE; XCC_ID), so tools/gemm_timeline.py can split a launch
// into dispatch skew, prologue, loop and epilogue and see how workgroups pack
// onto CUs.  The real kernel has none of this.
#ifdef SPI_GEMM_TIMELINE
__device__ unsigned long long g_gemm_timeline[65536 * 8];
// launches made by a thread inside spi_debug_gemm_timeline_enable(1) .. (0) carry KArgs::tl = 1
// (Model::profile_op on the repeated op), so other streams' launches never stamp
int& tl_thread() {
  static thread_local int on = 0;
  return on;
}
#define SPI_RT(v)                                                                  \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                             \
  } while (0)
#else
#define SPI_RT(v) \
  do {            \
  } while (0)
#endif

// Diagnostic builds: -DSPI_DIAG_NO_DMA issues no LDS-DMA (the tiles hold stale
// bytes), -DSPI_DIAG_NO_MFMA reads the fragments but issues no MFMA; timed
// against the real kernel (tools/ab_gemm.py) they split a launch into data
// movement and matrix work.  Outputs of both are meaningless.
#ifdef SPI_DIAG_NO_DMA
#define SPI_DMA(src, dst, sz, off, aux) \
  do {                                  \
    (void)(src);                        \
    (void)(dst);                        \
  } while (0)
#else
#define SPI_DMA(src, dst, sz, off, aux) __builtin_amdgcn_global_load_lds(src, dst, sz, off, aux)
#endif
// Diagnostic build -DSPI_DIAG_L2A: every A-operand DMA reads from the first 64 KiB
// of A (same instruction count and addressing work, almost no L2-miss traffic);
// timed against the real kernel it separates memory-side traffic from the rest.
// Diagnostic builds -DSPI_DIAG_NO_DMA_A / _W: drop only the A-operand (incl.
// halo) or only the weight DMAs.
#ifdef SPI_DIAG_NO_DMA_A
#define SPI_DMA_A(src, dst, sz, off, aux) \
  do {                                    \
    (void)(src);                          \
    (void)(dst);                          \
  } while (0)
#else
#define SPI_DMA_A SPI_DMA
#endif
#ifdef SPI_DIAG_NO_DMA_W
#define SPI_DMA_W(src, dst, sz, off, aux) \
  do {                                    \
    (void)(src);                          \
    (void)(dst);                          \
  } while (0)
#else
#define SPI_DMA_W SPI_DMA
#endif
#ifdef SPI_DIAG_L2A
#define SPI_A_SRC(ptr_) \
  (reinterpret_cast<const char*>(a.p.A) + ((reinterpret_cast<const char*>(ptr_) - reinterpret_cast<const char*>(a.p.A)) & 0xFFF0))
#else
#define SPI_A_SRC(ptr_) (ptr_)
#endif

// n / d for 0 <= n < 2^31 by one high multiply (host-computed magic, Granlund-Montgomery
// round-up form: 2^s < d <= 2^(s+1), magic = ceil(2^(32+s) / d) < 2^32, exact since the
// magic's error (< d) times n stays below 2^(32+s)); d = 1 is magic 0.  The prologue of a
// launch divides a dozen times (tile decode, output row -> image / row / column), and the
// compiler's generic 32-bit division is ~40 instructions of dependent SALU / VALU each.
struct FastDiv {
  unsigned magic;
  int shift;
};
__host__ __device__ inline FastDiv make_fastdiv(unsigned d) {
  if (d <= 1) return FastDiv{0u, 0};
  int s = 0;
  while ((2ull << s) < d) ++s;  // 2^s < d <= 2^(s+1)
  return FastDiv{(unsigned)(((1ull << (32 + s)) + d - 1) / d), s};
}
__device__ __forceinline__ int fdiv(int n, FastDiv f) {
  return f.magic ? (int)(__umulhi((unsigned)n, f.magic) >> f.shift) : n;
}

struct KArgs {
  GemmDesc d;
  GemmPtrs p;
  int k_per_split;  // elements, multiple of the k-step
  int tiles_m, tiles_n;
  int tiles;
  int cin_shift;
  int kw_mul;       // ceil(65536 / KW): cell / KW == (cell * kw_mul) >> 16 for cell < 2^12
  int cell_uniform; // conv with Cin >= k-step: one (kh, kw) cell per step
  int vec_ok;       // C / residual rows allow 16-byte vectors of 8 elements (epilogue)
  int xg_m, xg_n;   // XCD rectangles: tile rows in xg_m groups x tile columns in xg_n groups
  // the rectangles' first tile row per row group (rg_m0[xg_m] = tiles_m) and first tile
  // column per column group (cg_n0[xg_n] = tile columns), and the row-group heights as
  // FastDivs: the decode is compares and high multiplies, no loop, no division
  int rg_m0[9], cg_n0[9];
  FastDiv fd_rows[8];
  FastDiv fd_split;      // / splits
  FastDiv fd_ohw, fd_ow;  // conv: output row m -> image, then row / column
  FastDiv fd_tiles;       // grouped launches: / tiles
  FastDiv fd_period, fd_hwp;  // halo kinds: / h_period, / h_hwp
  int imgs;                   // conv: images (M / (OH * OW))
  // halo conv (kConvHalo): tile row block tm is the band of h_th "virtual" output
  // rows u in [tm * h_th, (tm + 1) * h_th) x the full width.  Virtual rows stack the
  // images with a period of h_period rows: image u / h_period, output row
  // u % h_period - h_off (valid when in [0, OH)).  Aligned bands (h_off 0,
  // h_period = bands per image x h_th) stay inside one image; stacked bands
  // (h_off 1, h_period = OH + 2: a zero row above and below every image) may span
  // several images, so one tile can cover whole small maps of several images and
  // the weights are re-read by fewer tiles.  The band's input rows (+1 pixel of
  // padding around) form an h_hwp-wide halo image of h_hp pixels; h_nblk channel
  // blocks, h_bps of them per split-K slice
  int h_th, h_period, h_off, h_hwp, h_hp, h_nblk, h_bps;
  int win_nblk_shift;  // window kind (kConvTapW): log2 of the channel blocks per tap
  int splits;  // split-K slices (the grid holds tiles x splits workgroups of this problem)
#ifdef SPI_GEMM_TIMELINE
  int tl;  // stamp this launch (tools/gemm_timeline.py)
#endif
};

// One launch, one or two independent problems of the same kernel instance (a
// grouped launch: ResNet's downsample 1x1 conv beside its block's first conv,
// both reading the block input).  Workgroups [0, wgs0) run a[0], the rest a[1].
struct KGroup {
  KArgs a[2];
  int wgs0;
};

template <int MODE>
struct Traits;
// RB: bytes of each A / W image row per k-step; ESTEP: k-values per step;
// EPC: A elements per 16-byte chunk.
template <>
struct Traits<(int)Prec::F16> {
  using A = _Float16;
  using Out = _Float16;
  static constexpr int RB = 128, ESTEP = 64, EPC = 8;
};
template <>
struct Traits<(int)Prec::F32> {
  using A = float;
  using Out = float;
  static constexpr int RB = 128, ESTEP = 32, EPC = 4;
};
template <>
struct Traits<(int)Prec::F16X3> {  // A: 32 fp32; W: [32 hi | 32 lo] (RB = 256 measured slower: VGPRs, LDS)
  using A = float;
  using Out = float;
  static constexpr int RB = 128, ESTEP = 32, EPC = 4;
};
// Kernel-internal mode: F16X3 whose A (and residual) are activations already
// stored split, [32 hi fp16 | 32 lo fp16] per 32 channels (GemmDesc::a_split).
// Byte-for-byte the same addressing as fp32 A (a 32-k block is 128 bytes either
// way), so only the fragment reads differ: A is read exactly like W.
constexpr int kF16X3S = 3;
template <>
struct Traits<kF16X3S> : Traits<(int)Prec::F16X3> {};

template <int MODE>
constexpr bool kSplitMode = MODE == (int)Prec::F16X3 || MODE == kF16X3S;

// Split layout index (in fp16 units) of logical element (m, n) of a row-major
// [rows][ld] tensor: hi at the returned index, lo 32 further on.
__device__ __forceinline__ size_t split_idx(int m, int n, int ld) {
  return (size_t)m * ld * 2 + (size_t)(n >> 5) * 64 + (n & 31);
}

__device__ __forceinline__ float apply_act(float v, Act act) {
  if (act == Act::Relu) return v > 0.f ? v : 0.f;
  if (act == Act::Gelu) return gelu(v);
  return v;
}

template <int MODE>
__device__ __forceinline__ float load_res(const KArgs& a, int m, int n) {
  using Out = typename Traits<MODE>::Out;
  if constexpr (MODE == kF16X3S) {  // split residual: hi + lo
    const _Float16* R = static_cast<const _Float16*>(a.p.res);
    const size_t i = split_idx(m, n, a.d.ldr);
    return static_cast<float>(R[i]) + static_cast<float>(R[i + 32]);
  }
  const size_t idx = (size_t)m * a.d.ldr + n;
  if (a.d.res_planes) {  // two fp16 planes: hi + lo
    const _Float16* R = static_cast<const _Float16*>(a.p.res);
    return static_cast<float>(R[idx]) + static_cast<float>(R[idx + a.d.plane]);
  }
  return a.d.res_f32 ? static_cast<const float*>(a.p.res)[idx]
                     : static_cast<float>(static_cast<const Out*>(a.p.res)[idx]);
}

__device__ __forceinline__ void split8(const u32x4& x0, const u32x4& x1, half8& hi, half8& lo) {
  const floatx4 f0 = __builtin_bit_cast(floatx4, x0);
  const floatx4 f1 = __builtin_bit_cast(floatx4, x1);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 a = static_cast<_Float16>(f0[e]);
    const _Float16 b = static_cast<_Float16>(f1[e]);
    hi[e] = a;
    hi[e + 4] = b;
    lo[e] = static_cast<_Float16>(f0[e] - static_cast<float>(a));
    lo[e + 4] = static_cast<_Float16>(f1[e] - static_cast<float>(b));
  }
}

// Wait for this wave's LDS-DMA down to N outstanding, then barrier.  One asm
// statement with a memory clobber so no LDS access moves across it.
template <int N>
__device__ __forceinline__ void dma_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// One 1-KiB LDS-DMA piece (lane l's 16 bytes from `src` to dst + 16 l) issued from inline
// asm, invisible to hipcc's waitcnt pass: the epilogue's residual prefetch lands in a stage
// region addressed at run time, and with the builtin hipcc would assume it may alias the
// last k-steps' fragment reads and drain it (vmcnt(0)) before them.  Counted by the
// k-loop's dma_wait_barrier<N> and waited for explicitly before the epilogue reads it.
__device__ __forceinline__ void glds16(const void* src, char* dst) {
  const lds_ptr_t lp = (lds_ptr_t)dst;
  const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lp);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(m0v)
               : "memory");
}

// The 4-byte form (a 256-byte piece: lane l's 4 bytes to dst + 4 l), same hand-counted contract.
__device__ __forceinline__ void glds4(const void* src, char* dst) {
  const lds_ptr_t lp = (lds_ptr_t)dst;
  const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lp);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(m0v)
               : "memory");
}

template <int RB>
__device__ __forceinline__ u32x4 rd_chunk(const char* img, int row, int c) {
  constexpr int CPR = RB / 16;  // 16-byte chunks per image row
  return *reinterpret_cast<const u32x4*>(img + row * RB + ((c ^ (row & (CPR - 1))) << 4));
}

// A-operand kinds: dense rows; conv with one (kh, kw) tap per k-step (Cin >= the
// k-step: scalar tap walk + per-row tap mask); conv in general (per-chunk taps:
// the stem); 3x3/s1/p1 conv from an LDS-resident input band (kConvHalo, below).
// Separate instantiations keep each kind's loop free of the others.
enum : int { kDense = 0, kConvTap = 1, kConvGen = 2, kConvHalo = 3, kConvHaloS = 4, kConvTapW = 5 };

// Split-K is compiled into the 64x64 and 128x64 tiles and the halo kinds (no plan
// rule splits 128x128; the reducer costs 36-120 VGPRs there).  Launch bounds ask
// for the occupancy each tile reaches within its registers: 4 / 3 / 2 waves per SIMD.
template <int BM, int BN, int KIND>
constexpr bool kSplitK = (BM == 64 && BN == 64) || (BM == 128 && BN == 64) || KIND == kConvHalo || KIND == kConvHaloS;

// kConvHalo.  An implicit-GEMM conv stages each (tap, channel block) A tile
// separately: every input pixel crosses the CU nine times, and the vector-memory
// ingest of a CU (~70 GB/s from L2, MI355X_MICROARCH.md "gather into LDS") is
// what bounds these layers (no-DMA diagnostic build: +64 % end to end).  Here a
// tile is a band of whole output rows of one image; per channel block the band's
// input rows plus the 1-pixel border -- (th + 2) x (W + 2) pixels, 128 bytes each,
// swizzled like the ring images -- are DMA'd once into one of two halo buffers,
// and the nine taps read their A fragments from it at a pixel offset of
// kh * (W + 2) + kw.  Only W goes through the per-step ring.  Halo pixels per
// buffer: HQ DMA instructions per wave x 4 waves x 8 pixels.
// kConvHaloS: the 64-row kind with 96-pixel buffers (14- and 7-wide layers):
// 48 KiB of LDS instead of 56, three workgroups per CU instead of two.
// NW = 8 (the 256-row kind, 4 x 2 waves): 6 pieces per wave = 384-pixel buffers.
template <int BM, int KIND, int NW>
constexpr int kHaloHQ = KIND == kConvHaloS ? 3 : NW == 8 ? 6 : BM == 64 ? 4 : 8;
template <int KIND>
constexpr bool kIsHalo = KIND == kConvHalo || KIND == kConvHaloS;
// kConvTapW (round 4): 3x3/s1/p1 tap walk with the three kw taps of a (kh, channel block)
// reading one A window.  For stride 1 and padding 1 (OH = H, OW = W) the input pixel of tap
// (kh, kw) of output row m is the global pixel m + (kh - 1) W + kw - 1, so the 64 rows of a
// tile read, for the three kw taps, the 66 consecutive pixels from m0 + (kh - 1) W - 1 on:
// one DMA'd window of BM + 8 rows (BM / 32 16-byte pieces + one 4-byte piece per wave) feeds
// 3 k-steps -- for 64-row tiles 9 KiB of A per 3 steps instead of 24 (a step's LDS ingest 16 ->
// 11 KiB; 128-row tiles 24 -> 13.7 KiB; the tap walks run at the per-CU ingest ceiling,
// DESIGN.md 3.1.5).
// Taps that fall into the padding read a real neighbour pixel of the window and are zeroed
// at fragment read by the row's tap mask.  Only W goes through the STAGES ring.
template <int BM>
constexpr int kWinRows = BM + 8;
// Dense kinds keep 2 x BM {mean, rstd} pairs past the ring for the LayerNorm fold (the tile's
// row statistics, computed once per row before the epilogue's walk).
template <int BM, int KIND>
constexpr int kLnBytes = KIND == kDense ? 2 * BM * 8 : 0;
// Window kind with NW = 8 (round 5): two K groups of 4 waves in one workgroup, each walking
// half of the slice's super-steps through its own LDS (ring + windows) and reducing through
// LDS at the end -- the intra-workgroup split-K of DESIGN.md 3.1.6.
template <int KIND, int NW>
constexpr int kKGroups = KIND == kConvTapW && NW == 8 ? 2 : 1;
// LDS bytes of one K group (the whole workgroup: kKGroups times this)
template <int BM, int BN, int STAGES, int KIND, int NW>
constexpr int kLdsBytes = kIsHalo<KIND> ? STAGES * BN * 128 + 2 * kHaloHQ<BM, KIND, NW> * NW * 8 * 128 + 16
                          : KIND == kConvTapW ? STAGES * BN * 128 + 2 * kWinRows<BM> * 128 + 16
                                              : STAGES * (BM + BN) * 128 + kLnBytes<BM, KIND> + 16;
// Occupancy asked of the register allocator: 4 / 3 / 2 waves per SIMD by tile
// size per wave (of a K group), capped by what the tile's LDS ring allows (NW / 4 waves
// per SIMD per block, 160 KiB of LDS per CU; RB = 128 bytes per row per stage in every mode).
template <int BM, int BN, int STAGES, int KIND, int NW>
constexpr int kMinWaves = std::max(
    1, std::min(BM * BN * 4 * kKGroups<KIND, NW> / NW <= 64 * 64 ? 4 : BM * BN * 4 * kKGroups<KIND, NW> / NW <= 128 * 64 ? 3 : 2,
                (160 * 1024) / (kKGroups<KIND, NW> * kLdsBytes<BM, BN, STAGES, KIND, NW>) * NW / 4));

// NW waves per workgroup in an (NW / 2) x 2 grid over the tile: wave (wm, wn)
// owns rows [wm * BM / (NW / 2), ...) x columns [wn * BN / 2, ...).
// The workgroup body: problem `a`, split-K slice `kslice`, linear tile `lin`.
// gemm_kernel passes its own arguments (constant kernarg offsets, preloadable);
// gemm_kernel_pair selects one of two problems at run time.
template <int MODE, int BM, int BN, int STAGES, int KIND, int NWA>
__device__ __forceinline__ void gemm_body(const KArgs& a, const int kslice_in, const int lin, const int hl) {
  constexpr bool CONV = KIND != kDense;
  constexpr bool TAP = KIND == kConvTap;
  constexpr bool HALO = kIsHalo<KIND>;
  constexpr bool WIN = KIND == kConvTapW;
  constexpr bool AR = !HALO && !WIN;  // A tiles go through the ring
  static_assert(!WIN || ((BM == 64 || BM == 128) && BN == 64 && STAGES == 3),
                "window kind: 64 / 128 x 64 tiles, 3 W stages");
  static_assert(NWA == 4 || NWA == 8, "4- or 8-wave workgroups");
  // KG K groups of NW waves: everything below is one group's (its waves, threads, LDS)
  constexpr int KG = kKGroups<KIND, NWA>;
  constexpr int NW = NWA / KG;
  static_assert(NW == 4 || NW == 8, "waves per K group");
  constexpr int NT = 64 * NW;  // threads per K group
  using TR = Traits<MODE>;
  using AT = typename TR::A;
  constexpr int ESTEP = TR::ESTEP, EPC = TR::EPC, RB = TR::RB;
  constexpr int CPR = RB / 16;             // chunks per image row
  constexpr int RPI = 64 / CPR;            // image rows per 1-KiB DMA instruction
  constexpr int IMG = (AR ? BM + BN : BN) * RB;  // bytes per ring stage (halo, window: W only)
  constexpr int AQ = BM / RPI / NW, BQ = BN / RPI / NW;  // DMA instructions per wave per step
  static_assert(!AR || AQ * RPI * NW == BM, "A image rows per wave");
  static_assert(BQ * RPI * NW == BN, "W image rows per wave");
  constexpr int QPS = (AR ? AQ : 0) + BQ;
  constexpr int HQ = HALO ? kHaloHQ<BM, KIND, NW> : 1;  // halo DMA instructions per wave per block
  constexpr int HBUF = HALO ? HQ * NW * RPI * RB : WIN ? kWinRows<BM> * RB : 0;  // bytes per halo / window buffer
  constexpr int XQ = BM / 32 + 1;  // window kind: DMA pieces per wave per window
  constexpr int LDSB = kLdsBytes<BM, BN, STAGES, KIND, NW>;
  static_assert(LDSB == STAGES * IMG + 2 * HBUF + kLnBytes<BM, KIND> + 16, "LDS layout");
  static_assert(!WIN || RB == 128, "window rows are 128-byte pixel blocks");
  static_assert(!HALO || (STAGES >= 3 && STAGES <= 6 && RPI == 8), "halo: 9 taps, the next halo at tap 10 - STAGES");
  __shared__ __attribute__((aligned(16))) char lds_wg[KG * LDSB];
  // K group (an SGPR) and its LDS: [0, LDSB) for group 0, [LDSB, 2 LDSB) for group 1
  const int grp = KG == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x / NT);
  char* const lds = KG == 1 ? lds_wg : lds_wg + grp * LDSB;
  int* s_flag = reinterpret_cast<int*>(lds + LDSB - 16);
  [[maybe_unused]] unsigned long long rt_e = 0, rt_l0 = 0, rt_l1 = 0, rt_p1 = 0, rt_p2 = 0;
  SPI_RT(rt_e);
#ifdef SPI_GEMM_TIMELINE
  // kind: 0 plain tile, 1 split-K slice that did not reduce, 2 the reducing slice
  auto tl_out = [&](int kind) {
    unsigned long long rt_x;
    SPI_RT(rt_x);
    if (threadIdx.x == 0 && a.tl) {
      unsigned long long* g = g_gemm_timeline + (size_t)((blockIdx.x + blockIdx.y * gridDim.x) & 65535) * 8;
      g[0] = rt_e;
      g[1] = rt_l0;
      g[2] = rt_l1;
      g[3] = rt_x;
      g[4] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
             ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
      g[5] = (unsigned long long)kind;
      g[6] = rt_p1;
      g[7] = rt_p2;
    }
  };
#else
  auto tl_out = [](int) {};
#endif

  const GemmDesc& d = a.d;
  // wave index in an SGPR: every LDS-DMA destination (M0) is then scalar math.
  const int tid = KG == 1 ? (int)threadIdx.x : (int)threadIdx.x & (NT - 1), lane = tid & 63,
            wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware remap: consecutive tiles (same weight columns) land on one XCD's L2.
  // hl: the workgroup's dispatch index inside this problem's range; the hardware deals
  // dispatch indices round-robin to the 8 XCDs, so hl & 7 names the XCD.  Number each
  // XCD's workgroups consecutively (bijective, chunks of q or q + 1).
  int tile = lin, kslice = kslice_in;
  const auto xcd_order = [](int idx, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = idx & 7, l = idx >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
  };
  if (kSplitK<BM, BN, KIND> && a.splits > 1) {
    // split-K: cut that order into tiles of `splits` consecutive slices
    const int wgid = xcd_order(hl, a.tiles * a.splits);
    tile = fdiv(wgid, a.fd_split);
    kslice = wgid - tile * a.splits;
  } else if (a.tiles >= 16) {
    tile = xcd_order(tile, a.tiles);
  }
  // Tile of linear index `tile`: the tile grid is cut into xg_m x xg_n
  // rectangles (row groups i-major), each walked with tm fastest; the chunk of
  // consecutive indices an XCD receives is then (about) one rectangle, so each
  // A row block is fetched by xg_n XCD L2s and each W column block by xg_m
  // (xg_m = 1: every XCD reads all of A -- the plain column-major order).
  int tm, tn;
  {
    const int TN = a.tiles_n;
    int mlo = 0, mhi = a.rg_m0[1];
    FastDiv fdm = a.fd_rows[0];
#pragma unroll
    for (int i = 1; i < 8; ++i)  // row group: the last whose first tile index is <= tile
      if (i < a.xg_m && a.rg_m0[i] * TN <= tile) {
        mlo = a.rg_m0[i];
        mhi = a.rg_m0[i + 1];
        fdm = a.fd_rows[i];
      }
    const int mi = mhi - mlo;
    const int l2 = tile - mlo * TN;  // index inside row group i: mi x TN tiles
    const int c = fdiv(l2, fdm);     // which tile column it falls in
    int nlo = 0;
#pragma unroll
    for (int j = 1; j < 8; ++j)
      if (j < a.xg_n && a.cg_n0[j] <= c) nlo = a.cg_n0[j];
    const int loc = l2 - mi * nlo;
    const int lq = fdiv(loc, fdm);
    tm = mlo + (loc - lq * mi);
    tn = nlo + lq;
  }
  const int n0 = tn * BN;
  SPI_RT(rt_p1);
  // m_lim: first row past this tile's valid rows.  Halo tiles map their rows to
  // output rows through the virtual-row bands (halo_m below) instead.
  int m0 = tm * BM, m_lim = d.M;
  if constexpr (!HALO) {
    if (d.pool_rows) {  // fused avgpool + FC: tile row tm = image tm's pixels
      m0 = tm * d.pool_rows;
      m_lim = m0 + d.pool_rows;
    }
  }
  // halo: first virtual output row of the band; halo_m(r) = output row of tile row
  // r (-1: a padding row of the virtual layout, or past the last image)
  const int h_u0 = HALO ? tm * a.h_th : 0;
  if constexpr (HALO) {
    if (!a.h_off) {  // aligned band: contiguous output rows [m0, m_lim) of one image
      const int img = fdiv(h_u0, a.fd_period), oy0 = h_u0 - img * a.h_period;
      m0 = (img * d.OH + oy0) * d.OW;
      m_lim = m0 + min(a.h_th, d.OH - oy0) * d.OW;
    }
  }
  [[maybe_unused]] auto halo_m = [&](int r) {
    const int ty = fdiv(r, a.fd_ow), tx = r - ty * d.OW;
    const int u = h_u0 + ty;
    const int img = fdiv(u, a.fd_period);
    const int oy = u - img * a.h_period - a.h_off;
    return (ty < a.h_th && img < a.imgs && (unsigned)oy < (unsigned)d.OH) ? (img * d.OH + oy) * d.OW + tx
                                                                                      : -1;
  };
  int kbeg = kslice * a.k_per_split;
  int kend = min(d.Kpad, kbeg + a.k_per_split);
  if constexpr (KG == 2) {
    // K groups: the first / second half of the slice's super-steps (the host plans an even
    // count per slice, so both groups run the same number of steps -- and of barriers)
    const int half = (kend - kbeg) / (6 * ESTEP) * (3 * ESTEP);
    if (grp == 0)
      kend = kbeg + half;
    else
      kbeg += half;
  }
  // halo: channel blocks [h_b0, h_b1) of this split-K slice, 9 taps each
  const int h_b0 = HALO ? kslice * a.h_bps : 0;
  const int h_b1 = HALO ? min(a.h_nblk, h_b0 + a.h_bps) : 0;
  const int nsteps = HALO ? (h_b1 - h_b0) * 9 : (kend - kbeg) / ESTEP;

  const char* zeros = static_cast<const char*>(a.p.zeros);
  const AT* __restrict__ Ap = static_cast<const AT*>(a.p.A);
  const char* __restrict__ Wb = static_cast<const char*>(a.p.W);

  // Per-lane source bookkeeping (fixed across k-steps).
  const int slot = lane & (CPR - 1);
  int a_koff[AQ], a_ih0[AQ], a_iw0[AQ];
  bool a_ok[AQ];
  const AT* a_base[AQ];
  const AT* a_pix[AQ];  // conv: image pointer at (ih0, iw0), may point before the image
  const AT* a_src[AQ];  // conv, one tap per step: a_pix + this lane's chunk offset
  // conv, one tap per step: bit (kh*KW + kw) set when that tap of this row lies
  // inside the image (0 for rows past M).  Indexed by the unrolled q only.
  uint32_t a_mask[AQ];
#pragma unroll
  for (int q = 0; q < (AR ? AQ : 0); ++q) {
    const int r = (wave * AQ + q) * RPI + lane / CPR;
    a_koff[q] = (slot ^ (r & (CPR - 1))) * EPC;
    const int m = m0 + r;
    a_ok[q] = m < d.M;
    const int mm = a_ok[q] ? m : 0;
    if constexpr (CONV) {
      const int img = fdiv(mm, a.fd_ohw);
      const int rem = mm - img * (d.OH * d.OW);
      const int oh = fdiv(rem, a.fd_ow);
      const int ow = rem - oh * d.OW;
      a_ih0[q] = oh * d.stride - d.pad;
      a_iw0[q] = ow * d.stride - d.pad;
      a_base[q] = Ap + (size_t)img * d.H * d.W * d.Cin;
      a_pix[q] = a_base[q] + ((ptrdiff_t)(a_ih0[q] * d.W + a_iw0[q]) << a.cin_shift);
      a_src[q] = a_pix[q] + a_koff[q];
      // valid taps: kh in [kh_lo, kh_hi) x kw in [kw_lo, kw_hi) -- one row of column bits
      // replicated per valid filter row (no per-tap compares)
      uint32_t mask = 0u;
      if (TAP && a_ok[q]) {
        const int kh_lo = max(0, -a_ih0[q]), kh_hi = min(d.KH, d.H - a_ih0[q]);
        const int kw_lo = max(0, -a_iw0[q]), kw_hi = min(d.KW, d.W - a_iw0[q]);
        const uint32_t cols = kw_hi > kw_lo ? (1u << kw_hi) - (1u << kw_lo) : 0u;
        for (int kh = kh_lo; kh < kh_hi; ++kh) mask |= cols << (kh * d.KW);
      }
      a_mask[q] = mask;
    } else {
      a_ih0[q] = a_iw0[q] = 0;
      a_base[q] = Ap + (size_t)mm * d.lda;
      a_pix[q] = a_base[q];
      a_src[q] = a_pix[q];
      a_mask[q] = 0u;
    }
  }
  const char* b_src[BQ];
#pragma unroll
  for (int q = 0; q < BQ; ++q) {
    const int r = (wave * BQ + q) * RPI + lane / CPR;
    const int c = slot ^ (r & (CPR - 1));
    // W rows are Kpad elements (F16/F32) or 2*Kpad fp16 (F16X3, 64-element blocks of hi|lo).
    const size_t row_bytes = (MODE == (int)Prec::F16) ? (size_t)d.Kpad * 2 : (size_t)d.Kpad * 4;
    b_src[q] = Wb + (size_t)(n0 + r) * row_bytes + c * 16;
  }

  // Halo bookkeeping.  DMA side: lane of instruction wave*HQ + q fills pixel p
  // (8 per instruction), slot s <- chunk s ^ (p & 7); h_src is its source for
  // channel block 0 (block b adds b * ESTEP elements), zeros when p lies in the
  // padding or past the halo.  Fragment side: h_row[i] = halo pixel of tap (0, 0)
  // for this lane's row of A fragment i (rows past the band read pixel 0; their
  // results are never stored).
  // Virtual input rows: aligned bands read rows of their own image only (row
  // oy0 - 1 + hy); stacked bands read virtual row u0 - 1 + hy, i.e. image
  // (u0 - 1 + hy) / period, row (u0 - 1 + hy) % period - 1 (the padding rows of the
  // stacked layout and rows past the last image read zeros).
  constexpr int WTM_ = BM / (NW / 2);  // rows per wave
  [[maybe_unused]] const AT* h_src[HQ];
  [[maybe_unused]] bool h_ok[HQ];
  [[maybe_unused]] int h_row[WTM_ / 16];
  if constexpr (HALO) {
    const int imgs = a.imgs;
#pragma unroll
    for (int q = 0; q < HQ; ++q) {
      const int p = (wave * HQ + q) * RPI + lane / CPR;
      const int c = slot ^ (p & (CPR - 1));
      const int hy = fdiv(p, a.fd_hwp), hx = p - hy * a.h_hwp;
      int img, iy;
      if (a.h_off) {
        const int vy = h_u0 - 1 + hy;
        img = vy < 0 ? imgs : fdiv(vy, a.fd_period);
        iy = vy - img * a.h_period - 1;
      } else {
        img = fdiv(h_u0, a.fd_period);
        iy = h_u0 - img * a.h_period - 1 + hy;
      }
      const int ix = hx - 1;
      h_ok[q] = p < a.h_hp && img < imgs && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
      h_src[q] = Ap + ((size_t)((h_ok[q] ? img : 0) * d.H + (h_ok[q] ? iy : 0)) * d.W + (h_ok[q] ? ix : 0)) * d.Cin +
                 c * EPC;
    }
#pragma unroll
    for (int i = 0; i < WTM_ / 16; ++i) {
      const int r = (wave >> 1) * WTM_ + i * 16 + (lane & 15);
      const int ty = fdiv(r, a.fd_ow), tx = r - ty * d.OW;
      h_row[i] = ty < a.h_th ? ty * a.h_hwp + tx : 0;
    }
  }
  auto issue_halo = [&](int blk, int buf) {
    if constexpr (HALO) {
      char* dst = lds + STAGES * IMG + buf * HBUF;
#pragma unroll
      for (int q = 0; q < HQ; ++q) {
        const char* src = h_ok[q] ? reinterpret_cast<const char*>(h_src[q] + (size_t)blk * ESTEP) : zeros;
        SPI_DMA_A((const void*)SPI_A_SRC(src), (lds_ptr_t)(dst + (wave * HQ + q) * 1024), 16, 0, 0);
      }
    }
  };
  // Window kind: super-step j of the slice is global super-step w_g0 + j = (kh, channel block
  // cb), kh-major (g = kh * nblk + cb); its k-step 3 j + kw reads W k-step (kh * 3 + kw) *
  // nblk + cb (k = tap * Cin + c).  DMA side of a window: pieces q < BM / 32 of wave w (16
  // bytes a lane) fill rows (BM / 4) w + 8 q + lane / 8, slot lane & 7; the last piece (4 bytes
  // a lane) rows BM + 2 w + lane / 32, slot (lane & 31) / 4 -- w_off: the source byte offset in
  // the pixel's 128-byte block (chunk slot ^ (row & 7), the ring images' swizzle).
  [[maybe_unused]] const int w_g0 = WIN ? kbeg / (3 * ESTEP) : 0;
  [[maybe_unused]] const int w_nbs = WIN ? a.win_nblk_shift : 0;
  [[maybe_unused]] int w_row[XQ], w_off[XQ];
  if constexpr (WIN) {
#pragma unroll
    for (int q = 0; q < XQ - 1; ++q) {
      const int r = wave * (BM / 4) + q * 8 + (lane >> 3);
      w_row[q] = r;
      w_off[q] = ((lane & 7) ^ (r & 7)) << 4;
    }
    const int r = BM + wave * 2 + (lane >> 5);
    w_row[XQ - 1] = r;
    w_off[XQ - 1] = ((((lane & 31) >> 2) ^ (r & 7)) << 4) + ((lane & 3) << 2);
  }
  auto issue_win = [&](int jj, int buf) {
    if constexpr (WIN) {
      constexpr int PSH = __builtin_ctz(sizeof(AT));
      const int g = w_g0 + jj, kh = g >> w_nbs, cb = g & ((1 << w_nbs) - 1);
      const int p0 = m0 + (kh - 1) * d.W - 1;  // global pixel of window row 0
      const char* base = reinterpret_cast<const char*>(Ap) + cb * RB;
      char* dst = lds + STAGES * IMG + buf * HBUF;
#pragma unroll
      for (int q = 0; q < XQ; ++q) {
        const int pix = p0 + w_row[q];
        const char* src = (unsigned)pix < (unsigned)d.M ? base + ((size_t)pix << (a.cin_shift + PSH)) + w_off[q] : zeros;
        if (q < XQ - 1)
          glds16(SPI_A_SRC(src), dst + (wave * (XQ - 1) + q) * 1024);
        else
          glds4(SPI_A_SRC(src), dst + BM * RB + wave * 256);
      }
    }
  };
  [[maybe_unused]] int w_tap0 = 0, w_j = 0;  // the running super-step's kh * 3 and index

  // halo: scalar (block, tap) walk of the issued W steps; k = tap * Cin + c, so
  // step (blk, tap) is W k-step tap * nblk + blk
  int hw_blk = h_b0, hw_tap = 0;
  int hw_blk_next = 0, hw_buf_next = 0;  // the halo issued at tap 7 of the current block

  // Cin >= k-step (one (kh, kw) tap per step): a scalar walk over (tap, channel
  // block), advanced once per issued step (issue() is called for steps 0, 1, 2 ...
  // in order): cu_cell = tap index, cu_off = element offset of (kh, kw, channel)
  // from the row's (ih0, iw0) pixel.  Taps past KH*KW (the Kpad tail) have no
  // mask bit, so they read zeros.
  int cu_cell = 0, cu_kw = 0, cu_ci = 0, cu_off = 0;
  if constexpr (TAP) {
    {
      const int kbeg_a = d.krep == 2 ? kbeg >> 1 : kbeg;  // A k of the slice's first step (slices hold whole krep groups)
      cu_cell = kbeg_a >> a.cin_shift;
      const int kh = (cu_cell * a.kw_mul) >> 16;
      cu_kw = cu_cell - kh * d.KW;
      cu_ci = kbeg_a & (d.Cin - 1);
      cu_off = ((kh * d.W + cu_kw) << a.cin_shift) + cu_ci;
    }
  }
  int w_kb = (kbeg / ESTEP) * RB;  // W byte offset of the next issued step
  auto issue = [&](int step, int stage) {
    const int k0 = kbeg + step * ESTEP;
    char* dst = lds + stage * IMG;
    if constexpr (HALO) {
      const int wstep = hw_tap * a.h_nblk + hw_blk;
#pragma unroll
      for (int q = 0; q < BQ; ++q)
        SPI_DMA_W((const void*)(b_src[q] + (size_t)wstep * RB), (lds_ptr_t)(dst + (wave * BQ + q) * 1024), 16, 0, 0);
      if (++hw_tap == 9) {
        hw_tap = 0;
        ++hw_blk;
      }
      return;
    } else if constexpr (WIN) {
      const int jj = step / 3, kw = step - jj * 3;
      const int g = w_g0 + jj, kh = g >> w_nbs, cb = g & ((1 << w_nbs) - 1);
      const int wstep = ((kh * 3 + kw) << w_nbs) + cb;
#pragma unroll
      for (int q = 0; q < BQ; ++q)
        SPI_DMA_W((const void*)(b_src[q] + (size_t)wstep * RB), (lds_ptr_t)(dst + (wave * BQ + q) * 1024), 16, 0, 0);
      return;
    } else if constexpr (CONV) {
      if constexpr (TAP) {
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
          const bool ok = (a_mask[q] >> cu_cell) & 1u;
          const char* src = ok ? reinterpret_cast<const char*>(a_src[q] + cu_off) : zeros;
          SPI_DMA_A((const void*)SPI_A_SRC(src), (lds_ptr_t)(dst + (wave * AQ + q) * 1024), 16, 0, 0);
        }
        // advance one k-step: next channel block, or the next tap (next pixel,
        // or the next filter row: W - KW + 1 pixels on); krep = 2: after the
        // second (lo-weight) step of the pair only
        if (d.krep == 1 || (step & 1)) {
          cu_ci += ESTEP;
          cu_off += ESTEP;
          if (cu_ci == d.Cin) {
            cu_ci = 0;
            ++cu_cell;
            if (++cu_kw == d.KW) {
              cu_kw = 0;
              cu_off += (d.W - d.KW) << a.cin_shift;
            }
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
          const char* src = zeros;
          const int k = k0 + a_koff[q];
          if (a_ok[q] && k < d.K) {
            const int cell = k >> a.cin_shift;
            const int c = k & (d.Cin - 1);
            const int kh = (cell * a.kw_mul) >> 16;
            const int kw = cell - kh * d.KW;
            const int ih = a_ih0[q] + kh, iw = a_iw0[q] + kw;
            if ((unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W)
              src = reinterpret_cast<const char*>(a_base[q] + ((size_t)(ih * d.W + iw) << a.cin_shift) + c);
          }
#ifndef SPI_DIAG_NO_DMA_GEN  // diagnostic build: general convs (the stem) issue no DMA
          SPI_DMA_A((const void*)SPI_A_SRC(src), (lds_ptr_t)(dst + (wave * AQ + q) * 1024), 16, 0, 0);
#endif
        }
      }
    } else {
      // krep = 2: packed steps 2s and 2s + 1 both stage A step s
      const int ka0 = d.krep == 2 ? (k0 / (2 * ESTEP)) * ESTEP : k0;
#pragma unroll
      for (int q = 0; q < AQ; ++q) {
        const int k = ka0 + a_koff[q];
        const char* src = (a_ok[q] && k < d.K) ? reinterpret_cast<const char*>(a_pix[q] + k) : zeros;
        SPI_DMA_A((const void*)SPI_A_SRC(src), (lds_ptr_t)(dst + (wave * AQ + q) * 1024), 16, 0, 0);
      }
    }
    // k-step byte offset inside a W row: RB bytes per step (advanced per issue).
#ifdef SPI_DIAG_NO_DMA_GEN
    if constexpr (KIND != kConvGen)
#endif
#pragma unroll
    for (int q = 0; q < BQ; ++q)
      SPI_DMA_W((const void*)(b_src[q] + w_kb), (lds_ptr_t)(dst + BM * RB + (wave * BQ + q) * 1024), 16, 0, 0);
    w_kb += RB;
  };

  const int fr = lane & 15, fq = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  constexpr int WTM = BM / (NW / 2), WTN = BN / 2;
  constexpr int TI = WTM / 16, TJ = WTN / 16;
  floatx4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // window kind: taps (bit kh * 3 + kw) inside the image for this lane's A fragment rows
  [[maybe_unused]] uint32_t w_mask[TI];
  if constexpr (WIN) {
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int m = m0 + wm * WTM + i * 16 + fr;
      uint32_t mask = 0u;
      if (m < d.M) {
        const int img = fdiv(m, a.fd_ohw), rem = m - img * (d.OH * d.OW);
        const int oh = fdiv(rem, a.fd_ow), ow = rem - oh * d.OW;
        const uint32_t cols = (ow > 0 ? 1u : 0u) | 2u | (ow + 1 < d.W ? 4u : 0u);
        mask = (oh > 0 ? cols : 0u) | (cols << 3) | (oh + 1 < d.H ? cols << 6 : 0u);
      }
      w_mask[i] = mask;
    }
  }

  // Residual tile prefetch (64 x 64 tiles on the vector epilogue path): the epilogue's
  // residual loads were the last dependent memory round trip of a launch (~0.5-1 us of a
  // ~1.2 us epilogue, tools/gemm_timeline.py).  The tile's residual rows go into LDS by
  // LDS-DMA at the first k-step that stages no further k-step (step nsteps - STAGES + 1),
  // into the stage region the step before it used (nsteps % STAGES); the epilogue parks its
  // fp32 tile in the last step's region ((nsteps - 1) % STAGES), so the two never meet.
  // Split-K tiles prefetch in the reducing slice only, after its ticket.  res_rb: bytes of a
  // residual tile row (64 fp16 = 128, 64 fp32 or split = 256); rpw: DMA pieces per wave.
  constexpr bool RPF = BM == 64 && BN == 64 && !HALO && NW == 4;
  // the LayerNorm fold lives in the dense fp16 instances only (the transformer GEMMs)
  constexpr bool LNF = KIND == kDense && MODE == (int)Prec::F16;
  // (residual planes: a row's 64 hi values, then its 64 lo values)
  [[maybe_unused]] const int res_rb =
      (MODE == kF16X3S || sizeof(typename TR::Out) == 4 || d.res_f32 || d.res_planes) ? 256 : 128;
  [[maybe_unused]] const int rpw = res_rb * BM / 1024 / NW;  // 2 or 4
  [[maybe_unused]] const bool rpf_tile = RPF && a.p.res && a.vec_ok && n0 + BN <= d.N && !d.pool_rows;
  // (window kind: into the window buffer the last super-step does not use -- 9 KiB, so fp16
  // residual rows only -- and the tile parks at 0)
  [[maybe_unused]] const bool rpf_loop = rpf_tile && a.splits == 1 && (!WIN || res_rb == 128) && grp == 0;
  [[maybe_unused]] const int rpf_step = max(0, nsteps - STAGES + 1);
  [[maybe_unused]] const int rpf_off = WIN ? STAGES * IMG + ((nsteps / 3) & 1) * HBUF : (nsteps % STAGES) * IMG;
  [[maybe_unused]] const int park_off = WIN ? 0 : ((nsteps - 1) % STAGES) * IMG;
  auto issue_res = [&](char* dst) {
    if constexpr (RPF) {
      const int rpp = 1024 / res_rb, cpr = res_rb / 16;  // rows per piece, 16-byte chunks per row
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q < rpw) {  // wave-uniform
          const int piece = wave * rpw + q;
          const int row = piece * rpp + lane / cpr, ch = lane % cpr;
          const int m = m0 + row;
          const char* src = zeros;
          if (m < m_lim) {
            if constexpr (MODE == kF16X3S)
              src = reinterpret_cast<const char*>(static_cast<const _Float16*>(a.p.res) + split_idx(m, n0, d.ldr)) + ch * 16;
            else if (d.res_planes)
              src = reinterpret_cast<const char*>(static_cast<const _Float16*>(a.p.res) + (size_t)m * d.ldr + n0 +
                                                  (ch >= 8 ? d.plane : 0)) + (ch & 7) * 16;
            else
              src = static_cast<const char*>(a.p.res) + ((size_t)m * d.ldr + n0) * (res_rb / 64) + ch * 16;
          }
          glds16(src, dst + piece * 1024);
        }
      }
    }
  };

  SPI_RT(rt_p2);
  if constexpr (HALO) issue_halo(h_b0, 0);  // lands before W step 0 (in-order vmcnt)
  if constexpr (WIN) issue_win(0, 0);
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nsteps) issue(s, s);

  // Epilogue through LDS (the K loop's ring is free by then; cdna_hip_programming.md
  // T21, store-issue-bound tails).  The waves park their raw accumulators as an fp32
  // [BM][BN] tile -- 16-column blocks XOR-swizzled by (row >> 2) & 3, so the
  // ds_write_b32 of a fragment (4 row groups x 16 columns) hits 64 distinct banks --
  // then every thread owns one 8-column group and walks rows, moving bias, residual
  // and output as 16-byte vectors (global_load/store_dwordx4) instead of the 2-4 byte
  // per-element accesses of the fragment layout (a 128x64 split tile: 16 vector
  // accesses per thread instead of 128 scalar ones).  All residual loads of a thread
  // go out before its first store (clamped rows: always-valid addresses, no branch).
  // Tiles crossing N, or unaligned strides, take the per-element path from LDS.
  // toff: byte offset of the parked tile in LDS; rl: the prefetched residual tile (issue_res)
  // or nullptr (the residual, if any, is read from global memory).
  auto finish = [&](floatx4 (&v)[TI][TJ], int toff, const char* rl) {
    using Out = typename TR::Out;
    static_assert(BM * BN * 4 <= LDSB - 16, "the C tile must fit the LDS");
    float* T = reinterpret_cast<float*>(lds + toff);
    // the bias row of this thread's column group, in flight across the park
    const int nb_ = n0 + (tid % (BN / 8)) * 8;
    floatx4 bv0 = floatx4{0.f, 0.f, 0.f, 0.f}, bv1 = bv0;
    if (a.vec_ok && n0 + BN <= d.N && a.p.bias) {
      bv0 = *reinterpret_cast<const floatx4*>(a.p.bias + nb_);
      bv1 = *reinterpret_cast<const floatx4*>(a.p.bias + nb_ + 4);
    }
    // LayerNorm fold: the tile rows' {mean, rstd} once per row into LDS past the ring ([0, BM):
    // the A rows' (consumer), [BM, 2 BM): the residual rows' (res_ln)); read after the park's barrier
    [[maybe_unused]] float2* const ln_s = reinterpret_cast<float2*>(lds + STAGES * IMG + 2 * HBUF);
    if constexpr (LNF) {
      if (d.ln_in_chunks > 0)
        ln_tile_stats(a.p.ln.in_stats, m0, BM, d.M, d.ln_in_chunks, d.ln_in_eps, ln_s, tid, NT);
      if (d.res_ln_chunks > 0)
        ln_tile_stats(a.p.ln.res_stats, m0, BM, d.M, d.res_ln_chunks, d.res_ln_eps, ln_s + BM, tid, NT);
    }
    __syncthreads();  // every wave is done reading the ring
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WTM + i * 16 + fq * 4 + r;
          const int col = (wn * WTN + j * 16 + fr) ^ (fq << 4);  // (row >> 2) & 3 == fq
          T[row * BN + col] = v[i][j][r];
        }
    if (rl) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's residual pieces
    __syncthreads();
    if constexpr (!HALO && BM * BN * 4 + 256 * 4 <= LDSB - 16) {
      if (d.pool_rows) {
        // fused avgpool + FC: column means of the tile's pool_rows valid rows,
        // four row-interleaved partial sums per column, combined through LDS
        constexpr int PARTS = NT / BN;
        float* red = T + BM * BN;
        const int col = tid % BN, part = tid / BN;
        float sum = 0.f;
        for (int r = part; r < d.pool_rows; r += PARTS) sum += T[r * BN + (col ^ (((r >> 2) & 3) << 4))];
        red[part * BN + col] = sum;
        __syncthreads();
        if (tid < BN) {
          float tot = 0.f;
#pragma unroll
          for (int q = 0; q < PARTS; ++q) tot += red[q * BN + tid];
          const int n = n0 + tid;
          if (n < d.N) {
            const float y = apply_act(tot / (float)d.pool_rows + (a.p.bias ? a.p.bias[n] : 0.f), d.act);
            if (d.out_f32 || sizeof(typename TR::Out) == 4)
              static_cast<float*>(a.p.C)[(size_t)tm * d.ldc + n] = y;
            else
              static_cast<_Float16*>(a.p.C)[(size_t)tm * d.ldc + n] = static_cast<_Float16>(y);
          }
        }
        return;
      }
    }
    constexpr int G = BN / 8, RSTEP = NT / G, ITEMS = BM / RSTEP;
    const int cg = tid % G, r0 = tid / G;
    const int nb = n0 + cg * 8;
    // 0 fp16, 1 fp32, 2 split layout, 3 two fp16 planes
    const int fmt = (kSplitMode<MODE> && d.out_split) ? 2 : d.out_planes ? 3 : d.out_f16 ? 0
                    : (d.out_f32 || sizeof(Out) == 4) ? 1 : 0;
    // output row of tile row `row`, -1 when it is not stored
    auto row_m = [&](int row) -> int {
      if constexpr (HALO) {
        if (a.h_off) return halo_m(row);
      }
      const int m = m0 + row;
      return m < m_lim ? m : -1;
    };
    auto tile_vals = [&](int row, float (&y)[8]) {
      const float* src = T + row * BN + ((cg * 8) ^ (((row >> 2) & 3) << 4));
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(src);
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(src + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] = x0[e];
        y[e + 4] = x1[e];
      }
    };
    auto finish_act = [&](auto& y) {
      constexpr int NI = sizeof(y) / sizeof(y[0]);
      auto apply = [&](auto act_tag) {
        constexpr Act act = decltype(act_tag)::value;
#pragma unroll
        for (int it = 0; it < NI; ++it)
#pragma unroll
          for (int e = 0; e < 8; ++e) y[it][e] = apply_act(y[it][e], act);
      };
      if (d.act == Act::Relu) {
        apply(std::integral_constant<Act, Act::Relu>{});
      } else if (d.act == Act::Gelu && fmt == 0) {
        // fp16 output: the packed degree-7/6 GELU (device_math.hpp gelu2, |erf error| 2.5e-6, 80x
        // under an fp16 half-ulp) at half the VALU of the scalar 13/8 form; fp32 / split outputs
        // keep the 4.5e-7 form (fp32 parity bar)
#pragma unroll
        for (int it = 0; it < NI; ++it)
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const float2v g2 = gelu2(float2v{y[it][e], y[it][e + 1]});
            y[it][e] = g2.x;
            y[it][e + 1] = g2.y;
          }
      } else if (d.act == Act::Gelu) {
        apply(std::integral_constant<Act, Act::Gelu>{});
      } else {
        apply(std::integral_constant<Act, Act::None>{});
      }
    };
    float b[8];
    if (a.vec_ok && n0 + BN <= d.N) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        b[e] = bv0[e];
        b[e + 4] = bv1[e];
      }
      // LayerNorm fold vectors of this thread's 8 columns: c1 (consumer), gain / bias of the
      // residual's LayerNorm (res_ln)
      [[maybe_unused]] float lnc1[8], lng[8], lnb[8];
      if constexpr (LNF) {
        const auto ld8 = [&](const float* v, float (&o)[8]) {
          const floatx4 x0 = *reinterpret_cast<const floatx4*>(v + nb);
          const floatx4 x1 = *reinterpret_cast<const floatx4*>(v + nb + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = x0[e];
            o[e + 4] = x1[e];
          }
        };
        if (d.ln_in_chunks > 0) ld8(a.p.ln.c1, lnc1);
        if (d.res_ln_chunks > 0) {
          ld8(a.p.ln.res_g, lng);
          ld8(a.p.ln.res_b, lnb);
        }
      }
      // rows in chunks of <= 4 per thread: the residual loads of a chunk are all in
      // flight before its first store, within a bounded register budget
      constexpr int CH = ITEMS < 4 ? ITEMS : 4;
#pragma unroll
      for (int c0 = 0; c0 < ITEMS; c0 += CH) {
        float y[CH][8];
#pragma unroll
        for (int it = 0; it < CH; ++it) {
#pragma unroll
          for (int e = 0; e < 8; ++e) y[it][e] = 0.f;
        }
        if (RPF && rl) {
          // the residual tile from LDS ([row][res_rb] as issue_res laid it out)
#pragma unroll
          for (int it = 0; it < CH; ++it) {
            const char* rr = rl + (r0 + (c0 + it) * RSTEP) * res_rb;
            if constexpr (MODE == kF16X3S) {
              const char* q = rr + (cg >> 2) * 128 + (cg & 3) * 16;
              const half8 hi = *reinterpret_cast<const half8*>(q);
              const half8 lo = *reinterpret_cast<const half8*>(q + 64);
#pragma unroll
              for (int e = 0; e < 8; ++e) y[it][e] = static_cast<float>(hi[e]) + static_cast<float>(lo[e]);
            } else if (d.res_planes) {
              const half8 hi = *reinterpret_cast<const half8*>(rr + cg * 16);
              const half8 lo = *reinterpret_cast<const half8*>(rr + 128 + cg * 16);
#pragma unroll
              for (int e = 0; e < 8; ++e) y[it][e] = static_cast<float>(hi[e]) + static_cast<float>(lo[e]);
            } else if (d.res_f32 || sizeof(Out) == 4) {
              const floatx4 r0v = *reinterpret_cast<const floatx4*>(rr + cg * 32);
              const floatx4 r1v = *reinterpret_cast<const floatx4*>(rr + cg * 32 + 16);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                y[it][e] = r0v[e];
                y[it][e + 4] = r1v[e];
              }
            } else {
              const half8 r = *reinterpret_cast<const half8*>(rr + cg * 16);
#pragma unroll
              for (int e = 0; e < 8; ++e) y[it][e] = static_cast<float>(r[e]);
            }
          }
        } else if (a.p.res) {
#pragma unroll
          for (int it = 0; it < CH; ++it) {
            const int mr = row_m(r0 + (c0 + it) * RSTEP);
            const int m = mr < 0 ? 0 : mr;  // skipped rows load row 0 (always valid)
            if constexpr (MODE == kF16X3S) {
              const _Float16* R = static_cast<const _Float16*>(a.p.res) + split_idx(m, nb, d.ldr);
              const half8 hi = *reinterpret_cast<const half8*>(R);
              const half8 lo = *reinterpret_cast<const half8*>(R + 32);
#pragma unroll
              for (int e = 0; e < 8; ++e) y[it][e] = static_cast<float>(hi[e]) + static_cast<float>(lo[e]);
            } else if (d.res_planes) {
              const _Float16* R = static_cast<const _Float16*>(a.p.res) + (size_t)m * d.ldr + nb;
              const half8 hi = *reinterpret_cast<const half8*>(R);
              const half8 lo = *reinterpret_cast<const half8*>(R + d.plane);
#pragma unroll
              for (int e = 0; e < 8; ++e) y[it][e] = static_cast<float>(hi[e]) + static_cast<float>(lo[e]);
            } else if (d.res_f32 || sizeof(Out) == 4) {
              const float* R = static_cast<const float*>(a.p.res) + (size_t)m * d.ldr + nb;
              const floatx4 r0v = *reinterpret_cast<const floatx4*>(R);
              const floatx4 r1v = *reinterpret_cast<const floatx4*>(R + 4);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                y[it][e] = r0v[e];
                y[it][e + 4] = r1v[e];
              }
            } else {
              const half8 r = *reinterpret_cast<const half8*>(static_cast<const _Float16*>(a.p.res) +
                                                              (size_t)m * d.ldr + nb);
#pragma unroll
              for (int e = 0; e < 8; ++e) y[it][e] = static_cast<float>(r[e]);
            }
          }
        }
        if constexpr (LNF) {
          // LayerNorm fold (ln_fold.hpp): the residual as LN(R) of the fp32 rows R loaded above
          if (d.res_ln_chunks > 0) {
#pragma unroll
            for (int it = 0; it < CH; ++it) {
              const float2 st = ln_s[BM + r0 + (c0 + it) * RSTEP];
#pragma unroll
              for (int e = 0; e < 8; ++e) y[it][e] = (y[it][e] - st.x) * st.y * lng[e] + lnb[e];
            }
          }
        }
#pragma unroll
        for (int it = 0; it < CH; ++it) {
          float t[8];
          tile_vals(r0 + (c0 + it) * RSTEP, t);
          if constexpr (LNF) {
            if (d.ln_in_chunks > 0) {  // consumer: y = rstd (acc - mean c1) + bias
              const float2 st = ln_s[r0 + (c0 + it) * RSTEP];
#pragma unroll
              for (int e = 0; e < 8; ++e) t[e] = st.y * (t[e] - st.x * lnc1[e]);
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) y[it][e] = t[e] + b[e] + y[it][e];  // acc + bias + residual
        }
        finish_act(y);
        if constexpr (LNF) {
          if (d.ln_out) {  // producer: chunk statistics + the fp16 copy of every output row
#pragma unroll
            for (int it = 0; it < CH; ++it) {
              const int m = row_m(r0 + (c0 + it) * RSTEP);
              float mean, m2;
              ln_chunk_stats(y[it], mean, m2);  // lanes of one row: consecutive cg
              if (m < 0) continue;
              if ((cg & 7) == 0)
                reinterpret_cast<float2*>(a.p.ln.out_stats)[(size_t)m * (d.N >> 6) + (nb >> 6)] = float2{mean, m2};
              if (a.p.ln.c16) {  // (two-plane outputs: the hi plane is the copy)
                half8 h;
#pragma unroll
                for (int e = 0; e < 8; ++e) h[e] = static_cast<_Float16>(y[it][e]);
                *reinterpret_cast<half8*>(a.p.ln.c16 + (size_t)m * d.ld16 + nb) = h;
              }
            }
          }
        }
#pragma unroll
        for (int it = 0; it < CH; ++it) {
          const int m = row_m(r0 + (c0 + it) * RSTEP);
          if (m < 0) continue;
          if (fmt == 2) {
            half8 hi, lo;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              hi[e] = static_cast<_Float16>(y[it][e]);
              lo[e] = static_cast<_Float16>(y[it][e] - static_cast<float>(hi[e]));
            }
            _Float16* C = static_cast<_Float16*>(a.p.C) + split_idx(m, nb, d.ldc);
            *reinterpret_cast<half8*>(C) = hi;
            *reinterpret_cast<half8*>(C + 32) = lo;
          } else if (fmt == 3) {
            half8 hi, lo;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              hi[e] = static_cast<_Float16>(y[it][e]);
              lo[e] = static_cast<_Float16>(y[it][e] - static_cast<float>(hi[e]));
            }
            _Float16* C = static_cast<_Float16*>(a.p.C) + (size_t)m * d.ldc + nb;
            *reinterpret_cast<half8*>(C) = hi;
            *reinterpret_cast<half8*>(C + d.plane) = lo;
          } else if (fmt == 1) {
            float* C = static_cast<float*>(a.p.C) + (size_t)m * d.ldc + nb;
            *reinterpret_cast<floatx4*>(C) = floatx4{y[it][0], y[it][1], y[it][2], y[it][3]};
            *reinterpret_cast<floatx4*>(C + 4) = floatx4{y[it][4], y[it][5], y[it][6], y[it][7]};
          } else {
            half8 h;
#pragma unroll
            for (int e = 0; e < 8; ++e) h[e] = static_cast<_Float16>(y[it][e]);
            *reinterpret_cast<half8*>(static_cast<_Float16*>(a.p.C) + (size_t)m * d.ldc + nb) = h;
          }
        }
      }
      return;
    }
    // per-element path (tiles crossing N, unaligned strides)
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = (a.p.bias && nb + e < d.N) ? a.p.bias[nb + e] : 0.f;
    for (int it = 0; it < ITEMS; ++it) {
      const int row = r0 + it * RSTEP, m = row_m(row);
      if (m < 0) continue;
      float y[8];
      tile_vals(row, y);
      for (int e = 0; e < 8; ++e) {
        const float r = (a.p.res && nb + e < d.N) ? load_res<MODE>(a, m, nb + e) : 0.f;
        y[e] = apply_act(y[e] + b[e] + r, d.act);
      }
      for (int e = 0; e < 8; ++e) {
        const int n = nb + e;
        if (n >= d.N) break;
        const float val = y[e];
        if (fmt == 2) {
          _Float16* C = static_cast<_Float16*>(a.p.C);
          const size_t k = split_idx(m, n, d.ldc);
          const _Float16 hi = static_cast<_Float16>(val);
          C[k] = hi;
          C[k + 32] = static_cast<_Float16>(val - static_cast<float>(hi));
        } else if (fmt == 3) {
          _Float16* C = static_cast<_Float16*>(a.p.C);
          const size_t k = (size_t)m * d.ldc + n;
          const _Float16 hi = static_cast<_Float16>(val);
          C[k] = hi;
          C[k + d.plane] = static_cast<_Float16>(val - static_cast<float>(hi));
        } else if (fmt == 1) {
          static_cast<float*>(a.p.C)[(size_t)m * d.ldc + n] = val;
        } else {
          static_cast<_Float16*>(a.p.C)[(size_t)m * d.ldc + n] = static_cast<_Float16>(val);
        }
      }
    }
  };

  [[maybe_unused]] unsigned long long st_t0 = 0, st_a = 0, st_b = 0, st_c = 0, st_d = 0, st_wait = 0, st_issue = 0, st_comp = 0;
  SPI_STAMP(st_t0);
  SPI_RT(rt_l0);
  // One k-step; U = t % STAGES is a compile-time constant (the loop below is
  // unrolled by STAGES), so every stage offset -- M0 of the DMAs, the base of
  // the fragment reads -- is an immediate.
  // Halo steps also take the tap (a constant), whether this is the slice's last
  // channel block, and that block's halo buffer.
  // steady_c (std::true_type): a step that issues step t + STAGES - 1, waits for the full ring
  // and is not at or after the residual prefetch -- no per-step checks at all (the loops below
  // run every step that far from the slice's end this way; round 4 had them checked per step,
  // ~55 SALU + 7 branches per step that made the ingest-bound loops 30 % slower)
  auto kstep = [&](int t, auto u_arg, auto tap_arg, bool last_blk, const char* Hs, auto steady_c) {
    const int U = u_arg;  // a constant when u_arg is a std::integral_constant
    constexpr int TP = decltype(tap_arg)::value;
    constexpr bool STEADY = decltype(steady_c)::value;
    SPI_STAMP(st_a);
    // Step t has landed once at most (issued steps after t) DMA groups remain.
    // Halo: W step t + 1 is in flight, and at tap 8 of a block that has a
    // successor the next block's halo too (issued at tap 7, before W step t + 2);
    // the last step of the slice waits for everything.
    if constexpr (HALO) {
      // G W groups in flight behind step t (fewer near the slice's end); the next
      // block's halo goes out at tap 10 - STAGES (before W step t + STAGES - 1 =
      // that block's tap 0), so the waits of the taps after it allow it too
      constexpr int G = STAGES - 2;
      constexpr int GL = G < 8 - TP ? G : 8 - TP;
      constexpr bool XH = TP >= 11 - STAGES;
      if (last_blk)
        dma_wait_barrier<GL * BQ>();
      else if (XH)
        dma_wait_barrier<G * BQ + HQ>();
      else
        dma_wait_barrier<G * BQ>();
    } else if constexpr (WIN) {
      // issue order: window j, ..., W(3j + 2) and window j + 1 at step 3j, W(3j + 3) at 3j + 1,
      // W(3j + 4) at 3j + 2.  Step 3j needs window j and W(3j) (W(3j + 1) in flight), 3j + 1
      // needs W(3j + 1) (W(3j + 2) and window j + 1 in flight), 3j + 2 needs W(3j + 2)
      // (window j + 1 and W(3j + 3)); last_blk: no super-step follows.  The residual
      // prefetch (issued at step 3j + 1 of the last super-step) stays in flight at 3j + 2.
      if constexpr (TP == 0) {
        dma_wait_barrier<BQ>();
      } else if constexpr (TP == 1) {
        if (last_blk)
          dma_wait_barrier<BQ>();
        else
          dma_wait_barrier<BQ + XQ>();
      } else {
        if (!last_blk)
          dma_wait_barrier<XQ + BQ>();
        else if (RPF && rpf_loop)
          dma_wait_barrier<2>();  // rpw = 2: 64 fp16 residual rows
        else
          dma_wait_barrier<0>();
      }
    } else if constexpr (STEADY) {
      dma_wait_barrier<(STAGES - 2) * QPS>();
    } else {
      // steps after the residual prefetch (rpf_loop, issued youngest at rpf_step) also leave
      // its rpw pieces in flight
      const bool rx = RPF && rpf_loop && t > rpf_step;
      auto wait = [&](auto n_c) {
        constexpr int N = decltype(n_c)::value;
        if (!rx)
          dma_wait_barrier<N>();
        else if (rpw == 2)
          dma_wait_barrier<N + 2>();
        else
          dma_wait_barrier<N + 4>();
      };
      if constexpr (STAGES == 4) {
        if (t + 2 < nsteps)
          wait(std::integral_constant<int, 2 * QPS>{});
        else if (t + 1 < nsteps)
          wait(std::integral_constant<int, QPS>{});
        else
          wait(std::integral_constant<int, 0>{});
      } else if constexpr (STAGES == 3) {
        if (t + 1 < nsteps)
          wait(std::integral_constant<int, QPS>{});
        else
          wait(std::integral_constant<int, 0>{});
      } else {
        wait(std::integral_constant<int, 0>{});
      }
    }
    SPI_STAMP(st_b);
    // All of this step's fragment reads go out first, then the next step's
    // DMAs (their issue cost overlaps the LDS latency), then the MFMAs.
    const char* As = lds + U * IMG;
    const char* Bs = AR ? As + BM * RB : As;
    // A fragment i: image and row (halo: pixel of this tap, kh * (W + 2) + kw on; window:
    // row + kw)
    const char* Ab = AR ? As : Hs;
    [[maybe_unused]] const int toff = HALO ? (TP / 3) * a.h_hwp + TP % 3 : 0;
    auto arow = [&](int i) {
      if constexpr (HALO)
        return h_row[i] + toff;
      else if constexpr (WIN)
        return wm * WTM + i * 16 + fr + TP;
      else
        return wm * WTM + i * 16 + fr;
    };
    // window kind: is tap (kh, TP) of fragment row i inside the image
    [[maybe_unused]] auto tap_ok = [&](int i) { return ((w_mask[i] >> (w_tap0 + TP)) & 1u) != 0u; };
    auto issue_next = [&] {
      if constexpr (HALO) {
        if (TP == 10 - STAGES && !last_blk) issue_halo(hw_blk_next, hw_buf_next);
      }
      if (STEADY || t + STAGES - 1 < nsteps) issue(t + STAGES - 1, (U + STAGES - 1) % STAGES);
      if constexpr (WIN) {
        if (TP == 0 && !last_blk) issue_win(w_j + 1, (w_j + 1) & 1);
      }
      if constexpr (!STEADY) {
        if (RPF && rpf_loop && t == rpf_step) issue_res(lds + rpf_off);
      }
    };
    if constexpr (MODE == (int)Prec::F16) {
      half8 af[2][TI], bf[2][TJ];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
          af[kk][i] = __builtin_bit_cast(half8, rd_chunk<RB>(Ab, arow(i), kk * 4 + fq));
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          bf[kk][j] = __builtin_bit_cast(half8, rd_chunk<RB>(Bs, wn * WTN + j * 16 + fr, kk * 4 + fq));
      }
      issue_next();
      SPI_STAMP(st_c);
      if constexpr (WIN) {
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const bool ok = tap_ok(i);
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) af[kk][i] = ok ? af[kk][i] : half8{};
        }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
#ifdef SPI_DIAG_NO_MFMA  // diagnostic build: fragments read, no matrix work
            asm volatile("" ::"v"(af[kk][i]), "v"(bf[kk][j]));
#else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[kk][i], bf[kk][j], acc[i][j], 0, 0, 0);
#endif
    } else if constexpr (kSplitMode<MODE>) {
      static_assert(ESTEP == 32, "one 32-k block per step");
      // fp32 A: two 16-byte chunks split into hi/lo below; split A: hi and lo
      // chunks read like W's (the same conflict-free pattern).
      u32x4 ar0[TI], ar1[TI];
      half8 bh[TJ], bl[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int row = arow(i);
        ar0[i] = rd_chunk<RB>(Ab, row, MODE == kF16X3S ? fq : 2 * fq);
        ar1[i] = rd_chunk<RB>(Ab, row, MODE == kF16X3S ? 4 + fq : 2 * fq + 1);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = wn * WTN + j * 16 + fr;
        bh[j] = __builtin_bit_cast(half8, rd_chunk<RB>(Bs, row, fq));
        bl[j] = __builtin_bit_cast(half8, rd_chunk<RB>(Bs, row, 4 + fq));
      }
      issue_next();
      SPI_STAMP(st_c);
      if constexpr (WIN) {
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const bool ok = tap_ok(i);
          ar0[i] = ok ? ar0[i] : u32x4{};
          ar1[i] = ok ? ar1[i] : u32x4{};
        }
      }
      half8 ah[TI], al[TI];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        if constexpr (MODE == kF16X3S) {
          ah[i] = __builtin_bit_cast(half8, ar0[i]);
          al[i] = __builtin_bit_cast(half8, ar1[i]);
        } else {
          split8(ar0[i], ar1[i], ah[i], al[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
#ifdef SPI_DIAG_NO_MFMA
          asm volatile("" ::"v"(al[i]), "v"(ah[i]), "v"(bh[j]), "v"(bl[j]));
#else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#endif
        }
    } else {
      floatx4 a0[TI], a1[TI], b0[TJ], b1[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int row = arow(i);
        a0[i] = __builtin_bit_cast(floatx4, rd_chunk<RB>(Ab, row, 2 * fq));
        a1[i] = __builtin_bit_cast(floatx4, rd_chunk<RB>(Ab, row, 2 * fq + 1));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = wn * WTN + j * 16 + fr;
        b0[j] = __builtin_bit_cast(floatx4, rd_chunk<RB>(Bs, row, 2 * fq));
        b1[j] = __builtin_bit_cast(floatx4, rd_chunk<RB>(Bs, row, 2 * fq + 1));
      }
      issue_next();
      SPI_STAMP(st_c);
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
#ifdef SPI_GEMM_STAMPS
    // MFMA results are consumed only at the end; force completion so the compute phase is timed.
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) asm volatile("" ::"v"(acc[i][j]));
#endif
    SPI_STAMP(st_d);
    st_wait += st_b - st_a;
    st_issue += st_c - st_b;
    st_comp += st_d - st_c;
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  if constexpr (HALO) {
    // one channel block per iteration, its 9 taps unrolled (3 stages: stage =
    // tap % 3, a constant; deeper rings: a scalar stage counter)
    const int nb = h_b1 - h_b0;
    int u = 0;
    for (int j = 0; j < nb; ++j) {
      const bool lb = j == nb - 1;
      const char* Hs = lds + STAGES * IMG + (j & 1) * HBUF;
      hw_blk_next = h_b0 + j + 1;
      hw_buf_next = (j + 1) & 1;
      const int t = j * 9;
      if constexpr (STAGES == 3) {
        kstep(t + 0, I0{}, std::integral_constant<int, 0>{}, lb, Hs, std::false_type{});
        kstep(t + 1, I1{}, std::integral_constant<int, 1>{}, lb, Hs, std::false_type{});
        kstep(t + 2, I2{}, std::integral_constant<int, 2>{}, lb, Hs, std::false_type{});
        kstep(t + 3, I0{}, std::integral_constant<int, 3>{}, lb, Hs, std::false_type{});
        kstep(t + 4, I1{}, std::integral_constant<int, 4>{}, lb, Hs, std::false_type{});
        kstep(t + 5, I2{}, std::integral_constant<int, 5>{}, lb, Hs, std::false_type{});
        kstep(t + 6, I0{}, std::integral_constant<int, 6>{}, lb, Hs, std::false_type{});
        kstep(t + 7, I1{}, std::integral_constant<int, 7>{}, lb, Hs, std::false_type{});
        kstep(t + 8, I2{}, std::integral_constant<int, 8>{}, lb, Hs, std::false_type{});
      } else {
        auto nx = [&] {
          const int v = u;
          u = u + 1 == STAGES ? 0 : u + 1;
          return v;
        };
        kstep(t + 0, nx(), std::integral_constant<int, 0>{}, lb, Hs, std::false_type{});
        kstep(t + 1, nx(), std::integral_constant<int, 1>{}, lb, Hs, std::false_type{});
        kstep(t + 2, nx(), std::integral_constant<int, 2>{}, lb, Hs, std::false_type{});
        kstep(t + 3, nx(), std::integral_constant<int, 3>{}, lb, Hs, std::false_type{});
        kstep(t + 4, nx(), std::integral_constant<int, 4>{}, lb, Hs, std::false_type{});
        kstep(t + 5, nx(), std::integral_constant<int, 5>{}, lb, Hs, std::false_type{});
        kstep(t + 6, nx(), std::integral_constant<int, 6>{}, lb, Hs, std::false_type{});
        kstep(t + 7, nx(), std::integral_constant<int, 7>{}, lb, Hs, std::false_type{});
        kstep(t + 8, nx(), std::integral_constant<int, 8>{}, lb, Hs, std::false_type{});
      }
    }
  } else if constexpr (WIN) {
    // one super-step (kh, channel block) per iteration, its three kw taps unrolled: the W
    // stage is kw (slices start at a multiple of 3 steps), the window buffer j & 1
    // (every super-step but the last one is steady: constant waits, no residual prefetch)
    const int ns = nsteps / 3;
    for (int j = 0; j < ns - 1; ++j) {
      const char* Ws = lds + STAGES * IMG + (j & 1) * HBUF;
      w_tap0 = ((w_g0 + j) >> w_nbs) * 3;
      w_j = j;
      kstep(3 * j, I0{}, I0{}, false, Ws, std::true_type{});
      kstep(3 * j + 1, I1{}, I1{}, false, Ws, std::true_type{});
      kstep(3 * j + 2, I2{}, I2{}, false, Ws, std::true_type{});
    }
    {
      const int j = ns - 1;
      const char* Ws = lds + STAGES * IMG + (j & 1) * HBUF;
      w_tap0 = ((w_g0 + j) >> w_nbs) * 3;
      w_j = j;
      kstep(3 * j, I0{}, I0{}, true, Ws, std::false_type{});
      kstep(3 * j + 1, I1{}, I1{}, true, Ws, std::false_type{});
      kstep(3 * j + 2, I2{}, I2{}, true, Ws, std::false_type{});
    }
  } else if constexpr (TAP) {
    // unrolled by STAGES: stage offsets are immediates (the conv loop is short;
    // unrolling the large dense-GEMM bodies measured 1-2 % slower end to end)
    // steady iterations while every step of the iteration issues a step (t + 2 STAGES - 2 <
    // nsteps), then the checked ones
    using S1 = std::true_type;
    using S0 = std::false_type;
    int t = 0;
    for (; t + 2 * STAGES - 1 <= nsteps; t += STAGES) {
      kstep(t, I0{}, I0{}, false, nullptr, S1{});
      kstep(t + 1, I1{}, I0{}, false, nullptr, S1{});
      if constexpr (STAGES > 2) kstep(t + 2, I2{}, I0{}, false, nullptr, S1{});
      if constexpr (STAGES > 3) kstep(t + 3, I3{}, I0{}, false, nullptr, S1{});
    }
    for (; t + STAGES <= nsteps; t += STAGES) {
      kstep(t, I0{}, I0{}, false, nullptr, S0{});
      kstep(t + 1, I1{}, I0{}, false, nullptr, S0{});
      if constexpr (STAGES > 2) kstep(t + 2, I2{}, I0{}, false, nullptr, S0{});
      if constexpr (STAGES > 3) kstep(t + 3, I3{}, I0{}, false, nullptr, S0{});
    }
    if (t < nsteps) kstep(t, I0{}, I0{}, false, nullptr, S0{});
    if constexpr (STAGES > 2)
      if (t + 1 < nsteps) kstep(t + 1, I1{}, I0{}, false, nullptr, S0{});
    if constexpr (STAGES > 3)
      if (t + 2 < nsteps) kstep(t + 2, I2{}, I0{}, false, nullptr, S0{});
  } else {
    // steady while step t + STAGES - 1 exists (then t < rpf_step too)
    int t = 0;
    for (; t + STAGES - 1 < nsteps; ++t) kstep(t, t % STAGES, I0{}, false, nullptr, std::true_type{});
    for (; t < nsteps; ++t) kstep(t, t % STAGES, I0{}, false, nullptr, std::false_type{});
  }

  SPI_STAMP(st_d);
  SPI_RT(rt_l1);
#ifdef SPI_GEMM_STAMPS
  if (threadIdx.x == 0) {
    unsigned long long* gs = g_gemm_stamps + (size_t)(blockIdx.x & 65535) * 8;
    gs[0] = st_d - st_t0;
    gs[1] = st_wait;
    gs[2] = st_issue;
    gs[3] = st_comp;
    gs[4] = (unsigned long long)nsteps;
  }
#endif
  if constexpr (KG == 2) {
    // K groups: group 1 parks its partial in fragment order (thread t's accumulator (i, j) is
    // 16 contiguous bytes at ((i TJ + j) NT + t) 16) in its own W stages 0-1 -- free since the
    // last step's barrier (that step reads stage 2 and a window) -- and exits; group 0 adds it
    // to its own and goes on alone (s_barrier waits for the surviving waves only).
    static_assert(TI * TJ * NT * 16 <= 2 * IMG, "group 1's partial fits its W stages 0-1");
    floatx4* const part = reinterpret_cast<floatx4*>(lds_wg + LDSB);
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) part[(i * TJ + j) * NT + tid] = acc[i][j];
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (grp == 1) return;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] += part[(i * TJ + j) * NT + tid];
  }
  if (!kSplitK<BM, BN, KIND> || a.splits == 1) {
    if (RPF && rpf_loop)
      finish(acc, park_off, lds + rpf_off);
    else
      finish(acc, 0, nullptr);
    tl_out(0);
    return;
  }
  if constexpr (kSplitK<BM, BN, KIND>) {

  // ---- split-K: the last slice to arrive reduces -----------------------------
  // Every slice publishes its slab write-through (sc1) in fragment order (thread tid's
  // accumulator (i, j) is 16 contiguous bytes at ((i*TJ + j)*NT + tid)*16), drains its stores
  // (vmcnt(0)) and takes a relaxed agent-scope ticket; the last to arrive resets the ticket,
  // prefetches the residual, reads the other slabs with sc1 loads (MI355X_MICROARCH.md, the
  // sc1 hand-off) and adds its own partial from registers.  (Round 4 tried tickets first --
  // only the non-last slices store, the last one polls a published-slab count: the poll made
  // the reducer ~1.2 us slower, tools/gemm_timeline.py.)  Partials are summed in split order
  // whichever slice arrives last: deterministic results.
  const int splits = a.splits;
  constexpr int SLAB = BM * BN;
  int* words = a.p.counters + tile;  // the tile's arrival ticket
  float* tile_slabs = a.p.partial + (size_t)tile * splits * SLAB;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(tile_slabs, (short)0, splits * SLAB * 4, 0x00020000);
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int off = (kslice * SLAB + ((i * TJ + j) * NT + tid) * 4) * 4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, off, 0, 16);
    }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (tid == 0) {
    const int ticket = __hip_atomic_fetch_add(words, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == splits - 1;
    if (last) __hip_atomic_store(words, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = last;
  }
  __syncthreads();
  if (!*s_flag) {
    tl_out(1);
    return;
  }
  const bool rpf_red = RPF && rpf_tile;
  char* const red_res = lds + (WIN ? STAGES * IMG : IMG);  // the parked tile takes [0, BM * BN * 4)
  if (rpf_red) issue_res(red_res);
  // ZR splits' slabs in flight per round (two for the small tiles, one when a slab is 8+
  // fragments per thread); loads past the last slab fall outside the descriptor's range and
  // return 0 (no branch, no per-load wait); this slice's own slot is loaded and ignored (its
  // partial is still in registers).
  constexpr int ZR = TI * TJ <= 4 ? 2 : 1;
  floatx4 sum[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) sum[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int z0 = 0; z0 < splits; z0 += ZR) {
    floatx4 v[ZR][TI][TJ];
#pragma unroll
    for (int zz = 0; zz < ZR; ++zz)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int off = ((z0 + zz) * SLAB + ((i * TJ + j) * NT + tid) * 4) * 4;
          v[zz][i][j] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
        }
#pragma unroll
    for (int zz = 0; zz < ZR; ++zz) {
      const bool own = z0 + zz == kslice;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) sum[i][j] += own ? acc[i][j] : v[zz][i][j];
    }
  }
  finish(sum, 0, rpf_red ? red_res : nullptr);
  tl_out(2);
  }
}

template <int MODE, int BM, int BN, int STAGES, int KIND, int NW = 4>
__global__ __launch_bounds__(64 * NW, (kMinWaves<BM, BN, STAGES, KIND, NW>)) void gemm_kernel(KArgs a) {
  gemm_body<MODE, BM, BN, STAGES, KIND, NW>(a, blockIdx.y, blockIdx.x, blockIdx.x + blockIdx.y * a.tiles);
}

// Grouped launch (KGroup): 1-D grid, problem-major, then slice, then tile.
template <int MODE, int BM, int BN, int STAGES, int KIND, int NW = 4>
__global__ __launch_bounds__(64 * NW, (kMinWaves<BM, BN, STAGES, KIND, NW>)) void gemm_kernel_pair(KGroup g) {
  // One body per problem (a branch on a workgroup-uniform condition), each with constant kernel
  // argument offsets: selecting the problem's KArgs by reference had every field become a select of
  // two loaded values -- SGPR spills to VGPR lanes and the tile decode's FastDiv tables copied to
  // scratch and read back with a dynamic offset (40 bytes of scratch per lane, round 6)
  const int lin = blockIdx.x;
  if (lin >= g.wgs0) {
    const int l1 = lin - g.wgs0;
    const int kslice = fdiv(l1, g.a[1].fd_tiles);
    gemm_body<MODE, BM, BN, STAGES, KIND, NW>(g.a[1], kslice, l1 - kslice * g.a[1].tiles, l1);
  } else {
    const int kslice = fdiv(lin, g.a[0].fd_tiles);
    gemm_body<MODE, BM, BN, STAGES, KIND, NW>(g.a[0], kslice, lin - kslice * g.a[0].tiles, lin);
  }
}

struct Plan {
  int bm, bn, stages, splits, k_per_split;
  // kConvHalo: waves per workgroup, virtual output rows per band, the virtual-row
  // period (rows per image) and offset (KArgs::h_off), band count, channel blocks
  // per slice
  int halo = 0, nw = 4, th = 0, period = 0, off = 0, tiles_m = 0, bps = 0;
  int win = 0;  // kConvTapW (64 x 64, 3 W stages; slices of whole 3-step super-steps)
};

int estep_of(Prec prec) {
  return prec == Prec::F16 ? Traits<(int)Prec::F16>::ESTEP
                           : prec == Prec::F32 ? Traits<(int)Prec::F32>::ESTEP : Traits<(int)Prec::F16X3>::ESTEP;
}

// Tuning knobs, read once (getenv on every launch cost ~0.5 us each, and the
// plan is evaluated three times per launch); spi_debug_gemm_reload_env()
// re-reads them for in-process sweeps and tests.  Variants measured and rejected
// in rounds 1-3 (latency plan rule, 128x64 split-K, 256x128 tiles, 3-stage
// 128x128 rings, 4-stage halo rings, XCD-local split-K, per-knob ring depths,
// DESIGN.md 6) are gone; what remains:
//   SPI_GEMM_PLAN="bm,bn,stages,splits"  force one plan for every GEMM (sweeps)
//   SPI_GEMM_MAXSPLIT=S                  cap split-K (default 8; 1: none, 0: uncapped)
//   SPI_GEMM_HALO_CFG                    halo candidates: "0" off, "rows,a|s" forced,
//                                        "OW:rows,a|s;..." per map width
//   SPI_GEMM_256_MIN / SPI_GEMM_256_LONGK  gemm256 routing (below)
struct Knobs {
  bool forced = false;
  Plan plan{};
  // SPI_GEMM_PLAN_LONGK="K,bm,bn,stages,splits": that plan for dense GEMMs with K >= K only (A/B sweeps)
  int longk_plan_k = 0;
  Plan longk_plan{};
  int target = 128;  // round 3 (with the joint pair plan): ResNet-18 fp16m +2 % over 192, BERT / ResNet-152 +-0
  // split-K cap: ResNet-18 bs1 (layer 4: 12 slices, layer 3: 4) +1.8 % at 8 or 6 over uncapped,
  // bs8 +-0.5 % (no conv splits past 6 there); round 6, profiles/r06/maxsplit/
  int max_split = 8;
  int halo = 1;  // 3x3/s1 convs from LDS-resident input bands (kConvHalo)
  // SPI_GEMM_WIN=0: 3x3/s1 tap walks without the kw window (kConvTapW); 2 / 3: 64 x 64 window
  // tiles as two K groups of 4 waves (8-wave workgroups), at the 4-wave plan's slices / half of them
  int win = 1;
  int g256_min = 128;      // SPI_GEMM_256_MIN="T256[,T128]": dense F16 GEMMs with >= T256 tiles of 256^2 -> gemm256 (0 = off)
  // ... else with >= T128 tiles of 128 x 256 -> gemm256's 128-row tile (round 5; 0 = off)
  // round 6: 64 tiles, two buffers -- BERT-base's FFN1 (96 tiles of 128 x 256, K = 768) four-stream
  // +1.5 % (24.25k -> 24.60k, profiles/r06/sweeps/); the long-K rule below keeps ViT-L's N = 1024
  // GEMMs on 256^2 tiles (128 x 256 there: -3 % with three buffers, -7 % with two).  Rounds 3-5
  // had it off (BERT -7 % with the three-buffer schedule, which also raced)
  int g128_min = 64;
  int g128_nbuf = 2;  // third field: k-tile buffers of the 128-row tile (2: 96 KiB, 3: 144 KiB)
  // SPI_GEMM_256_LONGK="tiles,K": also with >= `tiles` tiles when K >= `K` (round 3: 48,1024 -- ViT-L FFN2 /
  // out-proj, 52 tiles: one 256^2 workgroup per CU-time unit does ~1.7x the work of the 128x128 kernel, so
  // under four streams ViT-L goes 6.07k -> 6.70k inf/s though the launch alone is slower; BERT's K = 768
  // GEMMs stay off: -1.3 % with them)
  int g256_longk_tiles = 48, g256_longk_k = 1024;
  // SPI_GEMM_256_LONGK="tiles,K,S": gemm256 split-K up to S slices for grids under T tiles (default
  // 1: none -- round 4 measured ViT-L FFN2 at 3 slices 100 -> 73 us back to back but C5 under the
  // four streams 6.05k -> 5.09k inf/s: the slices' CU-time and slab traffic cost the other streams more)
  int g256_split = 1;
  // SPI_GEMM_256_ORDER: gemm256 tile order, 0 row blocks fastest, 1 column tiles fastest, -1 (default)
  // by shape: column tiles fastest when A is the larger operand (M > N), so an XCD's consecutive
  // workgroups share A row blocks (round 6, PMC FETCH_SIZE: ViT-L FFN2 142 -> 119 MB, out-proj
  // 47.7 -> 41.9 MB; FFN1 (N = 4096) 61 -> 78 MB the other way; C5 four-stream +0.2 %)
  int g256_order = -1;
  int halo_bm = 0;          // SPI_GEMM_HALO_CFG="rows,a|s": force a halo candidate (64 / 128 / 256 rows)
  bool halo_stacked = false;
  struct HaloPick {
    int ow, bm;
    bool stacked;
  };
  HaloPick halo_map[8] = {};  // SPI_GEMM_HALO_CFG="OW:rows,a|s;...": per map width
  int n_halo_map = 0;
};
// Fixed plan constants (each measured in rounds 1-3):
constexpr int kHaloStages = 3;     // W ring of the halo kinds
constexpr int kHaloMinH = 14;      // 7x7 maps: the implicit GEMM measured faster (77 % row use)
constexpr int kHaloMaxTiles = 64;  // halo only when the implicit GEMM has fewer 64x64 tiles
// Ring depth by k-steps per slice (variant builds: tools/build_variant.sh ... -DSPI_ST3_MIN=N /
// -DSPI_ST4_MIN=N).  Round 6: 3 stages from 12 k-steps, no 4-stage ring -- BERT-base's out-proj (12
// k-steps, was 2 stages) and FFN2 (48, was 4: +2.4 % in round 3) then share one kernel instance:
// C3 +1.2 %, each change alone +0.2 %; C2 / C4 +-0.3 % (profiles/r06/ring_depth/)
#ifndef SPI_ST3_MIN
#define SPI_ST3_MIN 12
#endif
#ifndef SPI_ST4_MIN
#define SPI_ST4_MIN (1 << 30)
#endif
constexpr int kSt3Min = SPI_ST3_MIN, kSt4Min = SPI_ST4_MIN;

Knobs read_knobs() {
  Knobs k;
  if (const char* e = std::getenv("SPI_GEMM_PLAN"); e && *e) {
    int bm = 0, bn = 0, st = 0, sp = 0;
    if (std::sscanf(e, "%d,%d,%d,%d", &bm, &bn, &st, &sp) == 4) {
      const bool ok_tile = (bm == 128 && bn == 128) || (bm == 128 && bn == 64) || (bm == 64 && bn == 64);
      const bool ok_st = st >= 2 && st <= 4 && !(bm == 128 && bn == 128 && st > 2) && !(bm == 128 && bn == 64 && st > 3);
      if (ok_tile && ok_st && sp >= 1) {
        k.forced = true;
        k.plan = Plan{bm, bn, st, sp, 0};
      }
    }
  }
  if (const char* e = std::getenv("SPI_GEMM_PLAN_LONGK"); e && *e) {
    int kk = 0, bm = 0, bn = 0, st = 0, sp = 0;
    if (std::sscanf(e, "%d,%d,%d,%d,%d", &kk, &bm, &bn, &st, &sp) == 5) {
      const bool ok_tile = (bm == 128 && bn == 128) || (bm == 128 && bn == 64) || (bm == 64 && bn == 64);
      const bool ok_st = st >= 2 && st <= 4 && !(bm == 128 && bn == 128 && st > 2) && !(bm == 128 && bn == 64 && st > 3);
      if (ok_tile && ok_st && sp >= 1 && kk > 0) {
        k.longk_plan_k = kk;
        k.longk_plan = Plan{bm, bn, st, sp, 0};
      }
    }
  }
  if (const char* e = std::getenv("SPI_GEMM_256_MIN"); e && *e) {
    int a = 0, b = 0, c = 3;
    const int n = std::sscanf(e, "%d,%d,%d", &a, &b, &c);
    k.g256_min = a;
    if (n >= 2) k.g128_min = b;
    if (n >= 3) k.g128_nbuf = c == 2 ? 2 : 3;
  }
  if (const char* e = std::getenv("SPI_GEMM_256_LONGK"); e && *e) {
    int t = 0, kk = 0, sp = 1;
    if (std::sscanf(e, "%d,%d,%d", &t, &kk, &sp) >= 2) {
      k.g256_longk_tiles = t;
      k.g256_longk_k = kk;
      k.g256_split = std::max(1, sp);
    } else {
      k.g256_longk_tiles = 0;  // e.g. "0": off
    }
  }
  if (const char* e = std::getenv("SPI_GEMM_HALO_CFG"); e && *e) {
    // "0": no halo kinds; "rows,a|s" for every halo conv, or per map width
    // "OW:rows,a|s;OW:rows,a|s;..." (OW 0 = any other width; rows 0 = not a halo conv)
    if (std::strcmp(e, "0") == 0) {
      k.halo = 0;
    } else if (std::strchr(e, ':')) {
      for (const char* q = e; q && *q;) {
        int ow = 0, bm = 0;
        char mode = 'a';
        if (std::sscanf(q, "%d:%d,%c", &ow, &bm, &mode) >= 2 && k.n_halo_map < 8)
          k.halo_map[k.n_halo_map++] = {ow, bm, mode == 's'};
        q = std::strchr(q, ';');
        if (q) ++q;
      }
    } else {
      int bm = 0;
      char mode = 'a';
      if (std::sscanf(e, "%d,%c", &bm, &mode) >= 1 && (bm == 64 || bm == 128 || bm == 256)) {
        k.halo_bm = bm;
        k.halo_stacked = mode == 's';
      }
    }
  }
  if (const char* e = std::getenv("SPI_GEMM_256_ORDER"); e && *e) k.g256_order = std::max(-1, std::min(1, std::atoi(e)));
  if (const char* e = std::getenv("SPI_GEMM_MAXSPLIT"); e && *e) k.max_split = std::max(0, std::atoi(e));  // 0: uncapped
  if (const char* e = std::getenv("SPI_GEMM_WIN"); e && *e) k.win = std::max(0, std::min(3, std::atoi(e)));
  return k;
}

Knobs& knobs() {
  static Knobs k = read_knobs();
  return k;
}

// gemm256 routing by desc (gemm() also needs 16-byte aligned A / W): the tile height it runs
// at, 0 = the general kernel.  256^2 tiles for grids of >= T256 of them, or of >= the long-K
// rule's tiles when K is long (ViT-L's N = 1024 GEMMs at bs16: 52 tiles); else 128 x 256 tiles
// for grids of >= T128 of those (BERT-base's FFN1 at bs8: 96).
int route_bm(const GemmDesc& d, Prec prec) {
  const Knobs& k = knobs();
  if (prec != Prec::F16) return 0;
  if (gemm256_eligible(d, prec, k.g256_min)) return 256;
  if (k.g256_longk_tiles > 0 && d.K >= k.g256_longk_k && gemm256_eligible(d, prec, k.g256_longk_tiles)) return 256;
  if (gemm256_eligible(d, prec, k.g128_min, 128)) return 128;
  return 0;
}
bool routes_256(const GemmDesc& d, Prec prec) { return route_bm(d, prec) != 0; }
int g256_splits(const GemmDesc& d) {
  const Knobs& k = knobs();
  const int cap = k.max_split > 0 ? std::min(k.max_split, k.g256_split) : k.g256_split;
  return cap > 1 ? gemm256_splits(d, k.target, cap, route_bm(d, Prec::F16)) : 1;
}

Plan finish_plan(Plan pl, int ksteps, int ES, int krep = 1) {
  const Knobs& k = knobs();
  if (k.max_split) pl.splits = std::min(pl.splits, k.max_split);
  if (pl.bn != 64 || (pl.bm != 64 && pl.bm != 128)) pl.splits = 1;  // split-K exists in the 64- and 128-row x 64 kernels only
  if (pl.bm == 128) pl.stages = pl.bn == 128 ? 2 : std::min(pl.stages, 3);  // the instantiated rings
  pl.splits = std::max(1, std::min(pl.splits, ksteps));
  int kt = (ksteps + pl.splits - 1) / pl.splits;
  kt = (kt + krep - 1) / krep * krep;  // krep: slices hold whole (hi, lo) step pairs
  pl.k_per_split = kt * ES;
  pl.splits = (ksteps + kt - 1) / kt;
  return pl;
}

// kConvHalo plan for 3x3/s1/p1 convs with whole channel blocks (split activations
// in F16X3).  Candidates (all 64 columns wide):
//   64 rows, 4 waves (kConvHaloS when the halo fits 96 pixels, else 128-pixel buffers)
//   128 rows, 4 waves (256-pixel buffers); 256 rows, 8 waves (384-pixel buffers)
// each with aligned bands (whole output rows of one image) or stacked bands
// (virtual rows spanning images, for maps too small to fill a tile).  th = as many
// (virtual) rows per band as fit the tile and the halo buffer; split-K over
// channel blocks up to ~T workgroups.  The default picks aligned 128 rows for maps
// wider than 32 pixels, else aligned 64 (the round-1 rule) -- SPI_GEMM_HALO_CFG =
// "rows,a|s" forces a candidate (tools/gemm_bench.py sweeps).  halo = 0 when the
// conv is not eligible.
Plan halo_candidate(const GemmDesc& d, Prec prec, int T, int bm, bool stacked, int smax) {
  Plan no{};
  const int ES = estep_of(prec);
  const int nw = bm == 256 ? 8 : 4;
  const int cap = (bm == 256 ? 6 * 8 : bm == 128 ? 8 * 4 : 4 * 4) * 8;  // kHaloHQ x NW x 8 pixels
  const int imgs = d.M / (d.OH * d.OW);
  int th = stacked ? bm / d.OW : std::min(bm / d.OW, d.OH);
  while (th > 0 && (th + 2) * (d.W + 2) > cap) --th;
  if (th == 0) return no;
  const bool small = bm == 64 && (th + 2) * (d.W + 2) <= 3 * 32;  // kConvHaloS
  const int nblk = d.Cin / ES;
  Plan h{bm, 64, kHaloStages, 1, 0};
  h.nw = nw;
  h.th = th;
  if (stacked) {
    h.off = 1;
    h.period = d.OH + 2;
    h.tiles_m = (imgs * h.period + th - 1) / th;
  } else {
    const int nb = (d.OH + th - 1) / th;
    h.off = 0;
    h.period = nb * th;
    h.tiles_m = imgs * nb;
  }
  const int tiles = h.tiles_m * (d.N / 64);
  int sp = 1;
  if (tiles < T) sp = std::min({(T + tiles - 1) / tiles, nblk, smax});
  if (knobs().max_split) sp = std::min(sp, knobs().max_split);
  const int bps = (nblk + sp - 1) / sp;
  h.splits = (nblk + bps - 1) / bps;
  h.halo = small ? 2 : 1;
  h.bps = bps;
  return h;
}

// kConvTapW: 3x3 / stride 1 / padding 1 convs with OH = H, OW = W (a tap's input pixel is
// the output pixel shifted by a constant), whole channel blocks, no Kpad tail, and A in
// 128-byte pixel blocks read as they are (fp16, split fp16x3).
bool window_ok(const GemmDesc& d, Prec prec) {
  const int ES = estep_of(prec);
  return knobs().win && d.conv && !d.pool_rows && d.KH == 3 && d.KW == 3 && d.stride == 1 && d.pad == 1 &&
         d.OH == d.H && d.OW == d.W && d.krep == 1 && d.Cin >= ES && d.Cin % ES == 0 && d.Kpad == d.K &&
         (prec == Prec::F16 || (prec == Prec::F16X3 && d.a_split));
}

Plan halo_plan(const GemmDesc& d, Prec prec, int T) {
  Plan no{};
  const int ES = estep_of(prec);
  if (!knobs().halo || knobs().forced || d.krep != 1 || !d.conv || d.KH != 3 || d.KW != 3 || d.stride != 1 || d.pad != 1 ||
      d.Cin < ES || d.Cin % ES || (prec == Prec::F16X3 && !d.a_split) || d.N % 64 || d.OH != d.H || d.OW != d.W)
    return no;
  if (knobs().halo_bm) return halo_candidate(d, prec, T, knobs().halo_bm, knobs().halo_stacked, 1 << 20);
  for (int i = 0; i < knobs().n_halo_map; ++i) {
    const auto& hm = knobs().halo_map[i];
    if (hm.ow == d.OW || hm.ow == 0) {
      if (hm.bm != 64 && hm.bm != 128 && hm.bm != 256) return no;
      return halo_candidate(d, prec, T, hm.bm, hm.stacked, 1 << 20);
    }
  }
  if (d.OH < kHaloMinH) return no;
  // Under the serving load (four worker streams) the implicit GEMM's many small,
  // LDS-light workgroups keep more kernels co-resident than the halo kinds'
  // 56-90 KiB ones: ResNet-18 bs8 59.3k vs 57.0k inf/s, ResNet-152 bs32 10.7k vs
  // 10.0k (tools/policy_sweep.py).  The halo kinds pay where the grid
  // is small and one forward's latency dominates (ResNet-18 bs1: 13.2k vs 12.1k).
  const auto ceil_div = [](int x, int y) { return (x + y - 1) / y; };
  if (ceil_div(d.M, 64) * ceil_div(d.N, 64) >= kHaloMaxTiles) return no;
  const int bm = d.OW > 32 ? 128 : 64;
  return halo_candidate(d, prec, T, bm, false, bm == 64 ? 1 << 20 : 1);  // round 1: only 64-row tiles split
}

// XCD rectangles (gemm_kernel's tile decode): the row x column group split
// gm x gn (gm * gn = 8, the XCDs) that minimises the bytes the XCDs' L2s fetch,
// A * gn + W * gm (A: the activation bytes a tile row block reads -- the input
// image for convs; W: the packed weights).
void xcd_groups(const GemmDesc& d, Prec prec, int TM, int TN, int& gm, int& gn) {
  gm = 1;
  gn = std::min(8, TN);
  if (TM * TN < 16) return;
  const double ea = prec == Prec::F16 ? 2 : 4, ew = prec == Prec::F16 ? 2 : 4;
  const double A = d.conv ? (double)(d.M / (d.OH * d.OW)) * d.H * d.W * d.Cin * ea : (double)d.M * d.K * ea;
  const double W = (double)d.N * d.Kpad * ew;
  double best = 1e300;
  for (int m = 1; m <= 8; m *= 2) {
    const int n = 8 / m;
    if (m > TM || n > TN) continue;
    const double cost = A * n + W * m;
    if (cost < best) {
      best = cost;
      gm = m;
      gn = n;
    }
  }
}

int plan_tiles(const GemmDesc& d, const Plan& pl) {
  if (pl.halo) return pl.tiles_m * ((d.N + pl.bn - 1) / pl.bn);
  if (d.pool_rows) return d.M / d.pool_rows * ((d.N + pl.bn - 1) / pl.bn);
  return ((d.M + pl.bm - 1) / pl.bm) * ((d.N + pl.bn - 1) / pl.bn);
}

// Plan rule: the largest tile that still yields >= T workgroups, split-K only
// when even 64x64 tiles fall short (then to ~T workgroups, >= 6 k-steps per
// slice).  T in 128..192 measured best with 4 concurrent worker streams
// (ResNet-18 bs8 fp16x3 +8 %, ResNet-152 bs32 +8 %, BERT-base +5 %, ViT-L +7 %
// over a single-stream latency rule); 128 since the joint pair
// plan (round 3).
Plan choose_plan(const GemmDesc& d, Prec prec) {
  const Knobs& k = knobs();
  const int ES = estep_of(prec);
  const int ksteps = d.Kpad / ES;
  if (k.forced) return finish_plan(k.plan, ksteps, ES, d.krep);
  if (k.longk_plan_k > 0 && !d.conv && !d.pool_rows && d.K >= k.longk_plan_k)
    return finish_plan(k.longk_plan, ksteps, ES, d.krep);
  const auto tiles_of = [&](int bm, int bn) { return ((d.M + bm - 1) / bm) * ((d.N + bn - 1) / bn); };
  // a deeper ring pays only on long K loops (4 stages only reach the 64x64 tiles, finish_plan caps the others)
  const auto stages_for = [](int kt) { return kt >= kSt4Min ? 4 : kt >= kSt3Min ? 3 : 2; };
#ifndef SPI_FC_SPLITS  // variant builds: split-K slices of the pooled FC (avgpool + FC in one GEMM)
#define SPI_FC_SPLITS 1
#endif
  if (d.pool_rows)  // one image per tile row
    return finish_plan(Plan{64, 64, stages_for((ksteps + SPI_FC_SPLITS - 1) / SPI_FC_SPLITS), SPI_FC_SPLITS, 0}, ksteps,
                       ES, d.krep);
  if (Plan h = halo_plan(d, prec, k.target); h.halo) return h;
  const int T = k.target;
  if (d.N > 64 && tiles_of(128, 128) >= T) return finish_plan(Plan{128, 128, 2, 1, 0}, ksteps, ES, d.krep);
  if (tiles_of(128, 64) >= T) {
    if (window_ok(d, prec)) {
      Plan w = finish_plan(Plan{128, 64, 3, 1, 0}, ksteps, ES, 3);
      w.win = 1;
      return w;
    }
    return finish_plan(Plan{128, 64, stages_for(ksteps), 1, 0}, ksteps, ES, d.krep);
  }
  const int t64 = tiles_of(64, 64);
  const int sp = t64 >= T ? 1 : std::max(1, std::min((T + t64 - 1) / t64, ksteps / 6));
  const Plan pl = finish_plan(Plan{64, 64, stages_for((ksteps + sp - 1) / sp), sp, 0}, ksteps, ES, d.krep);
  if (window_ok(d, prec)) {
    // the kw-window tap walk: slices of whole (kh, channel block) super-steps
    if (k.win >= 2 && ksteps % 6 == 0) {
      // two K groups per workgroup (8 waves): slices of an even number of super-steps,
      // SPI_GEMM_WIN=2 at the 4-wave plan's slice count, 3 at half of it
      const int sp2 = k.win == 3 ? (sp + 1) / 2 : sp;
      Plan w = finish_plan(Plan{64, 64, 3, sp2, 0}, ksteps, ES, 6);
      w.win = 1;
      w.nw = 8;
      return w;
    }
    Plan w = finish_plan(Plan{64, 64, 3, sp, 0}, ksteps, ES, 3);
    w.win = 1;
    return w;
  }
  return pl;
}

int ilog2(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

template <int MODE, int BM, int BN, int STAGES, int NW = 4>
void launch_tile(const KArgs& a, dim3 grid, hipStream_t s) {
  if (a.cell_uniform) {
    SPI_LAUNCH((gemm_kernel<MODE, BM, BN, STAGES, kConvTap, NW>), grid, dim3(64 * NW), 0, s, a);
  } else if (a.d.conv) {
    if constexpr (MODE != kF16X3S)  // split A needs one tap per step (checked in gemm())
      SPI_LAUNCH((gemm_kernel<MODE, BM, BN, STAGES, kConvGen, NW>), grid, dim3(64 * NW), 0, s, a);
  } else {
    SPI_LAUNCH((gemm_kernel<MODE, BM, BN, STAGES, kDense, NW>), grid, dim3(64 * NW), 0, s, a);
  }
}

// Kernel arguments of one problem under its plan.
template <int MODE>
KArgs make_args(const GemmDesc& d, const GemmPtrs& p, const Plan& pl) {
  KArgs a{};
  a.d = d;
  a.p = p;
  a.k_per_split = pl.k_per_split;
  a.splits = pl.splits;
  a.tiles = plan_tiles(d, pl);
  a.tiles_m = a.tiles / ((d.N + pl.bn - 1) / pl.bn);
#ifdef SPI_GEMM_TIMELINE
  a.tl = tl_thread();
#endif
  const int TM = a.tiles_m, TN = a.tiles / a.tiles_m;
  a.tiles_n = TN;
  xcd_groups(d, MODE == kF16X3S ? Prec::F16X3 : (Prec)MODE, TM, TN, a.xg_m, a.xg_n);
  if (pl.splits > 1) {  // split-K grids: the plain column-major order
    a.xg_m = 1;
    a.xg_n = std::min(8, TN);
  }
  for (int i = 0; i <= 8; ++i) {
    a.rg_m0[i] = std::min(i, a.xg_m) * TM / a.xg_m;
    a.cg_n0[i] = std::min(i, a.xg_n) * TN / a.xg_n;
  }
  for (int i = 0; i < 8; ++i) a.fd_rows[i] = make_fastdiv((unsigned)std::max(1, a.rg_m0[i + 1] - a.rg_m0[i]));
  a.fd_split = make_fastdiv((unsigned)std::max(1, pl.splits));
  a.fd_tiles = make_fastdiv((unsigned)std::max(1, a.tiles));
  if (d.conv) {
    a.fd_ohw = make_fastdiv((unsigned)(d.OH * d.OW));
    a.fd_ow = make_fastdiv((unsigned)d.OW);
    a.imgs = d.M / (d.OH * d.OW);
  }
  a.cin_shift = d.conv ? ilog2(d.Cin) : 0;
  a.kw_mul = (65536 + d.KW - 1) / d.KW;
  // one (kh, kw) tap per k-step; the per-row tap mask has 32 bits (taps + the Kpad tail step)
  a.cell_uniform = d.conv && d.Cin >= Traits<MODE>::ESTEP && d.KH * d.KW <= 31;
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  a.vec_ok = d.ldc % 8 == 0 && al16(p.C) && (!p.res || (d.ldr % 8 == 0 && al16(p.res))) && (!p.bias || al16(p.bias));
  if (pl.halo) {
    a.h_th = pl.th;
    a.h_period = pl.period;
    a.h_off = pl.off;
    a.h_hwp = d.W + 2 * d.pad;
    a.h_hp = (pl.th + 2) * a.h_hwp;
    a.h_nblk = d.Cin / Traits<MODE>::ESTEP;
    a.h_bps = pl.bps;
    a.fd_period = make_fastdiv((unsigned)std::max(1, pl.period));
    a.fd_hwp = make_fastdiv((unsigned)a.h_hwp);
  }
  if (pl.win) a.win_nblk_shift = ilog2(d.Cin / Traits<MODE>::ESTEP);
  return a;
}

// One problem under its plan: grid tiles x splits.
template <int MODE>
void dispatch(const Plan& pl, const KArgs& g, hipStream_t s) {
  const dim3 grid(g.tiles, pl.splits);
  if (pl.halo) {
    if constexpr (MODE != (int)Prec::F16X3) {  // fp32 A is split at fragment read: not a halo mode
      if (pl.bm == 256)
        SPI_LAUNCH((gemm_kernel<MODE, 256, 64, 3, kConvHalo, 8>), grid, dim3(512), 0, s, g);
      else if (pl.bm == 128)
        SPI_LAUNCH((gemm_kernel<MODE, 128, 64, 3, kConvHalo>), grid, dim3(256), 0, s, g);
      else if (pl.halo == 2)
        SPI_LAUNCH((gemm_kernel<MODE, 64, 64, 3, kConvHaloS>), grid, dim3(256), 0, s, g);
      else
        SPI_LAUNCH((gemm_kernel<MODE, 64, 64, 3, kConvHalo>), grid, dim3(256), 0, s, g);
    }
    return;
  }
  if (pl.win) {
    if constexpr (MODE == (int)Prec::F16 || MODE == kF16X3S) {
      if (pl.nw == 8) {
        // K groups: both must walk the same number of super-steps (their barriers pair up)
        const int ES = Traits<MODE>::ESTEP;
        if (pl.bm != 64 || pl.k_per_split % (6 * ES) || g.d.Kpad % (6 * ES))
          throw std::logic_error("window kind with K groups: slices of an even number of super-steps");
        SPI_LAUNCH((gemm_kernel<MODE, 64, 64, 3, kConvTapW, 8>), grid, dim3(512), 0, s, g);
      } else if (pl.bm == 128)
        SPI_LAUNCH((gemm_kernel<MODE, 128, 64, 3, kConvTapW>), grid, dim3(256), 0, s, g);
      else
        SPI_LAUNCH((gemm_kernel<MODE, 64, 64, 3, kConvTapW>), grid, dim3(256), 0, s, g);
    }
    return;
  }
  if (pl.bm == 128 && pl.bn == 128)
    launch_tile<MODE, 128, 128, 2>(g, grid, s);
  else if (pl.bm == 128 && pl.stages == 2)
    launch_tile<MODE, 128, 64, 2>(g, grid, s);
  else if (pl.bm == 128)
    launch_tile<MODE, 128, 64, 3>(g, grid, s);
  else if (pl.stages == 2)
    launch_tile<MODE, 64, 64, 2>(g, grid, s);
  else if (pl.stages == 4)
    launch_tile<MODE, 64, 64, 4>(g, grid, s);
  else
    launch_tile<MODE, 64, 64, 3>(g, grid, s);
}

// Two tap-walk conv problems sharing pl's tile shape and ring depth: one launch.
template <int MODE>
void dispatch_pair(const Plan& pl, const KGroup& g, int wgs, hipStream_t s) {
  const dim3 grid(wgs);
  if (pl.bm == 128 && pl.bn == 128)
    SPI_LAUNCH((gemm_kernel_pair<MODE, 128, 128, 2, kConvTap>), grid, dim3(256), 0, s, g);
  else if (pl.bm == 128 && pl.stages == 2)
    SPI_LAUNCH((gemm_kernel_pair<MODE, 128, 64, 2, kConvTap>), grid, dim3(256), 0, s, g);
  else if (pl.bm == 128)
    SPI_LAUNCH((gemm_kernel_pair<MODE, 128, 64, 3, kConvTap>), grid, dim3(256), 0, s, g);
  else if (pl.stages == 2)
    SPI_LAUNCH((gemm_kernel_pair<MODE, 64, 64, 2, kConvTap>), grid, dim3(256), 0, s, g);
  else if (pl.stages == 4)
    SPI_LAUNCH((gemm_kernel_pair<MODE, 64, 64, 4, kConvTap>), grid, dim3(256), 0, s, g);
  else
    SPI_LAUNCH((gemm_kernel_pair<MODE, 64, 64, 3, kConvTap>), grid, dim3(256), 0, s, g);
}

constexpr Prec prec_of_mode(int mode) { return mode == kF16X3S ? Prec::F16X3 : (Prec)mode; }

template <int MODE>
void launch(const GemmDesc& d, const GemmPtrs& p, hipStream_t s) {
  const Plan pl = choose_plan(d, prec_of_mode(MODE));
  dispatch<MODE>(pl, make_args<MODE>(d, p, pl), s);
}

// Two problems in one launch when their plans share a kernel instance (same
// tile, ring depth and A kind, neither a halo plan); otherwise two launches.
// Problem 1's split-K slabs and tickets follow problem 0's in the workspace.
template <int MODE>
void launch_pair(const GemmDesc& d0, const GemmPtrs& p0, const GemmDesc& d1, const GemmPtrs& p1, hipStream_t s) {
  const Prec pr = prec_of_mode(MODE);
  Plan q0 = choose_plan(d0, pr), q1 = choose_plan(d1, pr);
  if (!q0.halo && !q1.halo && q0.splits > 1 && q0.bm == 64 && q0.bn == 64 &&
      q1.bm == 64 && q1.bn == 64) {
    // Joint plan: the grouped launch is one grid, so problem 1's workgroups count
    // toward the T workgroups problem 0's split-K was sized for -- fewer slices,
    // fewer fp32 slabs through memory.  Problem 1 (the 1x1 downsample, a few
    // k-steps) takes problem 0's ring depth so the two still share a kernel.
    const int ES = estep_of(pr), ksteps = d0.Kpad / ES;
    const int t64 = plan_tiles(d0, q0), w1 = plan_tiles(d1, q1) * q1.splits;
    const int T0 = std::max(1, knobs().target - w1);
    const int sp = std::max(1, std::min({(T0 + t64 - 1) / t64, ksteps / 6, q0.splits}));
    if (sp < q0.splits) {
      const int kt = (ksteps + sp - 1) / sp;
      q0 = finish_plan(Plan{64, 64, kt >= kSt3Min ? 3 : 2, sp, 0}, ksteps, ES, d0.krep);
      if (q1.splits == 1) q1.stages = q0.stages;
    }
  }
  if (!q0.halo && !q1.halo && q0.splits == 1 && q1.splits == 1 && q0.bm == 64 &&
      q0.bn == 64 && q1.bm == 64 && q1.bn == 64) {
    // the largest common tile whose joint grid still reaches T
    // (the layer-2 pair: 98 + 98 tiles of 128 x 64 instead of 196 + 196 of 64 x 64)
    const auto t = [](const GemmDesc& d, int bm, int bn) { return ((d.M + bm - 1) / bm) * ((d.N + bn - 1) / bn); };
    if (t(d0, 128, 64) + t(d1, 128, 64) >= knobs().target) {
      const int ES = estep_of(pr), k0 = d0.Kpad / ES, k1 = d1.Kpad / ES;
      const int st = std::max(k0, k1) >= kSt3Min ? 3 : 2;
      q0 = finish_plan(Plan{128, 64, st, 1, 0}, k0, ES, d0.krep);
      q1 = finish_plan(Plan{128, 64, st, 1, 0}, k1, ES, d1.krep);
    }
  }
  KGroup g{};
  g.a[0] = make_args<MODE>(d0, p0, q0);
  GemmPtrs p1s = p1;
  if (q0.splits > 1) {  // keep clear of problem 0's slabs / tickets
    p1s.partial = p0.partial + (size_t)g.a[0].tiles * q0.splits * q0.bm * q0.bn;
    p1s.counters = p0.counters + g.a[0].tiles;
  }
  g.a[1] = make_args<MODE>(d1, p1s, q1);
  const bool same = !q0.halo && !q1.halo && !q0.win && !q1.win && q0.bm == q1.bm && q0.bn == q1.bn &&
                    q0.stages == q1.stages && q0.nw == 4 && q1.nw == 4 && g.a[0].cell_uniform &&
                    g.a[1].cell_uniform;
  if (!same) {
    launch<MODE>(d0, p0, s);
    launch<MODE>(d1, p1, s);
    return;
  }
  g.wgs0 = g.a[0].tiles * q0.splits;
  dispatch_pair<MODE>(q0, g, g.wgs0 + g.a[1].tiles * q1.splits, s);
}

}  // namespace

// Workspace of the general kernel's plan, or of gemm256's when gemm() may route the desc
// there (routing also needs 16-byte aligned A / W, unknown here: the larger of the two).
size_t gemm_partial_floats(const GemmDesc& d, Prec prec) {
  const Plan pl = choose_plan(d, prec);
  size_t f = pl.splits <= 1 ? 0 : (size_t)plan_tiles(d, pl) * pl.splits * pl.bm * pl.bn;
  if (const int bm = route_bm(d, prec); bm && g256_splits(d) > 1)
    f = std::max(f, (size_t)((d.M + bm - 1) / bm) * (d.N / 256) * g256_splits(d) * bm * 256);
  return f;
}

size_t gemm_counter_slots(const GemmDesc& d, Prec prec) {
  const Plan pl = choose_plan(d, prec);
  // general kernel: one arrival ticket per tile; gemm256 split-K: ticket + published-slab count
  size_t n = pl.splits <= 1 ? 0 : (size_t)plan_tiles(d, pl);
  if (const int bm = route_bm(d, prec); bm && g256_splits(d) > 1)
    n = std::max(n, 2 * (size_t)((d.M + bm - 1) / bm) * (d.N / 256));
  return n;
}

int gemm_kstep(Prec prec) { return estep_of(prec); }

extern "C" void spi_debug_gemm_reload_env(void) {
  knobs() = read_knobs();
  conv_wres_reload_env();
  gemm256_reload_env();
  attention_reload_env();
  qkv_attn_reload_env();
}

// The plan gemm() would pick for a conv (tests: which kind runs): out[0..7] = bm, bn, stages,
// splits, halo kind, window kind, waves, k per slice.  precision as spi_ops.h (3 = split).
extern "C" int spi_debug_conv_plan(int precision, int B, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                   int pad, int* out) {
  if (!out || precision < 0 || precision > 3) return 1;
  GemmDesc d;
  d.conv = true;
  d.H = H;
  d.W = W;
  d.Cin = Cin;
  d.KH = KH;
  d.KW = KW;
  d.stride = stride;
  d.pad = pad;
  d.OH = (H + 2 * pad - KH) / stride + 1;
  d.OW = (W + 2 * pad - KW) / stride + 1;
  d.M = B * d.OH * d.OW;
  d.N = Cout;
  d.K = KH * KW * Cin;
  d.Kpad = (d.K + 63) / 64 * 64;
  d.a_split = d.out_split = precision == 3;
  const Prec prec = precision == 0 ? Prec::F32 : precision == 1 ? Prec::F16 : Prec::F16X3;
  const Plan pl = choose_plan(d, prec);
  const int v[8] = {pl.bm, pl.bn, pl.stages, pl.splits, pl.halo, pl.win, pl.nw, pl.k_per_split};
  for (int i = 0; i < 8; ++i) out[i] = v[i];
  return 0;
}

#ifdef SPI_GEMM_STAMPS
extern "C" int spi_debug_gemm_stamps(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif
#ifdef SPI_GEMM_TIMELINE
extern "C" int spi_debug_gemm_timeline(unsigned long long* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_timeline), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
extern "C" void spi_debug_gemm_timeline_enable(int on, hipStream_t) { tl_thread() = on; }
extern "C" int spi_debug_gemm_timeline_clear(void) {
  static unsigned long long zeros[65536 * 8];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_timeline), zeros, sizeof(zeros)) == hipSuccess ? 0 : 1;
}
#endif

namespace {
void check_desc(const GemmDesc& d, Prec prec) {
  if (d.pool_rows && (d.conv || d.pool_rows > 64 || d.M % d.pool_rows))
    throw std::invalid_argument("pooled GEMM: dense A, pool_rows <= 64 dividing M");
  if (d.krep != 1 && (d.krep != 2 || prec != Prec::F16 || d.Kpad % (2 * estep_of(prec)) ||
                      (d.conv && (d.Cin < estep_of(prec) || d.KH * d.KW > 31))))
    throw std::invalid_argument("krep = 2 needs F16, a packed Kpad of whole step pairs and dense or one-tap-per-step A");
  if (prec == Prec::F16X3 && d.a_split && d.conv && (d.Cin < 32 || d.KH * d.KW > 31))
    throw std::invalid_argument("split activations need Cin >= 32 and <= 31 filter taps");
}
}  // namespace

void gemm_pair(const GemmDesc& d0, const GemmPtrs& p0, const GemmDesc& d1, const GemmPtrs& p1, Prec prec,
               hipStream_t s) {
  check_desc(d0, prec);
  check_desc(d1, prec);
  if (prec == Prec::F16X3 && d0.a_split != d1.a_split) {
    gemm(d0, p0, prec, s);
    gemm(d1, p1, prec, s);
    return;
  }
  switch (prec) {
    case Prec::F16:
      launch_pair<(int)Prec::F16>(d0, p0, d1, p1, s);
      break;
    case Prec::F32:
      launch_pair<(int)Prec::F32>(d0, p0, d1, p1, s);
      break;
    case Prec::F16X3:
      if (d0.a_split)
        launch_pair<kF16X3S>(d0, p0, d1, p1, s);
      else
        launch_pair<(int)Prec::F16X3>(d0, p0, d1, p1, s);
      break;
  }
}

void gemm(const GemmDesc& d, const GemmPtrs& p, Prec prec, hipStream_t s) {
  check_desc(d, prec);
  if (d.ln_in_chunks > 0 || d.res_ln_chunks > 0 || d.ln_out) {
    // the fold lives in the dense fp16 kernels' vector epilogue: whole 128-column tiles,
    // 16-byte aligned rows everywhere it reads or writes
    const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    const bool ok = prec == Prec::F16 && !d.conv && !d.pool_rows && d.N % 128 == 0 &&
                    d.ldc % 8 == 0 && al16(p.C) && (!p.bias || al16(p.bias)) &&
                    (!p.res || (d.ldr % 8 == 0 && al16(p.res))) &&
                    (d.ln_in_chunks == 0 || (p.ln.in_stats && p.ln.c1 && al16(p.ln.c1))) &&
                    (d.res_ln_chunks == 0 ||
                     (p.res && (d.res_f32 || d.res_planes) && p.ln.res_stats && al16(p.ln.res_g) && al16(p.ln.res_b))) &&
                    (!d.ln_out || (p.ln.out_stats && (p.ln.c16 ? al16(p.ln.c16) && d.ld16 % 8 == 0 : d.out_planes)));
    if (!ok) throw std::invalid_argument("LayerNorm fold: dense fp16 GEMM, N % 128 == 0, aligned vectors");
  }
  if (d.res_planes || d.out_planes) {
    // two fp16 planes: the F16 dense epilogue, 16-byte aligned rows and plane offset
    if (prec != Prec::F16 || d.conv || d.pool_rows || d.plane % 8 || (d.res_planes && (!p.res || d.res_f32)) ||
        (d.out_planes && (d.out_f32 || d.out_f16)))
      throw std::invalid_argument("two-plane residual / output: dense fp16 GEMM, plane offset a multiple of 8");
  }
  switch (prec) {
    case Prec::F16:
      if (conv_wres_eligible(d, prec, p))
        conv_wres(d, p, s);
      else if (routes_256(d, prec) && (reinterpret_cast<uintptr_t>(p.A) & 15) == 0 &&
               (reinterpret_cast<uintptr_t>(p.W) & 15) == 0)  // 16-byte LDS-DMA pieces
        gemm256(d, p, g256_splits(d), s, route_bm(d, prec), knobs().g128_nbuf,
                knobs().g256_order >= 0 ? knobs().g256_order : d.M > d.N);
      else
        launch<(int)Prec::F16>(d, p, s);
      break;
    case Prec::F32:
      launch<(int)Prec::F32>(d, p, s);
      break;
    case Prec::F16X3:
      // split A relies on one (kh, kw) cell per 32-k step (byte-identical to fp32 addressing)
      if (d.a_split)
        launch<kF16X3S>(d, p, s);
      else
        launch<(int)Prec::F16X3>(d, p, s);
      break;
  }
}

}  // namespace spi
