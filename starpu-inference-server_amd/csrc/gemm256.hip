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
#include "spi_kernels.hpp"

#include <cstdlib>
#include <stdexcept>

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
  int diag;  // diagnostic (SPI_G256_DIAG): 1 every k-tile re-reads k-tile 0 (L2-resident), 2 no DMA after the prologue
};

constexpr int kBufBytes = 65536;  // one k-tile: A 256 x 128 B + B 256 x 128 B
constexpr int kBOff = 32768;

// 8-row piece base (tile row) of piece pc (0..15) of quarter q
__device__ __forceinline__ int quarter_row(int q, int pc) {
  switch (q) {
    case 0: return pc < 8 ? pc * 8 : 128 + (pc - 8) * 8;
    case 1: return 64 * (pc >> 2) + (pc & 3) * 8;
    case 2: return 64 * (pc >> 2) + 32 + (pc & 3) * 8;
    default: return pc < 8 ? 64 + pc * 8 : 192 + (pc - 8) * 8;
  }
}

template <bool AHEAD>
__global__ __launch_bounds__(512) void gemm256_kernel(const G256Args g) {
  __shared__ __attribute__((aligned(16))) char lds[2 * kBufBytes];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // XCD-aware bijective remap: the workgroups one XCD receives get consecutive ids
  const int nwg = g.tiles_m * g.tiles_n, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tm = wgid % g.tiles_m, tn = wgid / g.tiles_m;
  const int m0 = tm * 256, n0 = tn * 256;
  const int KT = g.K >> 6;

  // per-lane DMA sources of each quarter's two pieces (k-tile 0); advance 128 B per k-tile
  const char* src[4][2];
  int dsto[4][2];
  {
    const int rl = lane >> 3, chunk = (lane & 7) ^ rl;  // row within the 8-row piece, swizzled chunk
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int base = quarter_row(q, wave * 2 + j);
        const int r = base + rl;
        if (q == 0 || q == 3) {
          const int m = min(m0 + r, g.M - 1);  // rows past M: a valid row, never stored
          src[q][j] = reinterpret_cast<const char*>(g.A + (size_t)m * g.lda) + chunk * 16;
          dsto[q][j] = base * 128;
        } else {
          src[q][j] = reinterpret_cast<const char*>(g.W + (size_t)(n0 + r) * g.ldw) + chunk * 16;
          dsto[q][j] = kBOff + base * 128;
        }
      }
  }
  auto stage = [&](int q, int kt) {
    char* buf = lds + (kt & 1) * kBufBytes;
    if (g.diag == 2 && kt > 0) return;
    const int kofs = g.diag == 1 ? 0 : kt * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[q][j] + kofs),
                                       (lds_ptr_t)(buf + dsto[q][j]), 16, 0, 0);
  };

  floatx4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  half8 fa[2][2][4];  // [m half][kk][i]
  half8 fb[2][2][2];  // [n half][kk][j]

  auto rd = [&](const char* img, int row, int c) -> half8 {
    return *reinterpret_cast<const half8*>(img + row * 128 + ((c ^ (row & 7)) << 4));
  };
  auto read_a = [&](const char* buf, int mq) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[mq][kk][i] = rd(buf, 128 * wr + 64 * mq + 16 * i + fr, kk * 4 + fq);
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

  // prologue: k-tile 0 into buffer 0
#pragma unroll
  for (int q = 0; q < 4; ++q) stage(q, 0);

  if constexpr (AHEAD) {
    // Fragment reads one phase ahead of their MFMAs: phase p's barrier retires the
    // quarter the NEXT phase's fragments come from, its reads go out, then its own
    // MFMAs run on registers read a phase earlier, so LDS latency hides behind
    // MFMAs.  Reads: phase 0 B_n1(t) [Q2], phase 1 A_m1(t) [Q3], phase 3 A_m0, B_n0
    // of t + 1 [Q0, Q1]; phase p still stages Q_p(t + 1).  Each quarter is in flight
    // two phases or more; every wait is vmcnt(2) (last tile: 2, 0).
    asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    read_a(lds, 0);
    read_b(lds, 0);
    auto ktile = [&](int kt, auto last_c) {
      constexpr bool LAST = decltype(last_c)::value;
      const char* buf = lds + (kt & 1) * kBufBytes;
      asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
      read_b(buf, 1);
      if constexpr (!LAST) stage(0, kt + 1);
      mma(0, 0);
      if constexpr (LAST)
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
      read_a(buf, 1);
      if constexpr (!LAST) stage(1, kt + 1);
      mma(0, 1);
      if constexpr (!LAST) stage(2, kt + 1);
      mma(1, 0);
      if constexpr (!LAST) {
        asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
        const char* nbuf = lds + ((kt + 1) & 1) * kBufBytes;
        read_a(nbuf, 0);
        read_b(nbuf, 0);
        stage(3, kt + 1);
      }
      mma(1, 1);
    };
    for (int kt = 0; kt < KT - 1; ++kt) ktile(kt, std::false_type{});
    ktile(KT - 1, std::true_type{});
  } else {
    // one k-tile; the vmcnt before phases 0 / 1 / 2: 4, 4, 4 (the last tile 4, 2, 0)
    auto ktile = [&](int kt, auto last_c) {
      constexpr bool LAST = decltype(last_c)::value;
      const char* buf = lds + (kt & 1) * kBufBytes;
      // phase 0: quadrant (0, 0)
      asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      read_a(buf, 0);
      read_b(buf, 0);
      if constexpr (!LAST) stage(0, kt + 1);
      mma(0, 0);
      // phase 1: quadrant (0, 1)
      if constexpr (LAST)
        asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      read_b(buf, 1);
      if constexpr (!LAST) stage(1, kt + 1);
      mma(0, 1);
      // phase 2: quadrant (1, 0)
      if constexpr (LAST)
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      read_a(buf, 1);
      if constexpr (!LAST) stage(2, kt + 1);
      mma(1, 0);
      // phase 3: quadrant (1, 1) from registers
      if constexpr (!LAST) stage(3, kt + 1);
      mma(1, 1);
    };
    for (int kt = 0; kt < KT - 1; ++kt) ktile(kt, std::false_type{});
    ktile(KT - 1, std::true_type{});
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
    if (act == Act::Gelu) return 0.5f * y * (1.f + erff(y * 0.70710678118654752f));
    return y;
  };
  if (!g.vec_ok) {
    float bv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) bv[b] = g.bias ? g.bias[n0 + 64 * wc + 16 * b + fr] : 0.f;
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = m0 + 128 * wr + 16 * a + 4 * fq + v;
        if (m >= g.M) continue;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int n = n0 + 64 * wc + 16 * b + fr;
          float y = acc[a][b][v] + bv[b];
          if (g.res) {  // residual before the activation, as the general kernel (conv + BN + x -> ReLU)
            const size_t ri = (size_t)m * g.ldr + n;
            y += g.res_f32 ? static_cast<const float*>(g.res)[ri]
                           : static_cast<float>(static_cast<const _Float16*>(g.res)[ri]);
          }
          y = finish(y);
          const size_t ci = (size_t)m * g.ldc + n;
          if (g.out_f32)
            static_cast<float*>(g.C)[ci] = y;
          else
            static_cast<_Float16*>(g.C)[ci] = static_cast<_Float16>(y);
        }
      }
    return;
  }
  float* T = reinterpret_cast<float*>(lds);
  const int cg = tid & 31, r0 = tid >> 5;  // 8-column group, first row of this thread
  const int nb = n0 + 8 * cg;
  float bias8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias8[e] = g.bias ? g.bias[nb + e] : 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();  // the k-loop's last reads / the previous round's walk are done
    if (wr == h) {
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int row = 16 * a + 4 * fq + v;
            const int col = (64 * wc + 16 * b + fr) ^ (((row >> 2) & 3) << 4);
            T[row * 256 + col] = acc[a][b][v];
          }
    }
    __syncthreads();
#pragma unroll 2
    for (int pass = 0; pass < 8; ++pass) {
      const int row = r0 + 16 * pass;
      const int m = m0 + 128 * h + row;
      if (m >= g.M) continue;
      const float* src = T + row * 256 + ((8 * cg) ^ (((row >> 2) & 3) << 4));
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(src);
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(src + 4);
      float y[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] = x0[e] + bias8[e];
        y[e + 4] = x1[e] + bias8[e + 4];
      }
      if (g.res) {
        const size_t ri = (size_t)m * g.ldr + nb;
        if (g.res_f32) {
          const floatx4 q0 = *reinterpret_cast<const floatx4*>(static_cast<const float*>(g.res) + ri);
          const floatx4 q1 = *reinterpret_cast<const floatx4*>(static_cast<const float*>(g.res) + ri + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            y[e] += q0[e];
            y[e + 4] += q1[e];
          }
        } else {
          const half8 q = *reinterpret_cast<const half8*>(static_cast<const _Float16*>(g.res) + ri);
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] += static_cast<float>(q[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = finish(y[e]);
      const size_t ci = (size_t)m * g.ldc + nb;
      if (g.out_f32) {
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

}  // namespace

bool gemm256_eligible(const GemmDesc& d, Prec prec, int min_tiles) {
  if (min_tiles <= 0 || prec != Prec::F16 || d.conv || d.krep != 1 || d.a_split || d.out_split || d.pool_rows ||
      d.out_f16)
    return false;
  if (d.N % 256 || d.K % 64 || d.Kpad != d.K || d.lda % 8 || d.M < 1) return false;
  return (d.M + 255) / 256 * (d.N / 256) >= min_tiles;
}

void gemm256(const GemmDesc& d, const GemmPtrs& p, hipStream_t s) {
  if (d.N % 256 || d.K % 64 || d.Kpad != d.K) throw std::invalid_argument("gemm256: N % 256, K % 64, Kpad == K");
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
  g.tiles_m = (d.M + 255) / 256;
  g.tiles_n = d.N / 256;
  g.act = static_cast<int>(d.act);
  g.res_f32 = d.res_f32;
  g.out_f32 = d.out_f32;
  static const int diag = [] {
    const char* e = std::getenv("SPI_G256_DIAG");
    return e && *e ? std::atoi(e) : 0;
  }();
  g.diag = diag;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  g.vec_ok = d.ldc % 8 == 0 && al16(p.C) && (!p.res || (d.ldr % 8 == 0 && al16(p.res))) ? 1 : 0;
  static const int sched = [] {
    const char* e = std::getenv("SPI_G256_SCHED");  // 1: fragment reads a phase ahead (default), 0: in-phase
    return e && *e ? std::atoi(e) : 1;
  }();
  if (sched)
    hipLaunchKernelGGL(gemm256_kernel<true>, dim3(g.tiles_m * g.tiles_n), dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL(gemm256_kernel<false>, dim3(g.tiles_m * g.tiles_n), dim3(512), 0, s, g);
}

}  // namespace spi
