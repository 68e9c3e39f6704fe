// Op-level C entry points (include/spi_ops.h): the individual kernels behind
// the forward passes, for kernel-level parity tests and micro-benchmarks.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "../../include/spi_ops.h"
#include "pack.hpp"
#include "spi_kernels.hpp"

extern "C" void spi_set_last_error(const char* msg);

namespace {

constexpr size_t kZeroBytes = 256;
constexpr size_t kTickets = 16384;
constexpr size_t kSlabFloats = (size_t)16 << 20;  // 64 MiB of split-K slabs (gemm256 at ViT-L FFN2: 40 MiB)

bool prec_of(int32_t p, spi::Prec* out) {
  if (p == 0) *out = spi::Prec::F32;
  else if (p == 1) *out = spi::Prec::F16;
  else if (p == 2 || p == 3) *out = spi::Prec::F16X3;  // 3: split activations
  else return false;
  return true;
}

constexpr int32_t kSplitPrecision = 3;

int fail(const std::string& m) {
  spi_set_last_error(m.c_str());
  return 1;
}

int check_launch() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

spi::GemmPtrs scratch(void* ws) {
  spi::GemmPtrs p;
  char* base = static_cast<char*>(ws);
  p.zeros = base;
  p.counters = reinterpret_cast<int*>(base + kZeroBytes);
  p.partial = reinterpret_cast<float*>(base + kZeroBytes + kTickets * sizeof(int));
  return p;
}

}  // namespace

extern "C" {

size_t spi_op_packed_bytes(int32_t precision, int32_t N, int32_t K, int32_t* Npad, int32_t* Kpad) {
  spi::Prec p;
  if (!prec_of(precision, &p) || N <= 0 || K <= 0) return 0;
  const int np = spi::round_up_to(N, 128), kp = spi::round_up_to(K, 64);
  if (Npad) *Npad = np;
  if (Kpad) *Kpad = kp;
  return spi::packed_bytes(p, np, kp);
}

int spi_op_pack_weight(int32_t precision, const float* w, int32_t N, int32_t K, void* dst) {
  spi::Prec p;
  if (!prec_of(precision, &p) || !w || !dst || N <= 0 || K <= 0) return fail("invalid pack arguments");
  const int np = spi::round_up_to(N, 128), kp = spi::round_up_to(K, 64);
  spi::pack_matrix_into(static_cast<char*>(dst), N, K, np, kp, p,
                        [&](int n, int k) { return w[(size_t)n * K + k]; });
  return 0;
}

size_t spi_op_workspace_bytes(void) { return kZeroBytes + kTickets * sizeof(int) + kSlabFloats * sizeof(float); }

int spi_op_gemm(int32_t precision, const void* A, int32_t M, int32_t K, int32_t lda, const void* W, int32_t N,
                const float* bias, const void* residual, int32_t res_f32, int32_t ldr, void* C, int32_t out_f32,
                int32_t ldc, int32_t act, void* workspace, void* stream) {
  spi::Prec p;
  if (!prec_of(precision, &p) || !A || !W || !C || !workspace || M <= 0 || N <= 0 || K <= 0 || lda < K ||
      ldc < N || act < 0 || act > 2)
    return fail("invalid gemm arguments");
  spi::GemmDesc d;
  d.M = M;
  d.N = N;
  d.K = K;
  d.Kpad = spi::round_up_to(K, 64);
  d.lda = lda;
  d.ldc = ldc;
  d.ldr = ldr;
  d.act = static_cast<spi::Act>(act);
  d.out_f32 = out_f32 != 0;
  d.res_f32 = res_f32 != 0;
  if (precision == kSplitPrecision) {
    if (K % 32 || N % 32 || lda % 32 || ldc % 32 || out_f32 || res_f32 || (residual && ldr % 32))
      return fail("split gemm needs K, N and strides multiples of 32, no fp32 operands");
    d.a_split = d.out_split = true;
  }
  if (spi::gemm_partial_floats(d, p) > kSlabFloats || spi::gemm_counter_slots(d, p) > kTickets)
    return fail("gemm too large for the op workspace");
  spi::GemmPtrs ptrs = scratch(workspace);
  ptrs.A = A;
  ptrs.W = W;
  ptrs.bias = bias;
  ptrs.res = residual;
  ptrs.C = C;
  spi::gemm(d, ptrs, p, static_cast<hipStream_t>(stream));
  return check_launch();
}

int spi_op_conv2d(int32_t precision, const void* x, int32_t B, int32_t H, int32_t W, int32_t Cin, const void* Wp,
                  int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad, const float* bias,
                  const void* residual, void* y, int32_t act, void* workspace, void* stream) {
  spi::Prec p;
  const int min_cin = precision == 1 ? 8 : 4;  // one 16-byte chunk: 8 fp16 or 4 fp32
  if (!prec_of(precision, &p) || !x || !Wp || !y || !workspace || B <= 0 || Cin < min_cin ||
      (Cin & (Cin - 1)) || Cout <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0 || act < 0 || act > 2)
    return fail("invalid conv arguments");
  spi::GemmDesc d;
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
  if (d.OH <= 0 || d.OW <= 0) return fail("empty conv output");
  d.M = B * d.OH * d.OW;
  d.N = Cout;
  d.K = KH * KW * Cin;
  d.Kpad = spi::round_up_to(d.K, 64);
  d.ldc = Cout;
  d.ldr = Cout;
  d.act = static_cast<spi::Act>(act);
  // W_packed comes from spi_op_pack_weight (spi_ops.h), which writes the image rows
  d.w_image = spi::packed_has_wres_image(p, Cout, d.K, spi::round_up_to(Cout, 128), d.Kpad);
  if (precision == kSplitPrecision) {
    if (Cin < 32 || Cout % 32 || KH * KW > 31)
      return fail("split conv needs Cin >= 32, Cout a multiple of 32 and <= 31 filter taps");
    d.a_split = d.out_split = true;
  }
  if (spi::gemm_partial_floats(d, p) > kSlabFloats || spi::gemm_counter_slots(d, p) > kTickets)
    return fail("conv too large for the op workspace");
  spi::GemmPtrs ptrs = scratch(workspace);
  ptrs.A = x;
  ptrs.W = Wp;
  ptrs.bias = bias;
  ptrs.res = residual;
  ptrs.C = y;
  spi::gemm(d, ptrs, p, static_cast<hipStream_t>(stream));
  return check_launch();
}

int spi_op_avgpool_fc(int32_t precision, const void* x, int32_t B, int32_t HW, int32_t C, const void* W, int32_t N,
                      const float* bias, float* y, int32_t act, void* workspace, void* stream) {
  spi::Prec p;
  if (!prec_of(precision, &p) || !x || !W || !y || !workspace || B <= 0 || HW <= 0 || HW > 64 || C <= 0 ||
      N <= 0 || act < 0 || act > 2)
    return fail("invalid avgpool_fc arguments");
  if (precision == kSplitPrecision && C % 32) return fail("split avgpool_fc needs C a multiple of 32");
  spi::GemmDesc d;
  d.M = B * HW;
  d.N = N;
  d.K = C;
  d.Kpad = spi::round_up_to(C, 64);
  d.lda = C;
  d.ldc = N;
  d.ldr = N;
  d.act = static_cast<spi::Act>(act);
  d.out_f32 = true;
  d.pool_rows = HW;
  d.a_split = precision == kSplitPrecision;
  spi::GemmPtrs ptrs = scratch(workspace);
  ptrs.A = x;
  ptrs.W = W;
  ptrs.bias = bias;
  ptrs.C = y;
  spi::gemm(d, ptrs, p, static_cast<hipStream_t>(stream));
  return check_launch();
}

size_t spi_op_stem_pool_bytes(void) { return spi::stem_pool_bytes(); }

int spi_op_stem_pool_pack(const float* w, void* dst) {
  if (!w || !dst) return fail("invalid stem_pool pack arguments");
  spi::stem_pool_pack(w, static_cast<_Float16*>(dst));
  return 0;
}

int spi_op_stem_pool(int32_t precision, const float* x, int32_t B, int32_t H, int32_t W, const void* Wp,
                     const float* bias, void* y, int32_t rows_per_block, void* stream) {
  if (precision < 1 || precision > 4 || !x || !Wp || !bias || !y || B <= 0 || H <= 0 || W <= 0 ||
      rows_per_block < 0 || rows_per_block > 2)
    return fail("invalid stem_pool arguments");
  if ((W + 6 - 7) / 2 + 1 > spi::kStemPoolMaxOW) return fail("stem_pool: image wider than 224");
  // stem_pool's lo: 0 fp16 weights, 1 hi + lo weights on the fp16 image (the model's fp16m stem),
  // 2 hi + lo weights on the split image (fp32-grade; fp16x3 and the split output)
  const int lo = precision == 1 ? 0 : precision == 2 ? 1 : 2;
  spi::stem_pool(x, Wp, bias, y, B, H, W, lo, precision == 3, rows_per_block, static_cast<hipStream_t>(stream));
  return check_launch();
}

int spi_op_attention(int32_t precision, const void* qkv, const float* mask_bias, void* ctx, int32_t B, int32_t S,
                     int32_t heads, float scale, void* stream) {
  if ((precision != 0 && precision != 1) || !qkv || !ctx || B <= 0 || S <= 0 || heads <= 0)
    return fail("invalid attention arguments");
  spi::attention(qkv, mask_bias, ctx, B, S, heads, 64, scale, precision == 1, static_cast<hipStream_t>(stream));
  return check_launch();
}

int spi_op_layernorm(int32_t precision, const float* x, const float* g, const float* b, float* yf, void* yt,
                     int32_t rows, int32_t D, float eps, void* stream) {
  if (precision < 0 || precision > 2 || !x || !g || !b || rows <= 0 || D <= 0 || D > 1024 || (!yf && !yt))
    return fail("invalid layernorm arguments");
  spi::layernorm(x, D, g, b, yf, yt, D, rows, D, eps, precision == 1, static_cast<hipStream_t>(stream));
  return check_launch();
}

}  // extern "C"
