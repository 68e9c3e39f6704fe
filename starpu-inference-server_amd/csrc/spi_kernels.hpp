// Internal launch interface of the HIP/CDNA4 kernels (gfx950 only).
// Every launcher enqueues on the given stream and never synchronises, so a
// forward pass can be captured into a hipGraph (cdna_hip_programming.md G9).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <vector>

namespace spi {

// Every kernel launch goes through SPI_LAUNCH.  While a forward is profiled
// (Model::launch_table) each launch is recorded with its kernel and grid, so a
// rocprofv3 kernel trace of graph-replayed forwards -- which knows kernels and grids,
// not ops -- can be attributed to the forward's ops (tools/trace_ops.py --launches).
// Outside profiling the cost is one thread-local pointer test per launch.
struct LaunchRec {
  const char* kernel;  // __PRETTY_FUNCTION__ of kernel_id<F>: "... [F = &spi::...::name<args>]"
  unsigned gx, gy, gz, block;
};
std::vector<LaunchRec>*& launch_log();
template <auto F>
inline const char* kernel_id() {
  return __PRETTY_FUNCTION__;
}
#define SPI_LAUNCH(F, G, B, SH, S, ...)                                                                  \
  do {                                                                                                   \
    if (auto* spi_log_ = ::spi::launch_log())                                                            \
      spi_log_->push_back({::spi::kernel_id<F>(), dim3(G).x, dim3(G).y, dim3(G).z, dim3(B).x});          \
    hipLaunchKernelGGL(F, G, B, SH, S, __VA_ARGS__);                                                     \
  } while (0)

enum class Act : int { None = 0, Relu = 1, Gelu = 2 };

// Contraction precision.  F16X3 = split fp16 (fp32 activations, hi/lo fp16
// operands, three MFMAs per fragment): fp32-grade results at the fp16 rate.
enum class Prec : int { F32 = 0, F16 = 1, F16X3 = 2 };

// C[M,N] = act(A[M,K] . W[N,K]^T + bias[N] + residual[M,N])
//
// A is either a dense row-major activation (lda) or, for conv-as-implicit-GEMM,
// an NHWC image gathered on the fly: row m = (img, oh, ow), column
// k = (kh*KW + kw)*Cin + c.  W is pre-packed [Npad][Kpad] (K contiguous,
// zero padded), so both MFMA operands are K-contiguous 16-byte chunks.  For
// Prec::F16X3 each W row is Kpad/32 blocks of [32 hi fp16 | 32 lo fp16].
struct GemmDesc {
  int M = 0, N = 0, K = 0;  // logical sizes
  int Kpad = 0;             // W row stride (multiple of 64)
  size_t wplane = 0;        // elements between the hi and lo weight planes (F16X3)
  int lda = 0;              // dense A row stride (elements)
  int ldc = 0;              // C row stride (elements)
  int ldr = 0;              // residual row stride (elements)
  // conv geometry (conv == true)
  bool conv = false;
  int H = 0, W = 0, Cin = 0, OH = 0, OW = 0, KH = 1, KW = 1, stride = 1, pad = 0;
  Act act = Act::None;
  bool out_f32 = false;  // C is float (else the compute type)
  bool out_f16 = false;  // C is fp16 although the mode's output type is fp32 (F16X3, plain stores)
  bool res_f32 = false;  // residual is float (else the compute type)
  // F16X3 activation split layout: per row, blocks of 32 elements stored as
  // [32 hi fp16 | 32 lo fp16] (128 bytes, the size of 32 fp32), hi = fp16(x),
  // lo = fp16(x - hi).  a_split: A and the residual are split (conv Cin >= 32);
  // out_split: C is written split.
  bool a_split = false;
  bool out_split = false;
  // Fused global average pool + linear layer (ResNet avgpool + fc): A holds
  // pool_rows consecutive rows (pixels) per image; output row b of C is
  // act(mean over image b's rows of A . W^T + bias).  Linearity lets the GEMM
  // run over every pixel and average its own C tile (64 x 64 tiles, one image
  // per tile row, pool_rows <= 64).  M = images x pool_rows.
  int pool_rows = 0;
  // krep = 2 (F16, dense or one-tap-per-step conv A): the packed W holds two k-steps per A
  // k-step -- fp16(w) then fp16(w - fp16(w)) for the same 64 k-values -- and each A k-step is
  // staged twice, so one launch accumulates x.w_hi + x.w_lo (~22-bit weights on fp16 MFMAs).
  // Kpad is the packed (W) row length; K stays the logical A length.
  int krep = 1;
  // W came from pack_matrix_into of an fp16 64 x 576 matrix, whose padding rows 64..127
  // hold the weight-resident conv's LDS image (pack.hpp); conv_wres requires it.
  bool w_image = false;
  // LayerNorm folded across GEMMs (transformer fp16 path; dense F16 A, the
  // vector epilogue only).  Row statistics travel as per-64-column-chunk partials
  // (mean, M2) -- [rows][chunks][2] fp32 -- combined by Chan's formula where they are used.
  //  ln_in_chunks > 0: A holds the rows x BEFORE a LayerNorm (an fp16 copy), W was packed
  //    with the gain folded in (W' = W diag(gamma)), and the epilogue applies
  //    y = rstd[m] * (acc - mean[m] * c1[n]) + bias[n] (bias = b + W beta, c1 = W' 1).
  //  res_ln_chunks > 0: the residual is LN(R) computed on the fly from the fp32 rows R and
  //    their statistics: (R - mean) * rstd * g + b (a post-LN block's input).
  //  ln_out: write the output rows' chunk statistics (N / 64 chunks) and an fp16 copy of
  //    the output (C16, row stride ld16) for the next, folding GEMM.
  int ln_in_chunks = 0;
  float ln_in_eps = 0.f;
  int res_ln_chunks = 0;
  float res_ln_eps = 0.f;
  bool ln_out = false;
  int ld16 = 0;
  // Two-plane fp16 residual stream (round 6, the transformer fold path): a row-major [rows][ld]
  // tensor x kept as hi = fp16(x) at the pointer and lo = fp16(x - hi) `plane` elements further on
  // -- ~22-bit values in the bytes of fp32, and the hi plane is already the fp16 operand the next
  // folding GEMM reads, so a producer writes no separate fp16 copy (LnPtrs::c16 may be null).
  // res_planes: the residual is such a pair; out_planes: C is written as one.
  bool res_planes = false;
  bool out_planes = false;
  size_t plane = 0;
};

// Pointers of the LayerNorm fold (GemmDesc::ln_in_chunks / res_ln_chunks / ln_out).
struct LnPtrs {
  const float* in_stats = nullptr;   // A rows' chunk statistics
  const float* c1 = nullptr;         // [N] per-column sum of the folded weights
  const float* res_stats = nullptr;  // residual rows' chunk statistics
  const float* res_g = nullptr;      // residual LayerNorm gain / bias
  const float* res_b = nullptr;
  float* out_stats = nullptr;        // output rows' chunk statistics
  _Float16* c16 = nullptr;           // fp16 copy of the output (none with GemmDesc::out_planes)
};

struct GemmPtrs {
  const void* A = nullptr;
  const void* W = nullptr;
  const float* bias = nullptr;
  const void* res = nullptr;
  void* C = nullptr;
  float* partial = nullptr;  // split-K slabs (gemm_partial_floats)
  int* counters = nullptr;   // split-K arrival tickets, zero-initialised (gemm_counter_slots)
  const void* zeros = nullptr;  // >= 256 zero bytes (padded / out-of-range chunks; conv_wres: a null bias)
  LnPtrs ln;
};

// Workspace needed by a GEMM with the chosen split-K (0 when not split).
size_t gemm_partial_floats(const GemmDesc& d, Prec prec);
size_t gemm_counter_slots(const GemmDesc& d, Prec prec);
// k-values per staged step (W rows must be padded to a multiple of it).
int gemm_kstep(Prec prec);
void gemm(const GemmDesc& d, const GemmPtrs& p, Prec prec, hipStream_t s);
// Two independent problems of one precision in a single launch when their plans
// share a kernel instance (else two launches); problem 1's split-K slabs and
// tickets follow problem 0's (size the workspace for both: gemm_partial_floats /
// gemm_counter_slots summed).
void gemm_pair(const GemmDesc& d0, const GemmPtrs& p0, const GemmDesc& d1, const GemmPtrs& p1, Prec prec,
               hipStream_t s);

// 8-wave phased fp16 GEMM (gemm256.hip), tiles of bm x 256 (bm = 256 or 128) for the dense
// F16 contractions; gemm() routes a desc to it when gemm256_eligible (N % 256 == 0,
// K % 64 == 0, at least min_tiles tiles of bm x 256; routing rule in gemm.hip).
bool gemm256_eligible(const GemmDesc& d, Prec prec, int min_tiles, int bm = 256);
// Split-K slices for a gemm256 problem: 1 with >= target tiles, else enough slices of >= 16
// k-tiles (at most 4, at most max_split when > 0) to reach ~target workgroups (ViT-L's
// N = 1024 GEMMs: 52 tiles -> FFN2 3 slices, out-proj none).
int gemm256_splits(const GemmDesc& d, int target, int max_split, int bm = 256);
void gemm256(const GemmDesc& d, const GemmPtrs& p, int splits, hipStream_t s, int bm = 256, int nbuf = 2,
             int n_fast = 0);
void gemm256_reload_env();  // no knobs left (kept for spi_debug_gemm_reload_env)

// Fused QKV projection + attention for S <= 128 (qkv_attn.hip): one workgroup per (sequence,
// head) runs the head's q | k | v GEMM (A rows lda apart, packed W rows ldw apart; with
// ln_stats: the LayerNorm consumer fold, ln_fold.hpp) and the attention on the LDS-resident
// result, writing ctx [B S][heads 64] fp16.
bool qkv_attention_eligible(int S, int heads, int hd, int K, int kpad, int krep, int lda, int ldw);
void qkv_attention(const void* A, int lda, const void* W, int ldw, const float* bias, const float* ln_stats,
                   const float* c1, int ln_chunks, float ln_eps, const float* mask_bias, void* ctx, int B, int S,
                   int heads, float scale, hipStream_t s);

// Weight-resident 3x3/s1/p1 conv, 64 -> 64 channels, fp16 NHWC (conv_wres.hip): the
// folded weights stay in LDS while a workgroup walks bands of output rows; gemm()
// routes an eligible desc to it (SPI_CONV_WRES=0: never).
bool conv_wres_eligible(const GemmDesc& d, Prec prec, const GemmPtrs& p);
void conv_wres(const GemmDesc& d, const GemmPtrs& p, hipStream_t s);
void conv_wres_reload_env();
void attention_reload_env();  // SPI_ATTN_WHOLE
void qkv_attn_reload_env();   // SPI_QKV_HP

// NCHW fp32 image -> NHWC (compute type) with channels zero-padded to cpad.
void ingest_nchw(const float* x, void* y, int B, int C, int H, int W, int cpad,
                 bool f16, hipStream_t s);
// Fused ResNet stem (stem.hip): NCHW fp32 image [B][3][H][W] -> 7x7/s2/p3 conv
// (64 output channels, folded BN) + ReLU -> 3x3/s2/p1 max pool -> NHWC [B][PH][PW][64]:
// fp16 (split false) or the split layout (split true, needs lo).  lo: hi + lo
// weights and image (three fp16 MFMAs per fragment, fp32-grade); else fp16 only.
// w: stem_pool_bytes() from stem_pool_pack(); pr: 0 auto, 1 / 2 pooled rows per 4-wave workgroup.
constexpr int kStemPoolMaxOW = 112;  // stem output width bound (images up to 224)
constexpr size_t stem_pool_bytes() { return (size_t)2 * 64 * 24 * 8 * sizeof(_Float16); }
void stem_pool_pack(const float* w_folded /* [64][3][7][7] */, _Float16* dst);
// lo: 0 fp16 weights, 1 hi + lo weights on the fp16 image (fp16m), 2 hi + lo weights on the split
// image (fp16x3; required for the split output)
void stem_pool(const float* x, const void* w, const float* bias, void* y, int B, int H, int W, int lo,
               bool split, int pr, hipStream_t s);
// 3x3/s2/p1 max pool on NHWC.
void maxpool_nhwc(const void* x, void* y, int B, int H, int W, int C, int OH,
                  int OW, int k, int stride, int pad, bool f16, hipStream_t s);
// Global average pool NHWC [B,HW,C] -> [B,C] (compute type).
void avgpool_nhwc(const void* x, void* y, int B, int HW, int C, bool f16,
                  hipStream_t s, bool out_f32 = false);  // out_f32: fp16 in, fp32 out
// The same two on F16X3 split activations (GemmDesc::a_split layout, C % 32 == 0):
// max pool split -> split, average pool split -> fp32 [B,C].
void maxpool_nhwc_split(const void* x, void* y, int B, int H, int W, int C, int OH,
                        int OW, int k, int stride, int pad, hipStream_t s);
void avgpool_nhwc_split(const void* x, float* y, int B, int HW, int C, hipStream_t s);
// Row LayerNorm over D: y = LN(x) * g + b.  x fp32 [rows, ldx]; writes fp32
// (yf, may alias x) and/or compute-type (yt) outputs.
void layernorm(const float* x, int ldx, const float* g, const float* b,
               float* yf, void* yt, int ldy, int rows, int D, float eps, bool f16,
               hipStream_t s);
// BERT embeddings: LN(word[ids] + pos[s] + type[0]) -> fp32 + compute type; with a mask, each
// token's additive attention bias too (mask_to_bias's, one launch fewer per forward).
void bert_embed(const int64_t* ids, const float* word, const float* pos,
                const float* type0, const float* g, const float* b, float* yf,
                void* yt, int B, int S, int D, int vocab, float eps, bool f16,
                hipStream_t s, const int64_t* mask = nullptr, float* mask_bias = nullptr);
// int64 attention mask [B,S] -> additive fp32 bias [B,S] (0 or finfo.min).
void mask_to_bias(const int64_t* mask, float* bias, int n, hipStream_t s);
// ViT: NCHW fp32 image -> patch rows [B*P, C*ps*ps] (compute type).
void patchify(const float* x, void* y, int B, int C, int H, int W, int ps,
              bool f16, hipStream_t s);
// ViT: x[b, 0] = cls + pos[0]; x[b, 1+p] = patch[b, p] + pos[1+p]  (fp32).
void vit_assemble(const float* patches, const float* cls, const float* pos,
                  float* x, int B, int P, int D, hipStream_t s);
// The same into the two-plane residual stream (GemmDesc::res_planes: hi at xh, lo plane elements
// on) plus, when stats is not null, each row's per-64-column chunk statistics [rows][D / 64][2]
// (ln_fold.hpp).
void vit_assemble_planes(const float* patches, const float* cls, const float* pos, _Float16* xh, size_t plane,
                         float* stats, int B, int P, int D, hipStream_t s);
// layernorm() over rows held in two fp16 planes (x = hi + lo), D <= 1024.
void layernorm_planes(const _Float16* xh, size_t plane, int ldx, const float* g, const float* b, float* yf, void* yt,
                      int ldy, int rows, int D, float eps, bool f16, hipStream_t s);
// Gather rows: y[i] = x[i * stride_rows] (fp32 -> compute type) for CLS pooling.
void gather_rows(const float* x, void* y, int rows, int stride_rows, int D,
                 bool f16, hipStream_t s);
// y = x * scale + shift, fp32 elementwise (AFFINE toy family).
void affine(const float* x, float* y, size_t n, float scale, float shift,
            hipStream_t s);

// Multi-head attention over a packed qkv buffer [B*S, 3*D] (compute type):
// ctx[b*S+i, h*hd:(h+1)*hd] = softmax(q k^T * scale + mask_bias[b]) v.
// mask_bias: fp32 [B, S] additive bias or nullptr.
void attention(const void* qkv, const float* mask_bias, void* ctx, int B, int S,
               int heads, int hd, float scale, bool f16, hipStream_t s);

}  // namespace spi
