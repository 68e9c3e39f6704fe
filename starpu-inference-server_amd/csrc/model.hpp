// Device-resident model replica: the MI355X replacement for the per-device
// TorchScript clones of inference_runner.cpp:251-275.  Weights are recognised
// by their torchvision / HF parameter names, BN is folded into the convs, every
// contraction weight is packed [Npad][Kpad] in the compute type, and the whole
// replica lives in one HBM blob.  Activations live in per-stream workspaces
// (one per StarPU worker stream: replicas are shared read-only by the workers
// of a device, starpu_setup.cpp:725-778 / docs/server_guide.md:116).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/spi_codelet.h"
#include "spi_kernels.hpp"

namespace spi {

struct ConvW {
  size_t w = 0, b = 0;  // blob offsets (packed weight, fp32 bias)
  int cout = 0, cin = 0, cin_pad = 0, kh = 1, kw = 1, stride = 1, pad = 0;
  int kpad = 0, npad = 0;
  size_t wplane = 0;
  Prec prec = Prec::F16;  // packing / contraction precision of this conv
  int krep = 1;           // 2: hi + lo weight steps per A step (GemmDesc::krep; SPI_PREC_F16M)
  bool w_image = false;   // the packed rows 64..127 hold conv_wres's LDS image (GemmDesc::w_image)
};

struct LinearW {
  size_t w = 0, b = 0;
  size_t c1 = 0;  // LayerNorm fold (GemmDesc::ln_in_chunks): sum_k W'[n][k] of the folded weights, else 0
  int n = 0, k = 0, kpad = 0, npad = 0;
  size_t wplane = 0;
  bool has_bias = true;
  Prec prec = Prec::F16;
  int krep = 1;
};

struct LnW {
  size_t g = 0, b = 0;
};

struct ResBlock {
  ConvW c1, c2, c3;  // c3 only for bottleneck
  bool has_ds = false;
  ConvW ds;  // SPI_PREC_F16M: packed hi + lo (krep = 2), fp32 output
};

struct TfLayer {  // BERT (post-LN) / ViT (pre-LN) encoder layer
  LinearW qkv, out, ff1, ff2;
  LnW ln1, ln2;
};

struct Workspace;

class Model {
 public:
  Model(int device, const spi_model_config& cfg, const spi_named_tensor* params, int n);
  ~Model();

  int device() const { return device_; }
  int family() const { return family_; }
  bool f16() const { return f16_; }
  int max_batch() const { return max_batch_; }
  size_t weight_bytes() const { return blob_bytes_; }
  uint64_t weight_digest() const { return digest_; }
  const std::string& describe() const { return desc_; }
  double flops(int64_t batch) const;
  void set_graphs(bool on) { graphs_ = on; }

  // Validates the task's I/O against the replica; throws std::runtime_error
  // with the reference's message wording on mismatch.
  void check_io(const spi_codelet_args& a, const size_t* in_bytes,
                const size_t* out_bytes) const;
  // Enqueue the forward on `s`; never synchronises.
  // S: BERT sequence length (ignored otherwise); n: AFFINE element count.
  void forward(hipStream_t s, int batch, int S, size_t n, const void* const* in, void* const* out);
  // Allocate the stream's workspace and capture its (batch, S, mask) graph ahead of serving.
  void warmup(hipStream_t s, int batch, int S, bool mask);

  // Per-op profile of one forward: each launch bracketed by hipEvents on `s`.
  struct OpRecord {
    std::string name;
    double flops;
    double bytes;
    hipEvent_t start, stop;
    int reps;  // launches between start and stop (profile_op)
    std::vector<LaunchRec> launches;  // the op's kernel launches (SPI_LAUNCH), in order
  };
  int profile(hipStream_t s, int batch, int S, const void* const* in, void* const* out, float* ms,
              double* flops, double* bytes, char* names, int name_len, int max_ops);
  // One profiled eager forward as text, one line per kernel launch:
  // "op_index\top_name\tkernel\tgrid_x\tgrid_y\tgrid_z\tblock\n" (spi_model_launch_table).
  std::string launch_table(hipStream_t s, int batch, int S, const void* const* in, void* const* out);
  // The same forward with op `name` launched `reps` times back to back; its time per launch.
  int profile_op(hipStream_t s, int batch, int S, const void* const* in, void* const* out, const char* name,
                 int reps, float* ms, double* flops, double* bytes);

  // Output element count per sample (for size checks).
  size_t out_elems_per_sample() const;
  int num_inputs_min() const;
  int num_inputs_max() const;

 private:
  void build_resnet(const std::map<std::string, const spi_named_tensor*>& p);
  void build_bert(const std::map<std::string, const spi_named_tensor*>& p);
  void build_vit(const std::map<std::string, const spi_named_tensor*>& p);
  Workspace* workspace(hipStream_t s);
  hipGraphExec_t graph(Workspace& w, int batch, int S, hipStream_t s);
  void body(Workspace& w, int batch, int S, hipStream_t s);
  void prologue(Workspace& w, int batch, int S, const void* const* in, hipStream_t s);
  void epilogue(Workspace& w, int batch, int S, void* const* out, hipStream_t s);
  // The LayerNorm fold of one transformer GEMM (ln_fold.hpp).
  struct LnSpec {
    const float* in_stats = nullptr;  // A rows are pre-LN: their chunk statistics (L.c1 folded in)
    const float* res_stats = nullptr;  // residual is LN(R): R's statistics, gain, bias
    const float* res_g = nullptr;
    const float* res_b = nullptr;
    float* out_stats = nullptr;  // write the output's statistics ...
    void* c16 = nullptr;         // ... and an fp16 copy
  };
  void run_gemm(const LinearW& L, const void* A, int M, int lda, void* C, int ldc,
                bool out_f32, Act act, const void* res, bool res_f32, int ldr, Workspace& ws,
                hipStream_t s, const LnSpec* ln = nullptr, size_t planes = 0);
  // QKV projection + attention of one transformer layer: the fused kernel (qkv_attn.hip) when
  // the shape allows it, else the QKV GEMM into qkv and the attention launch
  void run_qkv_attention(const LinearW& L, const void* x, const float* in_stats, void* qkv, void* ctx, int B,
                         int S, Workspace& ws, hipStream_t s);
  void run_conv(const ConvW& c, const void* x, int B, int H, int W, void* y, int& OH, int& OW,
                Act act, const void* res, Workspace& ws, hipStream_t s, bool out_f32 = false,
                bool res_f32 = false);
  struct ConvCall {
    GemmDesc d;
    GemmPtrs p;
    Prec prec = Prec::F16;
    std::string name;
    double flops = 0, bytes = 0;
  };
  ConvCall conv_call(const ConvW& c, const void* x, int B, int H, int W, void* y, int& OH, int& OW, Act act,
                     const void* res, Workspace& ws, bool out_f32, bool res_f32) const;
  void run_conv_pair(const ConvW& c0, const void* x, int B, int H, int W, void* y0, int& OH0, int& OW0, Act act0,
                     const ConvW& c1, void* y1, bool out1_f32, Workspace& ws, hipStream_t s);
  bool pooled_fc(int hw) const;
  void run_pooled_fc(const void* act, int B, int hw, void* out, Workspace& ws, hipStream_t s);
  size_t conv_partial(const ConvW& c, int B, int H, int W) const;
  size_t linear_partial(const LinearW& L, int M) const;
  GemmDesc pooled_fc_desc(int B, int hw) const;  // avgpool + FC as one GEMM (pool_rows = hw)
  template <typename P>
  const P* ptr(size_t off) const {
    return reinterpret_cast<const P*>(static_cast<const char*>(dblob_) + off);
  }

  int device_ = 0;
  int family_ = 0;
  Prec prec_ = Prec::F16;
  bool f16_ = true;  // activations stored as fp16 (Prec::F16 only)
  bool mixed_ = false;  // SPI_PREC_F16M on a ResNet (stem in F16X3, downsample + FC with krep = 2)
  // ResNet under Prec::F16X3: conv outputs / pool inputs in the split layout
  // (GemmDesc::a_split), so the GEMM main loop never splits A on the VALU.
  bool split_ = false;
  int max_batch_ = 1;
  bool graphs_ = false;
  std::string desc_;
  std::vector<char> hblob_;
  void* dblob_ = nullptr;
  size_t blob_bytes_ = 0;
  uint64_t digest_ = 0;

  // AFFINE
  float aff_scale_ = 1.f, aff_shift_ = 0.f;
  // ResNet
  bool bottleneck_ = false;
  std::vector<int> stage_blocks_;
  ConvW stem_;
  bool stem_fused_ = false;  // stem + max pool in one launch on the NCHW input (stem.hip)
#ifndef SPI_STEM_PR  // variant builds: 1 / 2 pooled rows per 4-wave workgroup (stem.hip)
#define SPI_STEM_PR 0
#endif
  int stem_pr_ = SPI_STEM_PR;  // its workgroup shape (0 = auto, stem.hip)
  size_t stem_pool_w_ = 0;   // its weights, [hi | lo][64][24][8] fp16
  std::vector<ResBlock> blocks_;
  LinearW fc_;
  int image_ = 224, classes_ = 1000, feat_ = 512;
  // transformers
  int D_ = 768, heads_ = 12, ffn_ = 3072, seq_ = 128, layers_ = 0, vocab_ = 0, maxpos_ = 0;
  float eps_ = 1e-12f;
  // LayerNorm folded across the GEMMs (fp16, D and FFN multiples of 128; SPI_LN_FOLD=0: the
  // separate LayerNorm launches): no LN launch inside the encoder stack
  bool ln_fold_ = false;
  // SPI_QKV_ATTN: 0 the QKV GEMM + attention launches (A/B); 1 (default) the fused kernel for S <= 128;
  // 2 also for 129..256 tokens (ViT-L at 197: correct, but -4 % under the four streams)
  int qkv_fused_ = 1;
  size_t word_ = 0, pos_ = 0, type0_ = 0;
  LnW emb_ln_, final_ln_;
  std::vector<TfLayer> tf_;
  // ViT
  int patch_ = 16, npatch_ = 196;
  LinearW patch_proj_, head_;
  size_t cls_ = 0, vpos_ = 0;

  std::mutex mu_;
  std::map<hipStream_t, std::unique_ptr<Workspace>> ws_;
  void run_profiled(hipStream_t s, int B, int S, const void* const* in, void* const* out, std::vector<OpRecord>& recs);
  // Set only inside profile(), on the profiling thread: forwards running on
  // other worker threads at the same time never see it.
  static thread_local std::vector<OpRecord>* prof_;
  struct ProfRepeat {
    std::string name;
    int reps;
    bool done;
  };
  static thread_local ProfRepeat* prof_rep_;
  // Starts an op record; returns how many times the op is to be launched (1, or
  // profile_op's repeat count for the op it names).
  int op_begin(hipStream_t s, const std::string& name, double flops, double bytes);
  void op_end(hipStream_t s);
  // Profiled launch (bytes = algorithmic traffic); a plain call when not profiling.
  template <typename F>
  void prof_op(hipStream_t s, const char* name, double bytes, F&& launch) {
    const int nrep = prof_ ? op_begin(s, name, 0, bytes) : 1;
    for (int r = 0; r < nrep; ++r) launch();
    if (prof_) op_end(s);
  }
  // LayerNorm over rows x D_: fp32 in + fp32 out (+ compute-type copy).
  double ln_bytes(double rows, bool f32_out) const {
    return rows * D_ * (4 + (f32_out ? 4 : 0) + (f16_ ? 2 : (f32_out ? 0 : 4)));
  }

  friend struct Workspace;
};

}  // namespace spi

struct spi_model {
  std::unique_ptr<spi::Model> impl;
};
