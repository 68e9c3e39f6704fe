// Model replica: recognise -> fold -> pack -> upload; per-stream workspaces;
// forward plans for ResNet (basic / bottleneck), BERT (post-LN) and ViT
// (pre-LN).  Reference counterparts: model loading and per-device clones
// (src/core/inference_runner.cpp:243-275), the forward that LibTorch runs
// inside the codelet (src/core/starpu_setup.cpp:610), and the model graphs the
// reference exports (models/import_resnet.py:25-73, models/import_vit.py:10-62,
// models/import_bert-base-uncased.py:8-39).
#include "model.hpp"
#include "pack.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <stdexcept>

namespace spi {

#define SPI_HIP(x)                                                                  \
  do {                                                                              \
    hipError_t e__ = (x);                                                           \
    if (e__ != hipSuccess)                                                          \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e__) + \
                               " at " #x);                                          \
  } while (0)

namespace {

using PMap = std::map<std::string, const spi_named_tensor*>;

int64_t numel(const spi_named_tensor* t) {
  int64_t n = 1;
  for (int i = 0; i < t->ndim; ++i) n *= t->shape[i];
  return n;
}

const float* fdata(const spi_named_tensor* t) {
  if (t->dtype != SPI_DTYPE_F32)
    throw std::runtime_error(std::string("parameter ") + t->name + " must be fp32");
  return static_cast<const float*>(t->data);
}

const spi_named_tensor* need(const PMap& p, const std::string& k) {
  auto it = p.find(k);
  if (it == p.end()) throw std::runtime_error("missing parameter '" + k + "'");
  return it->second;
}

bool has(const PMap& p, const std::string& k) { return p.count(k) != 0; }

int round_up(int v, int m) { return (v + m - 1) / m * m; }

}  // namespace

constexpr size_t kCounterSlots = 16384;  // >= tiles of any split GEMM (checked per launch)

// Graph capture vs allocation: a hipMalloc on one worker thread while another
// thread's stream is capturing invalidates that capture ("operation failed due
// to a previous error during capture").  Workspace allocation and graph capture
// therefore never overlap, process-wide (all replicas, all worker threads).
std::mutex g_capture_mu;

// ---------------------------------------------------------------------------
// Workspace: activation buffers for one stream at max_batch.
// ---------------------------------------------------------------------------
struct Workspace {
  std::vector<void*> bufs;
  float* partial = nullptr;
  float* mask_bias = nullptr;
  size_t partial_floats = 0;
  int* counters = nullptr;  // split-K tickets (zeroed once; the reducer re-zeroes its slot)
  bool has_mask = false;
  int final_buf = 6;  // ResNet: buffer holding the last stage's output
  int final_hw = 0;   // ... and its pixels per image (avgpool window)
  std::map<int, hipGraphExec_t> graphs;
  ~Workspace() {
    for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
    for (void* b : bufs) (void)hipFree(b);
    if (partial) (void)hipFree(partial);
    if (mask_bias) (void)hipFree(mask_bias);
    if (counters) (void)hipFree(counters);
  }
};

namespace {

class Blob {
 public:
  size_t add(const void* src, size_t bytes) {
    const size_t off = (data_.size() + 255) & ~size_t(255);
    data_.resize(off + bytes);
    if (src) std::memcpy(data_.data() + off, src, bytes);
    return off;
  }
  char* at(size_t off) { return data_.data() + off; }
  std::vector<char>& data() { return data_; }

 private:
  std::vector<char> data_;
};

// The blob being packed by this thread's Model constructor.  thread_local so
// replicas can be built concurrently (one per device, clone_model_to_gpus).
thread_local Blob* g_blob = nullptr;

// Pack a [N][K] fp32 matrix (row-major, K contiguous) into [Npad][Kpad] of the
// compute type.  get(n, k) supplies element (n, k) in packed-k order.
template <typename F>
size_t pack_matrix(int N, int K, int Npad, int Kpad, Prec prec, F get) {
  const size_t off = g_blob->add(nullptr, packed_bytes(prec, Npad, Kpad));
  pack_matrix_into(g_blob->at(off), N, K, Npad, Kpad, prec, get);
  return off;
}

size_t pack_vec(const float* v, int n) { return g_blob->add(v, (size_t)n * sizeof(float)); }

// Conv weight [Cout][Cin][KH][KW] (+ eval BN) -> folded [Npad][Kpad], k =
// (kh*KW + kw)*cin_pad + c; bias' = beta - mean * gamma / sqrt(var + eps).
// hilo (F16 only): pack every 64-k block of the folded weights twice -- fp16(w), then
// fp16(w - fp16(w)) -- for a krep = 2 contraction (GemmDesc::krep).
// Eval BatchNorm folded into a conv: w' = w * gamma / sqrt(var + eps) (fp64, then
// fp32), bias' = beta - mean * gamma / sqrt(var + eps) (or the conv's own bias).
struct FoldedConv {
  int cout = 0, cin = 0, kh = 1, kw = 1;
  std::vector<float> w;  // [cout][cin][kh][kw]
  std::vector<float> b;  // [cout]
};

FoldedConv fold_conv(const PMap& p, const std::string& wname, const std::string& bn, float bn_eps) {
  const spi_named_tensor* wt = need(p, wname + ".weight");
  if (wt->ndim != 4) throw std::runtime_error(wname + ".weight must be 4-D");
  FoldedConv f;
  f.cout = (int)wt->shape[0];
  f.cin = (int)wt->shape[1];
  f.kh = (int)wt->shape[2];
  f.kw = (int)wt->shape[3];
  std::vector<double> scale(f.cout, 1.0), shift(f.cout, 0.0);
  if (!bn.empty()) {
    const float* g = fdata(need(p, bn + ".weight"));
    const float* b = fdata(need(p, bn + ".bias"));
    const float* m = fdata(need(p, bn + ".running_mean"));
    const float* v = fdata(need(p, bn + ".running_var"));
    for (int o = 0; o < f.cout; ++o) {
      const double s = (double)g[o] / std::sqrt((double)v[o] + (double)bn_eps);
      scale[o] = s;
      shift[o] = (double)b[o] - (double)m[o] * s;
    }
  } else if (has(p, wname + ".bias")) {
    const float* b = fdata(need(p, wname + ".bias"));
    for (int o = 0; o < f.cout; ++o) shift[o] = b[o];
  }
  const float* w = fdata(wt);
  const size_t per = (size_t)f.cin * f.kh * f.kw;
  f.w.resize((size_t)f.cout * per);
  f.b.resize(f.cout);
  for (int o = 0; o < f.cout; ++o) {
    for (size_t i = 0; i < per; ++i) f.w[o * per + i] = (float)((double)w[o * per + i] * scale[o]);
    f.b[o] = (float)shift[o];
  }
  return f;
}

// Conv weight [Cout][Cin][KH][KW] (+ eval BN) -> folded [Npad][Kpad], k =
// (kh*KW + kw)*cin_pad + c.
// hilo (F16 only): pack every 64-k block of the folded weights twice -- fp16(w), then
// fp16(w - fp16(w)) -- for a krep = 2 contraction (GemmDesc::krep).
ConvW pack_conv(const PMap& p, const std::string& wname, const std::string& bn, int stride,
                int cin_pad, Prec prec, float bn_eps, bool hilo = false) {
  const FoldedConv f = fold_conv(p, wname, bn, bn_eps);
  ConvW c;
  c.cout = f.cout;
  c.cin = f.cin;
  c.kh = f.kh;
  c.kw = f.kw;
  c.stride = stride;
  c.pad = c.kh / 2;
  c.cin_pad = std::max(cin_pad, c.cin);
  const int K = c.kh * c.kw * c.cin_pad;
  c.kpad = round_up(K, 64);
  c.npad = round_up(c.cout, 128);
  if (hilo && prec != Prec::F16) throw std::runtime_error("hi/lo weight packing is an F16 layout");
  const int cin = c.cin, kh = c.kh, kw = c.kw, cp = c.cin_pad;
  c.prec = prec;
  auto folded = [&](int n, int k) -> float {
    const int cell = k / cp, ci = k % cp;
    if (ci >= cin) return 0.f;
    const int y = cell / kw, x = cell % kw;
    return f.w[(((size_t)n * cin + ci) * kh + y) * kw + x];
  };
  if (hilo) {
    c.krep = 2;
    c.kpad *= 2;
    c.w = pack_matrix(c.cout, c.kpad, c.npad, c.kpad, prec, [&](int n, int kp) -> float {
      const int k = (kp >> 7) * 64 + (kp & 63);  // 128-k packed block = [64 hi | 64 lo]
      if (k >= K) return 0.f;
      const float v = folded(n, k);
      return (kp & 64) ? v - static_cast<float>(static_cast<_Float16>(v)) : v;
    });
  } else {
    c.w = pack_matrix(c.cout, K, c.npad, c.kpad, prec, folded);
    c.w_image = packed_has_wres_image(prec, c.cout, K, c.npad, c.kpad);
  }
  c.wplane = (size_t)c.npad * c.kpad;
  c.b = pack_vec(f.b.data(), c.cout);
  return c;
}

LinearW pack_linear(const float* w, const float* b, int N, int K, Prec prec, bool hilo = false) {
  LinearW L;
  L.n = N;
  L.k = K;
  L.kpad = round_up(K, 64);
  L.npad = round_up(N, 128);
  L.prec = prec;
  if (hilo) {  // as pack_conv: [64 hi | 64 lo] per 64-k block, krep = 2
    if (prec != Prec::F16) throw std::runtime_error("hi/lo weight packing is an F16 layout");
    L.krep = 2;
    L.kpad *= 2;
    L.w = pack_matrix(N, L.kpad, L.npad, L.kpad, prec, [&](int n, int kp) -> float {
      const int k = (kp >> 7) * 64 + (kp & 63);
      if (k >= K) return 0.f;
      const float v = w[(size_t)n * K + k];
      return (kp & 64) ? v - static_cast<float>(static_cast<_Float16>(v)) : v;
    });
  } else {
    L.w = pack_matrix(N, K, L.npad, L.kpad, prec, [&](int n, int k) { return w[(size_t)n * K + k]; });
  }
  L.wplane = (size_t)L.npad * L.kpad;
  std::vector<float> zeros;
  if (!b) {
    zeros.assign(N, 0.f);
    b = zeros.data();
    L.has_bias = false;
  }
  L.b = pack_vec(b, N);
  return L;
}

LinearW pack_linear_named(const PMap& p, const std::string& name, Prec prec, bool hilo = false) {
  const spi_named_tensor* wt = need(p, name + ".weight");
  if (wt->ndim != 2) throw std::runtime_error(name + ".weight must be 2-D");
  const float* b = has(p, name + ".bias") ? fdata(need(p, name + ".bias")) : nullptr;
  return pack_linear(fdata(wt), b, (int)wt->shape[0], (int)wt->shape[1], prec, hilo);
}

// The weights of a GEMM whose input rows are LayerNorm'd (y = LN(x) W^T + b), packed for
// the fold (ln_fold.hpp): W' = W diag(gamma) in the compute type, bias' = b + W beta, and
// c1[n] = sum_k W'[n][k] over the packed (rounded) values, so the epilogue's
// rstd (x W'^T - mean c1) cancels exactly what the MFMAs accumulated.
// hilo (transformer F16M): W' packed hi + lo (krep = 2); c1 sums both halves as packed.
LinearW pack_linear_folded(const float* w, const float* b, int N, int K, Prec prec, const float* gamma,
                           const float* beta, bool hilo = false) {
  std::vector<float> wf((size_t)N * K), bf(N);
  std::vector<float> c1(N);
  for (int n = 0; n < N; ++n) {
    double bb = b ? b[n] : 0.0, cc = 0.0;
    for (int k = 0; k < K; ++k) {
      const float v = w[(size_t)n * K + k];
      const float f = v * gamma[k];
      wf[(size_t)n * K + k] = f;
      bb += (double)beta[k] * v;
      if (prec == Prec::F16) {
        const float hi = static_cast<float>(static_cast<_Float16>(f));
        cc += hilo ? (double)hi + (double)static_cast<float>(static_cast<_Float16>(f - hi)) : (double)hi;
      } else {
        cc += (double)f;
      }
    }
    bf[n] = (float)bb;
    c1[n] = (float)cc;
  }
  LinearW L = pack_linear(wf.data(), bf.data(), N, K, prec, hilo);
  L.c1 = pack_vec(c1.data(), N);
  return L;
}

// The LayerNorm fold is an fp16 path, on by default where it measured faster; SPI_LN_FOLD=0 / 1
// forces the separate launches / the fold (A/B runs).
bool ln_fold_enabled(Prec prec, bool by_default) {
  const char* e = std::getenv("SPI_LN_FOLD");
  const bool on = (e && *e) ? std::atoi(e) != 0 : by_default;
  return prec == Prec::F16 && on;
}
// BERT-base: fold +3.9 % four-stream (same process, round 4).  ViT-L: off in rounds 4-5 (5.93k
// folded against 6.30k, profiles/r04/fixed/vit_fold_ab.txt: the producer epilogues' fp16 copy and
// the consumers' statistics round trip + spills cost more than the 46 removed launches); on since
// round 6 over the two-plane residual stream (no copy; statistics loaded under the last k-tile):
// 6.68k folded against 6.59k (profiles/r06/vit_fold/)
constexpr bool kBertLnFold = true;
constexpr bool kVitLnFold = true;

LnW pack_ln(const PMap& p, const std::string& name) {
  LnW l;
  const spi_named_tensor* g = need(p, name + ".weight");
  l.g = pack_vec(fdata(g), (int)numel(g));
  l.b = pack_vec(fdata(need(p, name + ".bias")), (int)numel(g));
  return l;
}

// Strip the common prefix in front of an anchor name ("bert.embeddings..." ->
// "embeddings..."), so wrapped modules are recognised.
PMap strip_prefix(const PMap& in, const std::string& anchor) {
  std::string prefix;
  bool found = false;
  for (auto& kv : in) {
    const std::string& k = kv.first;
    if (k.size() >= anchor.size() && k.compare(k.size() - anchor.size(), anchor.size(), anchor) == 0) {
      const std::string pre = k.substr(0, k.size() - anchor.size());
      if (pre.empty() || pre.back() == '.') {
        prefix = pre;
        found = true;
        break;
      }
    }
  }
  if (!found || prefix.empty()) return in;
  PMap out;
  for (auto& kv : in)
    if (kv.first.compare(0, prefix.size(), prefix) == 0) out[kv.first.substr(prefix.size())] = kv.second;
  return out;
}

bool ends_with(const PMap& p, const std::string& anchor) {
  for (auto& kv : p) {
    const std::string& k = kv.first;
    if (k.size() >= anchor.size() && k.compare(k.size() - anchor.size(), anchor.size(), anchor) == 0)
      return true;
  }
  return false;
}

}  // namespace

// ---------------------------------------------------------------------------
// Construction
// ---------------------------------------------------------------------------
Model::Model(int device, const spi_model_config& cfg, const spi_named_tensor* params, int n)
    : device_(device), family_(cfg.family),
      prec_(cfg.precision == SPI_PREC_F16 || cfg.precision == SPI_PREC_F16M ? Prec::F16
            : cfg.precision == SPI_PREC_F16X3                               ? Prec::F16X3
                                                                            : Prec::F32),
      f16_(cfg.precision == SPI_PREC_F16 || cfg.precision == SPI_PREC_F16M),
      max_batch_(std::max(1, cfg.max_batch)) {
  if (cfg.precision != SPI_PREC_F16 && cfg.precision != SPI_PREC_F32 && cfg.precision != SPI_PREC_F16X3 &&
      cfg.precision != SPI_PREC_F16M)
    throw std::runtime_error("unsupported precision");
  PMap p;
  for (int i = 0; i < n; ++i) {
    if (!params[i].name) throw std::runtime_error("parameter without a name");
    p[params[i].name] = &params[i];
  }
  if (family_ == SPI_FAMILY_AUTO) {
    if (ends_with(p, "embeddings.word_embeddings.weight")) family_ = SPI_FAMILY_BERT;
    else if (ends_with(p, "conv_proj.weight") && ends_with(p, "class_token")) family_ = SPI_FAMILY_VIT;
    else if (ends_with(p, "layer1.0.conv1.weight")) family_ = SPI_FAMILY_RESNET;
    else throw std::runtime_error("unrecognised model: no ResNet/BERT/ViT parameter names");
  }
  Blob blob;
  g_blob = &blob;
  blob.add(nullptr, 256);  // offset 0: zero line read by the GEMM for padded chunks
  std::ostringstream os;
  if (family_ == SPI_FAMILY_AFFINE) {
    aff_scale_ = cfg.affine_scale;
    aff_shift_ = cfg.affine_shift;
    os << "affine(x*" << aff_scale_ << "+" << aff_shift_ << ") f32";
  } else if (family_ == SPI_FAMILY_RESNET) {
    mixed_ = cfg.precision == SPI_PREC_F16M;
    if (cfg.image_size > 0) image_ = cfg.image_size;
    eps_ = cfg.eps > 0 ? cfg.eps : 1e-5f;
    build_resnet(strip_prefix(p, "layer1.0.conv1.weight"));
    os << "resnet" << (bottleneck_ ? "-bottleneck[" : "-basic[");
    for (size_t i = 0; i < stage_blocks_.size(); ++i) os << (i ? "," : "") << stage_blocks_[i];
    os << "] img" << image_ << " classes" << classes_;
  } else if (family_ == SPI_FAMILY_BERT) {
    mixed_ = cfg.precision == SPI_PREC_F16M;  // hi + lo weights on every encoder GEMM
    if (const char* e = std::getenv("SPI_QKV_ATTN"); e && *e) qkv_fused_ = std::atoi(e);
    eps_ = cfg.eps > 0 ? cfg.eps : 1e-12f;
    ln_fold_ = ln_fold_enabled(prec_, kBertLnFold);
    heads_ = cfg.num_heads;
    seq_ = cfg.seq_len;
    build_bert(strip_prefix(p, "embeddings.word_embeddings.weight"));
    os << "bert L" << layers_ << " D" << D_ << " H" << heads_ << " FF" << ffn_ << " S<=" << seq_;
  } else if (family_ == SPI_FAMILY_VIT) {
    mixed_ = cfg.precision == SPI_PREC_F16M;
    if (const char* e = std::getenv("SPI_QKV_ATTN"); e && *e) qkv_fused_ = std::atoi(e);
    eps_ = cfg.eps > 0 ? cfg.eps : 1e-6f;
    ln_fold_ = ln_fold_enabled(prec_, kVitLnFold);
    heads_ = cfg.num_heads;
    if (cfg.image_size > 0) image_ = cfg.image_size;
    build_vit(strip_prefix(p, "conv_proj.weight"));
    os << "vit L" << layers_ << " D" << D_ << " H" << heads_ << " MLP" << ffn_ << " patch" << patch_
       << " img" << image_ << " classes" << classes_;
  } else {
    throw std::runtime_error("unsupported model family");
  }
  os << (mixed_ ? " f16m" : prec_ == Prec::F16 ? " f16" : prec_ == Prec::F16X3 ? " f16x3" : " f32") << " maxB"
     << max_batch_;
  desc_ = os.str();
  g_blob = nullptr;

  blob_bytes_ = blob.data().size();
  uint64_t h = 1469598103934665603ull;  // FNV-1a 64
  for (char c : blob.data()) h = (h ^ (uint8_t)c) * 1099511628211ull;
  digest_ = h;
  if (device_ < 0) return;  // host-only replica: recognised and packed, never uploaded
  SPI_HIP(hipSetDevice(device_));
  if (blob_bytes_) {
    SPI_HIP(hipMalloc(&dblob_, blob_bytes_));
    SPI_HIP(hipMemcpy(dblob_, blob.data().data(), blob_bytes_, hipMemcpyHostToDevice));
  }
}

Model::~Model() {
  ws_.clear();
  if (dblob_) (void)hipFree(dblob_);
}

void Model::build_resnet(const PMap& p) {
  // Stages: torchvision layer1..layer4, stride 2 on the first block of 2..4
  // (on conv1 for BasicBlock, conv2 for Bottleneck: torchvision v1.5).
  bottleneck_ = has(p, "layer1.0.conv3.weight");
  // Stem input channels padded to one 16-byte chunk per pixel: 4 fp32
  // (F32, and F16X3 whose A is fp32) or 8 fp16 (F16).
  // SPI_PREC_F16M: the stem reads the fp32 image with split weights (F16X3) and
  // writes fp16; the downsample convs and the (avgpool-fused) FC carry hi + lo
  // weights (krep = 2) (these layers set the fp16 error).
  const Prec stem_prec = mixed_ ? Prec::F16X3 : prec_;
  const int cin_pad = stem_prec == Prec::F16 ? 8 : 4;
  stem_ = pack_conv(p, "conv1", "bn1", 2, cin_pad, stem_prec, eps_);
  if (stem_.kh != 7 || stem_.cin != 3) throw std::runtime_error("resnet stem must be 7x7 over 3 channels");
  const FoldedConv stem_folded = fold_conv(p, "conv1", "bn1", eps_);
  for (int L = 1; L <= 4; ++L) {
    int nb = 0;
    while (has(p, "layer" + std::to_string(L) + "." + std::to_string(nb) + ".conv1.weight")) ++nb;
    if (nb == 0) throw std::runtime_error("resnet layer" + std::to_string(L) + " missing");
    stage_blocks_.push_back(nb);
    for (int i = 0; i < nb; ++i) {
      const std::string pre = "layer" + std::to_string(L) + "." + std::to_string(i) + ".";
      const int s = (L > 1 && i == 0) ? 2 : 1;
      ResBlock blk;
      if (bottleneck_) {
        blk.c1 = pack_conv(p, pre + "conv1", pre + "bn1", 1, 0, prec_, eps_);
        blk.c2 = pack_conv(p, pre + "conv2", pre + "bn2", s, 0, prec_, eps_);
        blk.c3 = pack_conv(p, pre + "conv3", pre + "bn3", 1, 0, prec_, eps_);
      } else {
        blk.c1 = pack_conv(p, pre + "conv1", pre + "bn1", s, 0, prec_, eps_);
        blk.c2 = pack_conv(p, pre + "conv2", pre + "bn2", 1, 0, prec_, eps_);
      }
      blk.has_ds = has(p, pre + "downsample.0.weight");
      if (blk.has_ds) blk.ds = pack_conv(p, pre + "downsample.0", pre + "downsample.1", s, 0, prec_, eps_, mixed_);
      blocks_.push_back(blk);
    }
  }
  // F16M: plain fp16 FC weights since round 5 (hi + lo kept the logits 0.06e-3 closer on 8 emulated
  // seeds and cost 1 % of C2); define SPI_FC_HILO=1 for the hi + lo packing
#ifndef SPI_FC_HILO
#define SPI_FC_HILO 0
#endif
  fc_ = pack_linear_named(p, "fc", prec_, mixed_ && SPI_FC_HILO);
  classes_ = fc_.n;
  feat_ = fc_.k;
  // Channel chain: every conv must read exactly the channels its producer
  // writes.  A grouped conv (ResNeXt, models/import_resnet.py variants) stores
  // weight.shape[1] = C/groups, which would otherwise be packed as a dense conv
  // over too few channels and give garbage without an error.
  {
    auto bad = [](const std::string& what) {
      throw std::runtime_error("resnet: grouped/unsupported conv (" + what + ")");
    };
    int ch = stem_.cout;
    for (size_t i = 0; i < blocks_.size(); ++i) {
      const ResBlock& b = blocks_[i];
      const std::string id = "block " + std::to_string(i);
      if (b.c1.cin != ch) bad(id + " conv1 reads " + std::to_string(b.c1.cin) + " of " + std::to_string(ch) + " channels");
      if (b.c2.cin != b.c1.cout) bad(id + " conv2 reads " + std::to_string(b.c2.cin) + " of " + std::to_string(b.c1.cout) + " channels");
      int out = b.c2.cout;
      if (bottleneck_) {
        if (b.c3.cin != b.c2.cout) bad(id + " conv3 reads " + std::to_string(b.c3.cin) + " of " + std::to_string(b.c2.cout) + " channels");
        out = b.c3.cout;
      }
      if (b.has_ds) {
        if (b.ds.cin != ch || b.ds.cout != out) bad(id + " downsample shape");
      } else if (ch != out) {
        bad(id + " identity residual with " + std::to_string(ch) + " -> " + std::to_string(out) + " channels");
      }
      ch = out;
    }
    if (fc_.k != ch) bad("fc reads " + std::to_string(fc_.k) + " of " + std::to_string(ch) + " features");
  }
  for (auto& b : blocks_) {
    const ConvW* cs[] = {&b.c1, &b.c2, &b.c3, &b.ds};
    for (const ConvW* c : cs)
      if (c->cout && (c->cin_pad % 8 != 0 || (c->cin_pad & (c->cin_pad - 1))))
        throw std::runtime_error("resnet conv channels must be a power of two >= 8");
  }
  // Split activations need every activation's channel count to be a multiple
  // of 32 (the split block) and every non-stem conv to read >= 32 channels.
  split_ = prec_ == Prec::F16X3 && stem_.cout % 32 == 0;
  for (auto& b : blocks_) {
    const ConvW* cs[] = {&b.c1, &b.c2, &b.c3, &b.ds};
    for (const ConvW* c : cs)
      if (c->cout && (c->cin_pad < 32 || c->cout % 32 != 0 || c->kh * c->kw > 31)) split_ = false;
  }
  // Fused stem (stem.hip: NCHW image -> conv + BN + ReLU -> max pool, one launch)
  // for the fp16-activation modes and split fp16x3; fp32 keeps ingest + stem GEMM +
  // max pool.  SPI_STEM_FUSED=0 selects the unfused path (A/B, tests).
  const char* fe = std::getenv("SPI_STEM_FUSED");
  const int stem_ow = (image_ + 6 - 7) / 2 + 1;
  stem_fused_ = !(fe && *fe && std::atoi(fe) == 0) && stem_.cout == 64 && stem_.stride == 2 &&
                stem_ow <= kStemPoolMaxOW && (prec_ == Prec::F16 || split_);
  if (stem_fused_) {
    std::vector<_Float16> packed(stem_pool_bytes() / sizeof(_Float16));
    stem_pool_pack(stem_folded.w.data(), packed.data());
    stem_pool_w_ = g_blob->add(packed.data(), stem_pool_bytes());
  }
}

void Model::build_bert(const PMap& p) {
  const spi_named_tensor* we = need(p, "embeddings.word_embeddings.weight");
  vocab_ = (int)we->shape[0];
  D_ = (int)we->shape[1];
  const spi_named_tensor* pe = need(p, "embeddings.position_embeddings.weight");
  maxpos_ = (int)pe->shape[0];
  if (heads_ <= 0) heads_ = D_ / 64;
  if (D_ % heads_ != 0 || D_ / heads_ != 64) throw std::runtime_error("attention head_dim must be 64");
  if (D_ % 64 != 0 || D_ > 1024) throw std::runtime_error("hidden size must be a multiple of 64, <= 1024");
  if (seq_ <= 0) seq_ = maxpos_;
  word_ = pack_vec(fdata(we), (int)numel(we));
  pos_ = pack_vec(fdata(pe), (int)numel(pe));
  const spi_named_tensor* te = need(p, "embeddings.token_type_embeddings.weight");
  type0_ = pack_vec(fdata(te), D_);  // token_type_ids buffer is all zeros
  emb_ln_ = pack_ln(p, "embeddings.LayerNorm");
  while (has(p, "encoder.layer." + std::to_string(layers_) + ".attention.self.query.weight")) ++layers_;
  if (layers_ == 0) throw std::runtime_error("bert: no encoder layers");
  for (int i = 0; i < layers_; ++i) {
    const std::string pre = "encoder.layer." + std::to_string(i) + ".";
    TfLayer L;
    // Q, K, V stacked into one [3D][D] projection.
    std::vector<float> w((size_t)3 * D_ * D_), b((size_t)3 * D_);
    const char* names[3] = {"query", "key", "value"};
    for (int j = 0; j < 3; ++j) {
      const std::string nm = pre + "attention.self." + names[j];
      std::memcpy(w.data() + (size_t)j * D_ * D_, fdata(need(p, nm + ".weight")), sizeof(float) * D_ * D_);
      std::memcpy(b.data() + (size_t)j * D_, fdata(need(p, nm + ".bias")), sizeof(float) * D_);
    }
    L.qkv = pack_linear(w.data(), b.data(), 3 * D_, D_, prec_, mixed_);
    L.out = pack_linear_named(p, pre + "attention.output.dense", prec_, mixed_);
    L.ln1 = pack_ln(p, pre + "attention.output.LayerNorm");
    L.ff1 = pack_linear_named(p, pre + "intermediate.dense", prec_, mixed_);
    L.ff2 = pack_linear_named(p, pre + "output.dense", prec_, mixed_);
    L.ln2 = pack_ln(p, pre + "output.LayerNorm");
    ffn_ = L.ff1.n;
    tf_.push_back(L);
  }
  // post-LN: FFN1 of layer i reads LN1_i(a), QKV of layer i >= 1 reads LN2_{i-1}(b)
  ln_fold_ = ln_fold_ && D_ % 128 == 0 && ffn_ % 128 == 0;
  if (ln_fold_) {
    for (int i = 0; i < layers_; ++i) {
      const std::string pre = "encoder.layer." + std::to_string(i) + ".";
      const std::string ln1 = pre + "attention.output.LayerNorm";
      const spi_named_tensor* f1 = need(p, pre + "intermediate.dense.weight");
      tf_[i].ff1 = pack_linear_folded(fdata(f1), fdata(need(p, pre + "intermediate.dense.bias")), ffn_, D_, prec_,
                                      fdata(need(p, ln1 + ".weight")), fdata(need(p, ln1 + ".bias")), mixed_);
      if (i == 0) continue;
      const std::string ln2 = "encoder.layer." + std::to_string(i - 1) + ".output.LayerNorm";
      std::vector<float> w((size_t)3 * D_ * D_), b((size_t)3 * D_);
      const char* names[3] = {"query", "key", "value"};
      for (int j = 0; j < 3; ++j) {
        const std::string nm = pre + "attention.self." + names[j];
        std::memcpy(w.data() + (size_t)j * D_ * D_, fdata(need(p, nm + ".weight")), sizeof(float) * D_ * D_);
        std::memcpy(b.data() + (size_t)j * D_, fdata(need(p, nm + ".bias")), sizeof(float) * D_);
      }
      tf_[i].qkv = pack_linear_folded(w.data(), b.data(), 3 * D_, D_, prec_, fdata(need(p, ln2 + ".weight")),
                                      fdata(need(p, ln2 + ".bias")), mixed_);
    }
  }
}

void Model::build_vit(const PMap& p) {
  const spi_named_tensor* cw = need(p, "conv_proj.weight");
  D_ = (int)cw->shape[0];
  patch_ = (int)cw->shape[2];
  if (cw->shape[1] != 3 || cw->shape[3] != patch_) throw std::runtime_error("vit conv_proj must be PxP over 3 channels");
  if (image_ % patch_) throw std::runtime_error("image size must be a multiple of the patch size");
  npatch_ = (image_ / patch_) * (image_ / patch_);
  if (heads_ <= 0) heads_ = D_ / 64;
  if (D_ % heads_ != 0 || D_ / heads_ != 64) throw std::runtime_error("attention head_dim must be 64");
  if (D_ % 64 != 0 || D_ > 1024) throw std::runtime_error("hidden size must be a multiple of 64, <= 1024");
  const int K = 3 * patch_ * patch_;
  patch_proj_ = pack_linear(fdata(cw), has(p, "conv_proj.bias") ? fdata(need(p, "conv_proj.bias")) : nullptr,
                            D_, K, prec_, mixed_);
  cls_ = pack_vec(fdata(need(p, "class_token")), D_);
  const spi_named_tensor* pe = need(p, "encoder.pos_embedding");
  if (numel(pe) != (int64_t)(npatch_ + 1) * D_) throw std::runtime_error("pos_embedding does not match image/patch size");
  vpos_ = pack_vec(fdata(pe), (int)numel(pe));
  while (has(p, "encoder.layers.encoder_layer_" + std::to_string(layers_) + ".ln_1.weight")) ++layers_;
  if (layers_ == 0) throw std::runtime_error("vit: no encoder layers");
  for (int i = 0; i < layers_; ++i) {
    const std::string pre = "encoder.layers.encoder_layer_" + std::to_string(i) + ".";
    TfLayer L;
    L.ln1 = pack_ln(p, pre + "ln_1");
    const spi_named_tensor* iw = need(p, pre + "self_attention.in_proj_weight");
    L.qkv = pack_linear(fdata(iw), fdata(need(p, pre + "self_attention.in_proj_bias")), (int)iw->shape[0],
                        (int)iw->shape[1], prec_, mixed_);
    L.out = pack_linear_named(p, pre + "self_attention.out_proj", prec_, mixed_);
    L.ln2 = pack_ln(p, pre + "ln_2");
    const std::string m1 = has(p, pre + "mlp.0.weight") ? pre + "mlp.0" : pre + "mlp.linear_1";
    const std::string m2 = has(p, pre + "mlp.3.weight") ? pre + "mlp.3" : pre + "mlp.linear_2";
    L.ff1 = pack_linear_named(p, m1, prec_, mixed_);
    L.ff2 = pack_linear_named(p, m2, prec_, mixed_);
    ffn_ = L.ff1.n;
    tf_.push_back(L);
  }
  // pre-LN: QKV of layer i >= 1 reads LN1_i(x) (layer 0's LN1 stays a launch, model body),
  // FFN1 of layer i reads LN2_i(x)
  ln_fold_ = ln_fold_ && D_ % 128 == 0 && ffn_ % 128 == 0;
  if (ln_fold_) {
    for (int i = 0; i < layers_; ++i) {
      const std::string pre = "encoder.layers.encoder_layer_" + std::to_string(i) + ".";
      const std::string m1 = has(p, pre + "mlp.0.weight") ? pre + "mlp.0" : pre + "mlp.linear_1";
      const spi_named_tensor* f1 = need(p, m1 + ".weight");
      tf_[i].ff1 = pack_linear_folded(fdata(f1), fdata(need(p, m1 + ".bias")), (int)f1->shape[0], (int)f1->shape[1],
                                      prec_, fdata(need(p, pre + "ln_2.weight")), fdata(need(p, pre + "ln_2.bias")),
                                      mixed_);
      if (i == 0) continue;
      const spi_named_tensor* iw = need(p, pre + "self_attention.in_proj_weight");
      tf_[i].qkv = pack_linear_folded(fdata(iw), fdata(need(p, pre + "self_attention.in_proj_bias")),
                                      (int)iw->shape[0], (int)iw->shape[1], prec_, fdata(need(p, pre + "ln_1.weight")),
                                      fdata(need(p, pre + "ln_1.bias")), mixed_);
    }
  }
  final_ln_ = pack_ln(p, "encoder.ln");
  head_ = pack_linear_named(p, "heads.head", prec_, mixed_);
  classes_ = head_.n;
  seq_ = npatch_ + 1;
}

// ---------------------------------------------------------------------------
// I/O contract
// ---------------------------------------------------------------------------
size_t Model::out_elems_per_sample() const {
  switch (family_) {
    case SPI_FAMILY_RESNET:
    case SPI_FAMILY_VIT:
      return (size_t)classes_;
    case SPI_FAMILY_BERT:
      return 0;  // depends on S: checked in check_io
    default:
      return 0;
  }
}

int Model::num_inputs_min() const { return 1; }
int Model::num_inputs_max() const { return family_ == SPI_FAMILY_BERT ? 2 : 1; }

void Model::check_io(const spi_codelet_args& a, const size_t* in_bytes, const size_t* out_bytes) const {
  const int ni = (int)a.num_inputs, no = (int)a.num_outputs;
  if (ni < num_inputs_min() || ni > num_inputs_max())
    throw std::runtime_error("model expects " + std::to_string(num_inputs_max()) + " input(s), got " +
                             std::to_string(ni));
  if (no != 1) throw std::runtime_error("Mismatch between model outputs and StarPU buffers");
  const int64_t B = a.dims[0][0];
  if (B < 1 || B > max_batch_)
    throw std::runtime_error("batch " + std::to_string(B) + " exceeds replica max_batch " +
                             std::to_string(max_batch_));
  auto elems = [&](int i) {
    int64_t e = 1;
    for (int d = 0; d < a.num_dims[i]; ++d) e *= a.dims[i][d];
    return e;
  };
  size_t expect_out = 0;
  if (family_ == SPI_FAMILY_AFFINE) {
    if (a.input_types[0] != SPI_DTYPE_F32) throw std::runtime_error("[ERROR] Input type mismatch");
    if (in_bytes[0] < (size_t)elems(0) * 4) throw std::runtime_error("[ERROR] Input buffer too small");
    expect_out = (size_t)elems(0) * 4;
  } else if (family_ == SPI_FAMILY_RESNET || family_ == SPI_FAMILY_VIT) {
    if (a.input_types[0] != SPI_DTYPE_F32) throw std::runtime_error("[ERROR] Input type mismatch");
    if (a.num_dims[0] != 4 || a.dims[0][1] != 3 || a.dims[0][2] != image_ || a.dims[0][3] != image_)
      throw std::runtime_error("[ERROR] Tensor layout mismatch: expected [B,3," + std::to_string(image_) + "," +
                               std::to_string(image_) + "]");
    if (in_bytes[0] < (size_t)elems(0) * 4) throw std::runtime_error("[ERROR] Input buffer too small");
    expect_out = (size_t)B * classes_ * 4;
  } else {  // BERT: input_ids [B,S] int64, optional attention_mask [B,S] int64
    for (int i = 0; i < ni; ++i) {
      if (a.input_types[i] != SPI_DTYPE_I64) throw std::runtime_error("[ERROR] Input type mismatch");
      if (a.num_dims[i] != 2 || a.dims[i][0] != B || a.dims[i][1] != a.dims[0][1])
        throw std::runtime_error("[ERROR] Tensor layout mismatch");
      if (in_bytes[i] < (size_t)elems(i) * 8) throw std::runtime_error("[ERROR] Input buffer too small");
    }
    const int64_t S = a.dims[0][1];
    if (S < 1 || S > seq_ || S > maxpos_)
      throw std::runtime_error("sequence length " + std::to_string(S) + " exceeds " + std::to_string(seq_));
    expect_out = (size_t)B * S * D_ * 4;
  }
  if (a.output_types[0] != SPI_DTYPE_F32) throw std::runtime_error("[ERROR] Output type mismatch");
  if (out_bytes[0] != expect_out) throw std::runtime_error("Output buffer size mismatch in bytes");
}

double Model::flops(int64_t B) const {
  double f = 0;
  auto conv_f = [&](const ConvW& c, int OH, int OW) {
    return 2.0 * B * OH * OW * c.cout * (double)c.kh * c.kw * c.cin;
  };
  if (family_ == SPI_FAMILY_RESNET) {
    int H = (image_ + 2 * 3 - 7) / 2 + 1;
    f += conv_f(stem_, H, H);
    H = (H + 2 - 3) / 2 + 1;
    for (const auto& b : blocks_) {
      if (bottleneck_) {
        f += conv_f(b.c1, H, H);
        const int H2 = (H + 2 * b.c2.pad - b.c2.kh) / b.c2.stride + 1;
        f += conv_f(b.c2, H2, H2) + conv_f(b.c3, H2, H2);
        if (b.has_ds) f += conv_f(b.ds, H2, H2);
        H = H2;
      } else {
        const int H2 = (H + 2 * b.c1.pad - b.c1.kh) / b.c1.stride + 1;
        f += conv_f(b.c1, H2, H2) + conv_f(b.c2, H2, H2);
        if (b.has_ds) f += conv_f(b.ds, H2, H2);
        H = H2;
      }
    }
    f += 2.0 * B * fc_.n * fc_.k;
  } else if (family_ == SPI_FAMILY_BERT || family_ == SPI_FAMILY_VIT) {
    const double S = family_ == SPI_FAMILY_BERT ? seq_ : npatch_ + 1;
    const double T = B * S;
    for (const auto& L : tf_)
      f += 2.0 * T * ((double)L.qkv.n * L.qkv.k + (double)L.out.n * L.out.k + (double)L.ff1.n * L.ff1.k +
                      (double)L.ff2.n * L.ff2.k) +
           4.0 * B * S * S * D_;
    if (family_ == SPI_FAMILY_VIT) f += 2.0 * B * npatch_ * (double)D_ * patch_proj_.k + 2.0 * B * head_.n * head_.k;
  }
  return f;
}

// ---------------------------------------------------------------------------
// Launch helpers
// ---------------------------------------------------------------------------
namespace {
GemmDesc conv_desc(const ConvW& c, int B, int H, int W, int& OH, int& OW) {
  OH = (H + 2 * c.pad - c.kh) / c.stride + 1;
  OW = (W + 2 * c.pad - c.kw) / c.stride + 1;
  GemmDesc d;
  d.M = B * OH * OW;
  d.N = c.cout;
  d.K = c.kh * c.kw * c.cin_pad;
  d.Kpad = c.kpad;
  d.ldc = c.cout;
  d.ldr = c.cout;
  d.conv = true;
  d.H = H;
  d.W = W;
  d.Cin = c.cin_pad;
  d.OH = OH;
  d.OW = OW;
  d.KH = c.kh;
  d.KW = c.kw;
  d.stride = c.stride;
  d.pad = c.pad;
  d.krep = c.krep;
  d.w_image = c.w_image;
  return d;
}

GemmDesc linear_desc(const LinearW& L, int M, int lda, int ldc) {
  GemmDesc d;
  d.M = M;
  d.N = L.n;
  d.K = L.k;
  d.Kpad = L.kpad;
  d.lda = lda;
  d.ldc = ldc;
  d.ldr = ldc;
  d.krep = L.krep;
  return d;
}
}  // namespace

size_t Model::conv_partial(const ConvW& c, int B, int H, int W) const {
  int OH, OW;
  GemmDesc d = conv_desc(c, B, H, W, OH, OW);
  d.a_split = split_ && &c != &stem_;  // as run_conv: the plan (halo, split-K) depends on it
  return gemm_partial_floats(d, c.prec);
}

size_t Model::linear_partial(const LinearW& L, int M) const {
  return gemm_partial_floats(linear_desc(L, M, L.k, L.n), L.prec);
}

Model::ConvCall Model::conv_call(const ConvW& c, const void* x, int B, int H, int W, void* y, int& OH, int& OW,
                                 Act act, const void* res, Workspace& ws, bool out_f32, bool res_f32) const {
  ConvCall k;
  GemmDesc& d = k.d;
  d = conv_desc(c, B, H, W, OH, OW);
  d.act = act;
  d.wplane = c.wplane;
  d.out_split = split_;
  d.a_split = split_ && &c != &stem_;  // the stem reads the ingested fp32 image
  d.out_f32 = out_f32;
  d.res_f32 = res_f32;
  d.out_f16 = f16_ && c.prec == Prec::F16X3 && !out_f32;  // F16M stem: F16X3 contraction, fp16 activations
  const size_t es = f16_ ? 2 : 4;
  k.name = "conv" + std::to_string(c.kh) + "x" + std::to_string(c.kw) + "_c" + std::to_string(c.cin) + "_k" +
           std::to_string(c.cout) + "_s" + std::to_string(c.stride) + "_M" + std::to_string(d.M);
  k.flops = 2.0 * d.M * d.N * (double)c.kh * c.kw * c.cin;
  k.bytes = (double)B * H * W * c.cin_pad * es + (double)c.cout * d.K * es + (double)d.M * d.N * es * (res ? 2 : 1);
  GemmPtrs& p = k.p;
  p.A = x;
  p.W = ptr<void>(c.w);
  p.bias = ptr<float>(c.b);
  p.res = res;
  p.C = y;
  p.partial = ws.partial;
  p.counters = ws.counters;
  p.zeros = dblob_;  // the blob starts with a zeroed 256-byte line
  k.prec = c.prec;
  return k;
}

void Model::run_conv(const ConvW& c, const void* x, int B, int H, int W, void* y, int& OH, int& OW,
                     Act act, const void* res, Workspace& ws, hipStream_t s, bool out_f32, bool res_f32) {
  const ConvCall k = conv_call(c, x, B, H, W, y, OH, OW, act, res, ws, out_f32, res_f32);
  if (gemm_partial_floats(k.d, k.prec) > ws.partial_floats || gemm_counter_slots(k.d, k.prec) > kCounterSlots)
    throw std::runtime_error("split-K workspace too small");
  const int nrep = !prof_ ? 1 : op_begin(s, k.name, k.flops, k.bytes);
  for (int r = 0; r < nrep; ++r) gemm(k.d, k.p, k.prec, s);
  if (prof_) op_end(s);
}

// A block's first conv and its downsample conv read the same input: one grouped
// launch (gemm_pair) instead of two dependent ones.
void Model::run_conv_pair(const ConvW& c0, const void* x, int B, int H, int W, void* y0, int& OH0, int& OW0,
                          Act act0, const ConvW& c1, void* y1, bool out1_f32, Workspace& ws, hipStream_t s) {
  int OH1, OW1;
  const ConvCall k0 = conv_call(c0, x, B, H, W, y0, OH0, OW0, act0, nullptr, ws, false, false);
  const ConvCall k1 = conv_call(c1, x, B, H, W, y1, OH1, OW1, Act::None, nullptr, ws, out1_f32, false);
  if (k0.prec != k1.prec) {
    run_conv(c0, x, B, H, W, y0, OH0, OW0, act0, nullptr, ws, s);
    run_conv(c1, x, B, H, W, y1, OH1, OW1, Act::None, nullptr, ws, s, out1_f32);
    return;
  }
  if (gemm_partial_floats(k0.d, k0.prec) + gemm_partial_floats(k1.d, k1.prec) > ws.partial_floats ||
      gemm_counter_slots(k0.d, k0.prec) + gemm_counter_slots(k1.d, k1.prec) > kCounterSlots)
    throw std::runtime_error("split-K workspace too small");
  const int nrep = !prof_ ? 1 : op_begin(s, k0.name + "+" + k1.name, k0.flops + k1.flops, k0.bytes + k1.bytes);
  for (int r = 0; r < nrep; ++r) gemm_pair(k0.d, k0.p, k1.d, k1.p, k0.prec, s);
  if (prof_) op_end(s);
}

void Model::run_gemm(const LinearW& L, const void* A, int M, int lda, void* C, int ldc, bool out_f32, Act act,
                     const void* res, bool res_f32, int ldr, Workspace& ws, hipStream_t s, const LnSpec* ln,
                     size_t planes) {
  GemmDesc d = linear_desc(L, M, lda, ldc);
  d.act = act;
  d.out_f32 = out_f32;
  d.res_f32 = res_f32;
  d.ldr = ldr;
  if (planes) {  // C (and an fp16-typed residual) in two fp16 planes `planes` elements apart
    d.out_planes = true;
    d.res_planes = res != nullptr && !res_f32;
    d.plane = planes;
  }
  d.wplane = L.wplane;
  LnPtrs lp;
  if (ln) {
    if (ln->in_stats) {
      if (!L.c1) throw std::runtime_error("LayerNorm fold: the GEMM's weights were not packed folded");
      d.ln_in_chunks = L.k / 64;
      d.ln_in_eps = eps_;
      lp.in_stats = ln->in_stats;
      lp.c1 = ptr<float>(L.c1);
    }
    if (ln->res_stats) {
      d.res_ln_chunks = L.n / 64;
      d.res_ln_eps = eps_;
      lp.res_stats = ln->res_stats;
      lp.res_g = ln->res_g;
      lp.res_b = ln->res_b;
    }
    if (ln->out_stats) {
      d.ln_out = true;
      d.ld16 = L.n;
      lp.out_stats = ln->out_stats;
      lp.c16 = static_cast<_Float16*>(ln->c16);
    }
  }
  const size_t es = f16_ ? 2 : 4;
  const int nrep = !prof_ ? 1 : op_begin(s, "gemm_M" + std::to_string(M) + "_N" + std::to_string(L.n) + "_K" + std::to_string(L.k),
             2.0 * M * L.n * (double)L.k,
             (double)M * L.k * es + (double)L.n * L.k * es + (double)M * L.n * (out_f32 || planes ? 4 : es) +
                 (res ? (double)M * L.n * (res_f32 || planes ? 4 : es) : 0.0));
  GemmPtrs p;
  p.A = A;
  p.W = ptr<void>(L.w);
  p.bias = ptr<float>(L.b);
  p.res = res;
  p.C = C;
  p.partial = ws.partial;
  p.counters = ws.counters;
  p.zeros = dblob_;  // the blob starts with a zeroed 256-byte line
  p.ln = lp;
  if (gemm_partial_floats(d, L.prec) > ws.partial_floats || gemm_counter_slots(d, L.prec) > kCounterSlots)
    throw std::runtime_error("split-K workspace too small");
  for (int r = 0; r < nrep; ++r) gemm(d, p, L.prec, s);
  if (prof_) op_end(s);
}

void Model::run_qkv_attention(const LinearW& L, const void* x, const float* in_stats, void* qkv, void* ctx, int B,
                              int S, Workspace& w, hipStream_t s) {
  const int T = B * S, hd = D_ / heads_;
  const float scale = 1.0f / std::sqrt((float)hd);
  const float* mask = w.has_mask ? w.mask_bias : nullptr;
  if (qkv_fused_ > 0 && S <= (qkv_fused_ >= 2 ? 256 : 128) && f16_ && L.prec == Prec::F16 &&
      qkv_attention_eligible(S, heads_, hd, L.k, L.kpad, L.krep, D_, L.kpad) && (!in_stats || L.c1)) {
    const int nrep = !prof_ ? 1 : op_begin(s, "qkv_attention_S" + std::to_string(S),
                                           2.0 * T * L.n * (double)L.k + 4.0 * B * S * S * D_,
                                           (double)T * D_ * 2 * 2 + (double)L.n * L.k * 2);
    for (int r = 0; r < nrep; ++r)
      qkv_attention(x, D_, ptr<void>(L.w), L.kpad, ptr<float>(L.b), in_stats, in_stats ? ptr<float>(L.c1) : nullptr,
                    D_ / 64, eps_, mask, ctx, B, S, heads_, scale, s);
    if (prof_) op_end(s);
    return;
  }
  LnSpec q;
  q.in_stats = const_cast<float*>(in_stats);
  run_gemm(L, x, T, D_, qkv, 3 * D_, false, Act::None, nullptr, false, 0, w, s, in_stats ? &q : nullptr);
  const int nrep = !prof_ ? 1 : op_begin(s, "attention_S" + std::to_string(S), 4.0 * B * S * S * D_,
                                         (double)T * 4 * D_ * (f16_ ? 2 : 4));
  for (int r = 0; r < nrep; ++r) attention(qkv, mask, ctx, B, S, heads_, hd, scale, f16_, s);
  if (prof_) op_end(s);
}

// avgpool + fc as one GEMM over every pixel of the last stage with a
// column-mean epilogue (GemmDesc::pool_rows): the split / fp16 / fp32 activation
// is the A operand as is, so the pooled vector never goes through HBM.
bool Model::pooled_fc(int hw) const { return hw > 0 && hw <= 64 && (!split_ || feat_ % 32 == 0); }

GemmDesc Model::pooled_fc_desc(int B, int hw) const {
  GemmDesc d = linear_desc(fc_, B * hw, feat_, classes_);
  d.pool_rows = hw;
  d.out_f32 = true;
  d.a_split = split_;
  d.wplane = fc_.wplane;
  return d;
}

void Model::run_pooled_fc(const void* act, int B, int hw, void* out, Workspace& ws, hipStream_t s) {
  const GemmDesc d = pooled_fc_desc(B, hw);
  if (gemm_partial_floats(d, fc_.prec) > ws.partial_floats || gemm_counter_slots(d, fc_.prec) > kCounterSlots)
    throw std::runtime_error("split-K workspace too small");
  const size_t es = f16_ ? 2 : 4;
  const int nrep = !prof_ ? 1 : op_begin(s, "avgpool_fc_M" + std::to_string(B * hw) + "_N" + std::to_string(classes_) + "_K" +
                    std::to_string(feat_),
             2.0 * B * classes_ * (double)feat_,
             (double)B * hw * feat_ * es + (double)fc_.n * fc_.k * es + (double)B * classes_ * 4);
  GemmPtrs p;
  p.A = act;
  p.W = ptr<void>(fc_.w);
  p.bias = ptr<float>(fc_.b);
  p.C = out;
  p.partial = ws.partial;
  p.counters = ws.counters;
  p.zeros = dblob_;
  for (int r = 0; r < nrep; ++r) gemm(d, p, fc_.prec, s);
  if (prof_) op_end(s);
}

// ---------------------------------------------------------------------------
// Workspaces
// ---------------------------------------------------------------------------
Workspace* Model::workspace(hipStream_t s) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = ws_.find(s);
  if (it != ws_.end()) return it->second.get();
  std::lock_guard<std::mutex> cap(g_capture_mu);
  auto w = std::make_unique<Workspace>();
  const size_t es = f16_ ? 2 : 4;
  const int B = max_batch_;
  size_t partial = 0;
  std::vector<size_t> sizes;  // bytes per buffer
  if (family_ == SPI_FAMILY_RESNET) {
    const int cp = stem_.cin_pad;
    sizes.push_back(stem_fused_ ? 256 : (size_t)B * image_ * image_ * cp * (stem_.prec == Prec::F16 ? 2 : 4));  // ingest
    // F16M: the downsample outputs are fp32 in the same pool
    const size_t ea = mixed_ ? 4 : es;
    int H = image_, OH, OW;
    size_t amax = 0;
    partial = std::max(partial, conv_partial(stem_, B, H, H));
    conv_desc(stem_, B, H, H, OH, OW);
    H = OH;
    if (!stem_fused_) amax = std::max(amax, (size_t)B * H * H * stem_.cout);  // else never materialised
    H = (H + 2 - 3) / 2 + 1;
    amax = std::max(amax, (size_t)B * H * H * stem_.cout);
    for (const auto& b : blocks_) {
      int H2;
      if (b.has_ds)  // conv1 + downsample in one grouped launch (run_conv_pair)
        partial = std::max(partial, conv_partial(b.c1, B, H, H) + conv_partial(b.ds, B, H, H));
      if (bottleneck_) {
        partial = std::max(partial, conv_partial(b.c1, B, H, H));
        amax = std::max(amax, (size_t)B * H * H * b.c1.cout);
        partial = std::max(partial, conv_partial(b.c2, B, H, H));
        conv_desc(b.c2, B, H, H, H2, OW);
        amax = std::max(amax, (size_t)B * H2 * H2 * b.c2.cout);
        partial = std::max(partial, conv_partial(b.c3, B, H2, H2));
        amax = std::max(amax, (size_t)B * H2 * H2 * b.c3.cout);
      } else {
        partial = std::max(partial, conv_partial(b.c1, B, H, H));
        conv_desc(b.c1, B, H, H, H2, OW);
        amax = std::max(amax, (size_t)B * H2 * H2 * b.c1.cout);
        partial = std::max(partial, conv_partial(b.c2, B, H2, H2));
      }
      if (b.has_ds) {
        partial = std::max(partial, conv_partial(b.ds, B, H, H));
        amax = std::max(amax, (size_t)B * H2 * H2 * b.ds.cout);
      }
      H = H2;
    }
    partial = std::max(partial, linear_partial(fc_, B));
    if (pooled_fc(H * H)) partial = std::max(partial, gemm_partial_floats(pooled_fc_desc(B, H * H), fc_.prec));
    for (int i = 0; i < 5; ++i) sizes.push_back(amax * ea);
    sizes.push_back((size_t)B * feat_ * ea);  // pooled (fp32 under F16M: the FC's A)
  } else if (family_ == SPI_FAMILY_BERT) {
    const size_t T = (size_t)B * seq_;
    sizes = {T * D_ * 4, T * D_ * es, T * 3 * D_ * es, T * D_ * es, T * D_ * 4, T * ffn_ * es,
             T * (D_ / 64) * 8, T * (D_ / 64) * 8};  // 6, 7: LayerNorm-fold row statistics S1, S2
    for (const auto& L : tf_)
      partial = std::max({partial, linear_partial(L.qkv, (int)T), linear_partial(L.out, (int)T),
                          linear_partial(L.ff1, (int)T), linear_partial(L.ff2, (int)T)});
    SPI_HIP(hipMalloc(&w->mask_bias, (size_t)B * seq_ * sizeof(float)));
  } else if (family_ == SPI_FAMILY_VIT) {
    const size_t S = npatch_ + 1, T = (size_t)B * S;
    sizes = {(size_t)B * npatch_ * patch_proj_.k * es,  // 0 patches
             (size_t)B * npatch_ * D_ * 4,              // 1 projected patches f32
             T * D_ * 4,                                // 2 residual stream x f32
             T * D_ * es,                               // 3 LN output
             T * 3 * D_ * es,                           // 4 qkv
             T * D_ * es,                               // 5 ctx
             T * ffn_ * es,                             // 6 mlp hidden
             (size_t)B * D_ * es,                       // 7 cls
             T * (D_ / 64) * 8};                        // 8 LayerNorm-fold row statistics of x
    partial = std::max(partial, linear_partial(patch_proj_, B * npatch_));
    for (const auto& L : tf_)
      partial = std::max({partial, linear_partial(L.qkv, (int)T), linear_partial(L.out, (int)T),
                          linear_partial(L.ff1, (int)T), linear_partial(L.ff2, (int)T)});
    partial = std::max(partial, linear_partial(head_, B));
  }
  for (size_t bytes : sizes) {
    void* b = nullptr;
    SPI_HIP(hipMalloc(&b, std::max<size_t>(bytes, 256)));
    w->bufs.push_back(b);
  }
  // Split-K slabs: choose_plan only splits grids of < 128 tiles into <= 512 +
  // tiles workgroups of 64x64, so 640 * 64 * 64 floats bounds every batch size.
  partial = std::max(partial, (size_t)640 * 64 * 64);
  w->partial_floats = partial;
  SPI_HIP(hipMalloc(&w->partial, partial * sizeof(float)));
  SPI_HIP(hipMalloc(&w->counters, kCounterSlots * sizeof(int)));
  // stream-ordered zeroing (a synchronous null-stream memset would also break
  // concurrent captures); it precedes every use of the tickets on this stream
  SPI_HIP(hipMemsetAsync(w->counters, 0, kCounterSlots * sizeof(int), s));
  Workspace* raw = w.get();
  ws_[s] = std::move(w);
  return raw;
}

// ---------------------------------------------------------------------------
// Forward: prologue (reads the task's input buffers) -> body (workspace only,
// graph-capturable) -> epilogue (writes the task's output buffer).
// ---------------------------------------------------------------------------
void Model::prologue(Workspace& w, int B, int S, const void* const* in, hipStream_t s) {
  if (family_ == SPI_FAMILY_RESNET && stem_fused_) {
    // the stem reads the task's NCHW buffer itself and writes the pooled map (buf 2)
    const int OH = (image_ + 6 - 7) / 2 + 1, PH = (OH + 2 - 3) / 2 + 1;
    const int nrep = !prof_ ? 1
                            : op_begin(s, "stem_pool", 2.0 * B * OH * OH * stem_.cout * 147.0,
                                       (double)B * 3 * image_ * image_ * 4 + (double)B * PH * PH * stem_.cout * (split_ ? 4 : 2));
    for (int r = 0; r < nrep; ++r)
      stem_pool(static_cast<const float*>(in[0]), ptr<void>(stem_pool_w_), ptr<float>(stem_.b), w.bufs[2], B, image_,
                image_, split_ ? 2 : stem_.prec != Prec::F16 ? 1 : 0, split_, stem_pr_, s);
    if (prof_) op_end(s);
  } else if (family_ == SPI_FAMILY_RESNET) {
    const int nrep = !prof_ ? 1 : op_begin(s, "ingest_nchw", 0, (double)B * 3 * image_ * image_ * 4 * 2);
    for (int r = 0; r < nrep; ++r)
      ingest_nchw(static_cast<const float*>(in[0]), w.bufs[0], B, 3, image_, image_, stem_.cin_pad,
                  stem_.prec == Prec::F16, s);
    if (prof_) op_end(s);
  } else if (family_ == SPI_FAMILY_BERT) {
    const double T = (double)B * S;
    // the attention mask's additive bias is written by the embedding kernel (round 6: one launch
    // fewer per forward than a separate mask_to_bias)
    w.has_mask = in[1] != nullptr;
    prof_op(s, "bert_embed", T * D_ * (4 * 3 + 4 + (f16_ ? 2 : 0)) + (w.has_mask ? T * 12 : 0), [&] {
      bert_embed(static_cast<const int64_t*>(in[0]), ptr<float>(word_), ptr<float>(pos_), ptr<float>(type0_),
                 ptr<float>(emb_ln_.g), ptr<float>(emb_ln_.b), static_cast<float*>(w.bufs[0]),
                 f16_ ? w.bufs[1] : nullptr, B, S, D_, vocab_, eps_, f16_, s,
                 w.has_mask ? static_cast<const int64_t*>(in[1]) : nullptr, w.has_mask ? w.mask_bias : nullptr);
    });
  } else if (family_ == SPI_FAMILY_VIT) {
    prof_op(s, "patchify", (double)B * 3 * image_ * image_ * (4 + (f16_ ? 2 : 4)),
            [&] { patchify(static_cast<const float*>(in[0]), w.bufs[0], B, 3, image_, image_, patch_, f16_, s); });
  }
}

void Model::body(Workspace& w, int B, int S_in, hipStream_t s) {
  if (family_ == SPI_FAMILY_RESNET) {
    int H = image_, OH, OW;
    void* const* buf = w.bufs.data();
    if (stem_fused_) {  // stem + max pool ran in the prologue
      OH = (H + 6 - 7) / 2 + 1;
      H = (OH + 2 - 3) / 2 + 1;
    } else {
      run_conv(stem_, buf[0], B, H, H, buf[1], OH, OW, Act::Relu, nullptr, w, s);
      H = OH;
      const int PH = (H + 2 - 3) / 2 + 1;
      const int nrep = !prof_ ? 1 : op_begin(s, "maxpool", 0, (double)B * (H * H + PH * PH) * stem_.cout * (f16_ ? 2 : 4));
      for (int r = 0; r < nrep; ++r) {
        if (split_)
          maxpool_nhwc_split(buf[1], buf[2], B, H, H, stem_.cout, PH, PH, 3, 2, 1, s);
        else
          maxpool_nhwc(buf[1], buf[2], B, H, H, stem_.cout, PH, PH, 3, 2, 1, f16_, s);
      }
      if (prof_) op_end(s);
      H = PH;
    }
    int cur = 2;
    auto pick = [&](std::initializer_list<int> busy) {
      for (int i = 1; i <= 5; ++i)
        if (std::find(busy.begin(), busy.end(), i) == busy.end()) return i;
      return -1;
    };
    for (const auto& b : blocks_) {
      int H2;
      if (bottleneck_) {
        const int t1 = pick({cur});
        int ident = cur;
        if (b.has_ds) {  // the downsample reads the block input too: grouped with conv1
          ident = pick({cur, t1});
          run_conv_pair(b.c1, buf[cur], B, H, H, buf[t1], OH, OW, Act::Relu, b.ds, buf[ident], false, w, s);
        } else {
          run_conv(b.c1, buf[cur], B, H, H, buf[t1], OH, OW, Act::Relu, nullptr, w, s);
        }
        const int t2 = pick({cur, t1, ident});
        run_conv(b.c2, buf[t1], B, H, H, buf[t2], H2, OW, Act::Relu, nullptr, w, s);
        const int o = pick({cur, t2, ident});
        run_conv(b.c3, buf[t2], B, H2, H2, buf[o], OH, OW, Act::Relu, buf[ident], w, s);
        cur = o;
      } else {
        const int t1 = pick({cur});
        int ident = cur;
        if (b.has_ds) {  // F16M: hi + lo weights, fp16 out like every conv (round 5: fp32 out kept nothing)
          ident = pick({cur, t1});
          run_conv_pair(b.c1, buf[cur], B, H, H, buf[t1], H2, OW, Act::Relu, b.ds, buf[ident], false, w, s);
        } else {
          run_conv(b.c1, buf[cur], B, H, H, buf[t1], H2, OW, Act::Relu, nullptr, w, s);
        }
        const int o = pick({cur, t1, ident});
        run_conv(b.c2, buf[t1], B, H2, H2, buf[o], OH, OW, Act::Relu, buf[ident], w, s);
        cur = o;
      }
      H = H2;
    }
    w.final_buf = cur;
    w.final_hw = H * H;
    if (!pooled_fc(H * H)) {  // else avgpool + fc run as one GEMM in the epilogue
      const int nrep = !prof_ ? 1 : op_begin(s, "avgpool", 0, (double)B * H * H * feat_ * (f16_ ? 2 : 4));
      for (int r = 0; r < nrep; ++r) {
        if (split_)
          avgpool_nhwc_split(buf[cur], static_cast<float*>(buf[6]), B, H * H, feat_, s);  // fp32 for the F16X3 FC
        else
          avgpool_nhwc(buf[cur], buf[6], B, H * H, feat_, f16_, s, mixed_);  // F16M: fp32 for the F16X3 FC
      }
      if (prof_) op_end(s);
      w.final_buf = 6;
    }
  } else if (family_ == SPI_FAMILY_BERT) {
    const int S = S_in, T = B * S;
    float* hf = static_cast<float*>(w.bufs[0]);
    void* ht = f16_ ? w.bufs[1] : w.bufs[0];
    void* qkv = w.bufs[2];
    void* ctx = w.bufs[3];
    float* a = static_cast<float*>(w.bufs[4]);
    void* ff = w.bufs[5];
    if (ln_fold_) {
      // Post-LN with the LayerNorms folded (ln_fold.hpp) over two-plane fp16 rows (round 6,
      // GemmDesc::res_planes: hi = fp16(x), lo = fp16(x - hi), a plane of T x D apart, the bytes of
      // fp32): buf 0 holds the embedding output (fp32, the prologue's), then each layer's pre-LN2
      // rows b as planes; buf 4 the pre-LN1 rows a as planes; S1 / S2 their row statistics.  The hi
      // planes are the folding GEMMs' fp16 A operands, so no producer writes an fp16 copy.
      // Layer i:
      //   qkv  = LN2_{i-1}(b) Wqkv  (folded; layer 0 reads the embedding's fp16 output ht)
      //   a    = ctx Wo + LN2_{i-1}(b)    -> S1   (layer 0: + the fp32 embedding output)
      //   ff   = GELU(LN1_i(a) W1)  (folded)
      //   b    = ff W2 + LN1_i(a)         -> S2
      // and the epilogue runs the one LayerNorm left, LN2 of the last layer.
      float* S1 = static_cast<float*>(w.bufs[6]);
      float* S2 = static_cast<float*>(w.bufs[7]);
      _Float16* bh = static_cast<_Float16*>(w.bufs[0]);
      _Float16* ah = static_cast<_Float16*>(w.bufs[4]);
      const size_t plane = (size_t)T * D_;
      for (int i = 0; i < layers_; ++i) {
        const TfLayer& L = tf_[i];
        run_qkv_attention(L.qkv, i > 0 ? bh : ht, i > 0 ? S2 : nullptr, qkv, ctx, B, S, w, s);
        LnSpec o;
        if (i > 0) {
          o.res_stats = S2;
          o.res_g = ptr<float>(tf_[i - 1].ln2.g);
          o.res_b = ptr<float>(tf_[i - 1].ln2.b);
        }
        o.out_stats = S1;
        run_gemm(L.out, ctx, T, D_, ah, D_, false, Act::None, i > 0 ? static_cast<void*>(bh) : hf, i == 0, D_, w, s,
                 &o, plane);
        LnSpec f1;
        f1.in_stats = S1;
        run_gemm(L.ff1, ah, T, D_, ff, ffn_, false, Act::Gelu, nullptr, false, 0, w, s, &f1);
        LnSpec f2;
        f2.res_stats = S1;
        f2.res_g = ptr<float>(L.ln1.g);
        f2.res_b = ptr<float>(L.ln1.b);
        f2.out_stats = S2;
        run_gemm(L.ff2, ff, T, ffn_, bh, D_, false, Act::None, ah, false, D_, w, s, &f2, plane);
      }
      return;
    }
    for (int i = 0; i < layers_; ++i) {
      const TfLayer& L = tf_[i];
      run_qkv_attention(L.qkv, ht, nullptr, qkv, ctx, B, S, w, s);
      run_gemm(L.out, ctx, T, D_, a, D_, true, Act::None, hf, true, D_, w, s);
      prof_op(s, "layernorm", ln_bytes(T, true), [&] {
        layernorm(a, D_, ptr<float>(L.ln1.g), ptr<float>(L.ln1.b), hf, f16_ ? ht : nullptr, D_, T, D_, eps_, f16_, s);
      });
      run_gemm(L.ff1, ht, T, D_, ff, ffn_, false, Act::Gelu, nullptr, false, 0, w, s);
      run_gemm(L.ff2, ff, T, ffn_, a, D_, true, Act::None, hf, true, D_, w, s);
      if (i + 1 < layers_)
        prof_op(s, "layernorm", ln_bytes(T, true), [&] {
          layernorm(a, D_, ptr<float>(L.ln2.g), ptr<float>(L.ln2.b), hf, f16_ ? ht : nullptr, D_, T, D_, eps_, f16_,
                    s);
        });
    }
  } else if (family_ == SPI_FAMILY_VIT) {
    const int S = npatch_ + 1, T = B * S;
    void* const* buf = w.bufs.data();
    float* x = static_cast<float*>(buf[2]);
    run_gemm(patch_proj_, buf[0], B * npatch_, patch_proj_.k, buf[1], D_, true, Act::None, nullptr, false, 0,
             w, s);
    if (!ln_fold_)
      prof_op(s, "vit_assemble", (double)T * D_ * 4 * 3, [&] {
        vit_assemble(static_cast<const float*>(buf[1]), ptr<float>(cls_), ptr<float>(vpos_), x, B, npatch_, D_, s);
      });
    if (ln_fold_) {
      // Pre-LN with the LayerNorms folded (ln_fold.hpp) over a two-plane residual stream (round 6,
      // GemmDesc::res_planes): x lives in buf 2 as hi = fp16(x) and lo = fp16(x - hi), a plane of
      // T x D apart -- the bytes of fp32, ~22-bit values.  vit_assemble_planes and the GEMMs that
      // update x (out-proj, FFN2: residual and output both two-plane, in place) write the rows'
      // chunk statistics Sx; the QKV GEMMs of layers >= 1 and every FFN1 GEMM read the hi plane as
      // their fp16 A operand with LN1 / LN2 folded in.  No producer writes an fp16 copy (the hi
      // plane is one).  Two LayerNorm launches are left: layer 0's LN1 (the stream's first rows
      // come from the patch embedding, whose row means make the folded form lose ~20 % of the fp16
      // margin: test_transformer_layernorm_fold, 8.5e-4 folded vs 7.0e-4 at this launch) and the
      // class-token LayerNorm at the end.
      float* Sx = static_cast<float*>(buf[8]);
      _Float16* xh = static_cast<_Float16*>(buf[2]);
      const size_t plane = (size_t)T * D_;
      prof_op(s, "vit_assemble", (double)T * D_ * 4 * 3, [&] {
        vit_assemble_planes(static_cast<const float*>(buf[1]), ptr<float>(cls_), ptr<float>(vpos_), xh, plane,
                            nullptr, B, npatch_, D_, s);
      });
      for (int i = 0; i < layers_; ++i) {
        const TfLayer& L = tf_[i];
        LnSpec q;
        if (i == 0) {
          prof_op(s, "layernorm", ln_bytes(T, false), [&] {
            layernorm_planes(xh, plane, D_, ptr<float>(L.ln1.g), ptr<float>(L.ln1.b), nullptr, buf[3], D_, T, D_,
                             eps_, f16_, s);
          });
        } else {
          q.in_stats = Sx;
        }
        run_qkv_attention(L.qkv, i == 0 ? buf[3] : xh, q.in_stats, buf[4], buf[5], B, S, w, s);
        LnSpec o;
        o.out_stats = Sx;
        run_gemm(L.out, buf[5], T, D_, xh, D_, false, Act::None, xh, false, D_, w, s, &o, plane);
        LnSpec f1;
        f1.in_stats = Sx;
        run_gemm(L.ff1, xh, T, D_, buf[6], ffn_, false, Act::Gelu, nullptr, false, 0, w, s, &f1);
        run_gemm(L.ff2, buf[6], T, ffn_, xh, D_, false, Act::None, xh, false, D_, w, s, &o, plane);
      }
      prof_op(s, "layernorm_cls", ln_bytes(B, false), [&] {
        layernorm_planes(xh, plane, S * D_, ptr<float>(final_ln_.g), ptr<float>(final_ln_.b), nullptr, buf[7], D_, B,
                         D_, eps_, f16_, s);
      });
      return;
    } else {
    for (const TfLayer& L : tf_) {
      prof_op(s, "layernorm", ln_bytes(T, false), [&] {
        layernorm(x, D_, ptr<float>(L.ln1.g), ptr<float>(L.ln1.b), f16_ ? nullptr : static_cast<float*>(buf[3]),
                  f16_ ? buf[3] : nullptr, D_, T, D_, eps_, f16_, s);
      });
      run_qkv_attention(L.qkv, buf[3], nullptr, buf[4], buf[5], B, S, w, s);
      run_gemm(L.out, buf[5], T, D_, x, D_, true, Act::None, x, true, D_, w, s);
      prof_op(s, "layernorm", ln_bytes(T, false), [&] {
        layernorm(x, D_, ptr<float>(L.ln2.g), ptr<float>(L.ln2.b), f16_ ? nullptr : static_cast<float*>(buf[3]),
                  f16_ ? buf[3] : nullptr, D_, T, D_, eps_, f16_, s);
      });
      run_gemm(L.ff1, buf[3], T, D_, buf[6], ffn_, false, Act::Gelu, nullptr, false, 0, w, s);
      run_gemm(L.ff2, buf[6], T, ffn_, x, D_, true, Act::None, x, true, D_, w, s);
    }
    }
    // final LN on the class-token rows only (torchvision: x = ln(x); x = x[:, 0])
    prof_op(s, "layernorm_cls", ln_bytes(B, false), [&] {
      layernorm(x, S * D_, ptr<float>(final_ln_.g), ptr<float>(final_ln_.b),
                f16_ ? nullptr : static_cast<float*>(buf[7]), f16_ ? buf[7] : nullptr, D_, B, D_, eps_, f16_, s);
    });
  }
}

void Model::epilogue(Workspace& w, int B, int S, void* const* out, hipStream_t s) {
  if (family_ == SPI_FAMILY_RESNET) {
    if (pooled_fc(w.final_hw))
      run_pooled_fc(w.bufs[w.final_buf], B, w.final_hw, out[0], w, s);
    else
      run_gemm(fc_, w.bufs[6], B, feat_, out[0], classes_, true, Act::None, nullptr, false, 0, w, s);
  } else if (family_ == SPI_FAMILY_BERT) {
    const TfLayer& L = tf_.back();
    const int T = B * S;
    prof_op(s, "layernorm_out", (double)T * D_ * 8, [&] {
      // the last layer's pre-LN2 rows: the two-plane b (buf 0) under the LayerNorm fold, else a
      if (ln_fold_)
        layernorm_planes(static_cast<const _Float16*>(w.bufs[0]), (size_t)T * D_, D_, ptr<float>(L.ln2.g),
                         ptr<float>(L.ln2.b), static_cast<float*>(out[0]), nullptr, D_, T, D_, eps_, f16_, s);
      else
        layernorm(static_cast<float*>(w.bufs[4]), D_, ptr<float>(L.ln2.g), ptr<float>(L.ln2.b),
                  static_cast<float*>(out[0]), nullptr, D_, T, D_, eps_, f16_, s);
    });
  } else if (family_ == SPI_FAMILY_VIT) {
    run_gemm(head_, w.bufs[7], B, D_, out[0], classes_, true, Act::None, nullptr, false, 0, w, s);
  }
}

void Model::forward(hipStream_t s, int B, int S, size_t n, const void* const* in, void* const* out) {
  if (device_ < 0) throw std::runtime_error("host-only replica (device < 0) cannot run a forward");
  if (family_ == SPI_FAMILY_AFFINE) {
    affine(static_cast<const float*>(in[0]), static_cast<float*>(out[0]), n, aff_scale_, aff_shift_, s);
    return;
  }
  if (family_ != SPI_FAMILY_BERT) S = 0;  // only BERT's graphs depend on the sequence length
  Workspace* w = workspace(s);
  prologue(*w, B, S, in, s);
  if (graphs_ && s != nullptr) {
    SPI_HIP(hipGraphLaunch(graph(*w, B, S, s), s));
  } else {
    body(*w, B, S, s);
  }
  epilogue(*w, B, S, out, s);
}

// The captured body for (batch, mask, S) on this stream's workspace, captured
// on first use (or ahead of time by warmup()).
hipGraphExec_t Model::graph(Workspace& w, int B, int S, hipStream_t s) {
  const int key = (B * 2 + (w.has_mask ? 1 : 0)) * 4096 + S;
  auto it = w.graphs.find(key);
  if (it != w.graphs.end()) return it->second;
  std::lock_guard<std::mutex> cap(g_capture_mu);
  SPI_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipGraph_t g = nullptr;
  try {
    body(w, B, S, s);
  } catch (...) {
    // Leave the worker stream usable: end the capture before rethrowing,
    // otherwise every later task on this stream fails.
    if (hipStreamEndCapture(s, &g) == hipSuccess && g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    throw;
  }
  SPI_HIP(hipStreamEndCapture(s, &g));
  hipGraphExec_t e = nullptr;
  const hipError_t ie = hipGraphInstantiate(&e, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  SPI_HIP(ie);
  return w.graphs.emplace(key, e).first->second;
}

// Per-worker warm-up (the reference warms each worker up before serving,
// inference_runner.cpp:507-560): allocate this stream's workspace and capture
// the body graph for (batch, S, mask) now, so no capture or allocation lands on
// a live request.  Runs nothing on the device.
void Model::warmup(hipStream_t s, int B, int S, bool mask) {
  if (device_ < 0) throw std::runtime_error("host-only replica (device < 0) cannot run a forward");
  if (family_ == SPI_FAMILY_AFFINE) return;
  if (B < 1 || B > max_batch_) throw std::runtime_error("warmup batch exceeds replica max_batch");
  if (family_ == SPI_FAMILY_BERT && (S < 1 || S > seq_)) throw std::runtime_error("warmup sequence length out of range");
  Workspace* w = workspace(s);
  if (!graphs_ || s == nullptr) return;
  w->has_mask = family_ == SPI_FAMILY_BERT && mask;
  (void)graph(*w, B, family_ == SPI_FAMILY_BERT ? S : 0, s);
}

}  // namespace spi

namespace spi {

thread_local std::vector<Model::OpRecord>* Model::prof_ = nullptr;

std::vector<LaunchRec>*& launch_log() {
  static thread_local std::vector<LaunchRec>* log = nullptr;
  return log;
}
thread_local Model::ProfRepeat* Model::prof_rep_ = nullptr;
#ifdef SPI_GEMM_TIMELINE
extern "C" void spi_debug_gemm_timeline_enable(int on, hipStream_t s);
#endif

int Model::op_begin(hipStream_t s, const std::string& name, double flops, double bytes) {
  OpRecord r{name, flops, bytes, nullptr, nullptr, 1};
  if (prof_rep_ && !prof_rep_->done && name == prof_rep_->name) {  // the op profile_op() repeats
    prof_rep_->done = true;
    r.reps = prof_rep_->reps;
#ifdef SPI_GEMM_TIMELINE
    spi_debug_gemm_timeline_enable(1, s);  // stamp only the repeated op's launches
#endif
  }
  SPI_HIP(hipEventCreate(&r.start));
  SPI_HIP(hipEventCreate(&r.stop));
  SPI_HIP(hipEventRecord(r.start, s));
  prof_->push_back(r);
  launch_log() = &prof_->back().launches;  // until op_end (no other record is pushed meanwhile)
  return r.reps;
}

void Model::op_end(hipStream_t s) {
  launch_log() = nullptr;
  SPI_HIP(hipEventRecord(prof_->back().stop, s));
#ifdef SPI_GEMM_TIMELINE
  if (prof_->back().reps > 1) spi_debug_gemm_timeline_enable(0, s);
#endif
}

void Model::run_profiled(hipStream_t s, int B, int S, const void* const* in, void* const* out,
                         std::vector<OpRecord>& recs) {
  if (device_ < 0) throw std::runtime_error("host-only replica (device < 0) cannot run a forward");
  Workspace* w = workspace(s);
  prof_ = &recs;
  try {
    prologue(*w, B, S, in, s);
    body(*w, B, S, s);
    epilogue(*w, B, S, out, s);
  } catch (...) {
    prof_ = nullptr;
    launch_log() = nullptr;
    for (auto& r : recs) {
      (void)hipEventDestroy(r.start);
      (void)hipEventDestroy(r.stop);
    }
    recs.clear();
    throw;
  }
  prof_ = nullptr;
  SPI_HIP(hipStreamSynchronize(s));
}

int Model::profile(hipStream_t s, int B, int S, const void* const* in, void* const* out, float* ms,
                   double* flops, double* bytes, char* names, int name_len, int max_ops) {
  if (family_ == SPI_FAMILY_AFFINE) return 0;
  std::vector<OpRecord> recs;
  run_profiled(s, B, S, in, out, recs);
  int n = 0;
  for (auto& r : recs) {
    if (n < max_ops) {
      float t = 0.f;
      SPI_HIP(hipEventElapsedTime(&t, r.start, r.stop));
      if (ms) ms[n] = t / r.reps;  // per launch
      if (flops) flops[n] = r.flops;
      if (bytes) bytes[n] = r.bytes;
      if (names && name_len > 0) std::snprintf(names + (size_t)n * name_len, name_len, "%s", r.name.c_str());
      ++n;
    }
    (void)hipEventDestroy(r.start);
    (void)hipEventDestroy(r.stop);
  }
  return n;
}

std::string Model::launch_table(hipStream_t s, int B, int S, const void* const* in, void* const* out) {
  if (family_ == SPI_FAMILY_AFFINE) return "";
  std::vector<OpRecord> recs;
  run_profiled(s, B, S, in, out, recs);
  std::string t;
  for (size_t i = 0; i < recs.size(); ++i) {
    for (const LaunchRec& l : recs[i].launches) {
      // kernel_id's __PRETTY_FUNCTION__: "... [F = &spi::(anonymous namespace)::name<args>]"
      std::string k = l.kernel;
      const size_t a = k.find("F = &");
      if (a != std::string::npos) k = k.substr(a + 5, k.size() - (a + 5) - (k.back() == ']' ? 1 : 0));
      t += std::to_string(i) + "\t" + recs[i].name + "\t" + k + "\t" + std::to_string(l.gx) + "\t" +
           std::to_string(l.gy) + "\t" + std::to_string(l.gz) + "\t" + std::to_string(l.block) + "\n";
    }
    (void)hipEventDestroy(recs[i].start);
    (void)hipEventDestroy(recs[i].stop);
  }
  return t;
}

int Model::profile_op(hipStream_t s, int B, int S, const void* const* in, void* const* out, const char* name,
                      int reps, float* ms, double* flops, double* bytes) {
  if (!name || reps < 1) throw std::runtime_error("profile_op: name and reps >= 1 required");
  ProfRepeat rep{name, reps, false};
  prof_rep_ = &rep;
  std::vector<float> t(4096);
  std::vector<double> f(4096), b(4096);
  std::vector<char> names((size_t)4096 * 96);
  int n = 0;
  try {
    n = profile(s, B, S, in, out, t.data(), f.data(), b.data(), names.data(), 96, 4096);
  } catch (...) {
    prof_rep_ = nullptr;
    throw;
  }
  prof_rep_ = nullptr;
  for (int i = 0; i < n; ++i)
    if (std::strcmp(names.data() + (size_t)i * 96, name) == 0) {
      if (ms) *ms = t[i];
      if (flops) *flops = f[i];
      if (bytes) *bytes = b[i];
      return 0;
    }
  throw std::runtime_error(std::string("profile_op: no op named ") + name);
}

}  // namespace spi
