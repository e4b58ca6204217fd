// C-ABI front end of libllmvox_hip.so (see include/llmvox.h).
//
// Owns: the device copies of all hot-path weights (converted / repacked for the kernels),
// the KV pool (max_streams slots x max_positions), the per-step scratch, the codec scratch,
// and the HIP graphs of the fused decode step.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "llmvox.h"
#include "lvx_internal.h"

using namespace lvx;

namespace lvx {
static const Opts kDefaultOpts{};
static thread_local const Opts* t_opts = nullptr;
const Opts& opts() { return t_opts ? *t_opts : kDefaultOpts; }
OptScope::OptScope(const Opts* o) : prev(t_opts) { t_opts = o; }
OptScope::~OptScope() { t_opts = prev; }
}  // namespace lvx

static constexpr int kMaxCodecL = 4096;
#ifndef LVX_GRAPH_STEPS
#define LVX_GRAPH_STEPS 16  // A/B builds (tools/build_variant.sh NAME -DLVX_GRAPH_STEPS=n)
#endif
static constexpr int kGraphSteps = LVX_GRAPH_STEPS;  // decode steps per captured graph

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Status of taken error bits (AR word | codec word << 16, as err_take_kernel reports them): the message
// names EVERY set condition; the code is the most specific one (index > state > capacity).
int bits_status(int32_t bits) {
  if (!bits) return LVX_OK;
  const int32_t ar = bits & 0xffff, cd = (bits >> 16) & 0xffff;
  std::string m;
  int code = 0;
  auto add = [&](int c, const char* what) {
    if (!m.empty()) m += "; ";
    m += what;
    if (code == 0 || (c == LVX_E_INDEX) || (c == LVX_E_STATE && code == LVX_E_CAPACITY)) code = c;
  };
  if (ar & 4) add(LVX_E_INDEX, "index out of range in self (a text id outside [0, 386) given to lvx_text_embed or a code "
                               "outside [0, 4096) given to lvx_codes_to_features)");
  if (cd & 4) add(LVX_E_INDEX, "index out of range in self (codec: a code outside [0, 4096) given to lvx_codec_decode_codes)");
  if (ar & 32) add(LVX_E_STATE, "a non-finite or out-of-range (|v| >= 2^25) partial in the fused MLP's fixed-point "
                                "accumulation (B <= 2): the logits of that step's rows are invalid");
  if (cd & 8) add(LVX_E_STATE, "ISTFT window envelope <= 1e-11 (spectral_ops.py:72 assertion)");
  if (ar & 1) add(LVX_E_CAPACITY, "a stream exceeded its KV capacity (max_positions)");
  if (ar & 2) add(LVX_E_CAPACITY, "a batch row ran past the end of its text plan (plan_stride)");
  if (!code) add(LVX_E_STATE, "unknown device error bits");
  char hex[32];
  snprintf(hex, sizeof hex, " [error bits 0x%x]", (unsigned)bits);
  return fail(code, m + hex);
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return fail(LVX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));         \
  } while (0)

struct WeightSpec {
  std::vector<int64_t> shape;
};

std::map<std::string, WeightSpec> make_specs() {
  std::map<std::string, WeightSpec> s;
  s["transformer.wpe.weight"] = {{BLOCK_SIZE, D}};
  for (int i = 0; i < N_LAYER; ++i) {
    std::string p = "transformer.h." + std::to_string(i) + ".";
    s[p + "ln_1.weight"] = {{D}};
    s[p + "attn.c_attn.weight"] = {{3 * D, D}};
    s[p + "attn.c_proj.weight"] = {{D, D}};
    s[p + "ln_2.weight"] = {{D}};
    s[p + "mlp.c_fc.weight"] = {{DFF, D}};
    s[p + "mlp.c_proj.weight"] = {{D, DFF}};
  }
  s["transformer.ln_f.weight"] = {{D}};
  s["lm_head.weight"] = {{VOCAB, D}};
  s["encoder.embed_tokens.weight"] = {{TEXT_VOCAB, TEXT_DIM}};
  s["feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed"] = {{4096, SPEECH_DIM}};
  const int CD = 768, CFF = 2304;
  s["backbone.embed.weight"] = {{CD, 512, 7}};
  s["backbone.embed.bias"] = {{CD}};
  s["backbone.norm.scale.weight"] = {{4, CD}};
  s["backbone.norm.shift.weight"] = {{4, CD}};
  for (int i : {0, 1, 3, 4}) {
    std::string p = "backbone.pos_net." + std::to_string(i) + ".";
    for (const char* n : {"norm1", "norm2"}) {
      s[p + n + ".weight"] = {{CD}};
      s[p + n + ".bias"] = {{CD}};
    }
    for (const char* n : {"conv1", "conv2"}) {
      s[p + n + ".weight"] = {{CD, CD, 3}};
      s[p + n + ".bias"] = {{CD}};
    }
  }
  s["backbone.pos_net.2.norm.weight"] = {{CD}};
  s["backbone.pos_net.2.norm.bias"] = {{CD}};
  for (const char* n : {"q", "k", "v", "proj_out"}) {
    s[std::string("backbone.pos_net.2.") + n + ".weight"] = {{CD, CD, 1}};
    s[std::string("backbone.pos_net.2.") + n + ".bias"] = {{CD}};
  }
  s["backbone.pos_net.5.weight"] = {{CD}};
  s["backbone.pos_net.5.bias"] = {{CD}};
  for (int i = 0; i < 12; ++i) {
    std::string p = "backbone.convnext." + std::to_string(i) + ".";
    s[p + "dwconv.weight"] = {{CD, 1, 7}};
    s[p + "dwconv.bias"] = {{CD}};
    s[p + "norm.scale.weight"] = {{4, CD}};
    s[p + "norm.shift.weight"] = {{4, CD}};
    s[p + "pwconv1.weight"] = {{CFF, CD}};
    s[p + "pwconv1.bias"] = {{CFF}};
    s[p + "pwconv2.weight"] = {{CD, CFF}};
    s[p + "pwconv2.bias"] = {{CD}};
    s[p + "gamma"] = {{CD}};
  }
  s["backbone.final_layer_norm.weight"] = {{CD}};
  s["backbone.final_layer_norm.bias"] = {{CD}};
  s["head.out.weight"] = {{1282, CD}};
  s["head.out.bias"] = {{1282}};
  return s;
}

const std::map<std::string, WeightSpec>& specs() {
  static const std::map<std::string, WeightSpec> s = make_specs();
  return s;
}

int64_t numel_of(const WeightSpec& w) {
  int64_t n = 1;
  for (auto d : w.shape) n *= d;
  return n;
}

}  // namespace

struct GraphKey {
  int B, stride, nsteps;
  const void *slots, *text, *rowstep, *tok, *margin;
  void* stream;
  bool operator<(const GraphKey& o) const {
    return std::tie(B, stride, nsteps, slots, text, rowstep, tok, margin, stream) <
           std::tie(o.B, o.stride, o.nsteps, o.slots, o.text, o.rowstep, o.tok, o.margin, o.stream);
  }
};

// host f32 -> OCP e4m3fn (gfx950 fp8), round to nearest even, saturated to +-448, NaN -> 0x7f
static uint8_t f32_to_e4m3_host(float x) {
  if (std::isnan(x)) return 0x7f;
  const uint8_t sign = std::signbit(x) ? 0x80 : 0x00;
  double a = std::fabs((double)x);
  if (a >= 448.0) return sign | 0x7e;
  if (a < std::ldexp(1.0, -6)) {  // subnormal: value = mant * 2^-9 (mant 8 is the smallest normal)
    const int q = (int)std::nearbyint(a * 512.0);
    return sign | (uint8_t)q;
  }
  int e;
  const double m = std::frexp(a, &e);  // a = m * 2^e, m in [0.5, 1)
  int mant = (int)std::nearbyint((m * 2.0 - 1.0) * 8.0);
  int ex = e - 1;
  if (mant == 8) { mant = 0; ++ex; }
  int code = ((ex + 7) << 3) | mant;
  if (code > 0x7e) code = 0x7e;
  return sign | (uint8_t)code;
}

struct lvx_ctx {
  lvx_config cfg{};
  std::map<std::string, std::vector<float>> host;  // staged fp32 weights (released at finalize)
  std::vector<void*> allocs;
  bool finalized = false;
  ArWeights arw;
  ArState st;
  CodecWeights cw;
  CodecScratch cs;
  float* window_override = nullptr;
  std::map<GraphKey, hipGraphExec_t> graphs;
  std::vector<hipGraph_t> graph_defs;
  bool use_graphs = true;
  Opts opts;                 // this context's kernel options (lvx_set_option, under mu)
  unsigned opt_epoch = 0;    // bumped by every lvx_set_option on this context (under mu)
  unsigned graph_epoch = 0;  // opt_epoch when the cached graphs were captured
  hipStream_t capture_stream = nullptr;  // lvx_set_capture_stream (not owned); null: capture on the caller's
  hipStream_t own_capture_stream = nullptr;  // created for null-stream callers only (cached_graph)
  std::mutex mu;

  // a snapshot of the options, taken under mu: the caller binds it (OptScope) for its launches
  Opts opts_snapshot() {
    std::lock_guard<std::mutex> lk(mu);
    return opts;
  }

  template <typename T>
  int dalloc(T** p, size_t n) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, n * sizeof(T) + 256);
    if (e != hipSuccess) return fail(LVX_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    allocs.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return 0;
  }
  int upload_f32(const std::vector<float>& v, const float** out) {
    float* d;
    if (int r = dalloc(&d, v.size())) return r;
    HIP_TRY(hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    *out = d;
    return 0;
  }
  // matrices in the weight dtype
  int upload_w(const std::vector<float>& v, const void** out) {
    if (cfg.weight_dtype == LVX_DTYPE_F32) return upload_f32(v, reinterpret_cast<const float**>(out));
    std::vector<bf16_t> h(v.size());
    for (size_t i = 0; i < v.size(); ++i) h[i] = f32_to_bf16(v[i]);
    bf16_t* d;
    if (int r = dalloc(&d, h.size())) return r;
    HIP_TRY(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    *out = d;
    return 0;
  }
  // codec GEMM weights: the weight dtype, or e4m3fn with one scale per output row (codec_dtype FP8:
  // s = max|w_row| / 448, q = RNE(w / s) saturated; dequantised exactly to bf16 in the GEMM loader)
  //
  // fp32 (parity mode) with K % 32 == 0: the matrix [rows][K] is followed in the same allocation by its
  // bf16x3 split image (same size, read by gemm_glds_kernel<float, SPLIT> in place of the fp32 rows):
  // per row and 32-k block kb, 16-B segment g (g < 4) holds bf16_rn(w) of k = kb + 4 g + e and
  // kb + 16 + 4 g + e (e = 0..3), segment 4 + g the lo parts bf16_rn(w - hi) of the same k (the k
  // order the kernel's A fragments are read in)
  int upload_cw(const std::vector<float>& v, int rows, const void** out, const float** scale_out) {
    const size_t K = v.size() / rows;
    if (cfg.codec_dtype != LVX_DTYPE_FP8 && cfg.weight_dtype == LVX_DTYPE_F32 && K % 32 == 0) {
      std::vector<float> both(2 * v.size());
      std::memcpy(both.data(), v.data(), v.size() * 4);
      bf16_t* sp = reinterpret_cast<bf16_t*>(both.data() + v.size());
      for (size_t n = 0; n < (size_t)rows; ++n)
        for (size_t kb = 0; kb < K; kb += 32) {
          bf16_t* o = sp + (n * K + kb) * 2;  // 128 B: 8 segments of 8 bf16
          for (int g = 0; g < 4; ++g)
            for (int h = 0; h < 2; ++h)
              for (int e = 0; e < 4; ++e) {
                const float x = v[n * K + kb + 16 * h + 4 * g + e];
                const bf16_t hi = f32_to_bf16(x);
                const uint32_t hb = (uint32_t)hi << 16;
                float hf;
                std::memcpy(&hf, &hb, 4);
                o[g * 8 + h * 4 + e] = hi;
                o[(4 + g) * 8 + h * 4 + e] = f32_to_bf16(x - hf);
              }
        }
      return upload_f32(both, reinterpret_cast<const float**>(out));
    }
    if (cfg.codec_dtype != LVX_DTYPE_FP8) return upload_w(v, out);
    std::vector<uint8_t> q(v.size());
    std::vector<float> sc(rows);
    for (int n = 0; n < rows; ++n) {
      float mx = 0.f;
      for (size_t k = 0; k < K; ++k) mx = std::max(mx, std::fabs(v[n * K + k]));
      const float s = mx > 0.f ? mx / 448.f : 1.f;
      sc[n] = s;
      for (size_t k = 0; k < K; ++k) q[n * K + k] = f32_to_e4m3_host(v[n * K + k] / s);
    }
    uint8_t* d;
    if (int r = dalloc(&d, q.size())) return r;
    HIP_TRY(hipMemcpy(d, q.data(), q.size(), hipMemcpyHostToDevice));
    *out = d;
    return upload_f32(sc, scale_out);
  }
  const std::vector<float>& H(const std::string& k) { return host.at(k); }
};

// conv weight [N][C][T] -> tap-major [N][T*C]
static std::vector<float> repack_conv(const std::vector<float>& w, int N, int C, int T) {
  std::vector<float> o((size_t)N * C * T);
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < C; ++c)
      for (int t = 0; t < T; ++t) o[(size_t)n * T * C + (size_t)t * C + c] = w[((size_t)n * C + c) * T + t];
  return o;
}

// mlp.c_proj [768][3072] -> [3072/16 blocks][256 threads][3][16]: block k's thread t holds
// W[t + 256 jj][16 k + j] as 96 contiguous bytes (bf16), the operand order of ar_mlp_fused_kernel
// mlp.c_proj [768][3072] for ar_mlp_fused_kernel: groups of 4 columns k4, then the output row's
// third jj (e = t + 256 jj), then thread t, 4 values: a wave's 8-byte load covers 512 contiguous bytes
static std::vector<float> pack_mproj(const std::vector<float>& w) {
  std::vector<float> o((size_t)D * DFF);
  size_t q = 0;
  for (int k4 = 0; k4 < DFF / 4; ++k4)
    for (int jj = 0; jj < 3; ++jj)
      for (int t = 0; t < 256; ++t)
        for (int j = 0; j < 4; ++j) o[q++] = w[(size_t)(t + 256 * jj) * DFF + 4 * k4 + j];
  return o;
}

// [N][K] -> [N / 16][K / 32][64 lanes][8]: lane l of fragment (T, j) holds W[16 T + l % 16][32 j + 8 (l / 16) ..+8],
// the A operand of v_mfma_f32_16x16x32_bf16 as the batched GEMMs load it (one contiguous KB per wave load)
static std::vector<float> pack_frag(const std::vector<float>& w, int N, int K) {
  std::vector<float> o((size_t)N * K);
  size_t q = 0;
  for (int t = 0; t < N / 16; ++t)
    for (int j = 0; j < K / 32; ++j)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e) o[q++] = w[(size_t)(16 * t + l % 16) * K + 32 * j + 8 * (l / 16) + e];
  return o;
}

// fp32 [N][K] -> [N / 16][K / 16][64 lanes][4]: lane l of fragment (T, j) holds
// W[16 T + l % 16][16 j + 4 (l / 16) .. +4] (ar_f32b_kernel: v_mfma_f32_16x16x4_f32 k-step 4 j + e takes
// element e)
static std::vector<float> pack_frag32(const std::vector<float>& w, int N, int K) {
  std::vector<float> o((size_t)N * K);
  size_t q = 0;
  for (int t = 0; t < N / 16; ++t)
    for (int j = 0; j < K / 16; ++j)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 4; ++e) o[q++] = w[(size_t)(16 * t + l % 16) * K + 16 * j + 4 * (l / 16) + e];
  return o;
}

extern "C" {

int lvx_version(void) { return 1; }

const char* lvx_last_error(void) { return g_err.c_str(); }

int lvx_create(const lvx_config* cfg, lvx_ctx** out) {
  if (!cfg || !out) return fail(LVX_E_ARG, "null argument");
  if (cfg->weight_dtype != LVX_DTYPE_F32 && cfg->weight_dtype != LVX_DTYPE_BF16)
    return fail(LVX_E_ARG, "weight_dtype must be LVX_DTYPE_F32 or LVX_DTYPE_BF16");
  if (cfg->kv_dtype != LVX_DTYPE_F32 && cfg->kv_dtype != LVX_DTYPE_BF16 && cfg->kv_dtype != LVX_DTYPE_FP8)
    return fail(LVX_E_ARG, "kv_dtype must be LVX_DTYPE_F32, LVX_DTYPE_BF16 or LVX_DTYPE_FP8");
  if (cfg->max_streams < 1 || cfg->max_streams > 1024) return fail(LVX_E_ARG, "max_streams out of range [1,1024]");
  if (cfg->max_positions < 1 || cfg->max_positions > BLOCK_SIZE)
    return fail(LVX_E_ARG, "max_positions out of range [1,8192] (GPTConfig.block_size)");
  if (cfg->max_codec_frames < 1) return fail(LVX_E_ARG, "max_codec_frames must be >= 1");
  if (cfg->codec_dtype != 0 && !(cfg->codec_dtype == LVX_DTYPE_FP8 && cfg->weight_dtype == LVX_DTYPE_BF16))
    return fail(LVX_E_ARG, "codec_dtype must be 0 or LVX_DTYPE_FP8 (with weight_dtype LVX_DTYPE_BF16)");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(LVX_E_HIP, "no HIP device available");
  if (cfg->device < 0 || cfg->device >= ndev) return fail(LVX_E_ARG, "device ordinal out of range");
  auto* c = new lvx_ctx();
  c->cfg = *cfg;
  *out = c;
  return LVX_OK;
}

void lvx_destroy(lvx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto g : c->graph_defs) (void)hipGraphDestroy(g);
  if (c->own_capture_stream) (void)hipStreamDestroy(c->own_capture_stream);
  for (void* p : c->allocs) (void)hipFree(p);
  delete c;
}

int lvx_set_weight(lvx_ctx* c, const char* name, const float* data, int64_t numel) {
  if (!c || !name || !data) return fail(LVX_E_ARG, "null argument");
  std::string k(name);
  if (c->finalized) return fail(LVX_E_STATE, "weights are frozen after lvx_finalize");
  if (k == "head.istft.window") {
    if (numel != 1280) return fail(LVX_E_ARG, "head.istft.window must have 1280 elements");
    c->host[k] = std::vector<float>(data, data + numel);
    return LVX_OK;
  }
  auto it = specs().find(k);
  if (it == specs().end()) return fail(LVX_E_NAME, "unknown weight name: " + k);
  if (numel != numel_of(it->second))
    return fail(LVX_E_ARG, "weight " + k + ": expected " + std::to_string(numel_of(it->second)) + " elements, got " +
                               std::to_string(numel));
  c->host[k] = std::vector<float>(data, data + numel);
  return LVX_OK;
}

int lvx_missing_weights(lvx_ctx* c, const char** first) {
  if (!c) return fail(LVX_E_ARG, "null ctx");
  if (c->finalized) return 0;
  int n = 0;
  static thread_local std::string name;
  for (auto& kv : specs())
    if (!c->host.count(kv.first)) {
      if (n == 0) name = kv.first;
      ++n;
    }
  if (first) *first = n ? name.c_str() : nullptr;
  return n;
}

int lvx_finalize(lvx_ctx* c) {
  if (!c) return fail(LVX_E_ARG, "null ctx");
  if (c->finalized) return LVX_OK;
  const char* miss = nullptr;
  if (lvx_missing_weights(c, &miss) > 0) return fail(LVX_E_STATE, std::string("missing weight: ") + miss);
  HIP_TRY(hipSetDevice(c->cfg.device));
  int r;
#define UP_F(key, dst) \
  if ((r = c->upload_f32(c->H(key), &(dst)))) return r;
#define UP_W(vec, dst) \
  if ((r = c->upload_w((vec), &(dst)))) return r;
  // ---- AR ----
  ArWeights& w = c->arw;
  UP_F("transformer.wpe.weight", w.wpe);
  UP_F("encoder.embed_tokens.weight", w.text_table);
  UP_F("feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed", w.codebook);
  for (int i = 0; i < N_LAYER; ++i) {
    std::string p = "transformer.h." + std::to_string(i) + ".";
    UP_F(p + "ln_1.weight", w.ln1[i]);
    UP_F(p + "ln_2.weight", w.ln2[i]);
    UP_W(c->H(p + "attn.c_attn.weight"), w.w_attn[i]);
    UP_W(c->H(p + "attn.c_proj.weight"), w.w_aproj[i]);
    UP_W(c->H(p + "mlp.c_fc.weight"), w.w_fc[i]);
    UP_W(c->H(p + "mlp.c_proj.weight"), w.w_mproj[i]);
    if (c->cfg.weight_dtype == LVX_DTYPE_BF16) {  // thread-packed copy for the fused MLP (ar_mlp_fused_kernel)
      UP_W(pack_mproj(c->H(p + "mlp.c_proj.weight")), w.w_mproj_pk[i]);
      UP_W(pack_frag(c->H(p + "attn.c_attn.weight"), 3 * D, D), w.f_attn[i]);
      UP_W(pack_frag(c->H(p + "attn.c_proj.weight"), D, D), w.f_aproj[i]);
      UP_W(pack_frag(c->H(p + "mlp.c_fc.weight"), DFF, D), w.f_fc[i]);
      UP_W(pack_frag(c->H(p + "mlp.c_proj.weight"), D, DFF), w.f_mproj[i]);
      // batched c_fc: LN2(x) . W^T = rstd * ((x * g) . W^T - mean * G), G[n] = sum_k g[k] W[n][k]
      // over the bf16 weights the GEMM multiplies (double accumulation, rounded once)
      const std::vector<float>& wf = c->H(p + "mlp.c_fc.weight");
      const std::vector<float>& g2 = c->H(p + "ln_2.weight");
      std::vector<float> gs(DFF);
      for (int n = 0; n < DFF; ++n) {
        double acc = 0.0;
        for (int k = 0; k < D; ++k) {
          const uint32_t hb = (uint32_t)f32_to_bf16(wf[(size_t)n * D + k]) << 16;
          float wv;
          std::memcpy(&wv, &hb, 4);
          acc += (double)g2[k] * (double)wv;
        }
        gs[n] = (float)acc;
      }
      if ((r = c->upload_f32(gs, &w.fc_gsum[i]))) return r;
    } else {  // fp32 parity mode: packed copies for the batched exact-fp32 MFMA GEMMs (ar_f32b_kernel)
      UP_W(pack_frag32(c->H(p + "attn.c_attn.weight"), 3 * D, D), w.f_attn[i]);
      UP_W(pack_frag32(c->H(p + "attn.c_proj.weight"), D, D), w.f_aproj[i]);
      UP_W(pack_frag32(c->H(p + "mlp.c_fc.weight"), DFF, D), w.f_fc[i]);
      UP_W(pack_frag32(c->H(p + "mlp.c_proj.weight"), D, DFF), w.f_mproj[i]);
    }
  }
  UP_F("transformer.ln_f.weight", w.lnf);
  UP_W(c->H("lm_head.weight"), w.w_lm);
  if (c->cfg.weight_dtype == LVX_DTYPE_BF16) {
    UP_W(pack_frag(c->H("lm_head.weight"), VOCAB, D), w.f_lm);
    // layer 0's c_attn as table rows (ArWeights q0_*): G on the host over the bf16 weights (as fc_gsum),
    // the three tables by a device GEMM over the uploaded bf16 c_attn weight
    const std::vector<float>& wa = c->H("transformer.h.0.attn.c_attn.weight");
    const std::vector<float>& g1 = c->H("transformer.h.0.ln_1.weight");
    std::vector<float> gq(3 * D);
    for (int n = 0; n < 3 * D; ++n) {
      double acc = 0.0;
      for (int k = 0; k < D; ++k) {
        const uint32_t hb = (uint32_t)f32_to_bf16(wa[(size_t)n * D + k]) << 16;
        float wv;
        std::memcpy(&wv, &hb, 4);
        acc += (double)g1[k] * (double)wv;
      }
      gq[n] = (float)acc;
    }
    if ((r = c->upload_f32(gq, &w.q0_g))) return r;
    float *tt, *tc, *tp;
    const int P = c->cfg.max_positions;
    if ((r = c->dalloc(&tt, (size_t)TEXT_VOCAB * 3 * D)) || (r = c->dalloc(&tc, (size_t)VOCAB * 3 * D)) ||
        (r = c->dalloc(&tp, (size_t)P * 3 * D)))
      return r;
    ar_launch_q0_tables(w, P, tt, tc, tp, nullptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    w.q0_text = tt;
    w.q0_code = tc;
    w.q0_pos = tp;
  } else {
    UP_W(pack_frag32(c->H("lm_head.weight"), VOCAB, D), w.f_lm);
  }
  // ---- codec ----
  CodecWeights& cw = c->cw;
  cw.codebook = w.codebook;
#define UP_CW(vec, rows, dst, sdst) \
  if ((r = c->upload_cw((vec), (rows), &(dst), &(sdst)))) return r;
  cw.wfp8 = c->cfg.codec_dtype == LVX_DTYPE_FP8;
  UP_CW(repack_conv(c->H("backbone.embed.weight"), 768, 512, 7), 768, cw.embed_w, cw.embed_s);
  UP_F("backbone.embed.bias", cw.embed_b);
  UP_F("backbone.norm.scale.weight", cw.ada_scale);
  UP_F("backbone.norm.shift.weight", cw.ada_shift);
  int ri = 0;
  for (int i : {0, 1, 3, 4}) {
    std::string p = "backbone.pos_net." + std::to_string(i) + ".";
    UP_F(p + "norm1.weight", cw.rn_n1w[ri]);
    UP_F(p + "norm1.bias", cw.rn_n1b[ri]);
    UP_F(p + "norm2.weight", cw.rn_n2w[ri]);
    UP_F(p + "norm2.bias", cw.rn_n2b[ri]);
    UP_CW(repack_conv(c->H(p + "conv1.weight"), 768, 768, 3), 768, cw.rn_c1w[ri], cw.rn_c1s[ri]);
    UP_F(p + "conv1.bias", cw.rn_c1b[ri]);
    UP_CW(repack_conv(c->H(p + "conv2.weight"), 768, 768, 3), 768, cw.rn_c2w[ri], cw.rn_c2s[ri]);
    UP_F(p + "conv2.bias", cw.rn_c2b[ri]);
    ++ri;
  }
  {
    const std::string p = "backbone.pos_net.2.";
    UP_F(p + "norm.weight", cw.at_nw);
    UP_F(p + "norm.bias", cw.at_nb);
    std::vector<float> qkv, qkvb;
    for (const char* n : {"q", "k", "v"}) {
      auto& m = c->H(p + n + ".weight");
      qkv.insert(qkv.end(), m.begin(), m.end());
      auto& b = c->H(p + n + ".bias");
      qkvb.insert(qkvb.end(), b.begin(), b.end());
    }
    UP_CW(qkv, 3 * 768, cw.at_qkv_w, cw.at_qkv_s);
    if ((r = c->upload_f32(qkvb, &cw.at_qkv_b))) return r;
    UP_CW(c->H(p + "proj_out.weight"), 768, cw.at_proj_w, cw.at_proj_s);
    UP_F(p + "proj_out.bias", cw.at_proj_b);
  }
  UP_F("backbone.pos_net.5.weight", cw.pn_w);
  UP_F("backbone.pos_net.5.bias", cw.pn_b);
  for (int i = 0; i < 12; ++i) {
    std::string p = "backbone.convnext." + std::to_string(i) + ".";
    {  // depthwise conv [768][1][7] -> tap-major [7][768] (16-byte weight loads in dwconv_adaln)
      const std::vector<float>& dwv = c->H(p + "dwconv.weight");
      std::vector<float> t(dwv.size());
      for (int ch = 0; ch < 768; ++ch)
        for (int k = 0; k < 7; ++k) t[(size_t)k * 768 + ch] = dwv[(size_t)ch * 7 + k];
      if ((r = c->upload_f32(t, &cw.dw_w[i]))) return r;
    }
    UP_F(p + "dwconv.bias", cw.dw_b[i]);
    UP_F(p + "norm.scale.weight", cw.cn_scale[i]);
    UP_F(p + "norm.shift.weight", cw.cn_shift[i]);
    UP_CW(c->H(p + "pwconv1.weight"), 2304, cw.pw1_w[i], cw.pw1_s[i]);
    UP_F(p + "pwconv1.bias", cw.pw1_b[i]);
    UP_CW(c->H(p + "pwconv2.weight"), 768, cw.pw2_w[i], cw.pw2_s[i]);
    UP_F(p + "pwconv2.bias", cw.pw2_b[i]);
    UP_F(p + "gamma", cw.gamma[i]);
  }
  UP_F("backbone.final_layer_norm.weight", cw.fln_w);
  UP_F("backbone.final_layer_norm.bias", cw.fln_b);
  UP_CW(c->H("head.out.weight"), 1282, cw.head_w, cw.head_s);
  UP_F("head.out.bias", cw.head_b);
  {
    std::vector<float> win(1280);
    if (c->host.count("head.istft.window")) win = c->H("head.istft.window");
    else
      for (int n = 0; n < 1280; ++n) win[n] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * n / 1280.0));
    if ((r = c->upload_f32(win, &cw.window))) return r;
    std::vector<float> tw(2 * 1280);
    for (int m = 0; m < 1280; ++m) {
      tw[2 * m] = (float)std::cos(2.0 * M_PI * m / 1280.0);
      tw[2 * m + 1] = (float)std::sin(2.0 * M_PI * m / 1280.0);
    }
    if ((r = c->upload_f32(tw, &cw.twiddle))) return r;
  }
#undef UP_F
#undef UP_W
#undef UP_CW
  // ---- AR state ----
  ArState& st = c->st;
  const int S = c->cfg.max_streams, P = c->cfg.max_positions;
  // the bf16 operand rows (xn, xb, hb) are stored and read in whole 16-row MFMA tiles when they are
  // fragment-packed (xfrag, 9 <= B <= 32): a partly filled tile spans 16 rows, so round up
  const int S16 = (S + 15) / 16 * 16;
  st.max_pos = P;
  st.max_streams = S;
  st.kv_chunks = (P + KV_CHUNK - 1) / KV_CHUNK;
  if ((r = c->dalloc(&st.slots, S)) || (r = c->dalloc(&st.pos, S)) || (r = c->dalloc(&st.prev, S)) ||
      (r = c->dalloc(&st.err, 4)) || (r = c->dalloc(&st.x, (size_t)S * D)) || (r = c->dalloc(&st.q, (size_t)S * D)) ||
      (r = c->dalloc(&st.part_o, (size_t)S * N_HEAD * NSPLIT * HD)) ||
      (r = c->dalloc(&st.part_ml, (size_t)S * N_HEAD * NSPLIT * 2)) || (r = c->dalloc(&st.h, (size_t)S * DFF)) ||
      (r = c->dalloc(&st.logits, (size_t)S * VOCAB)) || (r = c->dalloc(&st.rowinfo, S)) ||
      (r = c->dalloc(&st.rowinfo_n, S)) || (r = c->dalloc(&st.rowx, S)) || (r = c->dalloc(&st.rowx_n, S)) ||
      (r = c->dalloc(&st.selp, 4)) || (r = c->dalloc(&st.selrow, S)) ||
      (r = c->dalloc(&st.xn, (size_t)S16 * D)) || (r = c->dalloc(&st.hb, (size_t)S16 * DFF)) ||
      (r = c->dalloc(&st.xb, (size_t)S16 * D)) || (r = c->dalloc(&st.xstat, (size_t)(D / 16) * S * 2)) ||
      (r = c->dalloc(&st.lmbest, (size_t)LM_MAX_BLOCKS * 4 * 2)) ||
      (r = c->dalloc(&st.yacc, (size_t)YCOPIES * S * D)) || (r = c->dalloc(&st.qkvp, (size_t)4 * S * 3 * D)) ||
      (r = c->dalloc(&st.yfx, (size_t)YCOPIES * S * D)))
    return r;
  HIP_TRY(hipMemset(st.yfx, 0, (size_t)YCOPIES * S * D * 8));
  HIP_TRY(hipMemset(st.yacc, 0, (size_t)YCOPIES * S * D * 4));
  HIP_TRY(hipMemset(st.selp, 0, 16));
  HIP_TRY(hipMemset(st.part_o, 0, (size_t)S * N_HEAD * NSPLIT * HD * 4));
  HIP_TRY(hipMemset(st.part_ml, 0, (size_t)S * N_HEAD * NSPLIT * 2 * 4));
  HIP_TRY(hipMemset(st.pos, 0, S * 4));
  HIP_TRY(hipMemset(st.prev, 0, S * 4));
  HIP_TRY(hipMemset(st.err, 0, 16));
  const size_t kvn = (size_t)N_LAYER * st.kv_chunks * S * N_HEAD * KV_CHUNK * HD;
  const size_t kvb = c->cfg.kv_dtype == LVX_DTYPE_BF16 ? 2 : c->cfg.kv_dtype == LVX_DTYPE_FP8 ? 1 : 4;
  {
    char* k;
    char* v;
    if ((r = c->dalloc(&k, kvn * kvb)) || (r = c->dalloc(&v, kvn * kvb))) return r;
    st.kc = k;
    st.vc = v;
  }
  // ---- codec scratch ----
  CodecScratch& cs = c->cs;
  const int M = c->cfg.max_codec_frames;
  cs.max_frames = M;
  cs.ws_floats = (size_t)std::max(M, 256) * 2304 * 4;
  if ((r = c->dalloc(&cs.x, (size_t)M * 768)) || (r = c->dalloc(&cs.t1, (size_t)M * 2304)) ||
      (r = c->dalloc(&cs.t2, (size_t)(M + 4 * 64) * 2304 + (size_t)768 * 4 * M)) ||
      (r = c->dalloc(&cs.feats, (size_t)M * 512)) || (r = c->dalloc(&cs.gn, (size_t)M * 768)) ||
      (r = c->dalloc(&cs.ws, (size_t)std::max(M, 256) * 2304 * 4)) ||
      (r = c->dalloc(&cs.att, (size_t)M * (std::min(M, kMaxCodecL) + 4))) ||
      (r = c->dalloc(&cs.stats, (size_t)M * 32 * 2)) || (r = c->dalloc(&cs.spec, (size_t)M * 1282)) ||
      (r = c->dalloc(&cs.frames, (size_t)M * 1280)) || (r = c->dalloc(&cs.rowscale, (size_t)M)) ||
      (r = c->dalloc(&cs.tick, 4096)))
    return r;
  HIP_TRY(hipMemset(cs.tick, 0, 4096 * 4));
  cs.err = st.err + 1;  // the codec's own word (it may run on a second stream beside the AR)
  HIP_TRY(hipDeviceSynchronize());
  c->host.clear();
  c->finalized = true;
  return LVX_OK;
}

#define NEED_FINAL(c)                                                              \
  do {                                                                             \
    if (!(c)) return fail(LVX_E_ARG, "null ctx");                                  \
    if (!(c)->finalized) return fail(LVX_E_STATE, "call lvx_finalize first");      \
  } while (0)

int lvx_text_embed(lvx_ctx* c, const int64_t* ids, int n, float* out, void* stream) {
  NEED_FINAL(c);
  if (n < 0 || (n > 0 && (!ids || !out))) return fail(LVX_E_ARG, "bad ids/out");
  HIP_TRY(hipSetDevice(c->cfg.device));
  launch_text_embed(c->arw.text_table, ids, n, out, c->st.err, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

int lvx_codes_to_features(lvx_ctx* c, const int64_t* codes, int B, int L, float* feats, void* stream) {
  NEED_FINAL(c);
  if (B < 0 || L < 0 || ((B * L) > 0 && (!codes || !feats))) return fail(LVX_E_ARG, "bad codes/feats");
  HIP_TRY(hipSetDevice(c->cfg.device));
  launch_codes_to_features(c->arw.codebook, codes, B, L, feats, c->st.err, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

int lvx_stream_reset(lvx_ctx* c, int slot, void* stream) {
  NEED_FINAL(c);
  if (slot < 0 || slot >= c->cfg.max_streams) return fail(LVX_E_ARG, "slot out of range");
  HIP_TRY(hipSetDevice(c->cfg.device));
  HIP_TRY(hipMemsetAsync(c->st.pos + slot, 0, 4, (hipStream_t)stream));
  return LVX_OK;
}

int lvx_stream_set(lvx_ctx* c, int slot, int pos, int prev_token, void* stream) {
  NEED_FINAL(c);
  if (slot < 0 || slot >= c->cfg.max_streams) return fail(LVX_E_ARG, "slot out of range");
  if (pos < 0 || pos > c->cfg.max_positions) return fail(LVX_E_CAPACITY, "position out of range");
  if (prev_token < 0 || prev_token >= VOCAB) return fail(LVX_E_ARG, "prev_token out of range");
  HIP_TRY(hipSetDevice(c->cfg.device));
  launch_set_slot(c->st.pos, c->st.prev, slot, pos, prev_token, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

int lvx_stream_position(lvx_ctx* c, int slot, int* pos_out, void* stream) {
  NEED_FINAL(c);
  if (slot < 0 || slot >= c->cfg.max_streams || !pos_out) return fail(LVX_E_ARG, "bad slot/pos_out");
  HIP_TRY(hipSetDevice(c->cfg.device));
  int32_t v[2];
  launch_err_take(c->st.err, 1, 0, c->st.err + 3, (hipStream_t)stream);  // the capacity bit only
  HIP_TRY(hipMemcpyAsync(&v[0], c->st.pos + slot, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipMemcpyAsync(&v[1], c->st.err + 3, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  *pos_out = v[0];
  return bits_status(v[1]);
}

int lvx_set_option(lvx_ctx* c, const char* name, int value) {
  if (!c || !name) return fail(LVX_E_ARG, "null argument");
  std::string n(name);
  std::lock_guard<std::mutex> lk(c->mu);
  Opts& o = c->opts;  // this context only (round 4: the switches were process-wide globals)
  if (n == "defer_select") o.defer_select = value;
  else if (n == "fuse_mlp") o.fuse_mlp = value != 0;
  else if (n == "bt") o.bt = std::min(std::max(value, 0), 2);
  else if (n == "codec_g2") o.codec_g2 = value != 0;
  else if (n == "codec_skinny") o.codec_skinny = value != 0;
  else if (n == "codec_g3") o.codec_g3 = value != 0;
  else if (n == "codec_g3f") o.codec_g3f = value == 1 ? 1 : 2;  // 1: the exact-fp32 kernel (a test oracle)
  else if (n == "codec_exp") o.codec_exp = value;
  else if (n == "exp") o.exp = value;
  else if (n == "f32b") o.f32b = value != 0;
  else if (n == "ln_max") o.ln_max = std::min(std::max(value, 2), 8);
  else if (n == "l0q") o.l0q = value != 0;
  else return fail(LVX_E_NAME, "unknown option " + n);
  ++c->opt_epoch;  // this context's captured kernels change (checked in cached_graph)
  return LVX_OK;
}

int lvx_set_capture_stream(lvx_ctx* c, void* stream) {
  if (!c) return fail(LVX_E_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  c->capture_stream = (hipStream_t)stream;
  return LVX_OK;
}

int lvx_set_graphs(lvx_ctx* c, int enable) {
  if (!c) return fail(LVX_E_ARG, "null ctx");
  c->use_graphs = enable != 0;
  return LVX_OK;
}

int lvx_ar_forward_row(lvx_ctx* c, int slot, int pos, const float* emb_row, float* logits, void* stream) {
  NEED_FINAL(c);
  if (slot < 0 || slot >= c->cfg.max_streams) return fail(LVX_E_ARG, "slot out of range");
  if (pos < 0 || pos >= BLOCK_SIZE)
    return fail(LVX_E_CAPACITY, "Cannot forward sequence of length " + std::to_string(pos + 1) +
                                    ", block size is only " + std::to_string(BLOCK_SIZE));
  if (pos >= c->cfg.max_positions)
    return fail(LVX_E_CAPACITY, "position " + std::to_string(pos) + " exceeds the KV capacity " +
                                    std::to_string(c->cfg.max_positions));
  if (!emb_row || !logits) return fail(LVX_E_ARG, "null emb_row/logits");
  HIP_TRY(hipSetDevice(c->cfg.device));
  const Opts o = c->opts_snapshot();
  OptScope os(&o);
  ar_launch_step(c->arw, c->st, c->cfg.weight_dtype, c->cfg.kv_dtype, 1, 1, emb_row, slot, pos, logits,
                 (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

// Capture `launch(stream)` into a graph cached under `key` (instantiated once), then replay it on the
// caller's stream. The capture runs on the caller's stream unless lvx_set_capture_stream named another:
// torch's synchronous collectives record their completion events on the current stream, a process
// group's watchdog thread queries them, and HIP refuses a query of an event last recorded in a stream
// that is capturing (round 6: a configs[4] line with the one-rank RCCL group aborted mid-capture). The
// Python engine therefore hands over a pooled stream once an RCCL group exists; without one it keeps
// the caller's, since one more stream per process cost the two-ranks-on-one-GPU configs[3] rehearsal
// 6.5x (22.4k -> 3.4k tokens/s, profiles/r06/capture_stream_ab.txt) while a single rank per GPU saw no
// difference. (The legacy null stream cannot be captured: lvx_ar_step* null-stream callers launch the
// steps one by one; lvx_probe_kernel's capture on a stream the context creates.)
// Caller holds c->mu.
static int cached_graph(lvx_ctx* c, const GraphKey& key, hipStream_t s,
                        const std::function<void(hipStream_t)>& launch, hipGraphExec_t* out) {
  const unsigned epoch = c->opt_epoch;  // (caller holds c->mu)
  if (c->graph_epoch != epoch) {  // an option changed since these graphs were captured
    for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
    c->graphs.clear();
    c->graph_epoch = epoch;
  }
  auto it = c->graphs.find(key);
  if (it == c->graphs.end()) {
    hipStream_t cs = c->capture_stream ? c->capture_stream : s;
    if (!cs) {  // the legacy null stream cannot be captured (lvx_probe_kernel's null-stream callers)
      if (!c->own_capture_stream) HIP_TRY(hipStreamCreateWithFlags(&c->own_capture_stream, hipStreamNonBlocking));
      cs = c->own_capture_stream;
    }
    hipGraph_t g;
    HIP_TRY(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    launch(cs);
    hipError_t le = hipGetLastError();
    HIP_TRY(hipStreamEndCapture(cs, &g));
    if (le != hipSuccess) return fail(LVX_E_HIP, std::string("capture: ") + hipGetErrorString(le));
    hipGraphExec_t ex;
    HIP_TRY(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    c->graph_defs.push_back(g);
    it = c->graphs.emplace(key, ex).first;
  }
  *out = it->second;
  return 0;
}

static int ar_step_impl(lvx_ctx* c, int n_steps, int B, const int32_t* slots, const int32_t* text_plan,
                        int plan_stride, int32_t* rowstep, int32_t* tok_plan, float* margin_plan, void* stream) {
  NEED_FINAL(c);
  if (B < 1 || B > c->cfg.max_streams) return fail(LVX_E_ARG, "B out of range [1, max_streams]");
  if (plan_stride < 1) return fail(LVX_E_ARG, "plan_stride must be >= 1");
  if (n_steps < 0) return fail(LVX_E_ARG, "n_steps must be >= 0");
  if (!slots || !text_plan || !rowstep || !tok_plan) return fail(LVX_E_ARG, "null slots/text_plan/rowstep/tok_plan");
  if (n_steps == 0) return LVX_OK;
  HIP_TRY(hipSetDevice(c->cfg.device));
  ArState st = c->st;
  st.slots = const_cast<int32_t*>(slots);
  st.text_plan = text_plan;
  st.plan_stride = plan_stride;
  st.rowstep = rowstep;
  st.tok_plan = tok_plan;
  st.margin_plan = margin_plan;
  hipStream_t s = (hipStream_t)stream;
  ar_launch_rowinfo_init(st, B, s);  // per-row control records, then advanced by every step
  // null-stream callers (torch's default stream) launch the steps one by one: replaying the same
  // steps as graphs on a stream of their own measured no faster (round 1)
  if (!c->use_graphs || s == nullptr) {
    const Opts o = c->opts_snapshot();
    OptScope os(&o);
    for (int i = 0; i < n_steps; ++i)
      ar_launch_step(c->arw, st, c->cfg.weight_dtype, c->cfg.kv_dtype, B, 0, nullptr, 0, 0, nullptr, s);
    ar_launch_steps_end(st, c->cfg.weight_dtype, B, s);
    HIP_TRY(hipGetLastError());
    return LVX_OK;
  }
  std::lock_guard<std::mutex> lk(c->mu);
  const Opts o = c->opts;  // the options the cached graphs were captured under (epoch checked under mu)
  OptScope os(&o);
  // graphs of kGraphSteps consecutive steps (one replay per kGraphSteps tokens) + 1-step graph
  auto get_graph = [&](int nst, hipGraphExec_t* out) -> int {
    GraphKey key{B, plan_stride, nst, slots, text_plan, rowstep, tok_plan, margin_plan, stream};
    return cached_graph(c, key, s, [&](hipStream_t cs) {
      for (int i = 0; i < nst; ++i)
        ar_launch_step(c->arw, st, c->cfg.weight_dtype, c->cfg.kv_dtype, B, 0, nullptr, 0, 0, nullptr, cs);
    }, out);
  };
  int left = n_steps;
  if (left >= kGraphSteps) {
    hipGraphExec_t gx;
    if (int r = get_graph(kGraphSteps, &gx)) return r;
    for (; left >= kGraphSteps; left -= kGraphSteps) HIP_TRY(hipGraphLaunch(gx, s));
  }
  if (left > 0) {
    hipGraphExec_t g1;
    if (int r = get_graph(1, &g1)) return r;
    for (; left > 0; --left) HIP_TRY(hipGraphLaunch(g1, s));
  }
  ar_launch_steps_end(st, c->cfg.weight_dtype, B, s);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

int lvx_ar_step(lvx_ctx* c, int B, const int32_t* slots, const int32_t* text_plan, int plan_stride,
                int32_t* rowstep, int32_t* tok_plan, float* margin_plan, void* stream) {
  return ar_step_impl(c, 1, B, slots, text_plan, plan_stride, rowstep, tok_plan, margin_plan, stream);
}

int lvx_ar_steps(lvx_ctx* c, int n_steps, int B, const int32_t* slots, const int32_t* text_plan, int plan_stride,
                 int32_t* rowstep, int32_t* tok_plan, float* margin_plan, void* stream) {
  return ar_step_impl(c, n_steps, B, slots, text_plan, plan_stride, rowstep, tok_plan, margin_plan, stream);
}

int lvx_ar_logits(lvx_ctx* c, int B, float* dst, void* stream) {
  NEED_FINAL(c);
  if (B < 1 || B > c->cfg.max_streams || !dst) return fail(LVX_E_ARG, "bad B/dst");
  HIP_TRY(hipSetDevice(c->cfg.device));
  HIP_TRY(hipMemcpyAsync(dst, c->st.logits, (size_t)B * VOCAB * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return LVX_OK;
}

int lvx_check_errors(lvx_ctx* c, void* stream) {
  NEED_FINAL(c);
  HIP_TRY(hipSetDevice(c->cfg.device));
  int32_t v = 0;
  // both words taken atomically in stream order: a bit that a codec call in flight on another stream
  // sets afterwards stays in its word for the next check (round 4 cleared the word with a memset)
  launch_err_take(c->st.err, -1, -1, c->st.err + 2, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(&v, c->st.err + 2, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return bits_status(v);
}

int lvx_error_take(lvx_ctx* c, int which, int32_t* bits_dev, void* stream) {
  NEED_FINAL(c);
  if (!bits_dev || which < 1 || which > 3) return fail(LVX_E_ARG, "which must be LVX_ERRW_AR | LVX_ERRW_CODEC, bits_dev non-null");
  HIP_TRY(hipSetDevice(c->cfg.device));
  launch_err_take(c->st.err, (which & LVX_ERRW_AR) ? -1 : 0, (which & LVX_ERRW_CODEC) ? -1 : 0, bits_dev,
                  (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

int lvx_error_status(int bits) { return bits_status(bits); }

int lvx_probe_kernel(lvx_ctx* c, int which, int B, const int32_t* slots, int iters, void* stream) {
  NEED_FINAL(c);
  if (B < 1 || B > c->cfg.max_streams || !slots || iters < 1) return fail(LVX_E_ARG, "bad probe arguments");
  HIP_TRY(hipSetDevice(c->cfg.device));
  ArState st = c->st;  // no plan bound: text_plan / rowstep / tok_plan stay null
  st.slots = const_cast<int32_t*>(slots);
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> lk(c->mu);
  const Opts o = c->opts;
  OptScope os(&o);
  // a dry run (no launches) validates the op id / fused case before anything is captured
  const int pr = ar_probe(c->arw, st, c->cfg.weight_dtype, c->cfg.kv_dtype, B, which, 0, s);
  if (pr < 0) return fail(LVX_E_ARG, "unknown probe kernel id");
  if (pr > 0) return fail(LVX_E_STATE, "this op has no kernel of its own at this batch size (fused into the previous op)");
  if (!c->use_graphs) {
    ar_probe(c->arw, st, c->cfg.weight_dtype, c->cfg.kv_dtype, B, which, iters, s);
    HIP_TRY(hipGetLastError());
    return LVX_OK;
  }
  // the `iters` launches are replayed as one graph, as the decode step is: launched one by one
  // from the host, back-to-back kernels of 3-5 us measured the host's launch rate as much as
  // the kernel (the first call of a (op, B, slots, iters) captures; time the second)
  GraphKey key{B, -1 - which, iters, slots, nullptr, nullptr, nullptr, nullptr, stream};
  hipGraphExec_t gx;
  if (int r = cached_graph(c, key, s, [&](hipStream_t cs) {
        ar_probe(c->arw, st, c->cfg.weight_dtype, c->cfg.kv_dtype, B, which, iters, cs);
      }, &gx))
    return r;
  HIP_TRY(hipGraphLaunch(gx, s));
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

int lvx_select_probe(lvx_ctx* c, int path, int B, const int32_t* slots, const float* logits,
                     const int32_t* text_plan, int plan_stride, int32_t* rowstep, int32_t* tok_plan,
                     float* margin_plan, void* stream) {
  NEED_FINAL(c);
  if (B < 1 || B > c->cfg.max_streams || (path == 1 && B > 4) || (path == 3 && B > 8))
    return fail(LVX_E_ARG, "B out of range for this path");
  if (path < 0 || path > 3) return fail(LVX_E_ARG, "path must be 0, 1, 2 or 3");
  if (!slots || !logits || !text_plan || !rowstep || !tok_plan || plan_stride < 2)
    return fail(LVX_E_ARG, "null argument or plan_stride < 2");
  HIP_TRY(hipSetDevice(c->cfg.device));
  hipStream_t s = (hipStream_t)stream;
  ArState st = c->st;
  st.slots = const_cast<int32_t*>(slots);
  st.text_plan = text_plan;
  st.plan_stride = plan_stride;
  st.rowstep = rowstep;
  st.tok_plan = tok_plan;
  st.margin_plan = margin_plan;
  HIP_TRY(hipMemcpyAsync(st.logits, logits, (size_t)B * VOCAB * 4, hipMemcpyDeviceToDevice, s));
  const Opts o = c->opts_snapshot();
  OptScope os(&o);
  ar_select_probe(c->arw, st, B, path, s);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

static int codec_check(lvx_ctx* c, int B, int L, int bw) {
  if (B < 1 || L < 1) return fail(LVX_E_ARG, "B and L must be >= 1");
  if ((long long)B * L > c->cfg.max_codec_frames)
    return fail(LVX_E_CAPACITY, "B*L = " + std::to_string((long long)B * L) + " exceeds max_codec_frames " +
                                    std::to_string(c->cfg.max_codec_frames));
  if (L > kMaxCodecL) return fail(LVX_E_CAPACITY, "L exceeds the codec's max frames per stream (4096)");
  if (bw < 0 || bw > 3) return fail(LVX_E_ARG, "bandwidth_id out of range [0,3]");
  return 0;
}

int lvx_codec_decode_features(lvx_ctx* c, const float* feats, int B, int L, int bw, float* pcm, void* stream) {
  NEED_FINAL(c);
  if (int r = codec_check(c, B, L, bw)) return r;
  if (!feats || !pcm) return fail(LVX_E_ARG, "null feats/pcm");
  HIP_TRY(hipSetDevice(c->cfg.device));
  const Opts o = c->opts_snapshot();
  OptScope os(&o);
  codec_launch_decode(c->cw, c->cs, c->cfg.weight_dtype, feats, nullptr, B, L, bw, pcm, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

int lvx_codec_decode_codes(lvx_ctx* c, const int32_t* codes, int B, int L, int bw, float* pcm, void* stream) {
  NEED_FINAL(c);
  if (int r = codec_check(c, B, L, bw)) return r;
  if (!codes || !pcm) return fail(LVX_E_ARG, "null codes/pcm");
  HIP_TRY(hipSetDevice(c->cfg.device));
  const Opts o = c->opts_snapshot();
  OptScope os(&o);
  codec_launch_decode(c->cw, c->cs, c->cfg.weight_dtype, nullptr, codes, B, L, bw, pcm, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// WavTokenizer encoder (encode_infer): its own context, since its weights are not needed for TTS.
// ---------------------------------------------------------------------------
namespace {
constexpr const char* kEncPrefix = "feature_extractor.encodec.encoder.model.";
constexpr const char* kCodebookKey = "feature_extractor.encodec.quantizer.vq.layers.0._codebook.embed";
struct EncConv {
  std::string name;
  int cin, cout, k, stride, dil;
  bool elu;
};
// seanet.py:94-140 with n_filters 32, ratios [8, 5, 4, 2] reversed, compress 2 (llmvox_amd.weights.encoder_convs)
std::vector<EncConv> enc_convs() {
  std::vector<EncConv> v{{"0", 1, 32, 7, 1, 1, false}};
  int dim = 32, idx = 1;
  for (int ratio : {2, 4, 5, 8}) {
    v.push_back({std::to_string(idx) + ".block.1", dim, dim / 2, 3, 1, 1, true});
    v.push_back({std::to_string(idx) + ".block.3", dim / 2, dim, 1, 1, 1, true});
    v.push_back({std::to_string(idx) + ".shortcut", dim, dim, 1, 1, 1, false});
    v.push_back({std::to_string(idx + 2), dim, 2 * dim, 2 * ratio, ratio, 1, true});
    dim *= 2;
    idx += 3;
  }
  v.push_back({"15", 512, 512, 7, 1, 1, true});
  return v;
}
// SConv1d geometry (conv.py:54-61,79-96,195-211): left pad, reflect domain, output length
struct ConvGeo {
  int pl, lext, T;
};
ConvGeo conv_geo(int L, int k, int stride, int dil) {
  const int keff = (k - 1) * dil + 1, pt = keff - stride;
  const int nf = (L + stride - 1) / stride;  // ceil(n_frames) of get_extra_padding_for_conv1d (L >= 1)
  const int extra = nf * stride - L;
  const int pr = pt / 2, pl = pt - pr, right = pr + extra;
  const int max_pad = std::max(pl, right);
  const int ex0 = L <= max_pad ? max_pad - L + 1 : 0;
  return {pl, L + ex0, (pl + L + right - keff) / stride + 1};
}
int enc_frames_of(int n) {
  int L = n;
  for (const EncConv& cv : enc_convs()) L = conv_geo(L, cv.k, cv.stride, cv.dil).T;
  return L;
}
}  // namespace

struct lvx_enc {
  int device = 0;
  long long max_samples = 0;
  bool finalized = false;
  std::map<std::string, std::vector<float>> host;
  std::vector<void*> allocs;
  std::vector<EncConv> convs = enc_convs();
  std::vector<const float*> cw, cb;  // per conv: [cout][k][cin] weights, bias
  const float *wih[2] = {}, *bih[2] = {}, *whh[2] = {}, *bhh[2] = {};
  const float* codebook = nullptr;  // [4096][512]
  const float* esq = nullptr;       // [4096] |e|^2
  float* buf[4] = {};
  size_t buf_floats = 0;
  float *h = nullptr, *c = nullptr;  // [2][Bmax][512], [Bmax][512]
  int bmax = 0;
  int alloc(float** p, size_t n) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, n * 4 + 256);
    if (e != hipSuccess) return fail(LVX_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
    allocs.push_back(q);
    *p = reinterpret_cast<float*>(q);
    return 0;
  }
  int upload(const std::vector<float>& v, const float** out) {
    float* d;
    if (int r = alloc(&d, v.size())) return r;
    HIP_TRY(hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    *out = d;
    return 0;
  }
  std::map<std::string, size_t> expected() const {
    std::map<std::string, size_t> m;
    for (const EncConv& cv : convs) {
      m[std::string(kEncPrefix) + cv.name + ".conv.conv.weight"] = (size_t)cv.cout * cv.cin * cv.k;
      m[std::string(kEncPrefix) + cv.name + ".conv.conv.bias"] = cv.cout;
    }
    for (int l = 0; l < 2; ++l) {
      const std::string p = std::string(kEncPrefix) + "13.lstm.", sfx = "_l" + std::to_string(l);
      m[p + "weight_ih" + sfx] = m[p + "weight_hh" + sfx] = (size_t)2048 * 512;
      m[p + "bias_ih" + sfx] = m[p + "bias_hh" + sfx] = 2048;
    }
    m[kCodebookKey] = (size_t)4096 * 512;
    return m;
  }
};

extern "C" {

int lvx_enc_frames(int n_samples) { return n_samples >= 1 ? enc_frames_of(n_samples) : 0; }

int lvx_enc_create(int device, long long max_samples, lvx_enc** out) {
  if (!out) return fail(LVX_E_ARG, "null argument");
  if (max_samples < 1) return fail(LVX_E_ARG, "max_samples must be >= 1");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(LVX_E_HIP, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(LVX_E_ARG, "device ordinal out of range");
  auto* e = new lvx_enc();
  e->device = device;
  e->max_samples = max_samples;
  *out = e;
  return LVX_OK;
}

void lvx_enc_destroy(lvx_enc* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  for (void* p : e->allocs) (void)hipFree(p);
  delete e;
}

int lvx_enc_set_weight(lvx_enc* e, const char* name, const float* data, int64_t numel) {
  if (!e || !name || !data) return fail(LVX_E_ARG, "null argument");
  if (e->finalized) return fail(LVX_E_STATE, "weights are frozen after lvx_enc_finalize");
  const auto exp = e->expected();
  auto it = exp.find(name);
  if (it == exp.end()) return fail(LVX_E_NAME, std::string("unknown encoder weight name: ") + name);
  if ((size_t)numel != it->second)
    return fail(LVX_E_ARG, std::string("weight ") + name + ": expected " + std::to_string(it->second) + " elements");
  e->host[name] = std::vector<float>(data, data + numel);
  return LVX_OK;
}

int lvx_enc_finalize(lvx_enc* e) {
  if (!e) return fail(LVX_E_ARG, "null argument");
  if (e->finalized) return LVX_OK;
  for (auto& kv : e->expected())
    if (!e->host.count(kv.first)) return fail(LVX_E_STATE, "missing encoder weight: " + kv.first);
  HIP_TRY(hipSetDevice(e->device));
  int r;
  for (const EncConv& cv : e->convs) {
    const std::string p = std::string(kEncPrefix) + cv.name + ".conv.conv.";
    const float *w, *b;
    if ((r = e->upload(repack_conv(e->host[p + "weight"], cv.cout, cv.cin, cv.k), &w)) || (r = e->upload(e->host[p + "bias"], &b)))
      return r;
    e->cw.push_back(w);
    e->cb.push_back(b);
  }
  for (int l = 0; l < 2; ++l) {
    const std::string p = std::string(kEncPrefix) + "13.lstm.", sfx = "_l" + std::to_string(l);
    if ((r = e->upload(e->host[p + "weight_ih" + sfx], &e->wih[l])) || (r = e->upload(e->host[p + "bias_ih" + sfx], &e->bih[l])) ||
        (r = e->upload(e->host[p + "weight_hh" + sfx], &e->whh[l])) || (r = e->upload(e->host[p + "bias_hh" + sfx], &e->bhh[l])))
      return r;
  }
  const std::vector<float>& cbk = e->host[kCodebookKey];
  if ((r = e->upload(cbk, &e->codebook))) return r;
  std::vector<float> esq(4096);
  for (int n = 0; n < 4096; ++n) {  // |e|^2 (core_vq.py:180: embed.pow(2).sum(0)), double accumulation
    double a = 0.0;
    for (int k = 0; k < 512; ++k) a += (double)cbk[(size_t)n * 512 + k] * cbk[(size_t)n * 512 + k];
    esq[n] = (float)a;
  }
  if ((r = e->upload(esq, &e->esq))) return r;
  // activations: at most 32 channels per input sample through the SEANet stack; the LSTM gates
  // (2,048 per frame) and the quantiser scores (4,096 per frame) of up to 64 one-frame streams
  e->buf_floats = (size_t)e->max_samples * 32 + (size_t)64 * 4096;
  for (auto& b : e->buf)
    if ((r = e->alloc(&b, e->buf_floats))) return r;
  e->bmax = 1024;
  if ((r = e->alloc(&e->h, (size_t)2 * e->bmax * 512)) || (r = e->alloc(&e->c, (size_t)e->bmax * 512))) return r;
  HIP_TRY(hipDeviceSynchronize());
  e->host.clear();
  e->finalized = true;
  return LVX_OK;
}

// audio [B][N] -> features [B][512][T], codes [B][T] (device pointers; T = lvx_enc_frames(N))
int lvx_encode(lvx_enc* e, const float* audio, int B, int N, float* features, int32_t* codes, void* stream) {
  if (!e) return fail(LVX_E_ARG, "null argument");
  if (!e->finalized) return fail(LVX_E_STATE, "call lvx_enc_finalize first");
  if (B < 1 || N < 1 || !audio || !features || !codes) return fail(LVX_E_ARG, "bad audio / outputs");
  if ((long long)B * N > e->max_samples || B > e->bmax)
    return fail(LVX_E_CAPACITY, "B*N = " + std::to_string((long long)B * N) + " exceeds max_samples " + std::to_string(e->max_samples));
  HIP_TRY(hipSetDevice(e->device));
  hipStream_t s = (hipStream_t)stream;
  float** buf = e->buf;
  // the whole chain's sizes first (every intermediate within a buffer)
  {
    int L = N;
    for (const EncConv& cv : e->convs) {
      const ConvGeo g = conv_geo(L, cv.k, cv.stride, cv.dil);
      if ((size_t)B * g.T * cv.cout > e->buf_floats || (size_t)B * L * cv.cin > e->buf_floats)
        return fail(LVX_E_CAPACITY, "encoder activations exceed the scratch sized by max_samples");
      L = g.T;
    }
    if ((size_t)B * L * 4096 > e->buf_floats) return fail(LVX_E_CAPACITY, "quantiser scores exceed the scratch");
  }
  auto conv = [&](int i, const float* x, int L, float* y, const float* res) {
    const EncConv& cv = e->convs[i];
    const ConvGeo g = conv_geo(L, cv.k, cv.stride, cv.dil);
    enc_launch_conv(x, e->cw[i], e->cb[i], res, y, B, L, g.T, cv.cin, cv.cout, cv.k, cv.stride, cv.dil, g.pl, g.lext, cv.elu, s);
    return g.T;
  };
  // conv 0, then per ratio: t1 = block.1(ELU x), sc = shortcut(x), x' = block.3(ELU t1) + sc, down(ELU x')
  int L = conv(0, audio, N, buf[0], nullptr);
  for (int blk = 0; blk < 4; ++blk) {
    const int i = 1 + 4 * blk;
    conv(i, buf[0], L, buf[1], nullptr);
    conv(i + 2, buf[0], L, buf[2], nullptr);
    conv(i + 1, buf[1], L, buf[3], buf[2]);
    L = conv(i + 3, buf[3], L, buf[0], nullptr);
  }
  const int T = L;  // x = buf[0] [B][T][512]
  // SLSTM: layer 0 -> buf[2], layer 1 (+ skip from the LSTM input) -> buf[3]
  for (int l = 0; l < 2; ++l) {
    const float* xin = l == 0 ? buf[0] : buf[2];
    float* yout = l == 0 ? buf[2] : buf[3];
    enc_launch_conv(xin, e->wih[l], e->bih[l], nullptr, buf[1], B, T, T, 512, 2048, 1, 1, 1, 0, T, false, s);
    HIP_TRY(hipMemsetAsync(e->h, 0, (size_t)B * 512 * 4, s));
    HIP_TRY(hipMemsetAsync(e->c, 0, (size_t)B * 512 * 4, s));
    for (int t = 0; t < T; ++t)
      enc_launch_lstm_step(buf[1], e->whh[l], e->bhh[l], e->h + (size_t)(t & 1) * e->bmax * 512,
                           e->h + (size_t)((t + 1) & 1) * e->bmax * 512, e->c, yout, l == 1 ? buf[0] : nullptr, B, T, t, s);
  }
  conv(17, buf[3], T, buf[0], nullptr);  // ELU -> final conv: embedding [B][T][512]
  // quantiser: scores x . e (a 1-tap conv with the codebook as weights), then argmax + gather
  enc_launch_conv(buf[0], e->codebook, nullptr, nullptr, buf[1], B, T, T, 512, 4096, 1, 1, 1, 0, T, false, s);
  enc_launch_vq(buf[0], buf[1], e->esq, e->codebook, codes, features, B, T, s);
  HIP_TRY(hipGetLastError());
  return LVX_OK;
}

// test hook: the encoder's output before quantisation ([B][T][512], time-major) of the last lvx_encode
int lvx_enc_embedding(lvx_enc* e, float* dst, int B, int T, void* stream) {
  if (!e || !e->finalized || !dst) return fail(LVX_E_ARG, "bad arguments");
  HIP_TRY(hipMemcpyAsync(dst, e->buf[0], (size_t)B * T * 512 * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return LVX_OK;
}

}  // extern "C"
