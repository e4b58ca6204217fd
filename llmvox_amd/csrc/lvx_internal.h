// Internal (C++) interfaces between the C-ABI front end and the kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "lvx_common.h"
#include "llmvox.h"

namespace lvx {

constexpr int N_LAYER = 4, N_HEAD = 8, D = 768, HD = 96, DFF = 3072, VOCAB = 4096;
constexpr int TEXT_DIM = 256, SPEECH_DIM = 512, TEXT_VOCAB = 386, BLOCK_SIZE = 8192;
constexpr int NSPLIT = 16;  // max KV splits per (stream, head) in decode attention
// KV cache in chunks of KV_CHUNK positions, chunk-major over (slot, head): the positions a step reads
// (0..t-1 of every stream) lie in the first ceil(t / KV_CHUNK) chunks of a layer, whatever the
// capacity (max_positions) is
constexpr int KV_CHUNK = 64;
__host__ __device__ inline size_t kv_at(size_t layer, size_t chunks, size_t streams, int s, int head, int pos) {
  return (((((layer * chunks + (size_t)(pos / KV_CHUNK)) * streams + s) * 8 + head) * KV_CHUNK) + (size_t)(pos % KV_CHUNK)) * 96;
}
#ifndef LVX_YCOPIES
#define LVX_YCOPIES 4
#endif
constexpr int YCOPIES = LVX_YCOPIES;  // accumulator copies of the fused MLP (spreads atomic contention)
constexpr int LM_MAX_BLOCKS = 1024;  // lm_head blocks of the fused argmax tail (4096 rows / 8 per block = 512)
// Kernel-variant switches of ONE context (lvx_set_option; defaults = the production kernels). Each
// C-ABI call that launches or captures kernels binds a snapshot of its context's options to the
// calling thread for the duration of the call (OptScope); the launch helpers read them through
// opts(). Options set on one context therefore never change another context's kernels, and a
// launch never reads an option while another thread writes it.
struct Opts {
  int defer_select = 1;  // greedy select deferred into the next step's first kernel; 0: argmax kernel;
                         // 2: as 1 but 4 <= B <= 8 through ar_embed_select_kernel (cross-check)
  int fuse_mlp = 1;      // bf16, B <= 2: c_fc + gelu + mlp c_proj in one kernel; 0: two GEMV kernels
  int bt = 1;            // 1: batched v3 for 32 < B <= 64; 2: v3 for every batched B (cross-check); 0: off
  int codec_g2 = 1, codec_skinny = 1, codec_g3 = 1, codec_g3f = 2;  // codec GEMM kernels (cross-checks)
  int codec_exp = 0;     // codec A/B bits (bit-identical variants)
  int exp = 0;           // AR cross-check bits (fp32 tiles / one-launch forms: tests/test_gpu_f32b.py)
  int f32b = 1;          // fp32 batched steps on exact-fp32 MFMA; 0: the GEMV family
  int ln_max = 8;        // batched steps with the LayerNorm fused into the GEMM prologue for B <= ln_max
  int l0q = 1;           // bf16, B <= 32 (not 3): layer 0's q / k / v from the precomputed tables (ArWeights q0_*)
                         // in the embedding + select kernel; 0: that kernel + the c_attn GEMM (cross-check)
};
const Opts& opts();  // the calling thread's bound options (the defaults when none is bound)
struct OptScope {    // binds `o` to this thread until the scope ends
  explicit OptScope(const Opts* o);
  ~OptScope();
  OptScope(const OptScope&) = delete;
  OptScope& operator=(const OptScope&) = delete;
  const Opts* prev;
};

// Device-resident AR weights. Matrices are [out][in] row-major (torch Linear layout),
// in the context's weight dtype; vectors and gathered tables are fp32.
struct ArWeights {
  const float* wpe = nullptr;         // [8192][768]
  const float* text_table = nullptr;  // [386][256]
  const float* codebook = nullptr;    // [4096][512] (shared with the codec)
  const float* ln1[N_LAYER] = {};
  const float* ln2[N_LAYER] = {};
  const float* lnf = nullptr;
  const void* w_attn[N_LAYER] = {};   // [2304][768]
  const void* w_aproj[N_LAYER] = {};  // [768][768]
  const void* w_fc[N_LAYER] = {};     // [3072][768]
  const void* w_mproj[N_LAYER] = {};  // [768][3072]
  const void* w_mproj_pk[N_LAYER] = {};  // bf16 only: thread-packed copy for the fused MLP (pack_mproj)
  const float* fc_gsum[N_LAYER] = {};    // bf16 only: G[n] = sum_k ln_2.weight[k] * bf16(c_fc W[n][k]) (batched
                                         // c_fc: LayerNorm applied after the GEMM, ar_mfma2_kernel XM 1)
  const void* w_lm = nullptr;         // [4096][768]
  // bf16 only: layer 0's c_attn as table rows (ar_embed_select_kernel QKV). The step's input row is
  // x = cat(text_table[t], codebook[c]) / den + wpe[p] and c_attn multiplies LN1(x) = (x - mean) * rstd
  // * g, so W . LN1(x) = rstd * (W . (x * g) - mean * G) with W . (x * g) = (Tt[t] + Tc[c]) / den + Tp[p]:
  // Tt[t][n] = sum_k<256 g[k] W[n][k] text_table[t][k], Tc over k = 256.. 767 with the codebook, Tp with
  // wpe (bf16 W, fp32 sums), G[n] = sum_k g[k] W[n][k]
  const float* q0_text = nullptr;     // [386][2304]
  const float* q0_code = nullptr;     // [4096][2304]
  const float* q0_pos = nullptr;      // [max_positions][2304]
  const float* q0_g = nullptr;        // [2304]
  // MFMA-fragment-packed copies for the batched GEMMs, one contiguous KB per wave-wide 16-B load of
  // the A operand: bf16 [N / 16][K / 32][64][8] for v_mfma_f32_16x16x32_bf16 (pack_frag); fp32
  // [N / 16][K / 16][64][4] for v_mfma_f32_16x16x4_f32 (pack_frag32, the fp32 parity mode)
  const void* f_attn[N_LAYER] = {};
  const void* f_aproj[N_LAYER] = {};
  const void* f_fc[N_LAYER] = {};
  const void* f_mproj[N_LAYER] = {};
  const void* f_lm = nullptr;
};

// Device-resident decode state + scratch.
struct ArState {
  int32_t* slots = nullptr;      // [B] slot of batch row b (-1: idle row)
  const int32_t* text_plan = nullptr;  // [B][plan_stride] text id of row b at its step j
  int32_t* rowstep = nullptr;    // [B] next step j of row b (advanced by the step)
  int32_t* tok_plan = nullptr;   // [B][plan_stride] greedy token of row b at step j
  float* margin_plan = nullptr;  // [B][plan_stride] top1-top2 logit margin (optional)
  int plan_stride = 1;
  int4* rowinfo = nullptr;       // [B] {slot, pos, text id, prev token} of the step in flight
  int4* rowinfo_n = nullptr;     // [B] deferred select: records built by c_attn layer 0 (copied back by attention)
  int2* rowx = nullptr;          // [B] deferred select: {plan step j of the step in flight, text id of step j + 1}
  int2* rowx_n = nullptr;        // [B] its shadow (as rowinfo_n)
  uint32_t* selp = nullptr;      // [1] deferred select pending: lm_head granules not yet committed
  uint32_t* selrow = nullptr;    // [B] batched deferred select: row b's logits not yet committed
  int32_t* pos = nullptr;       // [max_streams] per-slot next position
  int32_t* prev = nullptr;      // [max_streams] per-slot previous token
  int32_t* err = nullptr;       // [4] error words: [0] AR (1 KV capacity, 2 plan overrun, 4 text id / code out
                                // of range in the drop-in gathers, 32 fused-MLP fixed-point range); [1] codec
                                // (4 code out of range, 8 ISTFT envelope); [2] / [3] take slots of
                                // lvx_check_errors / lvx_stream_position
  float* x = nullptr;           // [B][768] residual stream
  float* q = nullptr;           // [B][768]
  float* part_o = nullptr;      // [B][8][NSPLIT][96]
  float* part_ml = nullptr;     // [B][8][NSPLIT][2]
  float* h = nullptr;           // [B][3072]
  bf16_t* xn = nullptr;         // [B][768] bf16 operand rows (batched path)
  bf16_t* hb = nullptr;         // [B][3072] bf16 h (batched path)
  bf16_t* xb = nullptr;         // [B][768] bf16 copy of x after c_proj (batched path: c_fc's operand, normalised from xstat)
  float* xstat = nullptr;       // [max_streams][48 column blocks][2] (mean, M2) of x over 16 columns
  float* logits = nullptr;      // [B][4096]
  float* qkvp = nullptr;        // [4][max_streams][2304] c_attn K-slice partials (batched B > 16: summed by the attention)
  uint64_t* lmbest = nullptr;   // [LM_MAX_BLOCKS][4][2] per-block top1/top2 granules of lm_head (deferred select, B <= 2)
  unsigned long long* yfx = nullptr;  // [max_streams][YCOPIES][768] B <= 2 fused-MLP output, 2^-32 fixed point
                                     // (int64 atomics), a row's copies adjacent
  float* yacc = nullptr;        // [max_streams][YCOPIES][768] batched mlp c_proj K-slice partials (fp32);
                                // a row's copies adjacent: spaced by max_streams rows they shared
                                // L2 channels (B = 1: 82.6 vs 69.6 us/step at max_streams 32)
  void* kc = nullptr;           // [4][kv_chunks][max_streams][8][KV_CHUNK][96] (kv_at)
  void* vc = nullptr;
  int max_pos = 0, max_streams = 0, kv_chunks = 0;
};

// Launches the whole decode step (embed -> 4 blocks -> lm_head [-> argmax]).
// mode 0: fused step (inputs from st.slots/st.text_ids, argmax + state advance)
// mode 1: drop-in row forward (emb_row given, single stream, logits to `logits_out`)
void ar_launch_step(const ArWeights& w, const ArState& st, int wdtype, int kvdtype, int B, int mode,
                    const float* emb_row, int slot, int pos, float* logits_out, hipStream_t s);

int ar_probe(const ArWeights& w, const ArState& st, int wdtype, int kvdtype, int B, int which, int iters,
             hipStream_t s);
void ar_launch_rowinfo_init(const ArState& st, int B, hipStream_t s);
void ar_launch_steps_end(const ArState& st, int wdtype, int B, hipStream_t s);  // deferred select: commit the last step
int ar_select_probe(const ArWeights& w, const ArState& st, int B, int path, hipStream_t s);  // test hook
// ArWeights::q0_text / q0_code / q0_pos from the bf16 c_attn weight of layer 0 (lvx_finalize)
void ar_launch_q0_tables(const ArWeights& w, int max_pos, float* text, float* code, float* pos, hipStream_t s);
void launch_set_slot(int32_t* pos, int32_t* prev, int slot, int p, int tok, hipStream_t s);
void launch_err_take(int32_t* words, int mask_ar, int mask_codec, int32_t* out, hipStream_t s);
void launch_text_embed(const float* table, const int64_t* ids, int n, float* out, int32_t* err, hipStream_t s);
void launch_codes_to_features(const float* codebook, const int64_t* codes, int B, int L, float* feats,
                              int32_t* err, hipStream_t s);

// ---------------- codec ----------------
struct CodecWeights {
  const float* codebook = nullptr;      // [4096][512]
  const void* embed_w = nullptr;        // [768][7*512] (tap-major repack of [768][512][7])
  const float* embed_b = nullptr;
  const float* ada_scale = nullptr;     // backbone.norm.scale.weight [4][768]
  const float* ada_shift = nullptr;
  // pos_net resnet blocks 0,1,3,4 -> index 0..3
  const float* rn_n1w[4] = {}; const float* rn_n1b[4] = {};
  const float* rn_n2w[4] = {}; const float* rn_n2b[4] = {};
  const void* rn_c1w[4] = {};  const float* rn_c1b[4] = {};  // [768][3*768]
  const void* rn_c2w[4] = {};  const float* rn_c2b[4] = {};
  const float* at_nw = nullptr; const float* at_nb = nullptr;
  const void* at_qkv_w = nullptr; const float* at_qkv_b = nullptr;  // [2304][768], [2304]
  const void* at_proj_w = nullptr; const float* at_proj_b = nullptr;
  const float* pn_w = nullptr; const float* pn_b = nullptr;  // pos_net.5 GroupNorm
  const float* dw_w[12] = {};   // [7][768] (tap-major)
  const float* dw_b[12] = {};
  const float* cn_scale[12] = {}; const float* cn_shift[12] = {};  // [4][768]
  const void* pw1_w[12] = {}; const float* pw1_b[12] = {};  // [2304][768]
  const void* pw2_w[12] = {}; const float* pw2_b[12] = {};  // [768][2304]
  const float* gamma[12] = {};
  const float* fln_w = nullptr; const float* fln_b = nullptr;
  const void* head_w = nullptr; const float* head_b = nullptr;  // [1282][768]
  // codec_dtype FP8: every matrix above is e4m3fn [N][K] and *_s is its per-row scale [N]
  // (w = q * s); null in bf16 / fp32 storage
  int wfp8 = 0;
  const float* embed_s = nullptr;
  const float* rn_c1s[4] = {}; const float* rn_c2s[4] = {};
  const float* at_qkv_s = nullptr; const float* at_proj_s = nullptr;
  const float* pw1_s[12] = {}; const float* pw2_s[12] = {};
  const float* head_s = nullptr;
  const float* window = nullptr;  // [1280] periodic Hann
  const float* twiddle = nullptr; // FFT tables (see istft)
};

struct CodecScratch {
  float* x = nullptr;      // [M][768]
  float* t1 = nullptr;     // [M][2304] general temp
  float* t2 = nullptr;     // [M][2304]
  float* feats = nullptr;  // [M][512]
  float* gn = nullptr;     // [M][768] GroupNorm(+swish) output
  float* ws = nullptr;     // split-K partials
  size_t ws_floats = 0;
  uint32_t* tick = nullptr;  // [4096] per-tile arrival counters of the in-launch split-K combine (zero)
  float* att = nullptr;    // [sum_b L_b^2] scores
  float* stats = nullptr;  // [B][32][2]
  float* spec = nullptr;   // [M][1282]
  float* frames = nullptr; // [M][1280]
  float* rowscale = nullptr;  // [M] per-frame scale of an fp8 operand (codec_dtype FP8: pwconv1's)
  int32_t* err = nullptr;  // = ArState.err + 1, the codec's own word: bit 4 a code outside [0, 4096), bit 8 the ISTFT envelope <= 1e-11
  int max_frames = 0;
};

// feats_in: [B][512][L] (reference layout) when codes == nullptr; else codes [B][L]
void codec_launch_decode(const CodecWeights& w, const CodecScratch& sc, int wdtype, const float* feats_in,
                         const int32_t* codes, int B, int L, int bw, float* pcm, hipStream_t s);

// ---------------- encoder (encode_infer) ----------------
void enc_launch_conv(const float* x, const float* w, const float* bias, const float* res, float* y, int B, int L, int T,
                     int cin, int cout, int k, int stride, int dil, int pl, int lext, bool elu, hipStream_t s);
void enc_launch_lstm_step(const float* gin, const float* whh, const float* bhh, const float* hprev, float* hnext,
                          float* c, float* y, const float* skip, int B, int T, int t, hipStream_t s);
void enc_launch_vq(const float* emb, const float* scores, const float* esq, const float* cb, int32_t* codes,
                   float* feats, int B, int T, hipStream_t s);

}  // namespace lvx
