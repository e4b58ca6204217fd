// Speech-token GPT decode step for CDNA4 (gfx950).
//
// One decode step of src/model.py:201-237 (as driven by streaming_server.py:323-347) for
// B independent streams, each in its own KV slot:
//
//   embed      normalize(cat(text_table[id], codebook[prev] | 0)) + wpe[pos]      (a2-a4)
//   4 x block  LN1 -> c_attn (KV append at pos) -> split-KV decode attention ->
//              c_proj + residual -> LN2 -> c_fc -> gelu(tanh) -> c_proj + residual  (a6-a9)
//   ln_f -> lm_head -> argmax(first max)                                          (a10-a11)
//
// Kernel boundaries are placed only where a full-vector reduction seam exists (LayerNorm
// needs the whole residual row, attention needs the whole K/V history). LayerNorms are
// computed in the prologue of the consuming GEMV (each block re-normalises the <= 16 rows
// it needs from L2: 3 KB per row), the split-KV attention partials are merged in the
// prologue of c_proj, residual adds / GELU / KV-append are GEMV epilogues. The weight
// stream is the HBM-bound part: 62.9 MB (bf16) or 125.8 MB (fp32) per step, shared by the
// B streams of the step.
#include "lvx_internal.h"

// No implicit a*b+c contraction in this file: the compiler would choose per unrolled copy, so a
// batch row's rounding could depend on which copy (batch position) computed it. Fused
// multiply-adds are written out (fmaf / MFMA) where they are wanted.
#pragma clang fp contract(off)

namespace lvx {

// Development timeline of the batched step (tools/step_timeline.py; built only into the
// LVX_TIMING library variant, `make timing`): thread 0 of every block of the instrumented
// kernels records the 100 MHz real-time counter at entry, after its operands landed, and at
// exit, plus the XCC / hardware-id registers, under (tag, layer, block).
#ifdef LVX_TIMING
constexpr int TS_BLOCKS = 1024;
__device__ uint64_t g_lvx_ts[16 * 4 * TS_BLOCKS * 4];
#define TS_DECL uint64_t ts_[2] = {0, 0}
#define TS_MARK(i) do { if (threadIdx.x == 0) ts_[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TS_SAVE(tag, layer, blk)                                                                    \
  do {                                                                                               \
    if (threadIdx.x == 0) {                                                                          \
      const uint64_t te_ = __builtin_amdgcn_s_memrealtime();                                         \
      const uint64_t hw_ = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                    \
                           ((uint64_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32);              \
      uint64_t* p_ = g_lvx_ts + ((size_t)(((tag) * 4 + (layer)) * TS_BLOCKS + min((int)(blk), TS_BLOCKS - 1))) * 4; \
      p_[0] = ts_[0]; p_[1] = ts_[1]; p_[2] = te_; p_[3] = hw_;                                      \
    }                                                                                                \
  } while (0)
#else
#define TS_DECL do {} while (0)
#define TS_MARK(i) do {} while (0)
#define TS_SAVE(tag, layer, blk) do {} while (0)
#endif

// ---------------------------------------------------------------------------------
// GEMV family: out[b][n] = sum_k W[n][k] * in[b][k]   (W row-major [N][K], TW in {f32,bf16})
//   IN  0: in = LayerNorm(x[b]) * ln_w            (eps 1e-5, no bias; src/model.py:37-38)
//   IN  1: in = h[b] (fp32, K = 3072)
//   IN  2: in = merge of the split-KV attention partials (flash-decoding combine)
//   IN  4: in = LayerNorm(x[b] + sum_c yacc[b][c]) (the fused MLP's pending output)
//   IN  3: layer-0 c_attn: builds x[b] first (a2-a4: text row, codebook row of the previous
//          token or 0 at position 0, L2-normalise eps 1e-8, + wpe[pos]; or, for the drop-in
//          row forward, the caller's row + wpe[pos]), block 0 stores it, then LayerNorm.
//   OUT 0: c_attn: q -> st.q, k/v -> KV cache at the slot's position
//   OUT 1: residual: x[b][n] += out
//   OUT 2: h[b][n] = gelu_tanh(out)
//   OUT 3: logits: dst[b][n] = out
// A block is 4 waves; KW waves share the K range of the same RPW rows (KW in {1,4}). Each
// lane owns 4-element K chunks. All weight loads of the wave are issued before the input
// prologue (they do not depend on it), so the HBM/MALL latency overlaps the LN / merge /
// embed work, and the weights stay in registers across batch groups of BG rows.
// ---------------------------------------------------------------------------------
// Operand rows (bf16 [B][K]) in MFMA-fragment order, the B operand of v_mfma_f32_16x16x32_bf16 as
// the batched GEMMs load it: element (b, k) of tile b / 16, k-step k / 32, lane 16 ((k / 8) % 4) + b % 16,
// slot k % 8 — one wave-wide 16-B load reads one contiguous KB (row-major: 16 rows x 64 B)
__device__ __forceinline__ size_t xfrag(int b, int k, int K) {
  return ((((size_t)(b >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k >> 3) & 3) * 16 + (b & 15)) << 3) + (k & 7);
}

struct GemvArgs {
  ArState st;
  const void* W;
  const void* Wf;        // batched MFMA GEMMs: the fragment-packed copy of W (ArWeights f_*), or null
  int xpk;               // batched v2 steps at 9 <= B <= 32: the bf16 operand rows xn / xb / hb are kept
                         // fragment-packed (xfrag), as the GEMMs load them
  int N;
  int B;
  int layer;
  const float* ln_w;
  float* dst;
  int kv_dtype;          // LVX_DTYPE_F32 / BF16 / FP8
  // IN 3 inputs
  const float* text_table;
  const float* codebook;
  const float* wpe;
  const float* emb_row;  // drop-in row mode when non-null
  // fused MLP (ar_mlp_fused_kernel): its output sits in YCOPIES accumulators until c_proj folds it in
  float* yacc;           // batched steps: the mlp c_proj K-slice partials (fp32, plain stores)
  unsigned long long* yfx;  // B <= 2 fused MLP (non-null when the step runs it): its output as YCOPIES
                            // accumulators in 2^-32 fixed point (int64 atomics: order-independent sums)
  const float* gsum;     // batched c_fc (ar_mfma2_kernel XM 1): ArWeights::fc_gsum of the layer
  int add_y;             // c_proj: fold the accumulators into x (layers >= 1; 0 at layer 0 = just clear)
  int defer_sel;         // deferred greedy select (option "defer_select"). 1: B <= 2 GEMV step, lm_head
                         // publishes per-block granules, the next step's c_attn layer 0 reduces them;
                         // 2: batched step, the next step's embedding rows kernel reduces the logits
  int xmap;              // ar_mfma2_kernel launched as a 1-D grid with the XCD-aligned tile order:
                         // 1 = mlp c_proj (K slice = XCD mod 4), 2 = c_proj batch tiles (tile = XCD mod 2)
  // layer 0's c_attn as table rows (ArWeights q0_*; ar_embed_select_kernel QKV)
  const float* q0_text;
  const float* q0_code;
  const float* q0_pos;
  const float* q0_g;
};

// ---------------------------------------------------------------------------------
// greedy select (streaming_server.py:342-347): argmax with first-index ties, top1-top2 margin,
// then the slot's prev token / position / plan step advance (shared by ar_argmax_kernel and the
// fused lm_head tail).
// ---------------------------------------------------------------------------------
struct Best {
  float v, v2;
  int i;
};
__device__ __forceinline__ Best best_merge(Best a, Best c) {
  const bool cb = (c.v > a.v) || (c.v == a.v && c.i < a.i);
  Best r;
  if (cb) { r.v = c.v; r.i = c.i; r.v2 = fmaxf(c.v2, a.v); }
  else { r.v = a.v; r.i = a.i; r.v2 = fmaxf(a.v2, c.v); }
  return r;
}

__device__ __forceinline__ int4 make_rowinfo(const ArState& st, int b, int s, int p, int j, int prev);

// best_merge over the whole wave (exact: best_merge is commutative and associative), DPP within
// rows then the four row results through SGPRs; wave-uniform result
template <int CTRL>
__device__ __forceinline__ Best best_dpp(Best r) {
  return best_merge(r, Best{dpp_f32<CTRL>(r.v), dpp_f32<CTRL>(r.v2), dpp_i32<CTRL>(r.i)});
}
__device__ __forceinline__ Best best_lane(Best r, int lane) {
  return Best{lane_f32(r.v, lane), lane_f32(r.v2, lane), __builtin_amdgcn_readlane(r.i, lane)};
}
__device__ __forceinline__ Best best_wave(Best r) {
  r = best_dpp<0xB1>(r);
  r = best_dpp<0x4E>(r);
  r = best_dpp<0x128>(r);
  r = best_dpp<0x124>(r);
  return best_merge(best_merge(best_lane(r, 0), best_lane(r, 16)), best_merge(best_lane(r, 32), best_lane(r, 48)));
}

// The reference selects argmax(softmax(logits)) on the CPU in fp32 (streaming_server.py:343-346).
// ATen's last-dim softmax is exp(x - max) * (1 / sum): two probabilities are equal exactly when
// exp(x - max) rounds to 1.0f, i.e. x - max >= -2^-25 (exact subtraction this close to the max;
// exp behaves correctly rounded there: pinned against torch in tests/test_select_rule.py), and
// argmax then takes the first of them. best_merge's (top1, first index, top2) decides alone when
// top1 - top2 > 2^-25; otherwise the wave rescans the row for the first index within 2^-25 of the
// maximum (never taken on real logits short of an exact tie). r must be wave-uniform; returns
// the reference's index in r.i (r.v / r.v2 unchanged: the margin stays top1 - top2).
constexpr float SOFTMAX_TIE = 2.98023223876953125e-08f;  // 2^-25
__device__ __noinline__ int softmax_tie_scan(const float* __restrict__ row, float m, int lane) {
  int first = 0x7fffffff;
  const float4* p = reinterpret_cast<const float4*>(row);
  for (int k = 0; k < VOCAB / 256; ++k) {
    const float4 v = p[k * 64 + lane];
    const int i0 = (k * 64 + lane) * 4;
    if (v.w - m >= -SOFTMAX_TIE) first = i0 + 3;
    if (v.z - m >= -SOFTMAX_TIE) first = i0 + 2;
    if (v.y - m >= -SOFTMAX_TIE) first = i0 + 1;
    if (v.x - m >= -SOFTMAX_TIE) first = i0;
    if (first != 0x7fffffff) break;  // this lane's later chunks hold only larger indices
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o));
  return first;
}
__device__ __forceinline__ Best softmax_ties(const float* __restrict__ row, Best r, int lane) {
  if (!(r.v - r.v2 > SOFTMAX_TIE)) r.i = softmax_tie_scan(row, r.v, lane);
  return r;
}

// text id of row b at plan step j (-1: past the end of the plan; PAD when no plan is bound)
__device__ __forceinline__ int plan_tok(const ArState& st, int b, int j) {
  if (!st.text_plan) return 384;
  return (j < st.plan_stride) ? min(max(st.text_plan[(size_t)b * st.plan_stride + j], 0), TEXT_VOCAB - 1) : -1;
}

__device__ __forceinline__ void argmax_commit(const ArState& st, int b, int4 ri, Best r) {
  if (!st.rowstep) return;  // measurement probe: no plan bound, state is not advanced
  const int s = ri.x;
  const int j = st.rowstep[b];
  if (j < st.plan_stride) {
    st.tok_plan[(size_t)b * st.plan_stride + j] = r.i;
    if (st.margin_plan) st.margin_plan[(size_t)b * st.plan_stride + j] = r.v - r.v2;
  }
  st.prev[s] = r.i;
  st.pos[s] = ri.y + 1;
  st.rowstep[b] = j + 1;
  st.rowinfo[b] = make_rowinfo(st, b, s, ri.y + 1, j + 1, r.i);
}

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));

// Deferred select: lm_head (OUT 9) leaves one 16-byte granule {index << 32 | top1 bits, top2 bits}
// per (block, row) in st.lmbest; the next step's c_attn layer 0 (IN 5) or ar_select_final_kernel
// reduces a row's 512 granules with one wave: every load in flight at once, then a shuffle tree.
static_assert(NSPLIT == 16, "the split merges reduce one head's splits as one 16-lane DPP row");
constexpr int LM_SEL_BLOCKS = VOCAB / 8;  // lm_head blocks on the B <= 2 GEMV path (8 rows each)
struct LmGran {
  u64x2_t g[LM_SEL_BLOCKS / 64];
};
__device__ __forceinline__ void lmg_issue(const ArState& st, int b, int lane, LmGran& q) {
  const u64x2_t* base = reinterpret_cast<const u64x2_t*>(st.lmbest);
#pragma unroll
  for (int k = 0; k < LM_SEL_BLOCKS / 64; ++k) q.g[k] = base[(size_t)(lane + 64 * k) * 4 + b];
}
__device__ __forceinline__ Best lmg_reduce(const LmGran& q) {
  Best r{-INFINITY, -INFINITY, 0x7fffffff};
#pragma unroll
  for (int k = 0; k < LM_SEL_BLOCKS / 64; ++k)
    r = best_merge(r, Best{__uint_as_float((unsigned)q.g[k].x), __uint_as_float((unsigned)q.g[k].y),
                           (int)(q.g[k].x >> 32)});
  return best_wave(r);
}

// Batched deferred select at 4 <= B <= 8 (defer_sel 3): lm_head (ar_mfma_ln_kernel OUT 3, 16 vocabulary
// rows per block) leaves one granule per (block, row) in st.lmbest laid out [256 blocks][8 rows]; the
// next step's c_attn layer 0 (ar_mfma_ln_kernel MODE 7) reduces a row's 256 granules with one wave
constexpr int LM8_BLOCKS = VOCAB / 16, LM8_ROWS = 8;
struct LmGran8 {
  u64x2_t g[LM8_BLOCKS / 64];
};
__device__ __forceinline__ void lmg8_issue(const ArState& st, int b, int lane, LmGran8& q) {
  const u64x2_t* base = reinterpret_cast<const u64x2_t*>(st.lmbest);
#pragma unroll
  for (int k = 0; k < LM8_BLOCKS / 64; ++k) q.g[k] = base[(size_t)(lane + 64 * k) * LM8_ROWS + b];
}
__device__ __forceinline__ Best lmg8_reduce(const LmGran8& q) {
  Best r{-INFINITY, -INFINITY, 0x7fffffff};
#pragma unroll
  for (int k = 0; k < LM8_BLOCKS / 64; ++k)
    r = best_merge(r, Best{__uint_as_float((unsigned)q.g[k].x), __uint_as_float((unsigned)q.g[k].y),
                           (int)(q.g[k].x >> 32)});
  return best_wave(r);
}
__device__ __forceinline__ u64x2_t lm_granule(Best r) {
  u64x2_t g;
  g.x = ((unsigned long long)(unsigned)r.i << 32) | __float_as_uint(r.v);
  g.y = (unsigned long long)__float_as_uint(r.v2);
  return g;
}

// one K (which 0) or V (which 1) element of the KV cache in its dtype
__device__ __forceinline__ void store_kv(const GemvArgs& a, int which, size_t idx, float v) {
  void* base = which ? a.st.vc : a.st.kc;
  if (a.kv_dtype == LVX_DTYPE_BF16) reinterpret_cast<bf16_t*>(base)[idx] = f32_to_bf16(v);
  else if (a.kv_dtype == LVX_DTYPE_FP8) reinterpret_cast<fp8_t*>(base)[idx] = f32_to_fp8(v);
  else reinterpret_cast<float*>(base)[idx] = v;
}

template <typename TW> struct WReg;
template <> struct WReg<float> {
  typedef float4 T;
  __device__ __forceinline__ static T load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ __forceinline__ static float4 f(T v) { return v; }
  __device__ __forceinline__ static T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
template <> struct WReg<bf16_t> {
  typedef uint2 T;
  __device__ __forceinline__ static T load(const bf16_t* p) { return *reinterpret_cast<const uint2*>(p); }
  __device__ __forceinline__ static float4 f(T u) {
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
  __device__ __forceinline__ static T zero() { return make_uint2(0u, 0u); }
};

// LayerNorm of one 768-row held as 3 float4 per lane (one wave), written to xs
// gamma (3 float4 per lane, k = j * 256 + lane * 4) is loaded by the caller ahead of the weight
// stream: loaded here, after x, it was the last load issued, so waiting for it waited for every
// weight load in flight as well
__device__ __forceinline__ void wave_ln_to_lds(float4 (&v)[3], const float4 (&gam)[3], float* xs_row, int lane) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float dx = v[j].x - mean, dy = v[j].y - mean, dz = v[j].z - mean, dw = v[j].w - mean;
    q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
  }
  const float var = wave_sum(q) * (1.0f / D);
  const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int k = j * 256 + lane * 4;
    const float4 g = gam[j];
    *reinterpret_cast<float4*>(xs_row + k) =
        make_float4((v[j].x - mean) * rstd * g.x, (v[j].y - mean) * rstd * g.y, (v[j].z - mean) * rstd * g.z,
                    (v[j].w - mean) * rstd * g.w);
  }
}

// x[b] (IN 0) or x[b] + sum_c yacc[b][c] (IN 4) in the lane layout k = j * 256 + lane * 4: the
// loads are issued by xrow_issue and summed by xrow_sum, so a prefetch does not wait on them
// The fused MLP's fixed point (B <= 2): partial t -> round(t * 2^32) as int64, added with 64-bit
// integer atomics (exact, so the sum does not depend on the order the 192 blocks arrive in: the
// output is reproducible run to run), read back as (float)(sum of the copies) * 2^-32
typedef unsigned long long u64x2n __attribute__((ext_vector_type(2)));
// A partial outside +-2^25 (or NaN / inf) cannot be summed exactly by up to 48 adders per copy in
// int64 (and __float2ll_rn is undefined past 2^63): it is clamped and reported (error bit 32,
// lvx_check_errors -> LVX_E_STATE) instead of silently becoming an arbitrary finite value; the
// reference would carry the non-finite value into its logits. Activations here are O(1)-O(100).
constexpr float YFX_MAX = 33554432.0f;  // 2^25
__device__ __forceinline__ unsigned long long yfx_of(float t, int32_t* err) {
  if (!(fabsf(t) < YFX_MAX)) {
    atomicOr(err, 32);
    t = (t != t) ? 0.f : copysignf(YFX_MAX, t);
  }
  return (unsigned long long)__float2ll_rn(t * 4294967296.0f);
}
__device__ __forceinline__ float yfx_to_f(unsigned long long s) {
  return __ll2float_rn((long long)s) * 2.3283064365386963e-10f;
}

// FX = false: the batched steps' fp32 K-slice partials (ar_rows_kernel<4>); FX = true: the B <= 2
// fused MLP's fixed-point copies (GEMV IN 4)
template <int IN, bool FX = false>
struct XRow {
  float4 x[3];
  float4 y[(IN == 4 && !FX) ? YCOPIES : 1][3];
  u64x2n yf[(IN == 4 && FX) ? YCOPIES : 1][3][2];
};
template <int IN, bool FX = false>
__device__ __forceinline__ void xrow_issue(const GemvArgs& a, int b, int lane, XRow<IN, FX>& r) {
  const float* xr = a.st.x + (size_t)b * D;
#pragma unroll
  for (int j = 0; j < 3; ++j) r.x[j] = *reinterpret_cast<const float4*>(xr + j * 256 + lane * 4);
  if constexpr (IN == 4 && FX) {
#pragma unroll
    for (int c = 0; c < YCOPIES; ++c)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const u64x2n* yp = reinterpret_cast<const u64x2n*>(a.yfx + ((size_t)b * YCOPIES + c) * D + j * 256 + lane * 4);
        r.yf[c][j][0] = yp[0];
        r.yf[c][j][1] = yp[1];
      }
  } else if constexpr (IN == 4) {
#pragma unroll
    for (int c = 0; c < YCOPIES; ++c)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        r.y[c][j] = *reinterpret_cast<const float4*>(a.yacc + ((size_t)b * YCOPIES + c) * D + j * 256 + lane * 4);
  }
}
template <int IN, bool FX = false>
__device__ __forceinline__ void xrow_sum(const XRow<IN, FX>& r, float4 (&v)[3]) {
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float4 t = r.x[j];
    if constexpr (IN == 4 && FX) {
      u64x2n s0 = r.yf[0][j][0], s1 = r.yf[0][j][1];
#pragma unroll
      for (int c = 1; c < YCOPIES; ++c) { s0 += r.yf[c][j][0]; s1 += r.yf[c][j][1]; }
      t.x += yfx_to_f(s0.x); t.y += yfx_to_f(s0.y); t.z += yfx_to_f(s1.x); t.w += yfx_to_f(s1.y);
    } else if constexpr (IN == 4) {
#pragma unroll
      for (int c = 0; c < YCOPIES; ++c) { t.x += r.y[c][j].x; t.y += r.y[c][j].y; t.z += r.y[c][j].z; t.w += r.y[c][j].w; }
    }
    v[j] = t;
  }
}

// Kernels whose grid fills a fraction of the chip (B rows, 144 K-split blocks): with the default
// occupancy target the scheduler keeps few VGPRs live and issues part of the loads only after the
// first ones have landed (rows kernel: 12 loads, a wait, then gamma and 3 row loads; the K-split
// c_attn: weights two at a time), one more dependent round trip. Capping the target at 4 waves per
// SIMD (128 VGPRs) leaves them all in flight at once (round 3, checked in the ISA). Measured
// (tools/step_sweep.py, B = 32, t = 384-639, two A/B rounds on one box): bf16 129.2 / 133.0 vs
// 130.5 / 129.9 us/step, fp32 210.8 / 211.3 vs 211.5 / 211.3: within the noise; the late loads (gamma,
// lines already on their way to L2) return quickly.
#ifdef LVX_NO_LOADS_FIRST  // A/B builds (tools/build_variant.sh)
#define LVX_LOADS_FIRST
#else
#define LVX_LOADS_FIRST __attribute__((amdgpu_waves_per_eu(1, 4)))
#endif

template <int K, int IN, int BG = 0>
__device__ __forceinline__ void gemv_stage_input(const GemvArgs& a, float* xs, float* aux, const float4 (&gam)[3], int g0, int bg,
                                                 const XRow<IN == 4 ? 4 : 0, true>& xpre, int4 ripre, bool prefetched) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (IN == 0 || IN == 3 || IN == 4 || IN == 5) {
    for (int bb = wave; bb < bg; bb += 4) {  // one wave per row
      const int b = g0 + bb;
      const bool pre = prefetched && g0 == 0 && bb == wave;  // this row was prefetched before the weights
      float4 v[3];
      if (IN == 0 || IN == 4) {
        if (pre) {
          xrow_sum(xpre, v);
        } else {
          XRow<IN == 4 ? 4 : 0, true> xr;
          xrow_issue(a, b, lane, xr);
          xrow_sum(xr, v);
        }
      } else if (a.emb_row) {  // drop-in row forward: caller's normalised row + wpe[pos]
        const int p = a.st.rowinfo[0].y;
        const float* wr = a.wpe + (size_t)p * D;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int k = j * 256 + lane * 4;
          const float4 e = *reinterpret_cast<const float4*>(a.emb_row + k);
          const float4 pe = *reinterpret_cast<const float4*>(wr + k);
          v[j] = make_float4(e.x + pe.x, e.y + pe.y, e.z + pe.z, e.w + pe.w);
        }
        if (blockIdx.x == 0)
#pragma unroll
          for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + j * 256 + lane * 4) = v[j];
      } else {
        const int4 ri = pre ? ripre : a.st.rowinfo[b];  // {slot, pos, text id, prev}, validated by the producer
        if (ri.x < 0) {
#pragma unroll
          for (int j = 0; j < 3; ++j) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          const int p = ri.y, prev = ri.w;
          int tok = ri.z;
          // the wpe row goes out with the text / codebook rows (clamped row, unconditional:
          // issued behind the normalisation it was a round trip of its own)
          const float* wr = a.wpe + (size_t)min(max(p, 0), BLOCK_SIZE - 1) * D;
          float4 pe[3];
#pragma unroll
          for (int j = 0; j < 3; ++j) pe[j] = *reinterpret_cast<const float4*>(wr + j * 256 + lane * 4);
          if (tok < 0) {
            if (lane == 0 && blockIdx.x == 0) atomicOr(a.st.err, 2);
            tok = 384;
          }
          float ss = 0.f;
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const int k = j * 256 + lane * 4;  // j == 0: text part (k < 256), else speech part
            if (j == 0) v[j] = *reinterpret_cast<const float4*>(a.text_table + (size_t)tok * TEXT_DIM + k);
            else if (p == 0) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            else v[j] = *reinterpret_cast<const float4*>(a.codebook + (size_t)prev * SPEECH_DIM + (k - TEXT_DIM));
            ss += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
          }
          ss = wave_sum(ss);
          const float den = fmaxf(sqrtf(ss), 1e-8f);  // F.normalize: x / max(||x||_2, eps)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            v[j] = make_float4(v[j].x / den + pe[j].x, v[j].y / den + pe[j].y, v[j].z / den + pe[j].z,
                               v[j].w / den + pe[j].w);
        }
        if (blockIdx.x == 0)
#pragma unroll
          for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = v[j];
      }
      wave_ln_to_lds(v, gam, xs + bb * K, lane);
    }
  } else if (IN == 1) {
    for (int e = tid * 4; e < bg * K; e += 256 * 4)
      *reinterpret_cast<float4*>(xs + e) = *reinterpret_cast<const float4*>(a.st.h + (size_t)g0 * K + e);
  } else {
    // merge the split-KV partials: y = sum_s c_s o_s, c_s = e^{m_s - M} / sum_s' e^{m_s' - M} l_s'.
    // Phase A: one thread per (row, head) turns the (m, l) pairs into coefficients (zero for unused
    // splits); phase B: every element sums all NSPLIT partials unconditionally (part_o is zeroed at
    // allocation, so unused splits hold finite values), one round trip of independent loads.
    for (int q = tid; q < bg * N_HEAD; q += 256) {
      const int bb = q / N_HEAD, head = q - bb * N_HEAD, b = g0 + bb;
      const int4 ri = a.st.rowinfo[b];
      float* cf = aux + q * NSPLIT;
      const int t = ri.y + 1;
      const int ns = ri.x < 0 ? 0 : min(NSPLIT, (t + 63) / 64);
      const float* ml = a.st.part_ml + ((size_t)(b * N_HEAD + head) * NSPLIT) * 2;
      float m[NSPLIT], l[NSPLIT];
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) { m[i] = ml[2 * i]; l[i] = ml[2 * i + 1]; }
      float M = -INFINITY;
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) if (i < ns) M = fmaxf(M, m[i]);
      float den = 0.f;
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) {
        const float f = (i < ns && m[i] != -INFINITY) ? expf(m[i] - M) : 0.f;
        m[i] = f;
        den += f * l[i];
      }
      const float inv = ns ? 1.0f / den : 0.f;
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) cf[i] = m[i] * inv;
    }
    __syncthreads();
    if constexpr (BG == 2) {
      // B = 2 (bg == 2: 6 elements per thread): all 6 x NSPLIT partial loads in flight before the
      // first sum (the loop below waited for each element's 16 loads before issuing the next
      // element's: 6 dependent round trips); the same sum per element. tools/step_sweep.py B = 2,
      // t = 384-639: bf16 98.5-98.7 -> 96.3-96.5 us/step, fp32 110.9-112.3 -> 110.1-110.2
      constexpr int IT = 2 * D / 256;
      static_assert(2 * D % 256 == 0, "whole elements per thread");
      float pv[IT][NSPLIT];
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const int e = tid + 256 * k, bb = e / D, c = e - bb * D;
        const int head = c / HD, d = c - head * HD;
        const float* po = a.st.part_o + ((size_t)((g0 + bb) * N_HEAD + head) * NSPLIT) * HD + d;
#pragma unroll
        for (int i = 0; i < NSPLIT; ++i) pv[k][i] = po[(size_t)i * HD];
      }
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const int e = tid + 256 * k, bb = e / D, c = e - bb * D, head = c / HD;
        const float* cf = aux + (bb * N_HEAD + head) * NSPLIT;
        float y = 0.f;
#pragma unroll
        for (int i = 0; i < NSPLIT; ++i) y += cf[i] * pv[k][i];
        xs[bb * K + c] = y;
      }
      return;
    }
    for (int e = tid; e < bg * D; e += 256) {
      const int bb = e / D, c = e - bb * D;
      const int b = g0 + bb;
      const int head = c / HD, d = c - head * HD;
      const float* cf = aux + (bb * N_HEAD + head) * NSPLIT;
      const float* po = a.st.part_o + ((size_t)(b * N_HEAD + head) * NSPLIT) * HD + d;
      float pv[NSPLIT];
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) pv[i] = po[(size_t)i * HD];
      float y = 0.f;
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) y += cf[i] * pv[i];
      xs[bb * K + c] = y;
    }
  }
}

template <typename TW, int K, int KW, int RPW, int BG, int IN, int OUT>
__global__ __launch_bounds__(256) void ar_gemv_kernel(GemvArgs a) {
  constexpr int KC = K / KW;     // K columns per wave
  constexpr int NI = KC / 256;   // 4-element chunks per lane per row
  constexpr int WROWS = 4 / KW;  // row groups per block
  __shared__ __attribute__((aligned(16))) float xs[BG * K];
  __shared__ float part[4][RPW][BG];
  __shared__ float aux[IN == 2 ? BG * N_HEAD * NSPLIT : 1];
  __shared__ int4 ri_s[IN == 5 ? BG : 1];  // IN 5: the rows' new control records for the KV epilogue
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rg = wave / KW, kp = wave % KW;
  const int row0 = (blockIdx.x * WROWS + rg) * RPW;
  // inputs of the first batch group first (vmcnt retires in issue order): the LayerNorm /
  // embedding math then overlaps the weight stream instead of waiting behind it
  XRow<IN == 4 ? 4 : 0, true> xpre;
  int4 ripre = make_int4(-1, 0, 0, 0);
  const bool prefetched = wave < min(BG, a.B);
  // control record of this lane's epilogue row in the first batch group (bb = lane % BG): the
  // KV append needs (slot, pos); loading it here keeps it off the epilogue's critical path
  int4 riep = make_int4(-1, 0, 0, 0);
  if (OUT == 0 && IN != 5) riep = a.st.rowinfo[min(lane % BG, a.B - 1)];
  // residual epilogue (OUT 1): this lane's (row, batch row) of the first group is (row0 + lane / BG,
  // lane % BG); its x element (and, for c_proj after a fused MLP, the pending accumulators) is
  // loaded now instead of behind the dot products
  float xep = 0.f;
  unsigned long long yep[YCOPIES];
  if constexpr (OUT == 1) {
    const int n = row0 + lane / BG, b = lane % BG;
    if (lane < RPW * BG && n < a.N && b < a.B) {
      xep = a.st.x[(size_t)b * D + n];
      if (IN == 2 && a.yfx)
#pragma unroll
        for (int c = 0; c < YCOPIES; ++c) yep[c] = a.yfx[((size_t)b * YCOPIES + c) * D + n];
    }
  }
  if ((IN == 0 || IN == 3 || IN == 4) && prefetched) {
    if (IN == 0 || IN == 4) {
      xrow_issue(a, wave, lane, xpre);
    } else {
      ripre = a.st.rowinfo[wave];
    }
  }
  // IN 5 (deferred select, every row prefetched by its own wave): the previous step's lm_head
  // granules, the pending flag and the row's {step, next text id} come in the same round trip
  // as the control record
  LmGran lmg;
  int2 rxp = make_int2(0, 0);
  unsigned selpend = 0u;
  if constexpr (IN == 5) {  // every wave, clamped row (no loads under a branch); used by waves < B
    const int rb = min(wave, a.B - 1);
    ripre = a.st.rowinfo[rb];
    rxp = a.st.rowx[rb];
    selpend = *a.st.selp;
    lmg_issue(a.st, rb, lane, lmg);
  }
  float4 gam[3];  // LayerNorm gamma of the LN input modes, ahead of the weights
  if constexpr (IN == 0 || IN == 3 || IN == 4 || IN == 5) {
#pragma unroll
    for (int j = 0; j < 3; ++j) gam[j] = *reinterpret_cast<const float4*>(a.ln_w + j * 256 + lane * 4);
  }
  const TW* __restrict__ W = reinterpret_cast<const TW*>(a.W);
  typename WReg<TW>::T wr[RPW][NI];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int n = row0 + r;
#pragma unroll
    for (int it = 0; it < NI; ++it)
      // clamped row, unconditional load: a load under a branch makes the compiler drain every
      // outstanding load (the prefetched inputs) before the weights are even issued; rows past N
      // are never stored
      wr[r][it] = WReg<TW>::load(W + (size_t)min(n, a.N - 1) * K + kp * KC + it * 256 + lane * 4);
  }
  if constexpr (IN == 5) {
    // commit the previous step's greedy select (argmax_commit's state advance; block 0 writes
    // the shadow records, attention layer 0 copies them back) and build this step's record. The
    // reduction and the record select run unconditionally so that the granule loads stay in the
    // prologue (used only under a branch, the compiler sinks them into it: one more round trip).
    const Best r = softmax_ties(a.st.logits + (size_t)min(wave, a.B - 1) * VOCAB, lmg_reduce(lmg), lane);
    const int s = ripre.x, j = rxp.x, p = ripre.y + 1;
    const bool take = selpend && s >= 0;
    const int4 rn = take ? make_int4(s, min(p, a.st.max_pos - 1), rxp.y, min(max(r.i, 0), VOCAB - 1)) : ripre;
    if (prefetched && blockIdx.x == 0 && lane == 0) {
      const int b = wave;
      if (take) {
        if (p >= a.st.max_pos) atomicOr(a.st.err, 1);
        if (j < a.st.plan_stride) {
          a.st.tok_plan[(size_t)b * a.st.plan_stride + j] = r.i;
          if (a.st.margin_plan) a.st.margin_plan[(size_t)b * a.st.plan_stride + j] = r.v - r.v2;
        }
        a.st.prev[s] = r.i;
        a.st.pos[s] = p;
      }
      // the next text id is looked up by attention layer 0's copier (a dependent load here would
      // hold this block until its weight loads landed: vmcnt retires in order)
      a.st.rowx_n[b] = make_int2(take ? j + 1 : j, 0);
      a.st.rowinfo_n[b] = rn;
    }
    ripre = rn;
    if (prefetched && lane == 0) ri_s[wave] = rn;
  }
  for (int g0 = 0; g0 < a.B; g0 += BG) {
    const int bg = min(BG, a.B - g0);
    if (g0) __syncthreads();
    gemv_stage_input<K, IN, BG>(a, xs, aux, gam, g0, bg, xpre, ripre, prefetched);
    __syncthreads();
    float acc[RPW][BG];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int bb = 0; bb < BG; ++bb) acc[r][bb] = 0.f;
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int k = kp * KC + it * 256 + lane * 4;
#pragma unroll
      for (int bb = 0; bb < BG; ++bb) {
        if (bb < bg) {
          const float4 xv = *reinterpret_cast<const float4*>(xs + bb * K + k);
#pragma unroll
          for (int r = 0; r < RPW; ++r) {
            const float4 w = WReg<TW>::f(wr[r][it]);
            acc[r][bb] = dot4_fma(acc[r][bb], w, xv);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int bb = 0; bb < BG; ++bb) {
        if (bb >= bg) continue;
        const float v = wave_sum(acc[r][bb]);
        if (KW > 1) {
          if (lane == 0) part[wave][r][bb] = v;
        } else {
          acc[r][bb] = v;
        }
      }
    if (KW > 1) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int bb = 0; bb < BG; ++bb) {
          if (bb >= bg) continue;
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < KW; ++q) v += part[rg * KW + q][r][bb];
          acc[r][bb] = v;
        }
    }
    // epilogue: one lane per (row, batch row); with KW > 1 only the row group's first wave
    if (KW > 1 && kp != 0) continue;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = row0 + r;
#pragma unroll
      for (int bb = 0; bb < BG; ++bb) {
        if (bb >= bg || n >= a.N || lane != ((r * BG + bb) & 63)) continue;
        const float v = acc[r][bb];
        const int b = g0 + bb;
        if (OUT == 0) {
          if (n < D) {
            a.st.q[(size_t)b * D + n] = v;
          } else {
            const int c = (n - D) % D, which = (n - D) / D;
            const int head = c / HD, d = c - head * HD;
            const int4 ri = IN == 5 ? ri_s[bb] : g0 == 0 ? riep : a.st.rowinfo[b];
            const int s = ri.x, p = ri.y;
            if (s < 0) continue;
            const size_t idx =
                kv_at(a.layer, a.st.kv_chunks, a.st.max_streams, s, head, p) + d;
            store_kv(a, which, idx, v);
          }
        } else if (OUT == 1) {
          float* xp = a.st.x + (size_t)b * D + n;
          float t = g0 == 0 ? xep : *xp;
          if (IN == 2 && a.yfx) {  // c_proj: fold the fused MLP's accumulators into x and clear them
            unsigned long long ys = 0;
#pragma unroll
            for (int c = 0; c < YCOPIES; ++c) {
              unsigned long long* yp = a.yfx + ((size_t)b * YCOPIES + c) * D + n;
              ys += g0 == 0 ? yep[c] : *yp;
              *yp = 0ull;
            }
            if (a.add_y) t += yfx_to_f(ys);
          }
          *xp = t + v;
        } else if (OUT == 2) {
          a.st.h[(size_t)b * DFF + n] = gelu_tanh(v);
        } else {
          a.dst[(size_t)b * a.N + n] = v;
          if (OUT == 9) part[wave][r][bb] = v;
        }
      }
    }
  }
  if constexpr (OUT == 9) {
    // deferred select: this block's top1/top2 per row as one granule (plain store; the next
    // kernel boundary publishes it) and the pending flag
    __syncthreads();
    if (tid < a.B) {
      Best r{-INFINITY, -INFINITY, 0x7fffffff};
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
          const int n = (blockIdx.x * 4 + w) * RPW + rr;
          if (n < a.N) r = best_merge(r, Best{part[w][rr][tid], -INFINITY, n});
        }
      u64x2_t g;
      g.x = ((unsigned long long)(unsigned)r.i << 32) | __float_as_uint(r.v);
      g.y = (unsigned long long)__float_as_uint(r.v2);
      reinterpret_cast<u64x2_t*>(a.st.lmbest)[(size_t)blockIdx.x * 4 + tid] = g;
    }
    if (blockIdx.x == 0 && tid == 0) *a.st.selp = 1u;
  }
}

// GEMV / batched-GEMM epilogue store of output n of batch row b
template <int OUT>
__device__ __forceinline__ void gemv_store(const GemvArgs& a, int n, int b, float v) {
  if (OUT == 0) {
    if (n < D) {
      a.st.q[(size_t)b * D + n] = v;
    } else {
      const int c = (n - D) % D, which = (n - D) / D;
      const int head = c / HD, d = c - head * HD;
      const int4 ri = a.st.rowinfo[b];
      if (ri.x < 0) return;
      const size_t idx = kv_at(a.layer, a.st.kv_chunks, a.st.max_streams, ri.x, head, ri.y) + d;
      store_kv(a, which, idx, v);
    }
  } else if (OUT == 1) {
    float* xp = a.st.x + (size_t)b * D + n;
    float t = *xp;
    if (a.yacc && a.add_y)  // c_proj: fold the pending split-K partials of the previous mlp c_proj
#pragma unroll
      for (int c = 0; c < YCOPIES; ++c) t += a.yacc[((size_t)b * YCOPIES + c) * D + n];
    *xp = t + v;
  } else if (OUT == 2) {
    a.st.h[(size_t)b * DFF + n] = gelu_tanh(v);
  } else if (OUT == 6) {  // split-K partial of mlp c_proj (K slice blockIdx.y) -> pending copy
    a.yacc[((size_t)b * YCOPIES + blockIdx.y) * D + n] = v;
  } else {
    a.dst[(size_t)b * a.N + n] = v;
  }
}

__device__ __forceinline__ void wave_ln_regs(float4 (&v)[3], const float4 (&g)[3]) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    v[j].x -= mean; v[j].y -= mean; v[j].z -= mean; v[j].w -= mean;
    q += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) * (1.0f / D) + 1e-5f);
#pragma unroll
  for (int j = 0; j < 3; ++j)
    v[j] = make_float4(v[j].x * rstd * g[j].x, v[j].y * rstd * g[j].y, v[j].z * rstd * g[j].z, v[j].w * rstd * g[j].w);
}

// ---------------------------------------------------------------------------------
// c_proj for B = 1 with the split-KV merge in the prologue, one global round trip: every thread
// issues its partial loads (3 output elements x 16 splits) and one (m, l) pair of the 8 x 16
// (head, split) table BEFORE the weight rows; the per-head max / denominator are reduced over
// the 16 lanes of each head with shuffles, the coefficients go through LDS once.
// ---------------------------------------------------------------------------------
template <typename TW, int RPW, int NS>
__global__ __launch_bounds__(256) void ar_cproj_b1_kernel(GemvArgs a) {
  __shared__ float cf[N_HEAD * NSPLIT];
  __shared__ __attribute__((aligned(16))) float xs[D];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int4 ri = a.st.rowinfo[0];
  // (m, l) of (head = tid / 16, split = tid % 16) and the 48 partials of this thread's 3 elements
  float2 ml = make_float2(-INFINITY, 0.f);
  if (tid < N_HEAD * NSPLIT) ml = reinterpret_cast<const float2*>(a.st.part_ml)[tid];
  float pv[3][NS];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int e = tid + 256 * j, head = e / HD, d = e - head * HD;
    const float* po = a.st.part_o + ((size_t)head * NSPLIT) * HD + d;
#pragma unroll
    for (int i = 0; i < NS; ++i) pv[j][i] = po[(size_t)i * HD];
  }
  const int row0 = (blockIdx.x * 4 + wave) * RPW;
  // residual epilogue operands of lane r < RPW (row row0 + r): x and the fused MLP's accumulators
  float xep = 0.f;
  unsigned long long yep[YCOPIES];
  if (lane < RPW && row0 + lane < a.N) {
    xep = a.st.x[row0 + lane];
    if (a.yfx)
#pragma unroll
      for (int c = 0; c < YCOPIES; ++c) yep[c] = a.yfx[(size_t)c * D + row0 + lane];
  }
  const TW* __restrict__ W = reinterpret_cast<const TW*>(a.W);
  typename WReg<TW>::T wr[RPW][3];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int i = 0; i < 3; ++i)
      wr[r][i] = WReg<TW>::load(W + (size_t)min(row0 + r, a.N - 1) * D + i * 256 + lane * 4);  // clamped, unconditional
  if (tid < N_HEAD * NSPLIT) {
    const int t = ri.y + 1;
    const int ns = ri.x < 0 ? 0 : min(NS, (t + 63) / 64);
    const int sp = tid & (NSPLIT - 1);
    const bool on = sp < ns && ml.x != -INFINITY;
    float M = on ? ml.x : -INFINITY;
    M = row16_max(M);  // the NSPLIT == 16 splits of a head are one DPP row
    const float f = on ? expf(ml.x - M) : 0.f;
    float den = f * ml.y;
    den = row16_sum(den);
    cf[tid] = (ns > 0) ? f / den : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int e = tid + 256 * j, head = e / HD;
    float y = 0.f;
#pragma unroll
    for (int i = 0; i < NS; ++i) y += cf[head * NSPLIT + i] * pv[j][i];
    xs[e] = y;
  }
  __syncthreads();
  float acc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) acc[r] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 xv = *reinterpret_cast<const float4*>(xs + i * 256 + lane * 4);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const float4 w = WReg<TW>::f(wr[r][i]);
      acc[r] = dot4_fma(acc[r], w, xv);
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const float v = wave_sum(acc[r]);
    if (lane == r && row0 + r < a.N) {
      float t = xep;
      if (a.yfx) {
        unsigned long long ys = 0;
#pragma unroll
        for (int c = 0; c < YCOPIES; ++c) {
          ys += yep[c];
          a.yfx[(size_t)c * D + row0 + r] = 0ull;
        }
        if (a.add_y) t += yfx_to_f(ys);
      }
      a.st.x[row0 + r] = t + v;
    }
  }
}

// ---------------------------------------------------------------------------------
// Fused MLP for B <= 2 rows (bf16 weights; option "fuse_mlp"): block k owns h rows 16k..16k+15:
//   h = gelu_tanh(c_fc(LayerNorm(x) * ln_2))      (its 16 rows of c_fc, 24.6 KB of weights)
//   y += mlp.c_proj[:, 16k:16k+16] h               (its 16 columns of c_proj, thread-packed, 24.6 KB)
// The 768-wide partial is added into accumulator copy k % YCOPIES as 2^-32 fixed-point int64
// (no-return 64-bit integer atomics, yfx_of): integer sums are exact, so the result does not depend
// on the order the 192 blocks arrive in and a stream's tokens, margins and logits are reproducible
// run to run (round 3; fp32 atomics had varied at the 1e-7 level). The next c_attn / lm_head
// prologue reads x + the copies, the next c_proj folds them into x and clears them. This removes the
// c_fc -> c_proj kernel boundary (one of the per-layer seams, -6.7 us per step at B = 1); option
// fuse_mlp = 0 selects the two-kernel path (another summation order).
// ---------------------------------------------------------------------------------
template <int BG, int RB>
__global__ __launch_bounds__(256) void ar_mlp_fused_kernel(GemvArgs a, const bf16_t* __restrict__ Wfc,
                                                           const bf16_t* __restrict__ Wpk) {
  constexpr int RW = RB / 4;  // c_fc rows per wave
  __shared__ __attribute__((aligned(16))) float xs[BG][D];
  __shared__ float hs[BG][RB];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n0 = blockIdx.x * RB;
  // issue order: x rows (LayerNorm input), c_fc rows, packed c_proj columns
  float4 xv[3], gam[3];
  if (wave < BG) {
#pragma unroll
    for (int j = 0; j < 3; ++j) xv[j] = *reinterpret_cast<const float4*>(a.st.x + (size_t)wave * D + j * 256 + lane * 4);
#pragma unroll
    for (int j = 0; j < 3; ++j) gam[j] = *reinterpret_cast<const float4*>(a.ln_w + j * 256 + lane * 4);
  }
  uint2 wf[RW][3];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int i = 0; i < 3; ++i)
      wf[r][i] = *reinterpret_cast<const uint2*>(Wfc + (size_t)(n0 + wave * RW + r) * D + i * 256 + lane * 4);
  uint2 wp[RB / 4][3];  // column group g4 (4 columns), output third jj: 4 bf16 (pack_mproj layout)
#pragma unroll
  for (int g = 0; g < RB / 4; ++g)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
      wp[g][jj] = reinterpret_cast<const uint2*>(Wpk)[(((size_t)blockIdx.x * (RB / 4) + g) * 3 + jj) * 256 + tid];
  if (wave < BG) wave_ln_to_lds(xv, gam, xs[wave], lane);
  __syncthreads();
  float acc[RW][BG];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int bb = 0; bb < BG; ++bb) acc[r][bb] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int bb = 0; bb < BG; ++bb) {
      const float4 x4 = *reinterpret_cast<const float4*>(&xs[bb][i * 256 + lane * 4]);
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const float4 w = WReg<bf16_t>::f(wf[r][i]);
        acc[r][bb] = dot4_fma(acc[r][bb], w, x4);
      }
    }
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int bb = 0; bb < BG; ++bb) {
      const float v = wave_sum(acc[r][bb]);
      if (lane == 0) hs[bb][wave * RW + r] = gelu_tanh(v);
    }
  __syncthreads();
  // thread tid: outputs e = tid + 256 jj; pack g element jj * 16 + j = W[e][n0 + 16 g + j]
  unsigned long long* y = a.yfx + (size_t)(blockIdx.x % YCOPIES) * D;  // row bb's copies: y + bb * YCOPIES * D
#pragma unroll
  for (int bb = 0; bb < BG; ++bb) {
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < RB / 4; ++g) {
        const uint2 u = wp[g][jj];
        t = fmaf(__uint_as_float(u.x << 16), hs[bb][4 * g], t);
        t = fmaf(__uint_as_float(u.x & 0xffff0000u), hs[bb][4 * g + 1], t);
        t = fmaf(__uint_as_float(u.y << 16), hs[bb][4 * g + 2], t);
        t = fmaf(__uint_as_float(u.y & 0xffff0000u), hs[bb][4 * g + 3], t);
      }
      atomicAdd(y + (size_t)bb * YCOPIES * D + tid + 256 * jj, yfx_of(t, a.st.err));  // no-return int64 add
    }
  }
}

// Per-row control record of the step in flight: {slot, pos, text id, prev token}. Built once per
// lvx_ar_steps call (then advanced by the argmax kernel of every step), so the kernels of a step read
// one 16-byte record instead of chasing slots -> pos / prev / rowstep -> text_plan.
// text id -1 marks "past the end of the plan": reported by the step that would consume it.
__device__ __forceinline__ int4 make_rowinfo(const ArState& st, int b, int s, int p, int j, int prev) {
  if (s < 0) return make_int4(-1, 0, 0, 0);
  if (p >= st.max_pos) {
    atomicOr(st.err, 1);
    p = st.max_pos - 1;
  }
  return make_int4(s, p, plan_tok(st, b, j), min(max(prev, 0), VOCAB - 1));
}

__global__ void ar_rowinfo_init_kernel(ArState st, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int s = st.slots[b];
  const int j = st.rowstep ? st.rowstep[b] : 0;
  st.rowinfo[b] = s < 0 ? make_int4(-1, 0, 0, 0) : make_rowinfo(st, b, s, st.pos[s], j, st.prev[s]);
  st.rowx[b] = make_int2(j, plan_tok(st, b, j + 1));  // deferred select: step and next text id
  st.selrow[b] = 0u;
  if (b == 0) *st.selp = 0u;
}

// drop-in row mode: publish (slot, pos) for the kernels of the step
__global__ void ar_row_state_kernel(ArState st, int slot, int pos) {
  st.rowinfo[0] = make_int4(slot, pos, 0, 0);
  st.pos[slot] = pos;
}

// ---------------------------------------------------------------------------------
// split-KV decode attention (src/model.py:79-95 with T_q = 1, is_causal False, scale 1/sqrt(96)):
// grid (splits, 8 heads, B); a block owns a contiguous key range of its (stream, head). Partials
// (m, l, o) are merged in the c_proj prologue (B <= 2) or the merge kernel; with one split per
// (row, head) the block writes the normalised head output itself.
// ---------------------------------------------------------------------------------
constexpr int ATK = 64;  // keys per split granule

template <typename TKV> struct KvPiece;
template <> struct KvPiece<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void get(float* v) const {
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};
template <> struct KvPiece<bf16_t> {
  uint4 u;
  // (round 2: non-temporal KV loads, meant to keep the weights resident in the Infinity Cache while
  // the KV streams past, measured slower: B = 32 155.2 vs 140.5 us/step at t = 384-639, 297.6 vs
  // 255.9 at t = 2,048)
  __device__ __forceinline__ void load(const bf16_t* p) { u = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void get(float* v) const {
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
    v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
    v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
  }
};
template <> struct KvPiece<fp8_t> {
  uint2 u;
  __device__ __forceinline__ void load(const fp8_t* p) { u = *reinterpret_cast<const uint2*>(p); }
  __device__ __forceinline__ void get(float* v) const {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8(u.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8(u.x, true);
    const f2 c = __builtin_amdgcn_cvt_pk_f32_fp8(u.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8(u.y, true);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y; v[4] = c.x; v[5] = c.y; v[6] = d.x; v[7] = d.y;
  }
};

// (round 2, measured slower: keys stored in piece-major groups of 16 so that a 16-lane row reads
// one piece of 16 consecutive keys, 256 B contiguous per row and 8 lines per wave-instruction
// instead of 24: B = 32 10.83 vs 10.22 us at t = 512, 30.9 vs 29.95 at t = 2,048; every line of a
// wave's 3 KB key run is requested by its first load either way)
// No LDS in the key loop: a block walks its key range in 64-key
// tiles; lane quad (tid/4) owns one key per tile and lane tid%4 owns 24 of its 96 dims: the K and
// V pieces (48 B bf16 each) load straight to registers, the score needs two quad shuffles, and
// every wave keeps its own online-softmax state (m, l, o[24] per lane) so the loop has no
// barrier. The 4 wave states are merged once at the end through LDS.
// direct = 1 (batched path with one split per (row, head)): the normalised head output goes
// straight to the bf16 operand row xn, as the merge kernel would write it (o * (1 / l)), and the
// merge kernel is skipped.
// QKV (fp32 KV: the parity mode, 3 <= B <= 32): c_attn left its output as four K-slice partials
// (ar_qkv_ksplit_f32_kernel, st.qkvp); threads 0-287 sum them in K-slice order, q goes through LDS,
// and the split holding key t - 1 appends the new key's K / V to the cache and takes them from LDS in
// its last tile (its own store is not read back).
// Online softmax kept PER KEY SLOT (bf16 / fp8 KV; round 3): each lane quad owns one key slot of the
// tile (4 lanes x 24 dims) and keeps its own (m, l, o[24]) over the keys it sees, so a tile needs no
// wave-wide reduction (the wave-uniform form spent two DPP + readlane reductions and a 24-deep FMA
// chain per 64-key tile: the tile loop, not the KV stream, bounded the decode attention, ~0.65 us
// per tile whether the keys came from HBM or from LDS, in the round-3 persistent step's timeline). The score is
// four 6-term FMA chains summed pairwise. The slots are folded into the wave (max, rescale, DPP
// sums) once at the end. fp32 KV (the bit-exact parity mode) keeps the wave-uniform form.
__device__ __forceinline__ void slot_softmax_step(float& m, float& l, float (&o)[24], const float (&q)[24],
                                                  const float (&kf)[24], const float (&vf)[24], bool valid) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    s0 = fmaf(q[i], kf[i], s0);
    s1 = fmaf(q[6 + i], kf[6 + i], s1);
    s2 = fmaf(q[12 + i], kf[12 + i], s2);
    s3 = fmaf(q[18 + i], kf[18 + i], s3);
  }
  const float sc = quad_sum((s0 + s1) + (s2 + s3));  // every lane of the quad: the same bits
  if (!valid) return;
  const float mn = fmaxf(m, sc);
  const float alpha = expf(m - mn);  // m = -inf (first key of the slot): 0
  const float p = expf(sc - mn);
  l = l * alpha + p;
#pragma unroll
  for (int i = 0; i < 24; ++i) o[i] = fmaf(p, vf[i], o[i] * alpha);
  m = mn;
}
// bf16 KV: the same step on the raw bf16 pairs. The score is v_dot2_f32_bf16 of the key pairs with q
// split into bf16 hi + lo parts (q = hi + lo to ~2^-17: the products keep fp32-level accuracy) in
// four independent chains, and o is updated with packed fp32 math (v_pk_mul / v_pk_fma_f32): about
// half the VALU instructions per 64-key tile of the float form (no key conversions).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
struct QSplit {
  uint32_t hi[12], lo[12];  // bf16 pairs (dims 2j, 2j + 1)
};
__device__ __forceinline__ void qsplit_make(const float (&q)[24], QSplit& qs) {
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    const bf16_t h0 = f32_to_bf16(q[2 * j]), h1 = f32_to_bf16(q[2 * j + 1]);
    const bf16_t l0 = f32_to_bf16(q[2 * j] - bf16_to_f32(h0)), l1 = f32_to_bf16(q[2 * j + 1] - bf16_to_f32(h1));
    qs.hi[j] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    qs.lo[j] = (uint32_t)l0 | ((uint32_t)l1 << 16);
  }
}
__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
// the score of the lane quad's key (every lane of the quad: the same bits)
__device__ __forceinline__ float slot_score_bf16(const QSplit& qs, const uint4 (&kp)[3]) {
  uint32_t k[12];
#pragma unroll
  for (int i = 0; i < 3; ++i) { k[4 * i] = kp[i].x; k[4 * i + 1] = kp[i].y; k[4 * i + 2] = kp[i].z; k[4 * i + 3] = kp[i].w; }
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    s0 = dot2_bf16(qs.hi[j], k[j], s0);
    s1 = dot2_bf16(qs.hi[6 + j], k[6 + j], s1);
    s2 = dot2_bf16(qs.lo[j], k[j], s2);
    s3 = dot2_bf16(qs.lo[6 + j], k[6 + j], s3);
  }
  return quad_sum((s0 + s1) + (s2 + s3));
}
// the slot's online-softmax update with that score (split from the score so that a caller can
// compute the scores of two tiles before either update: independent chains, same bits)
__device__ __forceinline__ void slot_update_bf16(float& m, float& l, f32x2_t (&o)[12], float sc, const uint4 (&vp)[3],
                                                 bool valid) {
  uint32_t v[12];
#pragma unroll
  for (int i = 0; i < 3; ++i) { v[4 * i] = vp[i].x; v[4 * i + 1] = vp[i].y; v[4 * i + 2] = vp[i].z; v[4 * i + 3] = vp[i].w; }
  if (!valid) return;
  const float mn = fmaxf(m, sc);
  // 2^(x log2 e) on v_exp_f32 (arguments <= 0; m = -inf gives 0): ~1 ulp, two instructions instead
  // of expf's range-reduced sequence
  const float alpha = __builtin_amdgcn_exp2f((m - mn) * 1.4426950408889634f);
  const float p = __builtin_amdgcn_exp2f((sc - mn) * 1.4426950408889634f);
  l = l * alpha + p;
  const f32x2_t a2 = f32x2_t{alpha, alpha}, p2 = f32x2_t{p, p};
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    const f32x2_t vv = f32x2_t{__uint_as_float(v[j] << 16), __uint_as_float(v[j] & 0xffff0000u)};
    o[j] = __builtin_elementwise_fma(p2, vv, o[j] * a2);
  }
  m = mn;
}
__device__ __forceinline__ void slot_softmax_step_bf16(float& m, float& l, f32x2_t (&o)[12], const QSplit& qs,
                                                       const uint4 (&kp)[3], const uint4 (&vp)[3], bool valid) {
  slot_update_bf16(m, l, o, slot_score_bf16(qs, kp), vp, valid);
}

// fold the 16 slots of a wave: returns the wave's max; o / l rescaled to it (slots that saw no key: 0)
__device__ __forceinline__ float slot_fold_wave(float m, float& l, float (&o)[24]) {
  const float M = wave_max(m);
  const float f = (m == -INFINITY) ? 0.f : expf(m - M);
  l *= f;
#pragma unroll
  for (int i = 0; i < 24; ++i) o[i] *= f;
  return M;
}

// (round 4, measured slower: the per-key-slot form for fp32 KV too, B = 32 t = 384-639 214.1 vs
// 210.7 us/step; the fp32 parity mode keeps the wave-uniform form)
template <typename TKV, int DEPTH, int NW, bool QKV = false>
__global__ __launch_bounds__(NW * 64) void ar_attn_v2_kernel(ArState st, int layer, int ns_max, int direct,
                                                         int selcopy) {
  // NW waves: a tile is NW x 16 keys (4 lanes per key); NW = 8 doubles the bytes in flight per
  // block for long splits (batched steps)
  constexpr int TK = NW * 16;
  constexpr bool SLOT = sizeof(TKV) < 4;  // per-key-slot online softmax (bf16 / fp8 KV)
  static_assert(!QKV || (NW == 4 && sizeof(TKV) == 4), "the K-split c_attn: the fp32 parity mode's 4-wave blocks");
  constexpr int QH = QKV ? (3 * HD + NW * 64 - 1) / (NW * 64) : 1;  // q / k / v elements per thread (2 at 4 waves, 1 at 8)
  __shared__ float wm_s[NW], wl_s[NW];
  __shared__ float wo_s[NW][4][HD];  // [wave][16-lane row][part * 24 + i]
  __shared__ float qs_s[QKV ? HD : 1];
  __shared__ __attribute__((aligned(16))) TKV kvh_s[QKV ? 2 : 1][QKV ? HD : 1];  // QKV: the new key's K, V
  const int sp = blockIdx.x, head = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  TS_DECL;
  TS_MARK(0);
  // selcopy (layer 0 of a deferred-select step): the records c_attn just built are in the shadow
  // arrays; one block per row copies them back for the rest of the step and clears the flag
  // (the next text id, a dependent plan load, is looked up at the end of the block, when every
  // other load has landed)
  const int4 ri = selcopy ? st.rowinfo_n[b] : st.rowinfo[b];
  // QKV: thread tid owns elements e = tid and tid + 256 (tid < 32) of this head's (q, k, v) (element
  // e % 96 of q / k / v for e / 96 = 0 / 1 / 2); their four K-slice partials are issued with the
  // control record (clamped element: no load under a branch)
  float pq[QH][QKV ? 4 : 1];
  if constexpr (QKV) {
#pragma unroll
    for (int h = 0; h < QH; ++h) {
      const int e = min(tid + NW * 64 * h, 3 * HD - 1);
      const float* pp = st.qkvp + (size_t)b * (3 * D) + (e / HD) * D + head * HD + e % HD;
#pragma unroll
      for (int k = 0; k < 4; ++k) pq[h][k] = pp[(size_t)k * st.max_streams * (3 * D)];
    }
  }
  const bool cp = selcopy && sp == 0 && head == 0 && tid == 0;
  int jn = 0;
  if (cp) {
    jn = st.rowx_n[b].x;
    st.rowinfo[b] = ri;
    st.selrow[b] = 1u;  // (ar_q0_rows_kernel's pending select of the next step; unused by the granule forms)
    if (b == 0) *st.selp = 0u;
  }
  auto copy_tail = [&]() {
    if (cp) st.rowx[b] = make_int2(jn, plan_tok(st, b, jn + 1));
  };
  const int s = ri.x;
  if (s < 0) {
    copy_tail();
    // an idle row's fp32 operand is 0, as the merge would give it
    if (direct == 3 && sp == 0 && tid < HD) st.part_o[(size_t)(b * N_HEAD + head) * NSPLIT * HD + tid] = 0.f;
    return;
  }
  const int t = ri.y + 1;
  const int ns = min(ns_max, (t + ATK - 1) / ATK);
  if (sp >= ns) return;
  // SLOT (bf16 / fp8 KV): split ranges on whole 64-key tiles, so every tile is one KV chunk and a
  // lane's key address is the chunk base (wave-uniform) + a fixed lane offset (a trailing split
  // may be empty: it writes m = -inf, l = 0). fp32 KV keeps the unrounded ranges of the parity mode.
  const int chunk = SLOT ? (((t + ns - 1) / ns + ATK - 1) / ATK) * ATK : (t + ns - 1) / ns;
  const int k0 = sp * chunk, k1 = min(t, k0 + chunk);
  // key k of this (slot, head): chunk k / KV_CHUNK (cstride elements apart), row k % KV_CHUNK
  const size_t base = kv_at(layer, st.kv_chunks, st.max_streams, s, head, 0);
  const size_t cstride = (size_t)st.max_streams * N_HEAD * KV_CHUNK * HD;
  const TKV* __restrict__ Kg = reinterpret_cast<const TKV*>(st.kc) + base;
  const TKV* __restrict__ Vg = reinterpret_cast<const TKV*>(st.vc) + base;
  auto krow = [&](int k) { return (size_t)(k / KV_CHUNK) * cstride + (size_t)(k % KV_CHUNK) * HD; };
  const int part = tid & 3, kq = tid >> 2;  // key slot within the TK-key tile
  float q[24];
  if constexpr (!QKV) {
    const float* qg = st.q + (size_t)b * D + head * HD + part * 24;
#pragma unroll
    for (int i = 0; i < 24; i += 4) {
      const float4 v = *reinterpret_cast<const float4*>(qg + i);
      q[i] = v.x * 0.10206207261596575f; q[i + 1] = v.y * 0.10206207261596575f;
      q[i + 2] = v.z * 0.10206207261596575f; q[i + 3] = v.w * 0.10206207261596575f;
    }
  }
  float m = -INFINITY, l = 0.f, o[24];
#pragma unroll
  for (int i = 0; i < 24; ++i) o[i] = 0.f;
  // DEPTH tiles in flight: the register set of tile kb is refilled with tile kb + DEPTH * 64 right
  // after it is consumed, while the other sets are landing (DEPTH * 24 KB per block in flight: a
  // block streams at bytes-in-flight / latency, so the depth sets the per-CU rate). Loads are
  // unconditional (key clamped to the last valid one, invalid lanes masked after) so that no load
  // sits under a branch: the compiler's vmcnt for "this set has landed" then leaves the other sets
  // in flight instead of draining every outstanding load.
  KvPiece<TKV> kpr[DEPTH][3], vpr[DEPTH][3];
  const int klast = ((k1 - 1) / ATK) * ATK;  // SLOT: start of the last tile (a tile past it is clamped to it)
  auto issue = [&](int kb, KvPiece<TKV>(&kp)[3], KvPiece<TKV>(&vp)[3]) {
    if constexpr (SLOT) {  // keys past k1 in the last chunk: allocated rows, masked by `valid`
      // (a tile of NW * 16 keys spans NW / 4 chunks; chunks past the last one are clamped to it)
      const size_t off = (size_t)min((kb / KV_CHUNK) + (kq / KV_CHUNK), klast / KV_CHUNK) * cstride +
                         (size_t)(kq % KV_CHUNK) * HD + part * 24;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        kp[i].load(Kg + off + i * 8);
        vp[i].load(Vg + off + i * 8);
      }
      return;
    }
    const int key = min(kb + kq, k1 - 1);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      kp[i].load(Kg + krow(key) + part * 24 + i * 8);
      vp[i].load(Vg + krow(key) + part * 24 + i * 8);
    }
  };
  constexpr bool BF = SLOT && sizeof(TKV) == 2;  // bf16 pairs straight into v_dot2 / packed fp32 math
  f32x2_t o2[BF ? 12 : 1];
  if constexpr (BF) {
#pragma unroll
    for (int j = 0; j < 12; ++j) o2[j] = f32x2_t{0.f, 0.f};
  }
  QSplit qsp;
  auto tile = [&](int kb, const KvPiece<TKV>(&kp)[3], const KvPiece<TKV>(&vp)[3]) {
    const bool valid = kb + kq < k1;
    if constexpr (BF) {
      uint4 ku[3], vu[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) { ku[i] = reinterpret_cast<const uint4&>(kp[i]); vu[i] = reinterpret_cast<const uint4&>(vp[i]); }
      slot_softmax_step_bf16(m, l, o2, qsp, ku, vu, valid);
      return;
    }
    float kf[24], vf[24];
    if constexpr (QKV) {  // the tile holding key t - 1 (wave-uniform): that lane takes it from LDS
      KvPiece<TKV> kx[3], vx[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) { kx[i] = kp[i]; vx[i] = vp[i]; }
      if (kb + TK >= k1 && min(kb + kq, k1 - 1) == t - 1) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {  // 8 keys' worth of bytes from the LDS copy (fp8: uint2, bf16: uint4, fp32: 2 x float4)
          kx[i].load(kvh_s[0] + part * 24 + i * 8);
          vx[i].load(kvh_s[1] + part * 24 + i * 8);
        }
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) { kx[i].get(kf + 8 * i); vx[i].get(vf + 8 * i); }
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) { kp[i].get(kf + 8 * i); vp[i].get(vf + 8 * i); }
    }
    if constexpr (SLOT) {
      slot_softmax_step(m, l, o, q, kf, vf, valid);
      return;
    }
    float sc = 0.f;
#pragma unroll
    for (int i = 0; i < 24; ++i) sc = fmaf(q[i], kf[i], sc);
    sc = quad_sum(sc);
    if (!valid) sc = -INFINITY;
    const float mn = fmaxf(m, wave_max(sc));  // -inf while this wave has seen no key: alpha = p = 0
    if (DEPTH == 2 && mn == -INFINITY) return;  // (wave-uniform) skip the no-op update
    const float alpha = (m == -INFINITY) ? 0.f : expf(m - mn);
    const float p = valid ? expf(sc - mn) : 0.f;
    l = l * alpha + wave_sum(part == 0 ? p : 0.f);
#pragma unroll
    for (int i = 0; i < 24; ++i) o[i] = fmaf(valid ? p : 0.f, valid ? vf[i] : 0.f, o[i] * alpha);
    m = mn;
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) issue(k0 + d * TK, kpr[d], vpr[d]);
  if constexpr (QKV) {
    // the partials were issued before the tiles (vmcnt retires in issue order: this waits for them
    // alone); raw barrier after the LDS writes, the tiles stay in flight
#pragma unroll
    for (int h = 0; h < QH; ++h) {
      const int e = tid + NW * 64 * h;
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) v += pq[h][k];
      if (e < HD) {
        qs_s[e] = v;
      } else if (e < 3 * HD && k1 == t) {  // K / V of the new key (the last split): appended, kept in LDS
        const int which = e / HD - 1, d = e % HD;
        TKV hv;  // the value the one-launch c_attn stores (store_kv)
        if constexpr (sizeof(TKV) == 4) hv = v;
        else if constexpr (sizeof(TKV) == 2) hv = f32_to_bf16(v);
        else hv = f32_to_fp8(v);
        kvh_s[which][d] = hv;
        reinterpret_cast<TKV*>(which ? st.vc : st.kc)[base + krow(ri.y) + d] = hv;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 24; ++i) q[i] = qs_s[part * 24 + i] * 0.10206207261596575f;
  }
  if constexpr (BF) qsplit_make(q, qsp);
  // DEPTH 2 (few tiles per block, the B <= 2 step): leave after the last valid tile. DEPTH >= 4
  // (long splits, batched steps): whole groups of DEPTH tiles with no exit inside a group (a tile
  // past k1 is all-invalid: alpha = 1, p = 0), which keeps the compiler from draining every
  // outstanding load at the group boundary
  for (int kb = k0; kb < k1; kb += DEPTH * TK) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (DEPTH == 2 && d > 0 && kb + d * TK >= k1) break;
      tile(kb + d * TK, kpr[d], vpr[d]);
      issue(kb + (d + DEPTH) * TK, kpr[d], vpr[d]);
      if (DEPTH > 2) __builtin_amdgcn_sched_barrier(0);  // keep the refill right behind its tile
    }
  }
  if constexpr (BF) {
#pragma unroll
    for (int j = 0; j < 12; ++j) { o[2 * j] = o2[j].x; o[2 * j + 1] = o2[j].y; }
  }
  if constexpr (SLOT) {  // the slots' states folded into the wave's (m, l, o)
    m = slot_fold_wave(m, l, o);
    l = wave_sum(part == 0 ? l : 0.f);
  }
  // sum o over the 16 key slots of the wave (lanes with equal part): within each 16-lane row by
  // DPP (row_ror 8, 4), the four rows through LDS
#pragma unroll
  for (int i = 0; i < 24; ++i) {
    float v = o[i];
    v += dpp_f32<0x128>(v);
    v += dpp_f32<0x124>(v);
    o[i] = v;
  }
  if ((lane & 15) < 4) {
#pragma unroll
    for (int i = 0; i < 24; ++i) wo_s[wave][lane >> 4][(lane & 3) * 24 + i] = o[i];
  }
  TS_MARK(1);
  if (lane == 0) { wm_s[wave] = m; wl_s[wave] = l; }
  __syncthreads();
  TS_SAVE(2, layer, sp + gridDim.x * (head + N_HEAD * b));
  copy_tail();
  if (tid < HD) {
    float M = wm_s[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) M = fmaxf(M, wm_s[w]);
    float ov = 0.f, lv = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = (wm_s[w] == -INFINITY) ? 0.f : expf(wm_s[w] - M);
      ov += f * ((wo_s[w][0][tid] + wo_s[w][1][tid]) + (wo_s[w][2][tid] + wo_s[w][3][tid]));
      lv += f * wl_s[w];
    }
    if (direct == 3) {  // fp32 parity mode, one split: the normalised head output in split 0's slot
      st.part_o[(size_t)(b * N_HEAD + head) * NSPLIT * HD + tid] = ov * (1.0f / lv);
      return;
    }
    if (direct) {
      st.xn[direct == 2 ? xfrag(b, head * HD + tid, D) : (size_t)b * D + head * HD + tid] = f32_to_bf16(ov * (1.0f / lv));
      return;
    }
    st.part_o[((size_t)(b * N_HEAD + head) * NSPLIT + sp) * HD + tid] = ov;
    if (tid == 0) {
      float* ml = st.part_ml + ((size_t)(b * N_HEAD + head) * NSPLIT + sp) * 2;
      ml[0] = M;
      ml[1] = lv;
    }
  }
}

// ---------------------------------------------------------------------------------
// greedy select (streaming_server.py:342-347): argmax with first-index ties, top1-top2
// margin, then the slot's prev token / position / plan step advance.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ar_argmax_kernel(ArState st) {
  __shared__ float sv[4], sv2[4];
  __shared__ int si[4];
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int4 ri = st.rowinfo[b];
  const int s = ri.x;
  if (s < 0) return;
  const float4* lg = reinterpret_cast<const float4*>(st.logits + (size_t)b * VOCAB);
  Best bt{-INFINITY, -INFINITY, 0x7fffffff};
#pragma unroll
  for (int j = 0; j < VOCAB / 1024; ++j) {
    const float4 v = lg[j * 256 + tid];
    const int i0 = (j * 256 + tid) * 4;
    bt = best_merge(bt, Best{v.x, -INFINITY, i0});
    bt = best_merge(bt, Best{v.y, -INFINITY, i0 + 1});
    bt = best_merge(bt, Best{v.z, -INFINITY, i0 + 2});
    bt = best_merge(bt, Best{v.w, -INFINITY, i0 + 3});
  }
  bt = best_wave(bt);
  if (lane == 0) { sv[wave] = bt.v; sv2[wave] = bt.v2; si[wave] = bt.i; }
  __syncthreads();
  if (wave == 0) {
    Best r{sv[0], sv2[0], si[0]};
    for (int w = 1; w < 4; ++w) r = best_merge(r, Best{sv[w], sv2[w], si[w]});
    r = softmax_ties(st.logits + (size_t)b * VOCAB, r, lane);
    if (lane == 0) argmax_commit(st, b, ri, r);
  }
}

// ---------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------
// Kernel-variant switches kept for cross-checks (lvx_set_option): each selects between two correct
// implementations of the same step that tests/ compare (defaults are the measured-faster ones).
// option defer_select (default 1, Opts in lvx_internal.h): 1: greedy select deferred into the next
//   step's first kernel (B <= 2: c_attn layer 0 reduces lm_head's granules; B >= 4: ar_embed_select);
//   0: ar_argmax_kernel
// option fuse_mlp (default 1, Opts in lvx_internal.h): bf16, B <= 2: c_fc + gelu + mlp c_proj in one
//   kernel, its 192 blocks' c_proj partials added as 2^-32 fixed-point int64 (exact integer sums in any
//   arrival order: reproducible); 0: two GEMV kernels (another summation order)

template <typename TW, int K, int KW, int RPW, int IN, int OUT>
static void launch_gemv(const GemvArgs& a, hipStream_t s) {
  const int rows_per_block = (4 / KW) * RPW;
  dim3 grid((a.N + rows_per_block - 1) / rows_per_block);
  constexpr int BGMAX = (K == 768) ? 16 : 4;
  if constexpr (OUT == 9 || IN == 5) {  // select variants: one batch group of <= 4 rows (launch_op checks)
    if (a.B <= 1) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, 1, IN, OUT>), grid, dim3(256), 0, s, a);
    else if (a.B <= 2) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, 2, IN, OUT>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, 4, IN, OUT>), grid, dim3(256), 0, s, a);
  } else {
    if constexpr (IN == 2 && OUT == 1 && K == 768 && KW == 1) {
      if (a.B == 1) {  // B = 1 c_proj: the split merge once per block, 16 splits
        hipLaunchKernelGGL((ar_cproj_b1_kernel<TW, RPW, NSPLIT>), grid, dim3(256), 0, s, a);
        return;
      }
    }
    if (a.B <= 1) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, 1, IN, OUT>), grid, dim3(256), 0, s, a);
    else if (a.B <= 2) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, 2, IN, OUT>), grid, dim3(256), 0, s, a);
    else if (a.B <= 4 || BGMAX == 4) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, 4, IN, OUT>), grid, dim3(256), 0, s, a);
    else if (a.B <= 8) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, (BGMAX >= 8 ? 8 : 4), IN, OUT>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ar_gemv_kernel<TW, K, KW, RPW, BGMAX, IN, OUT>), grid, dim3(256), 0, s, a);
  }
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint2 pack4_bf16(float4 v) {
  return make_uint2((uint32_t)f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16),
                    (uint32_t)f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16));
}

#ifndef LVX_YCS
#define LVX_YCS 2
#endif
// pending copies of the mlp c_proj K slices at B <= ln_max, which every block of the next LayerNorm-
// prologue GEMM (c_attn, lm_head) folds for all B rows: 2 slices of 1,536 (96 blocks of 8 waves), so the
// prologues load 3 instead of 5 KB-rows per batch row (round 6, tools/ycs_ab.sh against 4 slices of 768,
// the LVX_YCS=4 build: B = 8 fp8 KV 94.8 / 95.1 -> 94.3 / 93.6 us per step, bf16 97.2 -> 96.7, B = 4
// 90.9 -> 90.5; configs[4] 82.0k -> 82.7k). B > ln_max keeps 4 slices (YCOPIES) for the rows kernel.
constexpr int YCS = LVX_YCS;
constexpr int MFMA_BATCH_MIN = 3;  // smallest B on the batched MFMA path (measured B = 3: 117 vs 154 us, B = 2: 119 vs 114)
// batched path: LayerNorm / embedding fused into the MFMA GEMM prologue for B <= this value
// (measured: B = 8 147 vs 156 us/step; B = 32 slower, every block re-normalising 32 rows)
// (runtime value: option "ln_max", for A/B of the two batched structures at small B)
// option ln_max (default 8, Opts in lvx_internal.h):
#define MFMA_LN_MAX (opts().ln_max)

// ---------------------------------------------------------------------------------
// Batched path v2 (bf16 weights, 4 < B <= 32): every per-row prologue runs ONCE per row into a
// bf16 operand buffer (LayerNorm / embedding+LayerNorm / split merge), then the weight GEMMs are
// pure MFMA GEMMs reading both operands from global: a block owns 16 weight rows and K is split
// over its waves (K/192 waves: 4 for K=768, 16 for K=3072); every lane issues all of its
// 16-byte fragment loads up front (one memory latency), partial tiles combine through LDS.
// ---------------------------------------------------------------------------------
// x row of the embedding (a2-a4) for control record ri, lane layout k = j * 256 + lane * 4:
// normalize(cat(text_table[id], codebook[prev] | 0 at position 0), eps 1e-8) + wpe[pos]
__device__ __forceinline__ void embed_row(const GemvArgs& a, int4 ri, int lane, float4 (&v)[3], float* rden = nullptr) {
  if (ri.x < 0) {
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int p = ri.y, prev = ri.w;
  const int tok = ri.z < 0 ? 384 : ri.z;
  // every load issued before any branch or use (the error flag's atomic and the position-0 zeros
  // came between them: one load went out a round trip late); prev is a valid codebook row
  float4 pe[3];
  const float* wr_ = a.wpe + (size_t)p * D;
#pragma unroll
  for (int j = 0; j < 3; ++j) pe[j] = *reinterpret_cast<const float4*>(wr_ + j * 256 + lane * 4);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int k = j * 256 + lane * 4;
    v[j] = j == 0 ? *reinterpret_cast<const float4*>(a.text_table + (size_t)tok * TEXT_DIM + k)
                  : *reinterpret_cast<const float4*>(a.codebook + (size_t)prev * SPEECH_DIM + (k - TEXT_DIM));
  }
  if (ri.z < 0 && lane == 0) atomicOr(a.st.err, 2);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (j > 0 && p == 0) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    ss += (v[j].x * v[j].x + v[j].y * v[j].y) + (v[j].z * v[j].z + v[j].w * v[j].w);
  }
  const float den = fmaxf(sqrtf(wave_sum(ss)), 1e-8f);
  if (rden) *rden = 1.0f / den;
#pragma unroll
  for (int j = 0; j < 3; ++j)
    v[j] = make_float4(v[j].x / den + pe[j].x, v[j].y / den + pe[j].y, v[j].z / den + pe[j].z, v[j].w / den + pe[j].w);
}


// 0: LayerNorm(x)  4: LayerNorm(x + pending copies)  3: embedding (+ stores x) then LayerNorm
// 5: as 4 with fp32 output rows in st.h ([B][768]; the batched fp32 parity mode's c_attn / lm_head
// operand, ar_qkv_ksplit_f32_kernel / ar_f32b_kernel IN 6: h is free between mlp c_proj and the next
// c_fc)  6: as 3 with the fp32 output rows of 5
template <int MODE>
__global__ __launch_bounds__(256) LVX_LOADS_FIRST void ar_rows_kernel(GemvArgs a) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int b = blockIdx.x * (blockDim.x >> 6) + wave;
  if (b >= a.B) return;
  TS_DECL;
  TS_MARK(0);
  float4 g[3], v[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) g[j] = *reinterpret_cast<const float4*>(a.ln_w + j * 256 + lane * 4);
  if (MODE == 0 || MODE == 4 || MODE == 5) {
    XRow<MODE == 5 ? 4 : MODE> r;
    xrow_issue(a, b, lane, r);
    __builtin_amdgcn_sched_barrier(0);  // gamma and the rows issued up front (the scheduler sank a
                                        // gamma load behind the variance: one more round trip)
    xrow_sum(r, v);
    if (MODE == 4 || MODE == 5)  // fold the pending copies into x here (one wave owns the row): the next c_proj
#pragma unroll      // then adds its output to a final x instead of re-reading the copies
      for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = v[j];
  } else {
    const int4 ri = a.st.rowinfo[b];
    embed_row(a, ri, lane, v);
#pragma unroll
    for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = v[j];
  }
  TS_MARK(1);
  wave_ln_regs(v, g);
  if constexpr (MODE == 5 || MODE == 6) {
#pragma unroll
    for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.h + (size_t)b * D + j * 256 + lane * 4) = v[j];
    return;
  }
  uint2* dst = reinterpret_cast<uint2*>(a.st.xn + (size_t)b * D);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (a.xpk) *reinterpret_cast<uint2*>(a.st.xn + xfrag(b, j * 256 + lane * 4, D)) = pack4_bf16(v[j]);
    else dst[j * 64 + lane] = pack4_bf16(v[j]);
  }
  TS_SAVE(a.N == VOCAB ? 8 : 0, a.layer, blockIdx.x);
}

// Batched deferred select (defer_sel 2): the previous step's greedy select of row b (the
// ar_argmax_kernel commit, streaming_server.py:342-347) and then the embedding + LayerNorm of the
// token it picked (ar_rows_kernel<3>). Four waves split the 4096 logits (one round trip with the
// row's control records), wave 0 commits and builds the operand row.
// F32OUT (the batched fp32 parity mode): the LayerNorm'd row in fp32 into st.h (ar_rows_kernel<6>'s
// output, read by ar_qkv_ksplit_f32_kernel)
// (With bf16 weights and option l0q the select runs in ar_q0_rows_kernel instead, which also computes
// layer 0's q / k / v from the q0 tables; round 6's first form of that, one block per row inside this
// kernel, took 1.1-1.7 us more per step and was removed.)
template <bool F32OUT = false>
__global__ __launch_bounds__(256) LVX_LOADS_FIRST void ar_embed_select_kernel(GemvArgs a) {
  __shared__ float sv[4], sv2[4];
  __shared__ int si[4];
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  TS_DECL;
  TS_MARK(0);
  int4 ri = a.st.rowinfo[b];
  const int2 rx = a.st.rowx[b];  // {plan step j, text id of step j + 1}
  const unsigned pend = a.st.selrow[b];
  float4 g[3];  // LN gamma first: the reduction's wait for the logits then covers it too
#pragma unroll
  for (int j = 0; j < 3; ++j) g[j] = *reinterpret_cast<const float4*>(a.ln_w + j * 256 + lane * 4);
  const float4* lg = reinterpret_cast<const float4*>(a.st.logits + (size_t)b * VOCAB);
  float4 lv[VOCAB / 1024];
#pragma unroll
  for (int k = 0; k < VOCAB / 1024; ++k) lv[k] = lg[k * 256 + tid];
  Best bt{-INFINITY, -INFINITY, 0x7fffffff};
#pragma unroll
  for (int k = 0; k < VOCAB / 1024; ++k) {
    const int i0 = (k * 256 + tid) * 4;
    bt = best_merge(bt, Best{lv[k].x, -INFINITY, i0});
    bt = best_merge(bt, Best{lv[k].y, -INFINITY, i0 + 1});
    bt = best_merge(bt, Best{lv[k].z, -INFINITY, i0 + 2});
    bt = best_merge(bt, Best{lv[k].w, -INFINITY, i0 + 3});
  }
  bt = best_wave(bt);
  TS_MARK(1);
  if (lane == 0) { sv[wave] = bt.v; sv2[wave] = bt.v2; si[wave] = bt.i; }
  __syncthreads();
  if (wave != 0) return;
  const bool take = pend && ri.x >= 0;
  if (take) {
    Best r{sv[0], sv2[0], si[0]};
#pragma unroll
    for (int w = 1; w < 4; ++w) r = best_merge(r, Best{sv[w], sv2[w], si[w]});
    r = softmax_ties(a.st.logits + (size_t)b * VOCAB, r, lane);
    const int s = ri.x, p = ri.y + 1, j = rx.x;
    const int4 rn = make_int4(s, min(p, a.st.max_pos - 1), rx.y, min(max(r.i, 0), VOCAB - 1));
    if (lane == 0) {  // argmax_commit
      if (p >= a.st.max_pos) atomicOr(a.st.err, 1);
      if (j < a.st.plan_stride) {
        a.st.tok_plan[(size_t)b * a.st.plan_stride + j] = r.i;
        if (a.st.margin_plan) a.st.margin_plan[(size_t)b * a.st.plan_stride + j] = r.v - r.v2;
      }
      a.st.prev[s] = r.i;
      a.st.pos[s] = p;
      a.st.rowstep[b] = j + 1;
      a.st.rowinfo[b] = rn;
    }
    ri = rn;
  }
  if (lane == 0) a.st.selrow[b] = 1u;  // this step's lm_head leaves the next pending select
  float4 v[3];
  embed_row(a, ri, lane, v);
#pragma unroll
  for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = v[j];
  wave_ln_regs(v, g);
  if constexpr (F32OUT) {
#pragma unroll
    for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.h + (size_t)b * D + j * 256 + lane * 4) = v[j];
  } else {
    uint2* dst = reinterpret_cast<uint2*>(a.st.xn + (size_t)b * D);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (a.xpk) *reinterpret_cast<uint2*>(a.st.xn + xfrag(b, j * 256 + lane * 4, D)) = pack4_bf16(v[j]);
      else dst[j * 64 + lane] = pack4_bf16(v[j]);
    }
  }
  // the plan load for the next text id last: waiting for it earlier held the embedding loads
  if (take && lane == 0) a.st.rowx[b] = make_int2(rx.x + 1, plan_tok(a.st, b, rx.x + 2));
  TS_SAVE(7, 0, b);
}

// B <= 2 GEMV steps with the deferred granule select (defer_sel 1) and option l0q (bf16): layer 0's
// c_attn from the q0 tables, as ar_embed_select_kernel<false, true> computes it, over 9 blocks of 256
// outputs instead of one block per row: every block reduces the rows' lm_head granules (as the GEMV's
// IN 5 prologue does; block 0 commits the select and leaves the new records in the shadow arrays that
// attention layer 0 copies back), loads its 256-column slices of Tt[t], Tp[p], G and Tc[c], and one
// wave per row builds the embedding row for (den, mean, rstd) (block 0 also stores x). Round 6: the
// single-block form cost the B = 1 step 6.6 us per launch (kernel trace) against 4.6-4.8 for its
// other kernels.
__global__ __launch_bounds__(256) LVX_LOADS_FIRST void ar_q0_gran_kernel(GemvArgs a) {
  constexpr int BM = 2;  // rows (the GEMV steps' B <= 2)
  __shared__ int4 rn_s[BM];
  __shared__ float4 sst[BM];  // {1 / den, mean, rstd} per row
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n = blockIdx.x * 256 + tid;  // this thread's output column (3 * D = 9 x 256)
  const int B = a.B;
  TS_DECL;
  TS_MARK(0);
  // every wave (row clamped: no load under a branch), as the IN 5 prologue: the record, the
  // {step, next text id}, the pending flag and the row's granules
  const int rb = min(wave, B - 1);
  const int4 ri = a.st.rowinfo[rb];
  const int2 rx = a.st.rowx[rb];
  const unsigned pend = *a.st.selp;
  LmGran lmg;
  lmg_issue(a.st, rb, lane, lmg);
  // this step's (text id, position) of every row as the commit sets them (they follow from the
  // records, not from the select): the Tt / Tp / G slices go out in the next round trip
  int4 rib[BM];
  int2 rxb[BM];
#pragma unroll
  for (int b = 0; b < BM; ++b) {
    rib[b] = a.st.rowinfo[min(b, B - 1)];
    rxb[b] = a.st.rowx[min(b, B - 1)];
  }
  float tq[BM], tpo[BM];
#pragma unroll
  for (int b = 0; b < BM; ++b) {
    const bool tk = pend && rib[b].x >= 0;
    const int p1 = min(max(tk ? rib[b].y + 1 : rib[b].y, 0), a.st.max_pos - 1);
    const int t1 = tk ? rxb[b].y : rib[b].z;
    tq[b] = a.q0_text[(size_t)(t1 < 0 ? 384 : t1) * (3 * D) + n];
    tpo[b] = a.q0_pos[(size_t)p1 * (3 * D) + n];
  }
  const float gq = a.q0_g[n];
  if (wave < B) {  // (wave-uniform) commit the previous step's greedy select of row `wave`
    const Best r = softmax_ties(a.st.logits + (size_t)wave * VOCAB, lmg_reduce(lmg), lane);
    const int sl = ri.x, j = rx.x, p = ri.y + 1;
    const bool take = pend && sl >= 0;
    const int4 rn = take ? make_int4(sl, min(p, a.st.max_pos - 1), rx.y, min(max(r.i, 0), VOCAB - 1)) : ri;
    if (blockIdx.x == 0 && lane == 0) {
      if (take) {
        if (p >= a.st.max_pos) atomicOr(a.st.err, 1);
        if (j < a.st.plan_stride) {
          a.st.tok_plan[(size_t)wave * a.st.plan_stride + j] = r.i;
          if (a.st.margin_plan) a.st.margin_plan[(size_t)wave * a.st.plan_stride + j] = r.v - r.v2;
        }
        a.st.prev[sl] = r.i;
        a.st.pos[sl] = p;
      }
      a.st.rowx_n[wave] = make_int2(take ? j + 1 : j, 0);
      a.st.rowinfo_n[wave] = rn;
    }
    if (lane == 0) rn_s[wave] = rn;
  }
  __syncthreads();
  // the codebook slice of each row's new token (every thread) beside the embedding rows (one wave per row)
  float tc[BM];
#pragma unroll
  for (int b = 0; b < BM; ++b) tc[b] = a.q0_code[(size_t)min(max(rn_s[min(b, B - 1)].w, 0), VOCAB - 1) * (3 * D) + n];
  if (wave < B) {
    const int4 rn = rn_s[wave];
    float4 v[3];
    float rden = 0.f;
    embed_row(a, rn, lane, v, &rden);
    if (blockIdx.x == 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)wave * D + j * 256 + lane * 4) = v[j];
    }
    float sm = 0.f;  // (mean, rstd) as wave_ln_regs computes them
#pragma unroll
    for (int j = 0; j < 3; ++j) sm += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    const float mean = wave_sum(sm) * (1.0f / D);
    float qs = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float4 d = make_float4(v[j].x - mean, v[j].y - mean, v[j].z - mean, v[j].w - mean);
      qs += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(qs) * (1.0f / D) + 1e-5f);
    if (lane == 0) sst[wave] = make_float4(rden, mean, rstd, 0.f);
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < BM; ++b) {
    if (b >= B) break;
    const int4 rn = rn_s[b];
    const float4 st = sst[b];
    const float cz = rn.y == 0 ? 0.f : 1.f;  // position 0: the codebook half of the input is zero
    const float o = rn.x < 0 ? 0.f : st.z * (((tq[b] + cz * tc[b]) * st.x + tpo[b]) - st.y * gq);
    if (n < D) {
      a.st.q[(size_t)b * D + n] = o;
    } else if (rn.x >= 0) {  // K / V append at the row's (slot, pos), as c_attn's epilogue
      const int c = (n - D) % D, which = (n - D) / D;
      const int head = c / HD, d = c - head * HD;
      store_kv(a, which, kv_at(0, a.st.kv_chunks, a.st.max_streams, rn.x, head, rn.y) + d, o);
    }
  }
  TS_SAVE(7, 0, blockIdx.x);
}

// Batched steps (4 <= B <= 32, bf16, option l0q; defer_sel 4): the previous step's greedy select and
// layer 0's c_attn from the q0 tables (as ar_embed_select_kernel<false, true> computes them) over a grid
// of 9 column slices x B rows: every block reduces its row's 4,096 logits (four waves, as
// ar_embed_select_kernel), loads 256-column slices of Tt[t], Tp[p], G and Tc[c] and builds the
// embedding row for (den, mean, rstd) with wave 0. The select is committed by the row's first block
// into the shadow records (rowinfo_n / rowx_n: the row's other blocks read rowinfo in this launch),
// which attention layer 0 copies back (it also sets the row's pending flag). Round 6: one block per row
// (ar_embed_select_kernel<false, true>) spent 4.7 us of the B = 32 step in this launch, its blocks
// each loading the 27 KB of table rows with the 16 KB of logits.
__global__ __launch_bounds__(256) LVX_LOADS_FIRST void ar_q0_rows_kernel(GemvArgs a) {
  __shared__ float sv[4], sv2[4];
  __shared__ int si[4];
  __shared__ float4 sst;  // {1 / den, mean, rstd}
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int cx = blockIdx.x, b = blockIdx.y;
  const int n = cx * 256 + tid;  // this thread's output column (3 * D = 9 x 256)
  TS_DECL;
  TS_MARK(0);
  const int4 ri = a.st.rowinfo[b];
  const int2 rx = a.st.rowx[b];
  const unsigned pend = a.st.selrow[b];
  const float4* lg = reinterpret_cast<const float4*>(a.st.logits + (size_t)b * VOCAB);
  float4 lv[VOCAB / 1024];
#pragma unroll
  for (int k = 0; k < VOCAB / 1024; ++k) lv[k] = lg[k * 256 + tid];
  const float gq = a.q0_g[n];
  // this step's (text id, position) as the commit sets them (from the records, not the select)
  const bool tk = pend && ri.x >= 0;
  const int p1 = min(max(tk ? ri.y + 1 : ri.y, 0), a.st.max_pos - 1);
  const int t1 = tk ? rx.y : ri.z;
  const float tq = a.q0_text[(size_t)(t1 < 0 ? 384 : t1) * (3 * D) + n];
  const float tpo = a.q0_pos[(size_t)p1 * (3 * D) + n];
  Best bt{-INFINITY, -INFINITY, 0x7fffffff};
#pragma unroll
  for (int k = 0; k < VOCAB / 1024; ++k) {
    const int i0 = (k * 256 + tid) * 4;
    bt = best_merge(bt, Best{lv[k].x, -INFINITY, i0});
    bt = best_merge(bt, Best{lv[k].y, -INFINITY, i0 + 1});
    bt = best_merge(bt, Best{lv[k].z, -INFINITY, i0 + 2});
    bt = best_merge(bt, Best{lv[k].w, -INFINITY, i0 + 3});
  }
  bt = best_wave(bt);
  if (lane == 0) { sv[wave] = bt.v; sv2[wave] = bt.v2; si[wave] = bt.i; }
  __syncthreads();
  int4 rn = ri;
  if (tk) {  // (block-uniform) every wave merges the four partials; the row's first block commits
    Best r{sv[0], sv2[0], si[0]};
#pragma unroll
    for (int w = 1; w < 4; ++w) r = best_merge(r, Best{sv[w], sv2[w], si[w]});
    r = softmax_ties(a.st.logits + (size_t)b * VOCAB, r, lane);
    const int sl = ri.x, p = ri.y + 1, j = rx.x;
    rn = make_int4(sl, min(p, a.st.max_pos - 1), rx.y, min(max(r.i, 0), VOCAB - 1));
    if (cx == 0 && tid == 0) {  // argmax_commit, with the records into the shadow arrays
      if (p >= a.st.max_pos) atomicOr(a.st.err, 1);
      if (j < a.st.plan_stride) {
        a.st.tok_plan[(size_t)b * a.st.plan_stride + j] = r.i;
        if (a.st.margin_plan) a.st.margin_plan[(size_t)b * a.st.plan_stride + j] = r.v - r.v2;
      }
      a.st.prev[sl] = r.i;
      a.st.pos[sl] = p;
      a.st.rowstep[b] = j + 1;
    }
  }
  if (cx == 0 && tid == 0) {
    a.st.rowinfo_n[b] = rn;
    a.st.rowx_n[b] = make_int2(tk ? rx.x + 1 : rx.x, 0);  // attention layer 0 looks up the next text id
  }
  const float tc = a.q0_code[(size_t)min(max(rn.w, 0), VOCAB - 1) * (3 * D) + n];
  if (wave == 0) {
    float4 v[3];
    float rden = 0.f;
    embed_row(a, rn, lane, v, &rden);
    if (cx == 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = v[j];
    }
    float sm = 0.f;  // (mean, rstd) as wave_ln_regs computes them
#pragma unroll
    for (int j = 0; j < 3; ++j) sm += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    const float mean = wave_sum(sm) * (1.0f / D);
    float qs = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float4 d = make_float4(v[j].x - mean, v[j].y - mean, v[j].z - mean, v[j].w - mean);
      qs += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(qs) * (1.0f / D) + 1e-5f);
    if (lane == 0) sst = make_float4(rden, mean, rstd, 0.f);
  }
  __syncthreads();
  const float4 st = sst;
  const float cz = rn.y == 0 ? 0.f : 1.f;  // position 0: the codebook half of the input is zero
  const float o = rn.x < 0 ? 0.f : st.z * (((tq + cz * tc) * st.x + tpo) - st.y * gq);
  if (n < D) {
    a.st.q[(size_t)b * D + n] = o;
  } else if (rn.x >= 0) {  // K / V append at the row's (slot, pos), as c_attn's epilogue
    const int c = (n - D) % D, which = (n - D) / D;
    const int head = c / HD, d = c - head * HD;
    store_kv(a, which, kv_at(0, a.st.kv_chunks, a.st.max_streams, rn.x, head, rn.y) + d, o);
  }
  TS_SAVE(7, 0, cx + 9 * b);
}

// split-KV merge for the batched path: y[b] (bf16) into st.xn. NS = ns_max (the attention's split
// count at this B): only the splits that can exist are loaded
template <int NS>
__global__ __launch_bounds__(256) void ar_merge_bf16_kernel(ArState st, int ns_max, int xpk) {
  __shared__ float cf[N_HEAD * NSPLIT];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int4 ri = st.rowinfo[b];
  // every load up front: one (m, l) pair per thread (8 heads x 16 splits) and 3 x 16 partials
  float2 ml = make_float2(-INFINITY, 0.f);
  if (tid < N_HEAD * NSPLIT) ml = reinterpret_cast<const float2*>(st.part_ml)[(size_t)b * N_HEAD * NSPLIT + tid];
  float pv[3][NS];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int e = tid + 256 * j, head = e / HD, d = e - head * HD;
    const float* po = st.part_o + ((size_t)(b * N_HEAD + head) * NSPLIT) * HD + d;
#pragma unroll
    for (int i = 0; i < NS; ++i) pv[j][i] = po[(size_t)i * HD];
  }
  if (tid < N_HEAD * NSPLIT) {
    const int ns = ri.x < 0 ? 0 : min(ns_max, (ri.y + 1 + 63) / 64);
    const bool on = (tid & (NSPLIT - 1)) < ns && ml.x != -INFINITY;
    float M = on ? ml.x : -INFINITY;
    M = row16_max(M);  // the NSPLIT == 16 splits of a head are one DPP row
    const float f = on ? expf(ml.x - M) : 0.f;
    float den = f * ml.y;
    den = row16_sum(den);
    cf[tid] = ns > 0 ? f / den : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int e = tid + 256 * j, head = e / HD;
    float y = 0.f;
#pragma unroll
    for (int i = 0; i < NS; ++i) y += cf[head * NSPLIT + i] * pv[j][i];
    st.xn[xpk ? xfrag(b, e, D) : (size_t)b * D + e] = f32_to_bf16(y);
  }
}

static void launch_merge_bf16(const ArState& st, int B, int nsm, hipStream_t s, int xpk = 0) {
  if (nsm <= 2) hipLaunchKernelGGL(ar_merge_bf16_kernel<2>, dim3(B), dim3(256), 0, s, st, nsm, xpk);
  else if (nsm <= 4) hipLaunchKernelGGL(ar_merge_bf16_kernel<4>, dim3(B), dim3(256), 0, s, st, nsm, xpk);
  else if (nsm <= 8) hipLaunchKernelGGL(ar_merge_bf16_kernel<8>, dim3(B), dim3(256), 0, s, st, nsm, xpk);
  else hipLaunchKernelGGL(ar_merge_bf16_kernel<NSPLIT>, dim3(B), dim3(256), 0, s, st, nsm, xpk);
}

// OUT as gemv_store, plus OUT 5: h (bf16) = gelu_tanh(v) for the batched mlp c_proj. A block
// covers K columns starting at blockIdx.y * K of rows of length KTOT (KTOT > K: split K, OUT 6).
// XM 1 (c_fc): LayerNorm applied after the GEMM. The operand is the bf16 copy of x * ln_2.weight
// the previous c_proj (OUT 7) left, multiplied as it is; the epilogue centres and scales:
// LN2(x) . W^T = rstd * ((x * g) . W^T - mean * G[n]), G = ArWeights::fc_gsum, with (mean, rstd)
// from the per-row statistics c_proj left in 48 column-block partials (mean, M2 over 16 columns
// each, combined here with Chan's formula while the operands load): no rows kernel and no
// per-element normalisation on the operand path (round 2: 4.1 -> ~2.7 us from entry to MFMA).
// OUT 7 (c_proj): x += v, plus that bf16 copy (x * ln_2.weight) and this block's (mean, M2) of its
// 16 columns.
template <int K, int NT, int OUT, int KTOT = K, int XM = 0>
__global__ __launch_bounds__(K / 192 * 64) void ar_mfma2_kernel(GemvArgs a) {
  constexpr int NW = K / 192;  // waves per block, each a 192-wide K slice (6 MFMA k-steps)
  __shared__ float red[NW][NT * 256];
  __shared__ float xo[OUT == 7 ? 16 * NT * 16 : 1];
  __shared__ float2 rs[XM == 1 ? NT * 16 : 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // XCD-aligned tile order (a.xmap, 1-D grid): workgroups are dealt to the 8 XCDs round robin, so
  // with this order XCD x runs only the tiles of K slice x mod 4 (mlp c_proj: its L2 fetches only
  // that part of the shared operand rows; the default order put every slice on every XCD: 8 copies
  // of all rows through the Infinity Fabric) or both batch tiles of its weight slices (c_proj: each
  // weight slice fetched once, the 49 KB of operand rows by every XCD)
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (a.xmap == 1) {
    const int x = bx & 7;
    by = x & 3;
    bx = (bx >> 3) * 2 + (x >> 2);
  } else if (a.xmap == 2) {
    // blocks b and b + 8 share an XCD: both batch tiles of weight slice (b / 16) * 8 + b % 8 run on
    // one XCD, so each 16-row weight slice crosses the fabric once (round 4; the round-3 order put
    // batch tile x & 1 on XCD x and fetched every slice into two XCDs' L2s: 2.04x the algorithmic
    // bytes)
    const int j = bx & 15;
    bz = j >> 3;
    bx = (bx >> 4) * 8 + (j & 7);
  }
  const int n0 = bx * 16;
  const int r0 = bz * (NT * 16);  // first batch row of this block's tile (grid.z batch tiles)
  const int B = a.B;
  TS_DECL;
  TS_MARK(0);
  const bf16_t* __restrict__ X = XM == 1 ? a.st.xb : ((KTOT == 768) ? a.st.xn : a.st.hb);
  const int k0 = by * K + wave * 192 + 8 * (lane >> 4);
  // epilogue operands first (a load in the epilogue is one more dependent round trip): thread tid
  // stores elements e = tid + k * NW * 64, all of batch row tid % (NT * 16) (NW * 64 is a multiple
  // of NT * 16): its control record (OUT 0, KV append) or its x values (OUT 7, residual)
  constexpr int EPT = (16 * NT * 16 + NW * 64 - 1) / (NW * 64);
  static_assert((NW * 64) % (NT * 16) == 0, "one batch row per thread in the epilogue");
  int4 ripre = make_int4(-1, 0, 0, 0);
  float xpre[(OUT == 7 || OUT == 1) ? EPT : 1];
  float gpre[(OUT == 7 || XM == 1) ? EPT : 1];  // OUT 7: ln_2.weight[n]; XM 1: G[n]
  if constexpr (OUT == 0) ripre = a.st.rowinfo[min(r0 + tid % (NT * 16), B - 1)];
  if constexpr (OUT == 1) {
    // (B <= 8 c_proj) x and the MLP's pending copies up front, summed in gemv_store<1>'s order
    // (x + c0 + c1 + c2 + c3, then + v): round 3, they were loaded in the epilogue, one more
    // dependent round trip after the MFMAs. The copies are loaded whether or not they are folded
    // (add_y: layers >= 1): no load under a branch.
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = min(tid + k * NW * 64, 16 * NT * 16 - 1), r = e / (NT * 16), b = min(r0 + e - r * (NT * 16), B - 1);
      const int n = min(n0 + r, a.N - 1);
      float t = a.st.x[(size_t)b * D + n];
      // (a.yacc is set on every MFMA step; a null one reads x itself, never folded)
      const float* yp = a.yacc ? a.yacc + (size_t)b * YCS * D + n : a.st.x + (size_t)b * D + n;
      const int ys = a.yacc ? D : 0;
      float yc[YCS];
#pragma unroll
      for (int c = 0; c < YCS; ++c) yc[c] = yp[c * ys];
      if (a.yacc && a.add_y)
#pragma unroll
        for (int c = 0; c < YCS; ++c) t += yc[c];
      xpre[k] = t;
    }
  }
  if constexpr (OUT == 7 || XM == 1) {
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = min(tid + k * NW * 64, 16 * NT * 16 - 1), r = e / (NT * 16), b = e - r * (NT * 16);
      const int n = min(n0 + r, a.N - 1);
      if constexpr (OUT == 7) xpre[k] = a.st.x[(size_t)min(r0 + b, B - 1) * D + n];
      gpre[k] = OUT == 7 ? a.ln_w[n] : a.gsum[n];
    }
  }
  // XM 1: the row statistics partials first (vmcnt retires in issue order, so the Chan combine
  // waits for them alone while the weights and operand rows stream), by every thread (clamped
  // row: no load under a branch), used by the first NT * 64
  float2 sp[XM == 1 ? 12 : 1];
  if constexpr (XM == 1) {
    const int rr = min(tid >> 2, NT * 16 - 1), q = tid & 3;
    const float2* xs = reinterpret_cast<const float2*>(a.st.xstat) + (size_t)min(r0 + rr, B - 1) * (D / 16) + q * 12;
#pragma unroll
    for (int j = 0; j < 12; ++j) sp[j] = xs[j];
    __builtin_amdgcn_sched_barrier(0);  // keep them ahead of the weight / operand loads
  }
  uint4 wf[6], xf[NT][6];
  // fragment-packed weights (a.Wf): the wave's 6 loads are 6 contiguous KB
  const bf16_t* wsrc = reinterpret_cast<const bf16_t*>(a.Wf) +
                       (((size_t)(n0 >> 4) * (KTOT / 32) + (by * K + wave * 192) / 32) * 64 + lane) * 8;
#pragma unroll
  for (int kk = 0; kk < 6; ++kk) wf[kk] = *reinterpret_cast<const uint4*>(wsrc + kk * 512);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int b = min(r0 + t * 16 + (lane & 15), B - 1);  // padded columns recompute row B-1, never stored
    // fragment-packed rows (a.xpk): the tile's 6 fragments are 6 contiguous KB (padded rows: whatever
    // the tile holds there, never stored)
    const bf16_t* xsrc = a.xpk ? X + ((((size_t)(r0 >> 4) + t) * (KTOT / 32) + (by * K + wave * 192) / 32) * 64 + lane) * 8
                               : X + (size_t)b * KTOT + k0;
    const int xstep = a.xpk ? 512 : 32;
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) xf[t][kk] = *reinterpret_cast<const uint4*>(xsrc + kk * xstep);
  }
  // every operand load in flight before the first MFMA (left to itself the scheduler interleaves
  // them with the MFMAs: ~7 KB in flight per wave instead of (6 + 6 NT) KB)
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (XM == 1) {  // (mean, rstd) per batch row into rs (read in the epilogue)
    if (tid < NT * 16 * 4) {  // 4 lanes per row, 12 column blocks each (loaded above)
      const int rr = tid >> 2, q = tid & 3;
      const float2 (&p)[12] = sp;
      float mean = 0.f, m2 = 0.f;  // Chan's combine of equal-count (16) groups, in a fixed order
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const float d = p[j].x - mean, w = 1.0f / (j + 1);
        mean = mean + d * w;
        m2 = m2 + p[j].y + d * d * (16.0f * j * w);
      }
#pragma unroll
      for (int o = 1; o < 4; o <<= 1) {  // pairs of equal counts n: M2 += (mb - ma)^2 n / 2
        // (whole waves: tid < NT * 64) partner lane xor o within the quad by DPP quad_perm
        const float mb = o == 1 ? dpp_f32<0xB1>(mean) : dpp_f32<0x4E>(mean);
        const float m2b = o == 1 ? dpp_f32<0xB1>(m2) : dpp_f32<0x4E>(m2);
        const float d = mb - mean;
        const float n = 192.0f * o;
        m2 = m2 + m2b + d * d * (n * 0.5f);
        mean = (mean + mb) * 0.5f;  // symmetric: both lanes of the pair hold the same result
      }
      if (q == 0) rs[rr] = make_float2(mean, 1.0f / sqrtf(m2 * (1.0f / D) + 1e-5f));
    }
  }
  f32x4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 6; ++kk)
#pragma unroll
    for (int t = 0; t < NT; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[kk]),
                                                       __builtin_bit_cast(bf16x8_t, xf[t][kk]), acc[t], 0, 0, 0);
  TS_MARK(1);
  // partial 16 x (NT*16) tiles -> LDS, element (row r, col c) at r * (NT*16) + c
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][(4 * (lane >> 4) + i) * (NT * 16) + t * 16 + (lane & 15)] = acc[t][i];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = tid + k * NW * 64;
    if (e >= 16 * NT * 16) break;
    const int r = e / (NT * 16), b = r0 + e - r * (NT * 16), n = n0 + r;
    if (b >= B || n >= a.N) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][e];
    if (OUT == 0 && n >= D) {  // K / V append at the row's (slot, pos), record prefetched
      const int c = (n - D) % D, which = (n - D) / D;
      const int head = c / HD, d = c - head * HD;
      if (ripre.x < 0) continue;
      const size_t idx = kv_at(a.layer, a.st.kv_chunks, a.st.max_streams, ripre.x, head, ripre.y) + d;
      store_kv(a, which, idx, v);
    } else if (OUT == 5) {
      if constexpr (XM == 1) {  // LayerNorm after the GEMM: rstd * (v - mean * G[n])
        const float2 st = rs[b - r0];
        v = (v - st.x * gpre[k]) * st.y;
      }
      a.st.hb[a.xpk ? xfrag(b, n, DFF) : (size_t)b * DFF + n] = f32_to_bf16(gelu_tanh(v));
    } else if (OUT == 7) {
      const float xn = xpre[k] + v;
      a.st.x[(size_t)b * D + n] = xn;
      a.st.xb[a.xpk ? xfrag(b, n, D) : (size_t)b * D + n] = f32_to_bf16(xn * gpre[k]);
      xo[e] = xn;
    } else if (OUT == 6) {  // split-K partial of mlp c_proj (K slice by) -> pending copy
      a.yacc[((size_t)b * (KTOT / K) + by) * D + n] = v;
    } else if (OUT == 1) {  // x (+ the folded copies, prefetched) + v
      a.st.x[(size_t)b * D + n] = xpre[k] + v;
    } else {
      gemv_store<OUT>(a, n, b, v);
    }
  }
  if constexpr (OUT == 7) {  // (mean, M2) of this block's 16 columns for every batch row
    __syncthreads();
    if (tid < NT * 16 && r0 + tid < B) {
      float mean = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) mean += xo[r * (NT * 16) + tid];
      mean *= 1.0f / 16;
      float m2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = xo[r * (NT * 16) + tid] - mean;
        m2 += d * d;
      }
      reinterpret_cast<float2*>(a.st.xstat)[(size_t)(r0 + tid) * (D / 16) + bx] = make_float2(mean, m2);
    }
  }
  TS_SAVE(OUT == 0 ? 1 : OUT == 7 ? 3 : OUT == 5 ? 4 : OUT == 6 ? 5 : 6, a.layer, blockIdx.x + gridDim.x * blockIdx.y);
}

// measured alternatives to the batched v2 layout (round 1/2, us/step at B = 32, t = 256-512), removed:
// 16-row batch tiles in grid.z (twice the blocks re-read the weights: 144.6 vs 142.2); LayerNorm of
// c_attn / lm_head from an unsplit mlp c_proj's row statistics (48 blocks of 16 waves: 178 vs 156);
// the split mlp c_proj combined in-launch by each column tile's last arriving slice (release /
// acquire fences: 182 vs 157; write-through slabs and sc1 loads, no fences: 171.9 vs 162-168)
template <int K, int OUT, int XM = 0>
static void launch_mfma2(const GemvArgs& a, hipStream_t s, bool btile = false) {
  dim3 grid((a.N + 15) / 16), block((K / 192) * 64);
  if (btile && a.B > 16) {  // 16-row batch tiles in grid.z: half the operand bytes per block
    grid.z = (a.B + 15) / 16;
    if (grid.z == 2 && grid.x % 8 == 0) {  // XCD-aligned order (xmap 2)
      GemvArgs b = a;
      b.xmap = 2;
      hipLaunchKernelGGL((ar_mfma2_kernel<K, 1, OUT, K, XM>), dim3(grid.x * 2), block, 0, s, b);
      return;
    }
    hipLaunchKernelGGL((ar_mfma2_kernel<K, 1, OUT, K, XM>), grid, block, 0, s, a);
  } else if (a.B <= 16) hipLaunchKernelGGL((ar_mfma2_kernel<K, 1, OUT, K, XM>), grid, block, 0, s, a);
  else if (a.B <= 32) hipLaunchKernelGGL((ar_mfma2_kernel<K, 2, OUT, K, XM>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((ar_mfma2_kernel<K, 4, OUT, K, XM>), grid, block, 0, s, a);
}

// (round 2-5: c_attn at 9 <= B <= 32 as four K-slice partials summed by the attention, the block's
// operand slice shared through LDS -- faster launched kernel by kernel on the null stream (B = 32
// 149.6 vs 154.3 us/step), slower under the HIP-graph replay every production path uses (B = 32
// t = 0 / 384 / 768: 103.8 / 130.5 / 160.6 vs 101.5 / 127.3 / 155.5 us/step); option "ksplit",
// off since round 3, removed in round 6 with its kernel. The fp32 parity mode keeps its K split:
// ar_qkv_ksplit_f32_kernel.)

// mlp c_proj (K = 3072) split into YCOPIES K slices of 768: 4x the blocks of the unsplit GEMM;
// each slice's partial goes to its pending copy (plain stores, deterministic), folded into x by
// the next c_proj and read as x + sum of copies by the next c_attn / lm_head prologue
template <int OUT>
static void launch_mproj_split(const GemvArgs& a, hipStream_t s) {
  static_assert(DFF == YCOPIES * 768, "one pending copy per K slice");
  dim3 grid((a.N + 15) / 16, YCOPIES), block(256);
  GemvArgs b = a;
  if (YCOPIES == 4 && grid.x % 2 == 0) {  // XCD-aligned order (xmap 1): 1-D grid
    b.xmap = 1;
    grid = dim3(grid.x * 4);
  }
  if (a.B <= 16) hipLaunchKernelGGL((ar_mfma2_kernel<768, 1, OUT, DFF>), grid, block, 0, s, b);
  else if (a.B <= 32) hipLaunchKernelGGL((ar_mfma2_kernel<768, 2, OUT, DFF>), grid, block, 0, s, b);
  else hipLaunchKernelGGL((ar_mfma2_kernel<768, 4, OUT, DFF>), grid, block, 0, s, b);
}

// Batched GEMM with the per-row prologue fused (K = 768; small B): every block builds the
// LayerNorm (MODE 0), LayerNorm of x + pending copies (MODE 4) or embedding + LayerNorm (MODE 3;
// block 0 also stores x) of all B rows into
// an LDS bf16 tile, then runs the MFMA 16 x (NT*16) tile of its 16 weight rows from it. The rows
// are recomputed by every block (B x 3 KB of x from L2) instead of paying a separate rows kernel
// and its launch boundary; the weight fragments are in flight while the rows are normalised.
// MODE 7 (c_attn layer 0 of the deferred select at 4 <= B <= 8, defer_sel 3): MODE 3 after committing
// the previous step's greedy select from lm_head's granules (block 0 writes the state and the shadow
// records, attention layer 0 copies them back, as the B <= 2 GEMV step's IN 5); every block builds the
// rows from the new records, which the KV append of the epilogue uses too. OUT 3 with defer_sel 3:
// the block's top-1 / top-2 per row as one granule, the pending flag set by block 0.
template <int NT, int OUT, int MODE>
__global__ __launch_bounds__(256) void ar_mfma_ln_kernel(GemvArgs a) {
  constexpr int K = 768, NW = 4, R = NT * 16, RW = R / NW;  // rows per wave
  constexpr int LDX = K + 8;                                 // bf16 row stride (16-B pad)
  static_assert(MODE != 7 || (NT == 1 && OUT == 0), "the deferred select's c_attn: B <= 8");
  constexpr int SR = MODE == 7 ? LM8_ROWS / NW : 1;          // rows per wave that can be live (B <= 8)
  __shared__ __attribute__((aligned(16))) bf16_t xs[R * LDX];
  __shared__ float red[NW][NT * 256];
  __shared__ float lgs[OUT == 3 && NT == 1 ? 16 * 17 : 1];
  __shared__ int4 ri_s[MODE == 7 ? LM8_ROWS : 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n0 = blockIdx.x * 16;
  const int B = a.B;
  // 1. row inputs (x rows or control records) first, then the weight fragments
  // (clamped rows, unconditional loads: a load under a branch drains everything in flight; the
  // pending copies of the first YR rows come with them, the rest are loaded in step 2)
  constexpr int YR = MODE == 4 ? (RW < 2 ? RW : 2) : 0;
  float4 xv[RW][3], ya[YR > 0 ? YR : 1][YCS][3];
  int4 ri[RW];
  // MODE 7: the select's inputs with the control records (clamped rows, unconditional loads)
  LmGran8 lmg[SR];
  int2 rxp[SR];
  unsigned selpend = 0u;
  if constexpr (MODE == 7) {
    selpend = *a.st.selp;
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      const int b = min(wave + NW * i, B - 1);
      rxp[i] = a.st.rowx[b];
      lmg8_issue(a.st, b, lane, lmg[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int b = min(wave + NW * i, B - 1);
    if (MODE == 0 || MODE == 4) {
#pragma unroll
      for (int j = 0; j < 3; ++j) xv[i][j] = *reinterpret_cast<const float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4);
    } else if (MODE != 7 || i < SR) {
      ri[i] = a.st.rowinfo[b];
    }
    if (i < YR)
#pragma unroll
      for (int c = 0; c < YCS; ++c)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          ya[i < YR ? i : 0][c][j] = *reinterpret_cast<const float4*>(a.yacc + ((size_t)b * YCS + c) * D + j * 256 + lane * 4);
  }
  const int k0 = wave * 192 + 8 * (lane >> 4);
  float4 g[3];  // gamma ahead of the weights (the first LayerNorm waits for it)
#pragma unroll
  for (int j = 0; j < 3; ++j) g[j] = *reinterpret_cast<const float4*>(a.ln_w + j * 256 + lane * 4);
  __builtin_amdgcn_sched_barrier(0);  // (the scheduler otherwise moves them behind the weights)
  uint4 wf[6];
#pragma unroll
  for (int kk = 0; kk < 6; ++kk)  // fragment-packed weights (a.Wf): 6 contiguous KB per wave
    wf[kk] = *reinterpret_cast<const uint4*>(
        reinterpret_cast<const bf16_t*>(a.Wf) + (((size_t)(n0 >> 4) * (K / 32) + wave * 6 + kk) * 64 + lane) * 8);
  if constexpr (MODE == 7) {
    // commit the previous step's select (ar_embed_select_kernel's argmax_commit, B <= 2 IN 5's shadow
    // records); reduction and record select unconditional so that the granule loads stay up front
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      const int b = wave + NW * i, bc = min(b, B - 1);
      const Best r = softmax_ties(a.st.logits + (size_t)bc * VOCAB, lmg8_reduce(lmg[i]), lane);
      const int4 r0 = ri[i];
      const int s = r0.x, j = rxp[i].x, p = r0.y + 1;
      const bool take = selpend && s >= 0;
      const int4 rn = take ? make_int4(s, min(p, a.st.max_pos - 1), rxp[i].y, min(max(r.i, 0), VOCAB - 1)) : r0;
      if (b < B && blockIdx.x == 0 && lane == 0) {
        if (take) {
          if (p >= a.st.max_pos) atomicOr(a.st.err, 1);
          if (j < a.st.plan_stride) {
            a.st.tok_plan[(size_t)b * a.st.plan_stride + j] = r.i;
            if (a.st.margin_plan) a.st.margin_plan[(size_t)b * a.st.plan_stride + j] = r.v - r.v2;
          }
          a.st.prev[s] = r.i;
          a.st.pos[s] = p;
          a.st.rowstep[b] = j + 1;
        }
        a.st.rowx_n[b] = make_int2(take ? j + 1 : j, 0);  // attention layer 0 looks up the next text id
        a.st.rowinfo_n[b] = rn;
      }
      ri[i] = rn;
      if (b < LM8_ROWS && lane == 0) ri_s[b] = rn;
    }
  }
  // 2. rows -> LayerNorm -> bf16 tile (rows >= B are zero: padded columns, never stored)
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int b = wave + NW * i;
    uint2* dst = reinterpret_cast<uint2*>(xs + b * LDX);
    if (b < B && (MODE != 7 || i < SR)) {
      if (MODE == 3 || MODE == 7) {
        embed_row(a, ri[i], lane, xv[i]);
        if (blockIdx.x == 0)
#pragma unroll
          for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = xv[i][j];
      } else if (MODE == 4) {  // + the pending split-K copies of the previous mlp c_proj
#pragma unroll
        for (int c = 0; c < YCS; ++c)
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const float4 y = i < YR ? ya[i < YR ? i : 0][c][j]
                                    : *reinterpret_cast<const float4*>(a.yacc + ((size_t)b * YCS + c) * D + j * 256 + lane * 4);
            xv[i][j].x += y.x; xv[i][j].y += y.y; xv[i][j].z += y.z; xv[i][j].w += y.w;
          }
      }
      wave_ln_regs(xv[i], g);
#pragma unroll
      for (int j = 0; j < 3; ++j) dst[j * 64 + lane] = pack4_bf16(xv[i][j]);
    } else {
#pragma unroll
      for (int j = 0; j < 3; ++j) dst[j * 64 + lane] = make_uint2(0u, 0u);
    }
  }
  __syncthreads();
  // 3. MFMA 16x16x32: A = weight rows (lane & 15), B = tile rows (lane & 15) of column block t
  f32x4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 6; ++kk)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const uint4 xf = *reinterpret_cast<const uint4*>(xs + (t * 16 + (lane & 15)) * LDX + k0 + kk * 32);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[kk]),
                                                       __builtin_bit_cast(bf16x8_t, xf), acc[t], 0, 0, 0);
    }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][(4 * (lane >> 4) + i) * (NT * 16) + t * 16 + (lane & 15)] = acc[t][i];
  __syncthreads();
  for (int e = tid; e < 16 * NT * 16; e += NW * 64) {
    const int r = e / (NT * 16), b = e - r * (NT * 16), n = n0 + r;
    if (b >= B || n >= a.N) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][e];
    if constexpr (OUT == 3 && NT == 1) lgs[r * 17 + b] = v;
    if constexpr (MODE == 7) {  // c_attn's store with this step's new record (gemv_store<0> reads rowinfo)
      if (n < D) {
        a.st.q[(size_t)b * D + n] = v;
      } else {
        const int c = (n - D) % D, which = (n - D) / D;
        const int head = c / HD, d = c - head * HD;
        const int4 rr = ri_s[b];
        if (rr.x >= 0) store_kv(a, which, kv_at(a.layer, a.st.kv_chunks, a.st.max_streams, rr.x, head, rr.y) + d, v);
      }
    } else if (OUT == 5) {
      a.st.hb[(size_t)b * DFF + n] = f32_to_bf16(gelu_tanh(v));
    } else {
      gemv_store<OUT>(a, n, b, v);
    }
  }
  if constexpr (OUT == 3 && NT == 1) {
    if (a.defer_sel == 3) {  // (kernel argument: uniform) this block's granule per row, pending flag
      // raw barrier after the LDS writes: __syncthreads() would also wait for the logits stores
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (tid < B) {
        Best r{-INFINITY, -INFINITY, 0x7fffffff};
#pragma unroll
        for (int rr = 0; rr < 16; ++rr)
          if (n0 + rr < a.N) r = best_merge(r, Best{lgs[rr * 17 + tid], -INFINITY, n0 + rr});
        reinterpret_cast<u64x2_t*>(a.st.lmbest)[(size_t)blockIdx.x * LM8_ROWS + tid] = lm_granule(r);
      }
      if (blockIdx.x == 0 && tid == 0) *a.st.selp = 1u;
    }
  }
}

template <int OUT, int MODE>
static void launch_mfma_ln(const GemvArgs& a, hipStream_t s) {
  dim3 grid((a.N + 15) / 16), block(256);
  if constexpr (MODE == 7) {  // (B <= 8 by defer_select_ln)
    hipLaunchKernelGGL((ar_mfma_ln_kernel<1, OUT, MODE>), grid, block, 0, s, a);
  } else {
    if (a.B <= 16) hipLaunchKernelGGL((ar_mfma_ln_kernel<1, OUT, MODE>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((ar_mfma_ln_kernel<2, OUT, MODE>), grid, block, 0, s, a);
  }
}

// ---------------------------------------------------------------------------------
// Batched path v3 (bf16 weights, MFMA_BATCH_MIN <= B <= 64; option "bt"): five kernels per
// layer and no pending partials, so every x row is final at each kernel boundary:
//   c_attn       LN1(x) prologue (layer 0: embedding, which also stores x), q / KV-append epilogue
//   attention    split-KV ar_attn_v2
//   c_proj       split-KV merge prologue, x += epilogue
//   c_fc         LN2(x) prologue, gelu -> hb (bf16) epilogue
//   mlp c_proj   hb operand straight from global, x += epilogue
// A block owns 16 weight rows (blockIdx.x) x R = NT*16 batch rows (blockIdx.y). K is split over
// its waves (192 columns = 6 MFMA k-steps each). The weight fragments are issued first (they do not
// depend on the step), then the per-row prologue builds the bf16 operand tile in LDS; the waves'
// partial 16 x R tiles are summed through LDS in fixed order (deterministic, equal rows bit-equal).
// ---------------------------------------------------------------------------------
template <int K, int NT, int IN, int OUT>
__global__ __launch_bounds__(K / 192 * 64) void ar_bt_kernel(GemvArgs a) {
  constexpr int NW = K / 192, R = NT * 16, NTH = NW * 64;
  constexpr bool STAGE = IN != 1;  // operand tile staged in LDS (K == 768)
  static_assert(!STAGE || K == 768, "the LDS operand tile holds K = 768 rows");
  constexpr int LDX = D + 8;  // bf16 row stride of the tile (16-B pad)
  __shared__ __attribute__((aligned(16))) bf16_t xs[STAGE ? R * LDX : 8];
  __shared__ float red[NW][16 * R];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n0 = blockIdx.x * 16, r0 = blockIdx.y * R;
  const int B = a.B;
  const bf16_t* __restrict__ W = reinterpret_cast<const bf16_t*>(a.W);
  const bf16_t* __restrict__ X = K == D ? a.st.xn : a.st.hb;  // IN 1 operand rows
  const int wrow = min(n0 + (lane & 15), a.N - 1);
  const int k0 = wave * 192 + 8 * (lane >> 4);
  uint4 wf[6];
  if constexpr (IN == 0 || IN == 3) {
    constexpr int RPW = R / NW;  // rows per wave, normalised 4 at a time
    float4 g[3];
#pragma unroll
    for (int gi = 0; gi < RPW; gi += 4) {
      float4 xv[4][3];
      int4 ri[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // clamped row, unconditional loads (rows past B are not stored)
        const int b = min(r0 + wave * RPW + gi + i, B - 1);
        if (IN == 0) {
#pragma unroll
          for (int j = 0; j < 3; ++j) xv[i][j] = *reinterpret_cast<const float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4);
        } else {
          ri[i] = a.st.rowinfo[b];
        }
      }
      if (gi == 0) {  // gamma, then the weights, behind the first row group's inputs (vmcnt retires in issue order)
#pragma unroll
        for (int j = 0; j < 3; ++j) g[j] = *reinterpret_cast<const float4*>(a.ln_w + j * 256 + lane * 4);
        __builtin_amdgcn_sched_barrier(0);  // (the scheduler otherwise moves them behind the weights)
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) wf[kk] = *reinterpret_cast<const uint4*>(W + (size_t)wrow * K + k0 + kk * 32);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = wave * RPW + gi + i, b = r0 + rr;
        uint2* dst = reinterpret_cast<uint2*>(xs + rr * LDX);
        if (b < B) {
          if (IN == 3) {
            embed_row(a, ri[i], lane, xv[i]);
            if (blockIdx.x == 0)
#pragma unroll
              for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = xv[i][j];
          }
          wave_ln_regs(xv[i], g);
#pragma unroll
          for (int j = 0; j < 3; ++j) dst[j * 64 + lane] = pack4_bf16(xv[i][j]);
        } else {
#pragma unroll
          for (int j = 0; j < 3; ++j) dst[j * 64 + lane] = make_uint2(0u, 0u);
        }
      }
    }
  } else {  // IN 1: bf16 operand rows (hb, or xn of the separate merge kernel) straight from global
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) wf[kk] = *reinterpret_cast<const uint4*>(W + (size_t)wrow * K + k0 + kk * 32);
  }
  if constexpr (STAGE) __syncthreads();
  f32x4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    uint4 xf[6];
    if constexpr (STAGE) {
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) xf[kk] = *reinterpret_cast<const uint4*>(xs + (t * 16 + (lane & 15)) * LDX + k0 + kk * 32);
    } else {
      const int b = min(r0 + t * 16 + (lane & 15), B - 1);  // padded columns recompute row B-1, never stored
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) xf[kk] = *reinterpret_cast<const uint4*>(X + (size_t)b * K + k0 + kk * 32);
    }
#pragma unroll
    for (int kk = 0; kk < 6; ++kk)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[kk]),
                                                       __builtin_bit_cast(bf16x8_t, xf[kk]), acc[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][(4 * (lane >> 4) + i) * R + t * 16 + (lane & 15)] = acc[t][i];
  __syncthreads();
  for (int e = tid; e < 16 * R; e += NTH) {
    const int r = e / R, c = e - r * R, n = n0 + r, b = r0 + c;
    if (b >= B || n >= a.N) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][e];
    if (OUT == 5) a.st.hb[(size_t)b * DFF + n] = f32_to_bf16(gelu_tanh(v));
    else if (OUT == 1) a.st.x[(size_t)b * D + n] += v;
    else gemv_store<OUT>(a, n, b, v);
  }
}

// ---------------------------------------------------------------------------------
// Batched fp32 parity mode (fp32 weights, 3 <= B <= 64; option "f32b"): the same five ops per layer
// as v3, on exact-fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 products and fp32 accumulation, no
// reduced-precision operands). A block owns 16 weight rows (blockIdx.x) x R = NT * 16 batch rows
// (blockIdx.y); K is split over its waves (192 columns = 48 MFMA k-steps each). Weights come from
// an MFMA-fragment-packed fp32 copy ([N / 16][K / 16][64 lanes][4]: one wave-wide 16-B load = one
// contiguous KB): lane l holds W[n0 + l % 16][16 j + 4 (l / 16) .. + 3], and MFMA k-step 4 j + e
// multiplies element e, so the operand row supplies the same k from its float4 at 16 j + 4 (l / 16).
// The per-row prologue (LayerNorm, layer 0's embedding, the split-KV merge) builds an fp32 operand
// tile in LDS once per block; mlp c_proj (K = 3072) reads the fp32 h rows from global. Wave partials
// are summed through LDS in wave order: deterministic, and a row's result never depends on its batch
// position (an MFMA column's dot product uses only that column's data).
// ---------------------------------------------------------------------------------
// KTOT > K (mlp c_proj, OUT 6): the K = 3072 reduction split over blockIdx.z into KTOT / K slices of
// 768, each slice's partial stored to its pending copy (st.yacc), folded into x by the rows kernel
// (ar_rows_kernel<5>) that normalises c_attn's / lm_head's operand rows (IN 6): 4x the blocks, a
// quarter of the bytes per block.
// CT column tiles per block (CT x K / 192 waves sharing the block's operand tile): CT = 2 halves the
// blocks of the wide ops (c_fc, lm_head, the mlp c_proj slices) so that 192-256 blocks cover the CUs
// once instead of 384-512 blocks loading two tiles' bytes on some CUs. Same bits either way.
template <int K, int NT, int IN, int OUT, int KTOT = K, int CT = 1>
__global__ __launch_bounds__(K / 192 * 64 * CT) void ar_f32b_kernel(GemvArgs a) {
  constexpr int NWK = K / 192, NW = NWK * CT, R = NT * 16, NTH = NW * 64;
  constexpr bool STAGE = IN != 1 || CT > 1;  // K == 768: the operand tile in LDS (shared by the column tiles)
  static_assert(KTOT == K || (IN == 1 && OUT == 6 && KTOT == YCOPIES * K), "split K: mlp c_proj into the pending copies");
  // IN 4 (c_proj after a one-split attention, direct == 3): the normalised rows are split 0 of part_o
  // IN 6 (c_attn / lm_head after ar_rows_kernel<5>): the LayerNorm'd fp32 rows in st.h
  static_assert(!STAGE || K == 768, "the LDS operand tile holds K = 768 rows");
  constexpr int LDX = D + 4;  // fp32 row stride: 16 rows x 4 banks apart, conflict-free 16-B reads
  __shared__ __attribute__((aligned(16))) float xs[STAGE ? R * LDX : 4];
  __shared__ float red[NW][16 * R];
  __shared__ float cf_s[IN == 2 ? R * N_HEAD * NSPLIT : 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int kw = wave % NWK;  // the wave's 192-wide K slice; wave / NWK its column tile
  const int nb = blockIdx.x * CT * 16, r0 = blockIdx.y * R, ks = KTOT > K ? blockIdx.z : 0;
  const int n0 = min(nb + (wave / NWK) * 16, a.N - 16);  // (a tile past N: the last one's weights, never stored)
  const int B = a.B;
  // weights (fragment-packed, the wave's 12 contiguous KB), issued first for IN 1 / IN 2; behind the
  // first row inputs for the LayerNorm modes (their statistics then overlap the weight stream)
  const float4* wsrc = reinterpret_cast<const float4*>(a.Wf) + ((size_t)(n0 >> 4) * (KTOT / 16) + ks * (K / 16) + kw * 12) * 64 + lane;
  float4 wf[12];
  if constexpr (IN == 1 || IN == 2 || IN == 4 || IN == 6) {
#pragma unroll
    for (int j = 0; j < 12; ++j) wf[j] = wsrc[j * 64];
    // all 12 in flight before anything else (left to itself the scheduler interleaved each load with
    // the MFMA that uses it: one memory latency per k group)
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (IN == 0 || IN == 3) {
    constexpr int RPW = R / NW;  // rows per wave (4 or 8), all inputs in flight at once
    float4 xv[RPW][3];
    int4 ri[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int b = min(r0 + wave * RPW + i, B - 1);  // clamped: no load under a branch
      if (IN == 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) xv[i][j] = *reinterpret_cast<const float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4);
      } else {
        ri[i] = a.st.rowinfo[b];
      }
    }
    float4 g[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) g[j] = *reinterpret_cast<const float4*>(a.ln_w + j * 256 + lane * 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 12; ++j) wf[j] = wsrc[j * 64];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int rr = wave * RPW + i, b = r0 + rr;
      float* dst = xs + rr * LDX;
      if (b < B) {
        if (IN == 3) {
          embed_row(a, ri[i], lane, xv[i]);
          if (blockIdx.x == 0)
#pragma unroll
            for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(a.st.x + (size_t)b * D + j * 256 + lane * 4) = xv[i][j];
        }
        wave_ln_regs(xv[i], g);
#pragma unroll
        for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(dst + j * 256 + lane * 4) = xv[i][j];
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) *reinterpret_cast<float4*>(dst + j * 256 + lane * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  } else if constexpr (IN == 2) {
    // split-KV merge (as gemv_stage_input IN 2): coefficients per (row, head, split), then every
    // element sums the partials of the nsm splits the attention ran at this B (attn_ns_max). The
    // splits past nsm have coefficient 0 (part_o is zeroed at allocation, finite): leaving them out
    // of the sum changes no bit, and at B = 32 (one split) it cuts the block's partial reads 16-fold
    int nsm = NSPLIT;
    while (nsm > 1 && nsm * N_HEAD * B > 256) nsm >>= 1;
    for (int q = tid; q < R * N_HEAD; q += NTH) {
      const int bb = q / N_HEAD, head = q - bb * N_HEAD, b = min(r0 + bb, B - 1);
      const int4 ri = a.st.rowinfo[b];
      float* cf = cf_s + q * NSPLIT;
      const int t = ri.y + 1;
      const int ns = (ri.x < 0 || r0 + bb >= B) ? 0 : min(nsm, (t + 63) / 64);
      const float* ml = a.st.part_ml + ((size_t)(b * N_HEAD + head) * NSPLIT) * 2;
      float m[NSPLIT], l[NSPLIT];
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) { m[i] = ml[2 * i]; l[i] = ml[2 * i + 1]; }
      float M = -INFINITY;
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) if (i < ns) M = fmaxf(M, m[i]);
      float den = 0.f;
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) {
        const float f = (i < ns && m[i] != -INFINITY) ? expf(m[i] - M) : 0.f;
        m[i] = f;
        den += f * l[i];
      }
      const float inv = ns ? 1.0f / den : 0.f;
#pragma unroll
      for (int i = 0; i < NSPLIT; ++i) cf[i] = m[i] * inv;
    }
    __syncthreads();
    auto merge = [&](auto nsc) {
      constexpr int NS = decltype(nsc)::value;
      for (int e = tid; e < R * D; e += NTH) {
        const int bb = e / D, c = e - bb * D;
        const int b = min(r0 + bb, B - 1);
        const int head = c / HD, d = c - head * HD;
        const float* cf = cf_s + (bb * N_HEAD + head) * NSPLIT;
        const float* po = a.st.part_o + ((size_t)(b * N_HEAD + head) * NSPLIT) * HD + d;
        float pv[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) pv[i] = po[(size_t)i * HD];
        float y = 0.f;
#pragma unroll
        for (int i = 0; i < NS; ++i) y += cf[i] * pv[i];
        xs[bb * LDX + c] = y;
      }
    };
    if (nsm == 1) merge(std::integral_constant<int, 1>{});
    else if (nsm == 2) merge(std::integral_constant<int, 2>{});
    else if (nsm == 4) merge(std::integral_constant<int, 4>{});
    else if (nsm == 8) merge(std::integral_constant<int, 8>{});
    else merge(std::integral_constant<int, NSPLIT>{});
  } else if constexpr (IN == 4) {
    // one round trip: the rows as the attention normalised them (the merge of one split: the same
    // product o * (1 / l), the same bits), 16 B per load, all in flight (round 3: the 4-B loads of a
    // strided loop were issued a few at a time: c_proj 12.4 us at B = 32)
    constexpr int NL = R * D / 4 / NTH;
    static_assert(R * D / 4 % NTH == 0, "whole float4 loads per thread");
    float4 rv[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = (tid + i * NTH) * 4, bb = e / D, c = e - bb * D;
      const int b = min(r0 + bb, B - 1), head = c / HD, d = c - head * HD;
      rv[i] = *reinterpret_cast<const float4*>(a.st.part_o + (size_t)(b * N_HEAD + head) * NSPLIT * HD + d);
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = (tid + i * NTH) * 4, bb = e / D, c = e - bb * D;
      *reinterpret_cast<float4*>(xs + bb * LDX + c) = rv[i];
    }
  } else if constexpr (IN == 6 || (IN == 1 && STAGE)) {
    // the rows kernel's LayerNorm'd rows (IN 6), or the K slice of the h rows (IN 1, two column
    // tiles), 16 B per thread and load, all in flight (padded rows: row B-1, never stored)
    constexpr int NL = R * D / 4 / NTH;
    static_assert(R * D / 4 % NTH == 0, "whole float4 loads per thread");
    float4 rv[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = (tid + i * NTH) * 4, bb = e / D, c = e - bb * D;
      rv[i] = *reinterpret_cast<const float4*>(a.st.h + (size_t)min(r0 + bb, B - 1) * (IN == 1 ? KTOT : D) + (IN == 1 ? ks * K : 0) + c);
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = (tid + i * NTH) * 4, bb = e / D, c = e - bb * D;
      *reinterpret_cast<float4*>(xs + bb * LDX + c) = rv[i];
    }
  }
  if constexpr (STAGE) __syncthreads();
  f32x4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int kq = 4 * (lane >> 4);  // this lane's k offset inside each 16-wide k group
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float4 xf[12];
    if constexpr (STAGE) {
      const float* xr = xs + (t * 16 + (lane & 15)) * LDX + kw * 192 + kq;
#pragma unroll
      for (int j = 0; j < 12; ++j) xf[j] = *reinterpret_cast<const float4*>(xr + 16 * j);
    } else {
      const int b = min(r0 + t * 16 + (lane & 15), B - 1);  // padded columns recompute row B-1, never stored
      const float* xr = a.st.h + (size_t)b * KTOT + ks * K + kw * 192 + kq;
#pragma unroll
      for (int j = 0; j < 12; ++j) xf[j] = *reinterpret_cast<const float4*>(xr + 16 * j);
    }
    __builtin_amdgcn_sched_barrier(0);  // the tile's 12 operand loads in flight together
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].x, xf[j].x, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].y, xf[j].y, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].z, xf[j].z, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].w, xf[j].w, acc[t], 0, 0, 0);
    }
  }
  // lane: C[n0 + 4 (lane >> 4) + i][t * 16 + (lane & 15)]
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][(4 * (lane >> 4) + i) * R + t * 16 + (lane & 15)] = acc[t][i];
  __syncthreads();
  for (int e = tid; e < CT * 16 * R; e += NTH) {
    const int ct = e / (16 * R), el = e - ct * (16 * R);
    const int r = el / R, c = el - r * R, n = nb + ct * 16 + r, b = r0 + c;
    if (b >= B || n >= a.N) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWK; ++w) v += red[ct * NWK + w][el];
    if constexpr (OUT == 6) a.yacc[((size_t)b * YCOPIES + ks) * D + n] = v;  // K slice ks -> its pending copy
    else gemv_store<OUT>(a, n, b, v);
  }
}

// c_attn of the batched fp32 parity mode (B <= 32), the K = 768 reduction split over the grid as in
// ar_qkv_ksplit_kernel: a block is 4 waves x 16 output rows of one 192-wide K slice (48 KB of
// fragment-packed fp32 weights) and stages the slice of the rows kernel's LayerNorm'd fp32 rows (st.h,
// NT * 16 x 192) once in LDS for its 4 waves; each wave stores its 16 x (NT * 16) partial to
// st.qkvp[slice]; the attention (ar_attn_v2_kernel<float, ..., QKV>) sums the four slices in slice
// order and appends the new key. 144 blocks of 48 + 24 KB instead of 144 of 48 + 96 KB. (Round 5,
// measured slower: 8-wave blocks whose two wave groups each multiply one of the two 16-row tiles, a
// 48-MFMA chain per wave instead of 96: B = 32 fp32 203.8 vs 201.4 us/step, bit-identical.)
template <int NT>
__global__ __launch_bounds__(256) LVX_LOADS_FIRST void ar_qkv_ksplit_f32_kernel(GemvArgs a) {
  constexpr int XR = NT * 16, XS = 196;  // rows, fp32 row stride (784 B: 16 rows 4 banks apart)
  __shared__ __attribute__((aligned(16))) float xs[XR * XS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n0 = (blockIdx.x * 4 + wave) * 16, ks = blockIdx.y;
  const int B = a.B;
  constexpr int XC = XR * 48 / 256;  // 16-B chunks per thread (3 / 6)
  static_assert(XR * 48 % 256 == 0, "whole chunks per thread");
  float4 xv[XC];
#pragma unroll
  for (int j = 0; j < XC; ++j) {  // the operand slice first (rows past B: row B-1, never stored)
    const int c = tid + 256 * j, r = c / 48, q = c - r * 48;
    xv[j] = *reinterpret_cast<const float4*>(a.st.h + (size_t)min(r, B - 1) * D + ks * 192 + q * 4);
  }
  const float4* wsrc = reinterpret_cast<const float4*>(a.Wf) + ((size_t)(n0 >> 4) * (D / 16) + ks * 12) * 64 + lane;
  float4 wf[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) wf[j] = wsrc[j * 64];
#pragma unroll
  for (int j = 0; j < XC; ++j) {
    const int c = tid + 256 * j, r = c / 48, q = c - r * 48;
    *reinterpret_cast<float4*>(xs + r * XS + q * 4) = xv[j];
  }
  __syncthreads();
  const int kq = 4 * (lane >> 4);
  f32x4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    float4 xf[12];
    const float* xr = xs + (t * 16 + (lane & 15)) * XS + kq;
#pragma unroll
    for (int j = 0; j < 12; ++j) xf[j] = *reinterpret_cast<const float4*>(xr + 16 * j);
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].x, xf[j].x, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].y, xf[j].y, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].z, xf[j].z, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j].w, xf[j].w, acc[t], 0, 0, 0);
    }
  }
  // lane: C[n0 + 4 (lane >> 4) + i][t * 16 + (lane & 15)], i = 0..3
  float* dst = a.st.qkvp + (size_t)ks * a.st.max_streams * (3 * D) + n0 + 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int b = t * 16 + (lane & 15);
    if (b < B) *reinterpret_cast<float4*>(dst + (size_t)b * (3 * D)) = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
  }
}

// option f32b (default 1, Opts in lvx_internal.h): 1: batched fp32 parity steps (3 <= B <= 64) on exact-fp32 MFMA; 0: the GEMV family

// 16-row batch tiles (NT = 1) for every op: a block's time is the bytes it loads (the N = 768 ops:
// 96 blocks of 16 rows instead of 48 of 32; round 3, c_fc and lm_head too: B = 32 248.3 -> 246.0
// us/step at t = 384-639). Option exp bit 8: 32-row tiles (NT = 2) at B > 16, the cross-check. Same
// bits either way (a column's dot product is its own).
template <int K, int IN, int OUT, int KTOT = K>
static void launch_f32b(const GemvArgs& a, hipStream_t s) {
  const bool nt1 = a.B <= 16 || !(opts().exp & 8);
  const int nbr = nt1 ? (a.B + 15) / 16 : (a.B + 31) / 32;
  // two column tiles per block when one per block would put more than 256 blocks on the chip
  // (round 5, B = 32 t = 384-639: 200.9 vs 210.9 us/step, c_fc 7.58 -> 6.37 us, lm_head 7.27 -> 6.40,
  // mlp c_proj with its h slice staged once per block; option exp bit 8192: one tile per block)
  const bool ct2 = nt1 && K == 768 && (a.N / 16) * nbr * (KTOT / K) > 256;
  dim3 grid((a.N + 15) / 16, nbr, KTOT / K), block(K / 192 * 64);
  if constexpr (K == 768) {
    if (ct2) {
      grid.x = (a.N + 31) / 32;
      block.x *= 2;
      hipLaunchKernelGGL((ar_f32b_kernel<K, 1, IN, OUT, KTOT, 2>), grid, block, 0, s, a);
      return;
    }
  }
  if (nt1) {
    hipLaunchKernelGGL((ar_f32b_kernel<K, 1, IN, OUT, KTOT>), grid, block, 0, s, a);
  } else {
    hipLaunchKernelGGL((ar_f32b_kernel<K, 2, IN, OUT, KTOT>), grid, block, 0, s, a);
  }
}

// Measured (round-1 sweep, us per step at positions 256-511): v3 saves kernels but every block
// re-reads the fp32 x rows of its batch tile, and per-CU load bandwidth (not launch count) sets the
// time of these short GEMMs: B = 8 / 16 / 32 v2 149 / 162 / 191 vs v3 172 / 181 / 203 (16-row
// tiles, separate merge); a fused merge re-reads ns_max partials per row and block: 271 / 302 / 266.
// v3 therefore runs only where v2 has no kernels (32 < B <= 64: 250 us, 16-row tiles).
// option exp (default 0, Opts in lvx_internal.h): development A/B bits (lvx_set_option "exp"), 0 = production kernels
// option bt (default 1, Opts in lvx_internal.h): 1: batched path v3 for 32 < B <= 64; 2: v3 for every batched B (cross-check of v2); 0: off

template <int K, int IN, int OUT>
static void launch_bt(const GemvArgs& a, hipStream_t s) {
  // 16 batch rows per block (32 / 64 measured slower: fewer blocks, more bytes each)
  dim3 grid((a.N + 15) / 16, (a.B + 15) / 16), block(K / 192 * 64);
  hipLaunchKernelGGL((ar_bt_kernel<K, 1, IN, OUT>), grid, block, 0, s, a);
}

// Attention launch shape, measured (tools/step_sweep.py, us/step): 4 waves per block (8 waves,
// 128-key tiles: B = 32 t = 256+ 153.7 vs 149.4; B = 64 211.1 vs 209.0), 2 KV tiles in flight per
// wave (4: B = 32 157.9 vs 152.0, B = 64 234.2 vs 216.3), splits until ns x 8 heads x B <= 256
// blocks (B = 32 at t = 256-511: 1024 blocks 164, 512 169, 256 = one split that writes xn
// itself 155.5; B = 16: 138 / 136 / 131; B = 8: 144 / 133 / 130).
constexpr int ATTN_BLOCKS = 256;
// (round 3, measured no faster: 8-wave blocks for the one-split bf16 attention at B = 32, 132.1 vs 130.3
// us/step at t = 0..1,023: the tile loop streams the KV history at ~7 TB/s either way)
static int attn_ns_max(int B) {  // enough splits to fill the chip, no more (early-exit blocks cost)
  int ns = NSPLIT;
  while (ns > 1 && ns * N_HEAD * B > ATTN_BLOCKS) ns >>= 1;
  return ns;
}

static void launch_attn(const ArState& st, int kvdtype, int B, int l, hipStream_t s, int ns_max = NSPLIT,
                        int direct = 0, int selcopy = 0, bool qkv = false, bool nw8 = false) {
  dim3 grid(ns_max, N_HEAD, B);
  // (round 4, measured slower: 16 waves and 256-key tiles for the one-split blocks at B <= 8, B = 8
  // t = 384-639 fp8 KV 103.9 vs 98.3 us/step, bf16 KV 109.6 vs 100.1)
  if (qkv && kvdtype != LVX_DTYPE_F32) return;  // (no such path: the K split is the fp32 parity mode's)
  if (nw8 && kvdtype == LVX_DTYPE_BF16)  // 8 waves, 128-key tiles: twice the KV bytes in flight per block
    hipLaunchKernelGGL((ar_attn_v2_kernel<bf16_t, 2, 8>), grid, dim3(512), 0, s, st, l, ns_max, direct, selcopy);
  // (round 5, measured slower: 3 / 4 fp8 KV tiles in flight per wave at B = 8, t = 384-639 99.2 / 100.1
  // vs 98.0 us/step)
  else if (nw8 && kvdtype == LVX_DTYPE_FP8)
    hipLaunchKernelGGL((ar_attn_v2_kernel<fp8_t, 2, 8>), grid, dim3(512), 0, s, st, l, ns_max, direct, selcopy);
  // (round 4, fp32 KV at B = 32, measured slower: 8 waves with 128-key tiles 212.6, 3 tiles in flight
  // per wave 218.0 vs 211.7 us/step)
  else if (qkv)  // fp32 parity mode: ar_qkv_ksplit_f32_kernel's partials (the only K-split c_attn)
    hipLaunchKernelGGL((ar_attn_v2_kernel<float, 2, 4, true>), grid, dim3(256), 0, s, st, l, ns_max, direct, selcopy);
  else if (kvdtype == LVX_DTYPE_BF16)
    hipLaunchKernelGGL((ar_attn_v2_kernel<bf16_t, 2, 4>), grid, dim3(256), 0, s, st, l, ns_max, direct, selcopy);
  else if (kvdtype == LVX_DTYPE_FP8)
    hipLaunchKernelGGL((ar_attn_v2_kernel<fp8_t, 2, 4>), grid, dim3(256), 0, s, st, l, ns_max, direct, selcopy);
  else
    hipLaunchKernelGGL((ar_attn_v2_kernel<float, 2, 4>), grid, dim3(256), 0, s, st, l, ns_max, direct, selcopy);
}

// ArWeights q0_* tables (lvx_finalize, once): out[r][n] = sum_k<K (src[r][k] * g[k0 + k]) * W[n][k0 + k],
// W = layer 0's bf16 c_attn weight [2304][768]; 64 x 64 output tiles, K staged 16 at a time through LDS
// (fp32 FMAs in k order)
__global__ __launch_bounds__(256) void q0_table_kernel(const float* __restrict__ src, int rows, int K, int k0,
                                                       const float* __restrict__ g, const bf16_t* __restrict__ W,
                                                       float* __restrict__ out) {
  __shared__ float As[16][65], Bs[16][65];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int r0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  float acc[4][4] = {};
  for (int kt = 0; kt < K; kt += 16) {
    for (int e = threadIdx.x; e < 1024; e += 256) {
      const int rr = e >> 4, kk = e & 15, r = r0 + rr;
      As[kk][rr] = r < rows ? src[(size_t)r * K + kt + kk] * g[k0 + kt + kk] : 0.f;
      Bs[kk][rr] = bf16_to_f32(W[(size_t)(n0 + rr) * D + k0 + kt + kk]);
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(As[kk][ty * 4 + i], Bs[kk][tx * 4 + j], acc[i][j]);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + ty * 4 + i;
    if (r < rows)
#pragma unroll
      for (int j = 0; j < 4; ++j) out[(size_t)r * (3 * D) + n0 + tx * 4 + j] = acc[i][j];
  }
}

void ar_launch_q0_tables(const ArWeights& w, int max_pos, float* text, float* code, float* pos, hipStream_t s) {
  static_assert((3 * D) % 64 == 0 && TEXT_DIM % 16 == 0 && SPEECH_DIM % 16 == 0 && D % 16 == 0, "q0 tiles");
  const bf16_t* W = reinterpret_cast<const bf16_t*>(w.w_attn[0]);
  const float* g = w.ln1[0];
  hipLaunchKernelGGL(q0_table_kernel, dim3(3 * D / 64, (TEXT_VOCAB + 63) / 64), dim3(256), 0, s, w.text_table,
                     TEXT_VOCAB, TEXT_DIM, 0, g, W, text);
  hipLaunchKernelGGL(q0_table_kernel, dim3(3 * D / 64, (VOCAB + 63) / 64), dim3(256), 0, s, w.codebook, VOCAB,
                     SPEECH_DIM, TEXT_DIM, g, W, code);
  hipLaunchKernelGGL(q0_table_kernel, dim3(3 * D / 64, (max_pos + 63) / 64), dim3(256), 0, s, w.wpe, max_pos, D, 0,
                     g, W, pos);
}

// one op of the decode step, with the B-dependent kernel choice (shared by the step and the probes)
// op: 0 c_attn (layer 0: + embedding) 1 attention 2 c_proj (+ split merge) 3 c_fc 4 mlp c_proj 5 lm_head
template <typename TW>
static bool use_mfma(int B) {
  return sizeof(TW) == 2 && B >= MFMA_BATCH_MIN && B <= 64;
}
template <typename TW>
static bool use_bt(int B) {
  return use_mfma<TW>(B) && opts().bt && (B > 32 || opts().bt == 2);
}

// batched path v3: one kernel per op (plus the attention), final x rows at every boundary
static void launch_op_bt(int op, GemvArgs& a, const ArWeights& w, int l, int kvdtype, int B, hipStream_t s) {
  const int nsm = attn_ns_max(B);
  a.layer = l;
  a.yacc = nullptr;
  a.add_y = 0;
  switch (op) {
    case 0:
      a.W = w.w_attn[l]; a.N = 3 * D; a.ln_w = w.ln1[l];
      if (l == 0 && a.defer_sel == 2) {  // embedding + the previous step's select, then c_attn
        hipLaunchKernelGGL(ar_embed_select_kernel<>, dim3(B), dim3(256), 0, s, a);
        launch_bt<768, 1, 0>(a, s);
      } else if (l == 0) {
        launch_bt<768, 3, 0>(a, s);
      } else {
        launch_bt<768, 0, 0>(a, s);
      }
      break;
    case 1: launch_attn(a.st, kvdtype, B, l, s, nsm); break;
    case 2:
      a.W = w.w_aproj[l]; a.N = D;
      launch_merge_bf16(a.st, B, nsm, s);
      launch_bt<768, 1, 1>(a, s);
      break;
    case 3: a.W = w.w_fc[l]; a.N = DFF; a.ln_w = w.ln2[l]; launch_bt<768, 0, 5>(a, s); break;
    case 4: a.W = w.w_mproj[l]; a.N = D; launch_bt<3072, 1, 1>(a, s); break;
    case 5: a.W = w.w_lm; a.N = VOCAB; a.ln_w = w.lnf; launch_bt<768, 0, 3>(a, s); break;
  }
}

// deferred select: every row of the step is prefetched by its own wave of c_attn layer 0 (B <= 2,
// one batch group) and lm_head runs LM_SEL_BLOCKS blocks of 8 rows
template <typename TW>
static bool defer_select(int B) {
  static_assert(LM_SEL_BLOCKS <= LM_MAX_BLOCKS && LM_SEL_BLOCKS % 64 == 0, "deferred select granules");
  return opts().defer_select && B <= 2 && !use_mfma<TW>(B);
}
template <typename TW>
static bool use_f32b(int B);
static bool f32b_qsplit(int B);
// 4 <= B <= 8 on the LayerNorm-prologue GEMMs (ar_mfma_ln_kernel): the select folded into c_attn layer
// 0's prologue from lm_head's granules (defer_sel 3) instead of ar_embed_select_kernel + the c_attn
// launch (option defer_select 2: the embedding + select kernel at these B too, the cross-check)
template <typename TW>
static bool defer_select_ln(int B) {
  return opts().defer_select == 1 && use_mfma<TW>(B) && B >= 4 && B <= MFMA_LN_MAX && B <= LM8_ROWS;
}
template <typename TW>
static bool defer_select_batched(int B) {
  // us/step (tools/step_sweep.py, t = 256+) argmax kernel / deferred: B = 3: 112.9 / 114.7 (B = 3
  // keeps the argmax kernel), B = 4: 106.0 / 104.9, 8: 120.7 / 118.3, 12: 123.0 / 120.5,
  // 16: 128.4 / 125.5, 32: 150.3 / 147.3, 64: 213.4 / 206.8
  // fp32 parity mode (round 3): with the K-split c_attn (its layer-0 rows kernel becomes
  // ar_embed_select_kernel<true>); B = 32 t = 384-639: 213.9 -> 210.8 us/step
  return opts().defer_select && ((use_mfma<TW>(B) && B >= 4) || use_bt<TW>(B) || (use_f32b<TW>(B) && B >= 4 && f32b_qsplit(B)));
}

// measured at B = 1 (round 1): 16 h rows per block (192 blocks) 76.7 us/step; 32 rows (96 blocks)
// +6.8 us; 12 rows (256 blocks, one per CU) 77.4 us; 8 accumulator copies slower than 4
template <typename TW>
static bool fused_mlp(int B) {
  return sizeof(TW) == 2 && opts().fuse_mlp && B <= 2 && !use_mfma<TW>(B);
}

template <typename TW>
static bool use_f32b(int B) {
  return sizeof(TW) == 4 && opts().f32b && B >= MFMA_BATCH_MIN && B <= 64;
}

// batched fp32 parity steps: five exact-fp32 MFMA kernels + the attention per layer; the split-KV
// partials are merged in c_proj's prologue; the select is the argmax kernel after lm_head.
// mlp c_proj runs as 4 K slices into the pending copies (384 blocks of 4 waves instead of 96 of 16:
// the 16-wave blocks each loaded 392 KB on 96 CUs); the rows kernel before c_attn (layers >= 1) and
// lm_head folds them into x and leaves the LayerNorm'd fp32 rows the GEMM stages (IN 6). Option exp
// bit 512: the unsplit mlp c_proj with x final at every boundary and the LayerNorm in the GEMM prologue.
static bool f32b_qsplit(int B) { return !(opts().exp & 512) && B <= 32 && !(opts().exp & 1024); }
static void launch_op_f32b(int op, GemvArgs& a, const ArWeights& w, int l, int kvdtype, int B, hipStream_t s) {
  const bool ksp = !(opts().exp & 512);
  a.layer = l;
  a.yacc = ksp ? a.st.yacc : nullptr;
  a.add_y = 0;
  a.xpk = 0;
  // c_attn split over K too (B <= 32), its partials summed by the attention; option exp bit 1024: one launch
  const bool qsp = f32b_qsplit(B);
  switch (op) {
    case 0:
      a.W = w.w_attn[l]; a.Wf = w.f_attn[l]; a.N = 3 * D; a.ln_w = w.ln1[l];
      if (qsp) {  // rows kernel (layer 0: embedding; else x + the MLP copies) -> fp32 rows, then the K slices
        if (l == 0 && a.defer_sel == 2) hipLaunchKernelGGL(ar_embed_select_kernel<true>, dim3(B), dim3(256), 0, s, a);
        else if (l == 0) hipLaunchKernelGGL((ar_rows_kernel<6>), dim3(B), dim3(64), 0, s, a);
        else hipLaunchKernelGGL((ar_rows_kernel<5>), dim3(B), dim3(64), 0, s, a);
        if (B <= 16) hipLaunchKernelGGL((ar_qkv_ksplit_f32_kernel<1>), dim3(3 * D / 64, 4), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((ar_qkv_ksplit_f32_kernel<2>), dim3(3 * D / 64, 4), dim3(256), 0, s, a);
      } else if (l == 0) {
        launch_f32b<768, 3, 0>(a, s);
      } else if (ksp) {
        hipLaunchKernelGGL((ar_rows_kernel<5>), dim3(B), dim3(64), 0, s, a);
        launch_f32b<768, 6, 0>(a, s);
      } else {
        launch_f32b<768, 0, 0>(a, s);
      }
      break;
    case 1: launch_attn(a.st, kvdtype, B, l, s, attn_ns_max(B), attn_ns_max(B) == 1 ? 3 : 0, 0, qsp); break;
    case 2:
      a.W = w.w_aproj[l]; a.Wf = w.f_aproj[l]; a.N = D;
      if (attn_ns_max(B) == 1) launch_f32b<768, 4, 1>(a, s);  // the attention wrote the rows (direct 3)
      else launch_f32b<768, 2, 1>(a, s);
      break;
    case 3: a.W = w.w_fc[l]; a.Wf = w.f_fc[l]; a.N = DFF; a.ln_w = w.ln2[l]; launch_f32b<768, 0, 2>(a, s); break;
    case 4:
      a.W = w.w_mproj[l]; a.Wf = w.f_mproj[l]; a.N = D;
      if (ksp) launch_f32b<768, 1, 6, DFF>(a, s);
      else launch_f32b<3072, 1, 1>(a, s);
      break;
    case 5:
      a.W = w.w_lm; a.Wf = w.f_lm; a.N = VOCAB; a.ln_w = w.lnf;
      if (ksp) {
        hipLaunchKernelGGL((ar_rows_kernel<5>), dim3(B), dim3(64), 0, s, a);
        launch_f32b<768, 6, 3>(a, s);
      } else {
        launch_f32b<768, 0, 3>(a, s);
      }
      break;
  }
}

// returns false when the op has no kernel of its own at this B (mlp c_proj inside the fused MLP)
template <typename TW>
static bool launch_op(int op, GemvArgs& a, const ArWeights& w, int l, int kvdtype, int B, hipStream_t s) {
  if (use_f32b<TW>(B) && !a.emb_row) {
    launch_op_f32b(op, a, w, l, kvdtype, B, s);
    return true;
  }
  if (use_bt<TW>(B) && !a.emb_row) {
    launch_op_bt(op, a, w, l, kvdtype, B, s);
    return true;
  }
  const bool mf = use_mfma<TW>(B);
  const bool fm = fused_mlp<TW>(B);
  // batched steps at B >= 9: one attention split per (row, head), the head output written straight
  // into the bf16 operand row (no merge kernel). Round 3, tools/step_sweep.py (graph replay, us per
  // step at t = 128 / 640): bf16 KV B = 12 104.3 / 113.0 -> 95.4 / 107.7, B = 16 107.1 / 126.7 ->
  // 97.4 / 119.0; fp8 KV B = 12 103.2 / 110.3 -> 95.4 / 108.4, B = 16 104.2 / 111.5 -> 96.1 / 109.2.
  // At B = 8 (64 blocks) one split loses at long histories (fp8 KV 102.4 -> 105.7 at t = 640 while
  // 98.1 -> 92.5 at t = 128): B <= 8 keeps the split-KV attention + merge.
  // 5 <= B <= 8: one split too, in 8-wave blocks (128-key tiles: twice the KV bytes in flight per
  // block, 40-64 blocks); tools/step_sweep.py, fp8 KV, B = 8, t = 128 / 640 / 896: 98.0 / 102.3 / 104.2
  // -> 92.6 / 102.8 / 106.5 us (bf16 KV 98.7 / 105.9 / 108.5 -> 95.1 / 105.3 / 108.8): ~1 % over a
  // 1,024-token utterance; at B = 4 it loses (91.9 / 94.5 / 95.5 -> 87.6 / 96.3 / 100.8). fp8 KV (half the bytes per
  // key) keeps the 8-wave blocks up to B = 16: B = 12 / 16, t = 128 / 640 / 896: 95.8 / 108.3 / 114.8 ->
  // 97.0 / 105.5 / 109.6 and 95.8 / 109.6 / 115.5 -> 97.0 / 106.8 / 110.2 us; bf16 KV there loses
  // (B = 16: 97.0 / 109.9 / 128.1 -> 100.8 / 112.5 / 130.5). (The switches restoring the older forms,
  // option exp bits 32 / 64 / 128, were removed in round 6.)
  const bool a8 = mf && B >= 5 && (B <= 8 || (kvdtype == LVX_DTYPE_FP8 && B <= 16));
  const int nsm = mf ? ((B > 8 || a8) ? 1 : attn_ns_max(B)) : NSPLIT;
  // the MFMA GEMMs read the fragment-packed weight copies (a.Wf; round 6: the row-major reads of option
  // exp bit 2, bit-identical and slower, removed)
  // fragment-packed operand rows on the v2 steps with the rows kernel (9 <= B <= 32)
  a.xpk = (mf && B > MFMA_LN_MAX && B <= 32) ? 1 : 0;
  a.layer = l;
  a.yacc = mf ? a.st.yacc : nullptr;
  a.yfx = fm ? a.st.yfx : nullptr;
  a.add_y = l > 0;
  switch (op) {
    case 0:
      a.W = w.w_attn[l]; a.Wf = w.f_attn[l]; a.N = 3 * D; a.ln_w = w.ln1[l];
      if (mf && l == 0 && a.defer_sel == 3) {  // the previous step's select + embedding in c_attn's prologue
        launch_mfma_ln<0, 7>(a, s);
      } else if (mf && l == 0 && a.defer_sel == 4) {  // select + c_attn from the q0 tables, 9 slices per row
        hipLaunchKernelGGL(ar_q0_rows_kernel, dim3(3 * D / 256, B), dim3(256), 0, s, a);
      } else if (mf && l == 0 && a.defer_sel == 2) {  // embedding + the previous step's select, then c_attn
        hipLaunchKernelGGL(ar_embed_select_kernel<>, dim3(B), dim3(256), 0, s, a);
        launch_mfma2<768, 0>(a, s);
      } else if (mf && B <= MFMA_LN_MAX) {
        if (l == 0) launch_mfma_ln<0, 3>(a, s);
        else launch_mfma_ln<0, 4>(a, s);
      } else if (mf) {  // rows kernel: LayerNorm (layer 0: of the embedding; else of x + the MLP copies)
        if (l == 0) hipLaunchKernelGGL((ar_rows_kernel<3>), dim3(B), dim3(64), 0, s, a);
        else hipLaunchKernelGGL((ar_rows_kernel<4>), dim3(B), dim3(64), 0, s, a);
        launch_mfma2<768, 0>(a, s);
      } else if (l == 0 && a.defer_sel == 1 && opts().l0q && a.q0_text) {  // B <= 2, the q0 tables
        hipLaunchKernelGGL(ar_q0_gran_kernel, dim3(3 * D / 256), dim3(256), 0, s, a);
      } else if (l == 0 && a.defer_sel) {
        launch_gemv<TW, 768, 1, 2, 5, 0>(a, s);  // + the previous step's select
      } else if (l == 0) {
        launch_gemv<TW, 768, 1, 2, 3, 0>(a, s);
      } else if (fm) {
        launch_gemv<TW, 768, 1, 2, 4, 0>(a, s);
      } else {
        launch_gemv<TW, 768, 1, 2, 0, 0>(a, s);
      }
      break;
    case 1:
      launch_attn(a.st, kvdtype, B, l, s, nsm, (mf && nsm == 1) ? 1 + a.xpk : 0,
                  (a.defer_sel == 1 || a.defer_sel == 3 || a.defer_sel == 4) && l == 0,
                  false, a8);
      break;
    case 2:
      a.W = w.w_aproj[l]; a.Wf = w.f_aproj[l]; a.N = D;
      if (mf) {
        if (B > MFMA_LN_MAX) a.add_y = 0;  // ar_rows_kernel<4> of this layer's c_attn folded them
        if (nsm > 1) launch_merge_bf16(a.st, B, nsm, s, a.xpk);  // nsm == 1: the attention wrote xn itself
        a.ln_w = w.ln2[l];  // OUT 7: the bf16 copy is x * ln_2.weight (c_fc's operand)
        // + bf16 x and row statistics for c_fc; 16-row batch tiles (B = 32: 96 blocks of 49 KB operands
        // instead of 48 of 74 KB: -3.4 us/step at t = 512-1,151)
        if (B > MFMA_LN_MAX) launch_mfma2<768, 7>(a, s, true);
        else launch_mfma2<768, 1>(a, s);
      } else {
        launch_gemv<TW, 768, 1, 1, 2, 1>(a, s);
      }
      break;
    case 3:
      a.W = w.w_fc[l]; a.Wf = w.f_fc[l]; a.N = DFF; a.ln_w = w.ln2[l];
      if (fm) {  // 16 h rows per block (192 blocks)
        const bf16_t* wfc = reinterpret_cast<const bf16_t*>(w.w_fc[l]);
        const bf16_t* wpk = reinterpret_cast<const bf16_t*>(w.w_mproj_pk[l]);
        if (B <= 1) hipLaunchKernelGGL((ar_mlp_fused_kernel<1, 16>), dim3(DFF / 16), dim3(256), 0, s, a, wfc, wpk);
        else hipLaunchKernelGGL((ar_mlp_fused_kernel<2, 16>), dim3(DFF / 16), dim3(256), 0, s, a, wfc, wpk);
      } else if (mf && B <= MFMA_LN_MAX) {
        launch_mfma_ln<5, 0>(a, s);
      } else if (mf) {
        a.gsum = w.fc_gsum[l];
        launch_mfma2<768, 5, 1>(a, s);  // LayerNorm from c_proj's row statistics, after the GEMM
      } else {
        launch_gemv<TW, 768, 1, 2, 0, 2>(a, s);
      }
      break;
    case 4:
      a.W = w.w_mproj[l]; a.Wf = w.f_mproj[l]; a.N = D;
      if (fm) return false;
      if (mf && YCS < YCOPIES && B <= MFMA_LN_MAX)  // YCS K slices of DFF / YCS into the YCS copies
        hipLaunchKernelGGL((ar_mfma2_kernel<DFF / YCS, 1, 6, DFF>), dim3(D / 16, YCS), dim3(DFF / YCS / 192 * 64), 0, s, a);
      else if (mf) launch_mproj_split<6>(a, s);
      else launch_gemv<TW, 3072, 4, 2, 1, 1>(a, s);
      break;
    case 5:
      a.W = w.w_lm; a.Wf = w.f_lm; a.N = VOCAB; a.ln_w = w.lnf;
      if (mf && B <= MFMA_LN_MAX) {
        launch_mfma_ln<3, 4>(a, s);
      } else if (mf) {
        hipLaunchKernelGGL((ar_rows_kernel<4>), dim3(B), dim3(64), 0, s, a);
        launch_mfma2<768, 3>(a, s);
      } else if (a.defer_sel == 1) {
        if (fm) launch_gemv<TW, 768, 1, 2, 4, 9>(a, s);
        else launch_gemv<TW, 768, 1, 2, 0, 9>(a, s);
      } else if (fm) {
        launch_gemv<TW, 768, 1, 2, 4, 3>(a, s);
      } else {
        launch_gemv<TW, 768, 1, 2, 0, 3>(a, s);
      }
      break;
  }
  return true;
}

template <typename TW>
static GemvArgs make_args(const ArWeights& w, const ArState& st, int kvdtype, int B, const float* emb_row) {
  GemvArgs a{};
  a.st = st;
  a.B = B;
  a.kv_dtype = kvdtype;
  a.text_table = w.text_table;
  a.codebook = w.codebook;
  a.wpe = w.wpe;
  a.emb_row = emb_row;
  a.q0_text = w.q0_text;
  a.q0_code = w.q0_code;
  a.q0_pos = w.q0_pos;
  a.q0_g = w.q0_g;
  return a;
}


// returns whether the greedy select is deferred into the next step (no argmax kernel after lm_head)
template <typename TW>
static bool ar_layers(const ArWeights& w, const ArState& st, int kvdtype, int B, const float* emb_row, int slot,
                      int pos, float* logits_dst, bool select, hipStream_t s) {
  GemvArgs a = make_args<TW>(w, st, kvdtype, B, emb_row);
  a.defer_sel = (select && !emb_row) ? (defer_select<TW>(B) ? 1 : defer_select_batched<TW>(B) ? (defer_select_ln<TW>(B) ? 3 : 2) : 0) : 0;
  // bf16 with option l0q, 4 <= B <= 32: the previous step's select and layer 0's c_attn from the q0
  // tables in one launch, ar_q0_rows_kernel (9 column slices per row; defer_sel 4): at B > 8 the c_attn
  // GEMM launch goes, at 4 <= B <= 8 the c_attn-with-select launch reads table rows instead of weight
  // slices (round 6, us per step at t = 384-639, each A/B on one box: the tables in one block per row
  // took B = 32 -2.9, B = 8 -1.8 / -2.5 (fp8 / bf16 KV), B = 4 -1.4 (l0q_ab.txt, b8_l0q_ab.txt); the 9
  // slices per row a further -1.1 / -1.7 / -1.7 (q0rows_ab.txt); the reference-agreement measures
  // unchanged). B <= 2 keep their granule select with the tables in ar_q0_gran_kernel.
  if ((a.defer_sel == 2 || a.defer_sel == 3) && use_mfma<TW>(B) && B <= 32 && opts().l0q && w.q0_text) a.defer_sel = 4;
  if (emb_row) hipLaunchKernelGGL(ar_row_state_kernel, dim3(1), dim3(1), 0, s, st, slot, pos);
  for (int l = 0; l < N_LAYER; ++l)
    for (int op = 0; op < 5; ++op) launch_op<TW>(op, a, w, l, kvdtype, B, s);
  a.dst = logits_dst;
  launch_op<TW>(5, a, w, N_LAYER - 1, kvdtype, B, s);
  return a.defer_sel != 0;
}

// Launch one op of the decode step `iters` times (bench.py times it with HIP events); layer 1.
template <typename TW>
static int ar_probe_impl(const ArWeights& w, const ArState& st, int kvdtype, int B, int which, int iters,
                         hipStream_t s) {
  if (which < 0 || which > 5) return -1;
  if (which == 4 && fused_mlp<TW>(B)) return 1;  // no kernel of its own at this B
  if (iters == 0) return 0;                       // validation only
  GemvArgs a = make_args<TW>(w, st, kvdtype, B, nullptr);
  a.dst = st.logits;
  hipLaunchKernelGGL(ar_rowinfo_init_kernel, dim3((B + 63) / 64), dim3(64), 0, s, st, B);
  for (int i = 0; i < iters; ++i)
    if (!launch_op<TW>(which, a, w, which == 5 ? N_LAYER - 1 : 1, kvdtype, B, s))
      return 1;  // no kernel of its own at this B
  return 0;
}

int ar_probe(const ArWeights& w, const ArState& st, int wdtype, int kvdtype, int B, int which, int iters,
             hipStream_t s) {
  return wdtype == LVX_DTYPE_BF16 ? ar_probe_impl<bf16_t>(w, st, kvdtype, B, which, iters, s)
                                  : ar_probe_impl<float>(w, st, kvdtype, B, which, iters, s);
}

void ar_launch_step(const ArWeights& w, const ArState& st, int wdtype, int kvdtype, int B, int mode,
                    const float* emb_row, int slot, int pos, float* logits_out, hipStream_t s) {
  float* dst = mode == 0 ? st.logits : logits_out;
  const float* er = mode == 0 ? nullptr : emb_row;
  const bool deferred = wdtype == LVX_DTYPE_BF16 ? ar_layers<bf16_t>(w, st, kvdtype, B, er, slot, pos, dst, mode == 0, s)
                                                : ar_layers<float>(w, st, kvdtype, B, er, slot, pos, dst, mode == 0, s);
  if (mode == 0 && !deferred) hipLaunchKernelGGL(ar_argmax_kernel, dim3(B), dim3(256), 0, s, st);
}

// test hook (select probe path 3): the 4 <= B <= 8 granule select as c_attn layer 0 (MODE 7) runs it
// (lmg8_reduce + softmax_ties), committed with argmax_commit
__global__ __launch_bounds__(64) void ar_select8_probe_kernel(ArState st) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int4 ri = st.rowinfo[b];
  LmGran8 q;
  lmg8_issue(st, b, lane, q);
  const Best r = softmax_ties(st.logits + (size_t)b * VOCAB, lmg8_reduce(q), lane);
  if (lane == 0 && ri.x >= 0) argmax_commit(st, b, ri, r);
}

// deferred select: the last step's lm_head granules are committed here (argmax_commit), once per
// lvx_ar_steps call, after the steps
__global__ __launch_bounds__(64) void ar_select_final_kernel(ArState st) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int4 ri = st.rowinfo[b];
  const int2 rx = st.rowx[b];
  LmGran q;
  lmg_issue(st, b, lane, q);
  const Best r = softmax_ties(st.logits + (size_t)b * VOCAB, lmg_reduce(q), lane);
  if (lane == 0) {
    if (b == 0) *st.selp = 0u;
    if (ri.x >= 0) {
      st.rowstep[b] = rx.x;  // the step being committed (argmax_commit advances it)
      argmax_commit(st, b, ri, r);
    }
  }
}

// Test hook (lvx_select_probe): the greedy select of each production path over given logits
// (st.logits). path 0: ar_argmax_kernel; 1: per-block lm_head granules formed as OUT 9 forms them
// (8 consecutive vocabulary rows per block), reduced by ar_select_final_kernel (lmg_reduce +
// softmax_ties, the same code as the deferred select in c_attn layer 0, IN 5); 2: the batched
// deferred select, ar_embed_select_kernel.
__global__ void ar_select_probe_prep_kernel(ArState st, int B, int path) {
  const int blk = blockIdx.x, b = threadIdx.x;
  if (b >= B) return;
  if (path == 3 && blk < LM8_BLOCKS) {  // as ar_mfma_ln_kernel OUT 3 forms them: 16 vocabulary rows per block
    Best r{-INFINITY, -INFINITY, 0x7fffffff};
    for (int n = blk * 16; n < blk * 16 + 16; ++n) r = best_merge(r, Best{st.logits[(size_t)b * VOCAB + n], -INFINITY, n});
    reinterpret_cast<u64x2_t*>(st.lmbest)[(size_t)blk * LM8_ROWS + b] = lm_granule(r);
  }
  if (path == 1) {
    Best r{-INFINITY, -INFINITY, 0x7fffffff};
    for (int n = blk * 8; n < blk * 8 + 8; ++n) r = best_merge(r, Best{st.logits[(size_t)b * VOCAB + n], -INFINITY, n});
    u64x2_t g;
    g.x = ((unsigned long long)(unsigned)r.i << 32) | __float_as_uint(r.v);
    g.y = (unsigned long long)__float_as_uint(r.v2);
    reinterpret_cast<u64x2_t*>(st.lmbest)[(size_t)blk * 4 + b] = g;
  }
  if (blk == 0) {
    st.selrow[b] = 1u;
    if (b == 0) *st.selp = 1u;
  }
}

int ar_select_probe(const ArWeights& w, const ArState& st, int B, int path, hipStream_t s) {
  if (path < 0 || path > 3 || B < 1 || (path == 1 && B > 4) || (path == 3 && B > LM8_ROWS)) return -1;
  hipLaunchKernelGGL(ar_rowinfo_init_kernel, dim3((B + 63) / 64), dim3(64), 0, s, st, B);
  hipLaunchKernelGGL(ar_select_probe_prep_kernel, dim3(LM_SEL_BLOCKS), dim3(64), 0, s, st, B, path);
  if (path == 0) {
    hipLaunchKernelGGL(ar_argmax_kernel, dim3(B), dim3(256), 0, s, st);
  } else if (path == 1) {
    hipLaunchKernelGGL(ar_select_final_kernel, dim3(B), dim3(64), 0, s, st);
  } else if (path == 3) {
    hipLaunchKernelGGL(ar_select8_probe_kernel, dim3(B), dim3(64), 0, s, st);
  } else {
    GemvArgs a = make_args<float>(w, st, LVX_DTYPE_F32, B, nullptr);
    a.ln_w = w.ln1[0];
    hipLaunchKernelGGL(ar_embed_select_kernel<>, dim3(B), dim3(256), 0, s, a);
  }
  return 0;
}

void ar_launch_steps_end(const ArState& st, int wdtype, int B, hipStream_t s) {
  const bool d = wdtype == LVX_DTYPE_BF16 ? defer_select<bf16_t>(B) : defer_select<float>(B);
  const bool db = wdtype == LVX_DTYPE_BF16 ? defer_select_batched<bf16_t>(B) : defer_select_batched<float>(B);
  if (d) hipLaunchKernelGGL(ar_select_final_kernel, dim3(B), dim3(64), 0, s, st);
  else if (db) hipLaunchKernelGGL(ar_argmax_kernel, dim3(B), dim3(256), 0, s, st);
}

// ---------------------------------------------------------------------------------
// gathers exposed through the drop-in members
// ---------------------------------------------------------------------------------
// An id outside the table raises IndexError in the reference (nn.Embedding): here the gather is
// clamped (never faults) and error bit 4 is set, reported by lvx_check_errors as LVX_E_INDEX.
__global__ void text_embed_kernel(const float* __restrict__ table, const int64_t* __restrict__ ids, int n,
                                  float* __restrict__ out, int32_t* err) {
  const int r = blockIdx.x;
  const int64_t raw = ids[r];
  if ((raw < 0 || raw >= TEXT_VOCAB) && threadIdx.x == 0) atomicOr(err, 4);
  const int64_t id = min(max(raw, (int64_t)0), (int64_t)(TEXT_VOCAB - 1));
  out[(size_t)r * TEXT_DIM + threadIdx.x] = table[(size_t)id * TEXT_DIM + threadIdx.x];
}

// codes [B][L] -> feats [B][512][L]
__global__ void codes_to_features_kernel(const float* __restrict__ cb, const int64_t* __restrict__ codes, int L,
                                         float* __restrict__ feats, int32_t* err) {
  const int b = blockIdx.y, c0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  for (int t = tid; t < L; t += 256) {
    const int64_t raw = codes[(size_t)b * L + t];
    if ((raw < 0 || raw > 4095) && blockIdx.x == 0) atomicOr(err, 4);  // reference: IndexError
    const int64_t code = min(max(raw, (int64_t)0), (int64_t)4095);
    for (int c = c0; c < c0 + 64; ++c) feats[((size_t)b * SPEECH_DIM + c) * L + t] = cb[(size_t)code * SPEECH_DIM + c];
  }
}

__global__ void set_slot_kernel(int32_t* pos, int32_t* prev, int slot, int p, int tok) {
  pos[slot] = p;
  prev[slot] = tok;
}

void ar_launch_rowinfo_init(const ArState& st, int B, hipStream_t s) {
  hipLaunchKernelGGL(ar_rowinfo_init_kernel, dim3((B + 63) / 64), dim3(64), 0, s, st, B);
}

void launch_set_slot(int32_t* pos, int32_t* prev, int slot, int p, int tok, hipStream_t s) {
  hipLaunchKernelGGL(set_slot_kernel, dim3(1), dim3(1), 0, s, pos, prev, slot, p, tok);
}

// Take (read and clear, one atomic per word) the masked bits of the AR word words[0] and the codec
// word words[1]: bits set meanwhile by kernels of another stream stay in their word for the next take.
// out = AR bits | codec bits << 16.
__global__ void err_take_kernel(int32_t* words, int32_t mask_ar, int32_t mask_codec, int32_t* out) {
  const int32_t a = mask_ar ? (atomicAnd(words, ~mask_ar) & mask_ar) : 0;
  const int32_t c = mask_codec ? (atomicAnd(words + 1, ~mask_codec) & mask_codec) : 0;
  out[0] = a | (c << 16);
}

void launch_err_take(int32_t* words, int mask_ar, int mask_codec, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(err_take_kernel, dim3(1), dim3(1), 0, s, words, mask_ar, mask_codec, out);
}

void launch_text_embed(const float* table, const int64_t* ids, int n, float* out, int32_t* err, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(text_embed_kernel, dim3(n), dim3(TEXT_DIM), 0, s, table, ids, n, out, err);
}

void launch_codes_to_features(const float* codebook, const int64_t* codes, int B, int L, float* feats,
                              int32_t* err, hipStream_t s) {
  if (B > 0 && L > 0)
    hipLaunchKernelGGL(codes_to_features_kernel, dim3(SPEECH_DIM / 64, B), dim3(256), 0, s, codebook, codes, L,
                       feats, err);
}

}  // namespace lvx

#ifdef LVX_TIMING
// timing build only (tools/step_timeline.py): copy / clear the step timeline records
extern "C" int lvx_debug_timeline(void* dst, size_t bytes, int clear) {
  if (bytes > sizeof(lvx::g_lvx_ts)) bytes = sizeof(lvx::g_lvx_ts);
  if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(lvx::g_lvx_ts), bytes) != hipSuccess) return -3;
  if (clear) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(lvx::g_lvx_ts)) != hipSuccess) return -3;
    if (hipMemset(p, 0, sizeof(lvx::g_lvx_ts)) != hipSuccess) return -3;
  }
  return (int)bytes;
}
#endif
