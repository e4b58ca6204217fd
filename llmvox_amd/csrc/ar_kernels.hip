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

namespace lvx {

// ---------------------------------------------------------------------------------
// embed: a2-a4 (+ wpe add of src/model.py:206-212, only the last row is ever used)
// ---------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void ar_embed_kernel(ArState st, const float* __restrict__ text_table,
                                                       const float* __restrict__ codebook,
                                                       const float* __restrict__ wpe,
                                                       const float* __restrict__ emb_row, int slot_arg,
                                                       int pos_arg) {
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  if (MODE == 1) {
    if (tid == 0) {
      st.slots[0] = slot_arg;
      st.pos[slot_arg] = pos_arg;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      int i = tid + 256 * j;
      st.x[i] = emb_row[i] + wpe[(size_t)pos_arg * D + i];
    }
    return;
  }
  const int s = st.slots[b];
  if (s < 0) {  // idle row: zero input, nothing else of the row is stored
#pragma unroll
    for (int j = 0; j < 3; ++j) st.x[(size_t)b * D + tid + 256 * j] = 0.f;
    return;
  }
  int p = st.pos[s];
  if (p >= st.max_pos) {
    if (tid == 0) atomicOr(st.err, 1);
    p = st.max_pos - 1;
  }
  int step = st.rowstep[b];
  if (step >= st.plan_stride) {  // ran past the end of the plan: flag, never read out of bounds
    if (tid == 0) atomicOr(st.err, 2);
    step = st.plan_stride - 1;
  }
  const int tok = min(max(st.text_plan[(size_t)b * st.plan_stride + step], 0), TEXT_VOCAB - 1);
  const int prev = min(max(st.prev[s], 0), VOCAB - 1);
  float v[3];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    int i = tid + 256 * j;
    float e;
    if (i < TEXT_DIM) e = text_table[(size_t)tok * TEXT_DIM + i];
    else e = (p == 0) ? 0.f : codebook[(size_t)prev * SPEECH_DIM + (i - TEXT_DIM)];
    v[j] = e;
    ss += e * e;
  }
  ss = block_sum<256>(ss, red);
  const float den = fmaxf(sqrtf(ss), 1e-8f);  // F.normalize: x / max(||x||_2, eps)
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    int i = tid + 256 * j;
    st.x[(size_t)b * D + i] = v[j] / den + wpe[(size_t)p * D + i];
  }
}

// ---------------------------------------------------------------------------------
// GEMV family: out[b][n] = sum_k W[n][k] * in[b][k]   (W row-major [N][K], TW in {f32,bf16})
//   IN  0: in = LayerNorm(x[b]) * ln_w   (eps 1e-5, no bias; src/model.py:37-38)
//   IN  1: in = h[b] (fp32)
//   IN  2: in = merge of the split-KV attention partials (flash-decoding combine)
//   OUT 0: c_attn: q -> st.q, k/v -> KV cache at the slot's position
//   OUT 1: residual: x[b][n] += out
//   OUT 2: h[b][n] = gelu_tanh(out)
//   OUT 3: logits: dst[b][n] = out
// 4 waves per block, RPW rows per wave; lanes split K in 4-element chunks (coalesced 1 KB /
// 512 B per wave-instruction), per-row partials reduced across the wave with DPP shuffles.
// ---------------------------------------------------------------------------------
struct GemvArgs {
  ArState st;
  const void* W;
  int N;
  int B;
  int layer;
  const float* ln_w;
  float* dst;
  int kv_bf16;
};

template <int K, int BG, int IN>
__device__ __forceinline__ void gemv_stage_input(const GemvArgs& a, float* xs, int g0, int bg, float* red) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (IN == 0) {
    // one wave per row: two-pass mean/var in fp32
    for (int bb = wave; bb < bg; bb += 4) {
      const float* xr = a.st.x + (size_t)(g0 + bb) * D;
      float4 v[3];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        v[j] = *reinterpret_cast<const float4*>(xr + j * 256 + lane * 4);
        s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
      }
      const float mean = wave_sum(s) * (1.0f / D);
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        float dx = v[j].x - mean, dy = v[j].y - mean, dz = v[j].z - mean, dw = v[j].w - mean;
        q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
      }
      const float var = wave_sum(q) * (1.0f / D);
      const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int k = j * 256 + lane * 4;
        const float4 g = *reinterpret_cast<const float4*>(a.ln_w + k);
        float4 o = make_float4((v[j].x - mean) * rstd * g.x, (v[j].y - mean) * rstd * g.y,
                               (v[j].z - mean) * rstd * g.z, (v[j].w - mean) * rstd * g.w);
        *reinterpret_cast<float4*>(xs + bb * K + k) = o;
      }
    }
  } else if (IN == 1) {
    for (int e = tid * 4; e < bg * K; e += 256 * 4) {
      *reinterpret_cast<float4*>(xs + e) = *reinterpret_cast<const float4*>(a.st.h + (size_t)g0 * K + e);
    }
  } else {
    // merge NSPLIT partials per (b, head): y = sum_s e^{m_s-M} o_s / sum_s e^{m_s-M} l_s
    for (int e = tid; e < bg * D; e += 256) {
      const int bb = e / D, c = e - bb * D;
      const int b = g0 + bb;
      const int head = c / HD, d = c - head * HD;
      const int s = a.st.slots[b];
      if (s < 0) { xs[bb * K + c] = 0.f; continue; }
      const int t = min(a.st.pos[s], a.st.max_pos - 1) + 1;
      const int ns = min(NSPLIT, (t + 63) / 64);
      const float* ml = a.st.part_ml + ((size_t)(b * N_HEAD + head) * NSPLIT) * 2;
      const float* po = a.st.part_o + ((size_t)(b * N_HEAD + head) * NSPLIT) * HD + d;
      float M = -INFINITY;
      for (int i = 0; i < ns; ++i) M = fmaxf(M, ml[2 * i]);
      float num = 0.f, den = 0.f;
      for (int i = 0; i < ns; ++i) {
        const float m = ml[2 * i];
        const float f = (m == -INFINITY) ? 0.f : expf(m - M);
        num += f * po[(size_t)i * HD];
        den += f * ml[2 * i + 1];
      }
      xs[bb * K + c] = num / den;
    }
  }
  (void)red;
}

template <typename TW, int K, int BG, int IN, int OUT, int RPW>
__global__ __launch_bounds__(256) void ar_gemv_kernel(GemvArgs a) {
  __shared__ __attribute__((aligned(16))) float xs[BG * K];
  __shared__ float red[8];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = (blockIdx.x * 4 + wave) * RPW;
  const TW* __restrict__ W = reinterpret_cast<const TW*>(a.W);
  for (int g0 = 0; g0 < a.B; g0 += BG) {
    const int bg = min(BG, a.B - g0);
    __syncthreads();
    gemv_stage_input<K, BG, IN>(a, xs, g0, bg, red);
    __syncthreads();
    float acc[RPW][BG];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int bb = 0; bb < BG; ++bb) acc[r][bb] = 0.f;
#pragma unroll 3
    for (int it = 0; it < K / 256; ++it) {
      const int k = it * 256 + lane * 4;
      float4 w[RPW];
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const int n = row0 + r;
        w[r] = (n < a.N) ? Ld<TW>::load4(W + (size_t)n * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int bb = 0; bb < BG; ++bb) {
        if (bb < bg) {
          const float4 xv = *reinterpret_cast<const float4*>(xs + bb * K + k);
#pragma unroll
          for (int r = 0; r < RPW; ++r)
            acc[r][bb] += (w[r].x * xv.x + w[r].y * xv.y) + (w[r].z * xv.z + w[r].w * xv.w);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = row0 + r;
#pragma unroll
      for (int bb = 0; bb < BG; ++bb) {
        if (bb >= bg) continue;
        const float v = wave_sum(acc[r][bb]);
        if (n >= a.N || lane != ((r * BG + bb) & 63)) continue;
        const int b = g0 + bb;
        if (OUT == 0) {
          if (n < D) {
            a.st.q[(size_t)b * D + n] = v;
          } else {
            const int c = (n - D) % D, which = (n - D) / D;
            const int head = c / HD, d = c - head * HD;
            const int s = a.st.slots[b];
            if (s < 0) continue;
            const int p = min(a.st.pos[s], a.st.max_pos - 1);
            const size_t idx =
                ((((size_t)a.layer * a.st.max_streams + s) * N_HEAD + head) * a.st.max_pos + p) * HD + d;
            if (a.kv_bf16) reinterpret_cast<bf16_t*>(which ? a.st.vc : a.st.kc)[idx] = f32_to_bf16(v);
            else reinterpret_cast<float*>(which ? a.st.vc : a.st.kc)[idx] = v;
          }
        } else if (OUT == 1) {
          a.st.x[(size_t)b * D + n] += v;
        } else if (OUT == 2) {
          a.st.h[(size_t)b * DFF + n] = gelu_tanh(v);
        } else {
          a.dst[(size_t)b * a.N + n] = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// split-KV decode attention (src/model.py:79-95 with T_q = 1, is_causal False):
// grid (NSPLIT/4, 8 heads, B), one wave per split. Lane = key for the scores (each lane
// reads its key's 96-element row), online softmax per wave, P.V with lane = output dim.
// Partials (m, l, o) are merged in the c_proj prologue.
// ---------------------------------------------------------------------------------
template <typename TKV>
__global__ __launch_bounds__(256) void ar_attn_kernel(ArState st, int layer) {
  __shared__ __attribute__((aligned(16))) float qs[HD];
  const int head = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int s = st.slots[b];
  if (s < 0) return;
  const int t = min(st.pos[s], st.max_pos - 1) + 1;
  if (tid < HD) qs[tid] = st.q[(size_t)b * D + head * HD + tid] * 0.10206207261596575f;  // 1/sqrt(96)
  __syncthreads();
  const int ns = min(NSPLIT, (t + 63) / 64);
  const int sp = blockIdx.x * 4 + wave;
  if (sp >= ns) return;
  const int chunk = (t + ns - 1) / ns;
  const int k0 = sp * chunk, k1 = min(t, k0 + chunk);
  const size_t base = (((size_t)layer * st.max_streams + s) * N_HEAD + head) * st.max_pos;
  const TKV* __restrict__ K = reinterpret_cast<const TKV*>(st.kc) + base * HD;
  const TKV* __restrict__ V = reinterpret_cast<const TKV*>(st.vc) + base * HD;
  float m = -INFINITY, l = 0.f, o0 = 0.f, o1 = 0.f;
  for (int kb = k0; kb < k1; kb += 64) {
    const int key = kb + lane;
    const bool valid = key < k1;
    float sc = -INFINITY;
    if (valid) {
      const TKV* kr = K + (size_t)key * HD;
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int d = 0; d < HD; d += 8) {
        const float4 k4a = Ld<TKV>::load4(kr + d);
        const float4 k4b = Ld<TKV>::load4(kr + d + 4);
        const float4 qa = *reinterpret_cast<const float4*>(qs + d);
        const float4 qb = *reinterpret_cast<const float4*>(qs + d + 4);
        a0 += (qa.x * k4a.x + qa.y * k4a.y) + (qa.z * k4a.z + qa.w * k4a.w);
        a1 += (qb.x * k4b.x + qb.y * k4b.y) + (qb.z * k4b.z + qb.w * k4b.w);
      }
      sc = a0 + a1;
    }
    const float mt = wave_max(sc);
    const float mn = fmaxf(m, mt);
    const float p = valid ? expf(sc - mn) : 0.f;
    const float alpha = (m == -INFINITY) ? 0.f : expf(m - mn);
    l = l * alpha + wave_sum(p);
    o0 *= alpha;
    o1 *= alpha;
    const int nk = min(64, k1 - kb);
    for (int j = 0; j < nk; ++j) {
      const float pj = __shfl(p, j, 64);
      const TKV* vr = V + (size_t)(kb + j) * HD;
      o0 += pj * Ld<TKV>::load1(vr + lane);
      if (lane < HD - 64) o1 += pj * Ld<TKV>::load1(vr + 64 + lane);
    }
    m = mn;
  }
  float* po = st.part_o + ((size_t)(b * N_HEAD + head) * NSPLIT + sp) * HD;
  po[lane] = o0;
  if (lane < HD - 64) po[64 + lane] = o1;
  if (lane == 0) {
    float* ml = st.part_ml + ((size_t)(b * N_HEAD + head) * NSPLIT + sp) * 2;
    ml[0] = m;
    ml[1] = l;
  }
}

// ---------------------------------------------------------------------------------
// greedy select (streaming_server.py:342-347): argmax with first-index ties, top1-top2
// margin, then the slot's prev token / position advance.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ar_argmax_kernel(ArState st) {
  __shared__ float sv[256], sv2[256];
  __shared__ int si[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* lg = st.logits + (size_t)b * VOCAB;
  float bv = -INFINITY, bv2 = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = tid; i < VOCAB; i += 256) {
    const float v = lg[i];
    if (v > bv) { bv2 = bv; bv = v; bi = i; }
    else if (v > bv2) bv2 = v;
  }
  sv[tid] = bv; sv2[tid] = bv2; si[tid] = bi;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      float av = sv[tid], av2 = sv2[tid]; int ai = si[tid];
      float cv = sv[tid + off], cv2 = sv2[tid + off]; int ci = si[tid + off];
      const bool c_better = (cv > av) || (cv == av && ci < ai);
      float nv, nv2; int ni;
      if (c_better) { nv = cv; ni = ci; nv2 = fmaxf(cv2, av); }
      else { nv = av; ni = ai; nv2 = fmaxf(av2, cv); }
      sv[tid] = nv; sv2[tid] = nv2; si[tid] = ni;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const int s = st.slots[b];
    if (s < 0) return;
    const int j = st.rowstep[b];
    if (j >= st.plan_stride) return;  // flagged by the embed kernel
    st.tok_plan[(size_t)b * st.plan_stride + j] = si[0];
    if (st.margin_plan) st.margin_plan[(size_t)b * st.plan_stride + j] = sv[0] - sv2[0];
    st.prev[s] = si[0];
    st.pos[s] = st.pos[s] + 1;
    st.rowstep[b] = j + 1;
  }
}

// ---------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------
template <typename TW, int K, int IN, int OUT, int RPW>
static void launch_gemv_bg(const GemvArgs& a, hipStream_t s) {
  const int rows_per_block = 4 * RPW;
  dim3 grid((a.N + rows_per_block - 1) / rows_per_block);
  constexpr int BGMAX = (K == 768) ? 16 : 4;
  if (a.B <= 1) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, 1, IN, OUT, RPW>), grid, dim3(256), 0, s, a);
  else if (a.B <= 2) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, 2, IN, OUT, RPW>), grid, dim3(256), 0, s, a);
  else if (a.B <= 4 || BGMAX == 4) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, 4, IN, OUT, RPW>), grid, dim3(256), 0, s, a);
  else if (a.B <= 8) hipLaunchKernelGGL((ar_gemv_kernel<TW, K, (BGMAX >= 8 ? 8 : 4), IN, OUT, RPW>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((ar_gemv_kernel<TW, K, BGMAX, IN, OUT, RPW>), grid, dim3(256), 0, s, a);
}

template <typename TW>
static void ar_layers(const ArWeights& w, const ArState& st, int kvdtype, int B, float* logits_dst,
                      hipStream_t s) {
  GemvArgs a{};
  a.st = st;
  a.B = B;
  a.kv_bf16 = kvdtype == LVX_DTYPE_BF16;
  for (int l = 0; l < N_LAYER; ++l) {
    a.layer = l;
    // LN1 + c_attn (+ KV append)
    a.W = w.w_attn[l]; a.N = 3 * D; a.ln_w = w.ln1[l];
    launch_gemv_bg<TW, 768, 0, 0, 2>(a, s);
    if (kvdtype == LVX_DTYPE_BF16)
      hipLaunchKernelGGL((ar_attn_kernel<bf16_t>), dim3(NSPLIT / 4, N_HEAD, B), dim3(256), 0, s, st, l);
    else
      hipLaunchKernelGGL((ar_attn_kernel<float>), dim3(NSPLIT / 4, N_HEAD, B), dim3(256), 0, s, st, l);
    a.W = w.w_aproj[l]; a.N = D;
    launch_gemv_bg<TW, 768, 2, 1, 1>(a, s);
    a.W = w.w_fc[l]; a.N = DFF; a.ln_w = w.ln2[l];
    launch_gemv_bg<TW, 768, 0, 2, 2>(a, s);
    a.W = w.w_mproj[l]; a.N = D;
    launch_gemv_bg<TW, 3072, 1, 1, 1>(a, s);
  }
  a.W = w.w_lm; a.N = VOCAB; a.ln_w = w.lnf; a.dst = logits_dst;
  launch_gemv_bg<TW, 768, 0, 3, 2>(a, s);
}

void ar_launch_step(const ArWeights& w, const ArState& st, int wdtype, int kvdtype, int B, int mode,
                    const float* emb_row, int slot, int pos, float* logits_out, hipStream_t s) {
  if (mode == 0)
    hipLaunchKernelGGL((ar_embed_kernel<0>), dim3(B), dim3(256), 0, s, st, w.text_table, w.codebook, w.wpe,
                       nullptr, 0, 0);
  else
    hipLaunchKernelGGL((ar_embed_kernel<1>), dim3(1), dim3(256), 0, s, st, w.text_table, w.codebook, w.wpe,
                       emb_row, slot, pos);
  float* dst = mode == 0 ? st.logits : logits_out;
  if (wdtype == LVX_DTYPE_BF16) ar_layers<bf16_t>(w, st, kvdtype, B, dst, s);
  else ar_layers<float>(w, st, kvdtype, B, dst, s);
  if (mode == 0) hipLaunchKernelGGL(ar_argmax_kernel, dim3(B), dim3(256), 0, s, st);
}

// ---------------------------------------------------------------------------------
// gathers exposed through the drop-in members
// ---------------------------------------------------------------------------------
__global__ void text_embed_kernel(const float* __restrict__ table, const int64_t* __restrict__ ids, int n,
                                  float* __restrict__ out) {
  const int r = blockIdx.x;
  const int64_t id = min(max(ids[r], (int64_t)0), (int64_t)(TEXT_VOCAB - 1));  // clamp: never fault
  out[(size_t)r * TEXT_DIM + threadIdx.x] = table[(size_t)id * TEXT_DIM + threadIdx.x];
}

// codes [B][L] -> feats [B][512][L]
__global__ void codes_to_features_kernel(const float* __restrict__ cb, const int64_t* __restrict__ codes, int L,
                                         float* __restrict__ feats) {
  const int b = blockIdx.y, c0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
  for (int t = tid; t < L; t += 256) {
    const int64_t code = min(max(codes[(size_t)b * L + t], (int64_t)0), (int64_t)4095);
    for (int c = c0; c < c0 + 64; ++c) feats[((size_t)b * SPEECH_DIM + c) * L + t] = cb[(size_t)code * SPEECH_DIM + c];
  }
}

__global__ void set_slot_kernel(int32_t* pos, int32_t* prev, int slot, int p, int tok) {
  pos[slot] = p;
  prev[slot] = tok;
}

void launch_set_slot(int32_t* pos, int32_t* prev, int slot, int p, int tok, hipStream_t s) {
  hipLaunchKernelGGL(set_slot_kernel, dim3(1), dim3(1), 0, s, pos, prev, slot, p, tok);
}

void launch_text_embed(const float* table, const int64_t* ids, int n, float* out, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(text_embed_kernel, dim3(n), dim3(TEXT_DIM), 0, s, table, ids, n, out);
}

void launch_codes_to_features(const float* codebook, const int64_t* codes, int B, int L, float* feats,
                              hipStream_t s) {
  if (B > 0 && L > 0)
    hipLaunchKernelGGL(codes_to_features_kernel, dim3(SPEECH_DIM / 64, B), dim3(256), 0, s, codebook, codes, L,
                       feats);
}

}  // namespace lvx
