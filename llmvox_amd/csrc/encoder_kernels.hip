// WavTokenizer encoder (encode_infer) for CDNA4 (gfx950), fp32.
//
// Reference: WavTokenizer/decoder/pretrained.py:185-190 -> feature_extractors.py:122-133: the
// SEANet encoder (encoder/modules/seanet.py:94-143; SConv1d conv.py:54-96,195-211; SLSTM lstm.py:31-39)
// and the 1-codebook quantizer (quantization/vq.py:115-140, core_vq.py:171-231,245-276).
//
// Activations are time-major [stream][frame][channel] as in the decoder. Every SConv1d is one
// launch of enc_conv_kernel: implicit GEMM over (tap, input channel), the reflect padding of
// SConv1d (incl. the extra right padding that makes the last strided window full, and the zero
// extension of inputs shorter than the pad) resolved in the operand loader, the ELU that precedes
// most convs applied there too, bias and the residual-block sum as the epilogue. The LSTM's input
// projections (x W_ih^T + b_ih over all frames) and the quantiser's scores (x . e over the 4,096
// codes) are the same kernel with a 1-tap "conv". The recurrence runs one launch per (layer, frame):
// a wave per hidden unit computes its four gate rows of h W_hh^T for every stream and updates (c, h)
// in PyTorch's order. The quantiser picks argmax of -((|x|^2 - 2 x.e) + |e|^2), first index on ties
// (core_vq.py:175-183), and writes the codes and the codebook rows (features, [B][512][T]).
#include "lvx_internal.h"

#pragma clang fp contract(off)

namespace lvx {

struct EncConvArgs {
  const float* x;  // [B][L][cin]
  const float* w;  // [cout][k][cin] (tap-major)
  const float* bias;  // [cout] or null
  const float* res;   // [B][T][cout] added after the bias, or null
  float* y;           // [B][T][cout]
  int B, L, T, cin, cout, k, stride, dil;
  int pl, lext;  // left reflect pad; reflect domain length (L + zero extension)
  int elu;
};

__device__ __forceinline__ float elu1(float v) { return v > 0.f ? v : expm1f(v); }

// 64 output frames x 64 output channels per block, 256 threads of 4 x 4 outputs, K in chunks of
// 16 (one tap, 16 input channels) through LDS.
__global__ __launch_bounds__(256) void enc_conv_kernel(EncConvArgs a) {
  __shared__ float xs[16][64 + 4];
  __shared__ float ws[16][64 + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int M = a.B * a.T;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int kc_per_tap = (a.cin + 15) / 16, nk = a.k * kc_per_tap;
  // loader: thread -> (row r = tid / 4, 4 channels c4 = (tid & 3) * 4) of the 64 x 16 chunk
  const int lr = tid >> 2, lc = (tid & 3) * 4;
  const int m = min(m0 + lr, M - 1);
  const int b = m / a.T, to = m - b * a.T;
  const int n = min(n0 + lr, a.cout - 1);
  float acc[4][4] = {};
  for (int kc = 0; kc < nk; ++kc) {
    const int j = kc / kc_per_tap, c0 = (kc - j * kc_per_tap) * 16 + lc;
    // input frame of tap j (SConv1d reflect padding, conv.py:79-96,195-211)
    int i = to * a.stride + j * a.dil - a.pl;
    if (i < 0) i = -i;
    if (i >= a.lext) i = 2 * (a.lext - 1) - i;
    const bool inl = i < a.L;
    const float* xp = a.x + ((size_t)b * a.L + (inl ? i : 0)) * a.cin;
    const float* wp = a.w + ((size_t)n * a.k + j) * a.cin;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c0 + e;
      float xv = (inl && c < a.cin) ? xp[c] : 0.f;
      if (a.elu) xv = elu1(xv);
      xs[lc + e][lr] = xv;
      ws[lc + e][lr] = c < a.cin ? wp[c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float xv[4], wv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) xv[r] = xs[kk][ty * 4 + r];
#pragma unroll
      for (int q = 0; q < 4; ++q) wv[q] = ws[kk][tx * 4 + q];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[r][q] = fmaf(xv[r], wv[q], acc[r][q]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int mo = m0 + ty * 4 + r;
    if (mo >= M) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int co = n0 + tx * 4 + q;
      if (co >= a.cout) continue;
      float v = acc[r][q] + (a.bias ? a.bias[co] : 0.f);
      if (a.res) v = a.res[(size_t)mo * a.cout + co] + v;
      a.y[(size_t)mo * a.cout + co] = v;
    }
  }
}

// One LSTM step of one layer for every stream (aten LSTMCell order: gates = (h W_hh^T + b_hh) +
// (x W_ih^T + b_ih); i, f, o sigmoid, g tanh; c' = f c + i g; h' = o tanh(c')). A wave per hidden
// unit u: its four gate rows u + 512 q of W_hh against h_{t-1} of every stream (8 values per lane),
// DPP/shuffle sums, then lane b updates stream b. y[b][t][u] = h' (+ skip[b][t][u] at the last layer).
constexpr int ENC_H = 512;
__global__ __launch_bounds__(256) void enc_lstm_step_kernel(const float* __restrict__ gin, const float* __restrict__ whh,
                                                            const float* __restrict__ bhh, const float* __restrict__ hprev,
                                                            float* __restrict__ hnext, float* __restrict__ cst,
                                                            float* __restrict__ y, const float* __restrict__ skip, int B,
                                                            int T, int t) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u = blockIdx.x * 4 + wave;
  float w[4][8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4* p = reinterpret_cast<const float4*>(whh + (size_t)(q * ENC_H + u) * ENC_H + lane * 8);
    const float4 a = p[0], c = p[1];
    w[q][0] = a.x; w[q][1] = a.y; w[q][2] = a.z; w[q][3] = a.w;
    w[q][4] = c.x; w[q][5] = c.y; w[q][6] = c.z; w[q][7] = c.w;
  }
  for (int b0 = 0; b0 < B; b0 += 16) {
    float mine[4] = {0.f, 0.f, 0.f, 0.f};  // lane b - b0 keeps stream b's gate sums
    for (int b = b0; b < min(B, b0 + 16); ++b) {
      const float4* hp = reinterpret_cast<const float4*>(hprev + (size_t)b * ENC_H + lane * 8);
      const float4 h0 = hp[0], h1 = hp[1];
      const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) s = fmaf(w[q][e], hv[e], s);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == b - b0) mine[q] = s;
      }
    }
    const int b = b0 + lane;
    if (lane < 16 && b < B) {
      const float* g = gin + ((size_t)b * T + t) * (4 * ENC_H);
      float gate[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) gate[q] = (mine[q] + bhh[q * ENC_H + u]) + g[q * ENC_H + u];
      const float ig = 1.f / (1.f + expf(-gate[0]));
      const float fg = 1.f / (1.f + expf(-gate[1]));
      const float cg = tanhf(gate[2]);
      const float og = 1.f / (1.f + expf(-gate[3]));
      const float c = fg * cst[(size_t)b * ENC_H + u] + ig * cg;
      const float h = og * tanhf(c);
      cst[(size_t)b * ENC_H + u] = c;
      hnext[(size_t)b * ENC_H + u] = h;
      const size_t yi = ((size_t)b * T + t) * ENC_H + u;
      y[yi] = skip ? h + skip[yi] : h;
    }
  }
}

// Quantiser: row m of the scores s = x . e (4,096 codes) -> code = argmax of -((|x|^2 - 2 s) + |e|^2)
// (first index on ties, as torch's max), features[b][c][t] = codebook[code][c] (reference layout).
__global__ __launch_bounds__(256) void enc_vq_select_kernel(const float* __restrict__ emb, const float* __restrict__ s,
                                                            const float* __restrict__ esq, const float* __restrict__ cb,
                                                            int32_t* __restrict__ codes, float* __restrict__ feats, int T) {
  __shared__ float red_v[4];
  __shared__ int red_i[4];
  __shared__ float xsq_s;
  const int m = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (wave == 0) {
    float q = 0.f;
    for (int c = lane; c < 512; c += 64) {
      const float v = emb[(size_t)m * 512 + c];
      q = fmaf(v, v, q);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    if (lane == 0) xsq_s = q;
  }
  __syncthreads();
  const float xsq = xsq_s;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int n = tid; n < 4096; n += 256) {  // ascending per thread: strict > keeps the first index
    const float d = -((xsq - 2.f * s[(size_t)m * 4096 + n]) + esq[n]);
    if (d > best) { best = d; bi = n; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  if (lane == 0) { red_v[wave] = best; red_i[wave] = bi; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (red_v[w] > best || (red_v[w] == best && red_i[w] < bi)) { best = red_v[w]; bi = red_i[w]; }
    red_i[0] = bi;
    codes[m] = bi;
  }
  __syncthreads();
  const int code = red_i[0];
  const int b = m / T, t = m - b * T;
  for (int c = tid; c < 512; c += 256) feats[((size_t)b * 512 + c) * T + t] = cb[(size_t)code * 512 + c];
}

void enc_launch_conv(const float* x, const float* w, const float* bias, const float* res, float* y, int B, int L, int T,
                     int cin, int cout, int k, int stride, int dil, int pl, int lext, bool elu, hipStream_t s) {
  EncConvArgs a{x, w, bias, res, y, B, L, T, cin, cout, k, stride, dil, pl, lext, elu ? 1 : 0};
  dim3 grid((B * T + 63) / 64, (cout + 63) / 64);
  hipLaunchKernelGGL(enc_conv_kernel, grid, dim3(256), 0, s, a);
}

void enc_launch_lstm_step(const float* gin, const float* whh, const float* bhh, const float* hprev, float* hnext,
                          float* c, float* y, const float* skip, int B, int T, int t, hipStream_t s) {
  hipLaunchKernelGGL(enc_lstm_step_kernel, dim3(ENC_H / 4), dim3(256), 0, s, gin, whh, bhh, hprev, hnext, c, y, skip, B, T, t);
}

void enc_launch_vq(const float* emb, const float* scores, const float* esq, const float* cb, int32_t* codes,
                   float* feats, int B, int T, hipStream_t s) {
  hipLaunchKernelGGL(enc_vq_select_kernel, dim3(B * T), dim3(256), 0, s, emb, scores, esq, cb, codes, feats, T);
}

}  // namespace lvx
