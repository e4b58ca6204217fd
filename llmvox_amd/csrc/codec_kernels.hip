// WavTokenizer decoder (VocosBackbone + ISTFTHead) for CDNA4 (gfx950).
//
// Reference: WavTokenizer/decoder/pretrained.py:192-239, models.py:152-235, modules.py:8-86,
// heads.py:24-67, spectral_ops.py:7-75.
//
// Activations are kept time-major ([stream][frame][channel], channels contiguous) so that every
// Conv1d is an implicit GEMM whose A-tile rows are contiguous channel segments of neighbouring
// frames, and every 1x1 conv / Linear is a plain GEMM. GroupNorm(+swish) is applied while a GEMM
// stages its A tile (statistics come from a small reduction kernel), bias / GELU / layer-scale /
// residual are GEMM epilogues. GEMMs run on the fp32-input MFMA (v_mfma_f32_32x32x2_f32, exact
// fp32 products) — the reference is fp32 end to end; bf16 weights are widened on the way into LDS.
// The iSTFT is a per-frame LDS Stockham FFT (640-point complex, radices 4,4,4,2,5) wrapped as a
// 1280-point C2R, followed by a gather-form overlap-add with the window-envelope divide.
#include <algorithm>

#include "lvx_internal.h"

namespace lvx {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int CD = 768, CFF = 2304, CIN = 512, NFFT = 1280, HOPL = 320, NB = 641, GN_G = 32;

enum { A_PLAIN = 0, A_CONV = 1 };
enum { E_BIAS = 0, E_BIAS_GELU = 1, E_BIAS_GAMMA_RES = 2, E_BIAS_RES = 3, E_SCALE = 4 };

struct GemmArgs {
  const float* A; int lda;
  const void* W; int ldw;
  float* C; int ldc;
  const float* bias; const float* gamma; const float* res; int ldr;
  int M, N, K;
  long long sA, sW, sC, sR;  // per-batch strides (elements)
  int L;                     // frames per stream (rows per stream)
  int cin, taps;
  float alpha;
  int ksplit;                // >1: deterministic split-K through the fp32 workspace `ws`
  float* ws;
};

template <typename T> __device__ __forceinline__ void load8(const T* p, float* v);
template <> __device__ __forceinline__ void load8<float>(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <> __device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint4 pack_bf16x8(const float* v) {
  uint4 u;
  u.x = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
  u.y = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
  u.z = (uint32_t)f32_to_bf16(v[4]) | ((uint32_t)f32_to_bf16(v[5]) << 16);
  u.w = (uint32_t)f32_to_bf16(v[6]) | ((uint32_t)f32_to_bf16(v[7]) << 16);
  return u;
}

template <int EPI>
__device__ __forceinline__ float gemm_epi(const GemmArgs& g, const float* R, int row, int col, float v, float bias,
                                          float gam) {
  if (EPI == E_BIAS) return v + bias;
  if (EPI == E_BIAS_GELU) return gelu_erf(v + bias);
  if (EPI == E_BIAS_GAMMA_RES) return R[(size_t)row * g.ldr + col] + gam * (v + bias);
  if (EPI == E_BIAS_RES) return R[(size_t)row * g.ldr + col] + (v + bias);
  return v * g.alpha;
}

// 64x64 block tile, BK 32, 4 waves in 2x2 (each a 32x32 accumulator tile).
//   BF = true : operands rounded to bf16 into LDS, v_mfma_f32_32x32x16_bf16 (bf16 weight mode)
//   BF = false: fp32 operands, v_mfma_f32_32x32x2_f32 (exact fp32 products; parity mode)
// Software pipeline: the next k-tile's global loads are issued into registers before the MFMAs
// of the current LDS tile, so one memory latency is exposed per block, not one per k-step.
// A operand loaders: A_PLAIN (row-major, lda) or A_CONV (implicit Conv1d over time-major
// [stream][frame][cin] activations, taps centred, zero padding at every stream's edges).
// grid.z = batch x ksplit; with ksplit > 1 every split writes its raw partial tile to ws and
// gemm_splitk_reduce applies the epilogue (fixed summation order: deterministic).
constexpr int BM = 64, BN = 64, BK = 32;
constexpr int LDF = BK + 1;  // fp32 LDS row (conflict-free b32 column reads)
constexpr int LDH = BK + 8;  // bf16 LDS row (80 B)

template <bool BF, typename TB, int AMODE, int EPI>
__global__ __launch_bounds__(256) void gemm_mfma_kernel(GemmArgs g) {
  constexpr int LDSZ = BF ? (BM * LDH / 2) : (BM * LDF);  // in floats
  __shared__ __attribute__((aligned(16))) float As_[LDSZ];
  __shared__ __attribute__((aligned(16))) float Bs_[LDSZ];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int zb = blockIdx.z / g.ksplit, ks = blockIdx.z - zb * g.ksplit;
  const float* A = g.A + zb * g.sA;
  const TB* W = reinterpret_cast<const TB*>(g.W) + zb * g.sW;
  const int lrow = tid >> 2, lseg = (tid & 3) * 8;
  const int am = m0 + lrow, bn = n0 + lrow;
  int ab = 0, at = 0;
  if (AMODE == A_CONV && am < g.M) { ab = am / g.L; at = am - ab * g.L; }
  const int nkt = (g.K + BK - 1) / BK;
  const int kt_per = (nkt + g.ksplit - 1) / g.ksplit;
  const int kt0 = ks * kt_per, kt1 = min(nkt, kt0 + kt_per);

  auto load_tile = [&](int kt, float* av, float* bv) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { av[i] = 0.f; bv[i] = 0.f; }
    const int k = kt * BK + lseg;
    if (am < g.M) {
      if (AMODE == A_PLAIN) {
        const float* ap = A + (size_t)am * g.lda + k;
        if (k + 8 <= g.K) load8<float>(ap, av);
        else {
#pragma unroll
          for (int i = 0; i < 8; ++i) av[i] = (k + i < g.K) ? ap[i] : 0.f;
        }
      } else {
        const int tap = k / g.cin, c = k - tap * g.cin;
        const int tt = at + tap - (g.taps - 1) / 2;
        if (tt >= 0 && tt < g.L) load8<float>(A + ((size_t)ab * g.L + tt) * g.cin + c, av);
      }
    }
    if (bn < g.N) {
      const TB* wp = W + (size_t)bn * g.ldw + k;
      if (k + 8 <= g.K) load8<TB>(wp, bv);
      else {
#pragma unroll
        for (int i = 0; i < 8; ++i) bv[i] = (k + i < g.K) ? Ld<TB>::load1(wp + i) : 0.f;
      }
    }
  };

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float av[8], bv[8];
  if (kt0 < kt1) load_tile(kt0, av, bv);
  for (int kt = kt0; kt < kt1; ++kt) {
    __syncthreads();  // the previous tile's LDS reads are done
    if (BF) {
      bf16_t* As = reinterpret_cast<bf16_t*>(As_);
      bf16_t* Bs = reinterpret_cast<bf16_t*>(Bs_);
      *reinterpret_cast<uint4*>(As + lrow * LDH + lseg) = pack_bf16x8(av);
      *reinterpret_cast<uint4*>(Bs + lrow * LDH + lseg) = pack_bf16x8(bv);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        As_[lrow * LDF + lseg + i] = av[i];
        Bs_[lrow * LDF + lseg + i] = bv[i];
      }
    }
    __syncthreads();
    if (kt + 1 < kt1) load_tile(kt + 1, av, bv);  // in flight during the MFMAs below
    if (BF) {
      const bf16_t* As = reinterpret_cast<const bf16_t*>(As_);
      const bf16_t* Bs = reinterpret_cast<const bf16_t*>(Bs_);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(As + (wm * 32 + (lane & 31)) * LDH + kk + 8 * (lane >> 5));
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(Bs + (wn * 32 + (lane & 31)) * LDH + kk + 8 * (lane >> 5));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
      }
    } else {
      const float* Ar = As_ + (wm * 32 + (lane & 31)) * LDF + (lane >> 5);
      const float* Br = Bs_ + (wn * 32 + (lane & 31)) * LDF + (lane >> 5);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ar[kk], Br[kk], acc, 0, 0, 0);
    }
  }
  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= g.N) return;
  if (g.ksplit > 1) {  // raw partial tile -> ws[ks][zb][M][N]
    float* P = g.ws + ((size_t)ks * gridDim.z / g.ksplit + zb) * (size_t)g.M * g.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.M) P[(size_t)row * g.N + col] = acc[r];
    }
    return;
  }
  float* C = g.C + zb * g.sC;
  const float* R = g.res ? g.res + zb * g.sR : nullptr;
  const float bias = (EPI != E_SCALE && g.bias) ? g.bias[col] : 0.f;
  const float gam = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[col] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < g.M) C[(size_t)row * g.ldc + col] = gemm_epi<EPI>(g, R, row, col, acc[r], bias, gam);
  }
}

// sum the ksplit partials in split order, then the epilogue
template <int EPI>
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmArgs g, int batch) {
  const size_t MN = (size_t)g.M * g.N;
  const size_t total = MN * batch;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int zb = (int)(i / MN);
    const size_t e = i - (size_t)zb * MN;
    const int row = (int)(e / g.N), col = (int)(e - (size_t)row * g.N);
    float v = 0.f;
    for (int ks = 0; ks < g.ksplit; ++ks) v += g.ws[((size_t)ks * batch + zb) * MN + e];
    const float* R = g.res ? g.res + zb * g.sR : nullptr;
    const float bias = (EPI != E_SCALE && g.bias) ? g.bias[col] : 0.f;
    const float gam = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[col] : 0.f;
    g.C[zb * g.sC + (size_t)row * g.ldc + col] = gemm_epi<EPI>(g, R, row, col, v, bias, gam);
  }
}

static size_t g_ws_floats = 0;  // capacity of the split-K workspace (set by the front end)

template <bool BF, typename TB, int AMODE, int EPI>
static void gemm_launch(GemmArgs g, int batch, hipStream_t s) {
  const int tiles = ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM) * batch;
  const int nkt = (g.K + BK - 1) / BK;
  int ks = 1;
  // split K until the grid covers the chip (>= ~256 blocks), >= 4 k-tiles per split,
  // and the partials fit the workspace
  while (tiles * ks * 2 <= 320 && nkt / (ks * 2) >= 4 && (size_t)(ks * 2) * g.M * g.N * batch <= g_ws_floats) ks *= 2;
  g.ksplit = ks;
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, batch * ks);
  hipLaunchKernelGGL((gemm_mfma_kernel<BF, TB, AMODE, EPI>), grid, dim3(256), 0, s, g);
  if (ks > 1) {
    const size_t total = (size_t)g.M * g.N * batch;
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 2048);
    hipLaunchKernelGGL((gemm_splitk_reduce<EPI>), dim3(blocks), dim3(256), 0, s, g, batch);
  }
}

// weight GEMMs: bf16 weights -> bf16 MFMA; fp32 weights -> exact fp32 MFMA (parity mode)
template <typename TW, int AMODE, int EPI>
static void gemm_w(const GemmArgs& g, int batch, hipStream_t s) {
  if constexpr (sizeof(TW) == 2) gemm_launch<true, bf16_t, AMODE, EPI>(g, batch, s);
  else gemm_launch<false, float, AMODE, EPI>(g, batch, s);
}
// activation x activation GEMMs (AttnBlock scores / P.V): operands are fp32 in memory
template <typename TW, int EPI>
static void gemm_act(const GemmArgs& g, int batch, hipStream_t s) {
  if constexpr (sizeof(TW) == 2) gemm_launch<true, float, A_PLAIN, EPI>(g, batch, s);
  else gemm_launch<false, float, A_PLAIN, EPI>(g, batch, s);
}

// ---------------------------------------------------------------------------------
// GroupNorm (32 groups, eps 1e-6, affine) [+ swish] applied once per (stream, group): statistics
// (two-pass fp32) and the transformed output in one kernel, so the following conv / 1x1 GEMM
// reads a ready operand (decoder/models.py:15-16, 59-68, 109).
// ---------------------------------------------------------------------------------
template <bool SWISH>
__global__ __launch_bounds__(256) void gn_apply_kernel(const float* __restrict__ x, int L, const float* __restrict__ gw,
                                                       const float* __restrict__ gb, float* __restrict__ y) {
  __shared__ float red[4];
  const int gi = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  constexpr int CG = CD / GN_G;  // 24 channels
  const size_t off = (size_t)b * L * CD + gi * CG;
  const int n = L * CG;
  float s = 0.f;
  for (int e = tid; e < n; e += 256) {
    const int t = e / CG, c = e - t * CG;
    s += x[off + (size_t)t * CD + c];
  }
  const float mean = block_sum<256>(s, red) / n;
  float q = 0.f;
  for (int e = tid; e < n; e += 256) {
    const int t = e / CG, c = e - t * CG;
    const float d = x[off + (size_t)t * CD + c] - mean;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(block_sum<256>(q, red) / n + 1e-6f);
  for (int e = tid; e < n; e += 256) {
    const int t = e / CG, c = e - t * CG, ch = gi * CG + c;
    float v = (x[off + (size_t)t * CD + c] - mean) * rstd * gw[ch] + gb[ch];
    if (SWISH) v = swishf(v);
    y[off + (size_t)t * CD + c] = v;
  }
}

// ---------------------------------------------------------------------------------
// GroupNorm statistics (decoder/models.py:15-16: 32 groups, eps 1e-6): per (stream, group)
// mean and 1/sqrt(var + eps) over L frames x 24 channels, two-pass fp32.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gn_stats_kernel(const float* __restrict__ x, int L, float* __restrict__ stats) {
  __shared__ float red[4];
  const int gi = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  constexpr int CG = CD / GN_G;  // 24
  const float* xb = x + (size_t)b * L * CD + gi * CG;
  const int n = L * CG;
  float s = 0.f;
  for (int e = tid; e < n; e += 256) {
    const int t = e / CG, c = e - t * CG;
    s += xb[(size_t)t * CD + c];
  }
  const float mean = block_sum<256>(s, red) / n;
  float q = 0.f;
  for (int e = tid; e < n; e += 256) {
    const int t = e / CG, c = e - t * CG;
    const float d = xb[(size_t)t * CD + c] - mean;
    q += d * d;
  }
  const float var = block_sum<256>(q, red) / n;
  if (tid == 0) {
    stats[((size_t)b * GN_G + gi) * 2] = mean;
    stats[((size_t)b * GN_G + gi) * 2 + 1] = 1.0f / sqrtf(var + 1e-6f);
  }
}

// LayerNorm over 768 channels of a row held as 3 values per thread (256 threads)
__device__ __forceinline__ void row_ln(float (&v)[3], float eps, float* red) {
  float s = v[0] + v[1] + v[2];
  const float mean = block_sum<256>(s, red) * (1.0f / CD);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) { v[j] -= mean; q += v[j] * v[j]; }
  const float var = block_sum<256>(q, red) * (1.0f / CD);
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int j = 0; j < 3; ++j) v[j] *= rstd;
}

// end of pos_net: GroupNorm (pos_net.5, affine) then AdaLayerNorm (backbone.norm, id bw)
__global__ __launch_bounds__(256) void gn_adaln_kernel(const float* __restrict__ x, int L, const float* __restrict__ stats,
                                                       const float* __restrict__ gw, const float* __restrict__ gb,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       float* __restrict__ y) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x, b = m / L;
  float v[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j, gi = c / (CD / GN_G);
    v[j] = (x[(size_t)m * CD + c] - stats[((size_t)b * GN_G + gi) * 2]) * stats[((size_t)b * GN_G + gi) * 2 + 1] * gw[c] + gb[c];
  }
  row_ln(v, 1e-6f, red);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
    y[(size_t)m * CD + c] = v[j] * scale[c] + shift[c];
  }
}

// ConvNeXt prologue (modules.py:45-50): depthwise conv k7 pad 3 (+bias) then AdaLN
__global__ __launch_bounds__(256) void dwconv_adaln_kernel(const float* __restrict__ x, int L, const float* __restrict__ dw,
                                                           const float* __restrict__ dwb, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, float* __restrict__ y) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x, b = m / L, t = m - b * L;
  float v[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int tt = t + k - 3;
      if (tt >= 0 && tt < L) a += dw[c * 7 + k] * x[((size_t)b * L + tt) * CD + c];
    }
    v[j] = a + dwb[c];
  }
  row_ln(v, 1e-6f, red);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
    y[(size_t)m * CD + c] = v[j] * scale[c] + shift[c];
  }
}

// final_layer_norm (affine, eps 1e-6)
__global__ __launch_bounds__(256) void ln_affine_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bb, float* __restrict__ y) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  float v[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) v[j] = x[(size_t)m * CD + tid + 256 * j];
  row_ln(v, 1e-6f, red);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
    y[(size_t)m * CD + c] = v[j] * w[c] + bb[c];
  }
}

// features [B][512][L] -> [B*L][512]
__global__ void feats_transpose_kernel(const float* __restrict__ f, int L, float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, c0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, t = t0 + tx;
    tile[i][tx] = (t < L) ? f[((size_t)b * CIN + c) * L + t] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, c = c0 + tx;
    if (t < L) out[((size_t)b * L + t) * CIN + c] = tile[tx][i];
  }
}

// codes [B*L] -> [B*L][512]
__global__ void codes_gather_kernel(const float* __restrict__ cb, const int32_t* __restrict__ codes, float* __restrict__ out) {
  const int m = blockIdx.x;
  const int code = min(max(codes[m], 0), 4095);
  const float4 v = reinterpret_cast<const float4*>(cb + (size_t)code * CIN)[threadIdx.x];
  reinterpret_cast<float4*>(out + (size_t)m * CIN)[threadIdx.x] = v;
}

// v rows of qkv [B*L][2304] (cols 1536..2303) -> Vt [B][768][ldv]
__global__ void v_transpose_kernel(const float* __restrict__ qkv, int L, int ldv, float* __restrict__ vt) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, c0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, c = c0 + tx;
    tile[i][tx] = (t < L) ? qkv[((size_t)b * L + t) * CFF + 2 * CD + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, t = t0 + tx;
    if (t < ldv) vt[((size_t)b * CD + c) * ldv + t] = (t < L) ? tile[tx][i] : 0.f;
  }
}

// in-place row softmax of attention scores (already scaled), rows of length L, stride ld
__global__ __launch_bounds__(256) void softmax_rows_kernel(float* __restrict__ S, int L, int ld) {
  __shared__ float red[4];
  float* row = S + (size_t)blockIdx.x * ld;
  const int tid = threadIdx.x;
  float mx = -INFINITY;
  for (int j = tid; j < L; j += 256) mx = fmaxf(mx, row[j]);
  mx = wave_max(mx);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s = 0.f;
  for (int j = tid; j < L; j += 256) {
    const float e = expf(row[j] - mx);
    row[j] = e;
    s += e;
  }
  s = block_sum<256>(s, red);
  const float inv = 1.0f / s;
  for (int j = tid; j < L; j += 256) row[j] = row[j] * inv;
}

// ---------------------------------------------------------------------------------
// iSTFT (spectral_ops.py:33-75, padding "same"): per frame, X = min(exp(mag),100) e^{i p},
// irfft n=1280 (imag of DC / Nyquist ignored, 1/N scale) via a 640-point complex inverse FFT
// (Stockham, radices 4,4,4,2,5, LDS resident), times the periodic Hann window.
// tw[m] = e^{+2 pi i m / 1280}, m in [0,1280) (host double precision).
// ---------------------------------------------------------------------------------
constexpr int FM = 640;

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <int R>
__device__ __forceinline__ void stockham_pass(const float2* __restrict__ src, float2* __restrict__ dst, int Ns,
                                              const float2* __restrict__ tw) {
  // twiddle for e^{+2 pi i k r / (Ns R)} over the 640-point transform = tw[2 * (640/(Ns R)) * k * r]
  for (int j = threadIdx.x; j < FM / R; j += blockDim.x) {
    const int k = j % Ns;
    const int step = FM / (Ns * R);
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float2 x = src[j + r * (FM / R)];
      const int ti = (2 * step * k * r) % (2 * FM);
      v[r] = (r == 0) ? x : cmul(x, tw[ti]);
    }
    float2 y[R];
    if constexpr (R == 2) {
      y[0] = make_float2(v[0].x + v[1].x, v[0].y + v[1].y);
      y[1] = make_float2(v[0].x - v[1].x, v[0].y - v[1].y);
    } else if constexpr (R == 4) {
      const float2 a0 = make_float2(v[0].x + v[2].x, v[0].y + v[2].y);
      const float2 a1 = make_float2(v[0].x - v[2].x, v[0].y - v[2].y);
      const float2 a2 = make_float2(v[1].x + v[3].x, v[1].y + v[3].y);
      const float2 d = make_float2(v[1].x - v[3].x, v[1].y - v[3].y);
      const float2 a3 = make_float2(-d.y, d.x);  // i * (v1 - v3): inverse transform
      y[0] = make_float2(a0.x + a2.x, a0.y + a2.y);
      y[2] = make_float2(a0.x - a2.x, a0.y - a2.y);
      y[1] = make_float2(a1.x + a3.x, a1.y + a3.y);
      y[3] = make_float2(a1.x - a3.x, a1.y - a3.y);
    } else {  // R == 5: direct 5-point DFT with e^{+2 pi i rq/5} = tw[256 * ((r q) mod 5)]
#pragma unroll
      for (int q = 0; q < R; ++q) {
        float2 accv = v[0];
#pragma unroll
        for (int r = 1; r < R; ++r) {
          const float2 c = cmul(v[r], tw[256 * ((r * q) % 5)]);
          accv.x += c.x;
          accv.y += c.y;
        }
        y[q] = accv;
      }
    }
    const int base = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) dst[base + r * Ns] = y[r];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void istft_frames_kernel(const float* __restrict__ spec, const float2* __restrict__ tw,
                                                           const float* __restrict__ window, float* __restrict__ frames) {
  __shared__ float2 bufA[FM], bufB[FM];
  __shared__ float2 X[NB];
  const int f = blockIdx.x, tid = threadIdx.x;
  const float* row = spec + (size_t)f * (2 * NB);
  for (int k = tid; k < NB; k += 256) {
    const float mag = fminf(expf(row[k]), 100.0f);
    const float ph = row[NB + k];
    float2 x = make_float2(mag * cosf(ph), mag * sinf(ph));
    if (k == 0 || k == NB - 1) x.y = 0.f;  // C2R ignores imag of DC and Nyquist
    X[k] = x;
  }
  __syncthreads();
  // Z[k] = Xe[k] + i Xo[k];  Xe = (X[k] + conj X[M-k]) / 2,  Xo = (X[k] - conj X[M-k]) e^{+2 pi i k/N} / 2
  for (int k = tid; k < FM; k += 256) {
    const float2 a = X[k];
    const float2 bc = make_float2(X[FM - k].x, -X[FM - k].y);
    const float2 xe = make_float2(0.5f * (a.x + bc.x), 0.5f * (a.y + bc.y));
    const float2 xo = cmul(make_float2(0.5f * (a.x - bc.x), 0.5f * (a.y - bc.y)), tw[k]);
    bufA[k] = make_float2(xe.x - xo.y, xe.y + xo.x);
  }
  __syncthreads();
  stockham_pass<4>(bufA, bufB, 1, tw);
  stockham_pass<4>(bufB, bufA, 4, tw);
  stockham_pass<4>(bufA, bufB, 16, tw);
  stockham_pass<2>(bufB, bufA, 64, tw);
  stockham_pass<5>(bufA, bufB, 128, tw);
  float* out = frames + (size_t)f * NFFT;
  const float sc = 1.0f / FM;
  for (int m = tid; m < FM; m += 256) {
    const float2 zz = bufB[m];
    out[2 * m] = zz.x * sc * window[2 * m];
    out[2 * m + 1] = zz.y * sc * window[2 * m + 1];
  }
}

// overlap-add (fold, hop 320) + trim 480 + divide by the window-square envelope
__global__ void istft_ola_kernel(const float* __restrict__ frames, const float* __restrict__ window, int L,
                                 float* __restrict__ pcm) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int T = HOPL * L;
  if (j >= T) return;
  const int n = j + (NFFT - HOPL) / 2;
  int f_lo = (n - NFFT + HOPL) / HOPL;  // ceil((n - 1279) / 320) for n >= 1279
  if (n < NFFT - 1) f_lo = 0;
  const int f_hi = min(L - 1, n / HOPL);
  float y = 0.f, env = 0.f;
  for (int f = max(f_lo, 0); f <= f_hi; ++f) {
    const int o = n - f * HOPL;
    if (o < 0 || o >= NFFT) continue;
    y += frames[((size_t)b * L + f) * NFFT + o];
    env += window[o] * window[o];
  }
  pcm[(size_t)b * T + j] = y / env;
}

// ---------------------------------------------------------------------------------
// the decode pipeline
// ---------------------------------------------------------------------------------
template <typename TW>
static void decode_impl(const CodecWeights& w, const CodecScratch& sc, const float* feats_in, const int32_t* codes,
                        int B, int L, int bw, float* pcm, hipStream_t s) {
  const int M = B * L;
  float* x = sc.x;
  float* t1 = sc.t1;
  float* t2 = sc.t2;
  // a3: features, time-major [M][512]
  if (codes) hipLaunchKernelGGL(codes_gather_kernel, dim3(M), dim3(CIN / 4), 0, s, w.codebook, codes, sc.feats);
  else hipLaunchKernelGGL(feats_transpose_kernel, dim3((L + 31) / 32, CIN / 32, B), dim3(256), 0, s, feats_in, L, sc.feats);

  float* gn = sc.gn;  // [M][768] normalised operand of the next conv / 1x1
  g_ws_floats = sc.ws_floats;
  GemmArgs g{};
  g.ws = sc.ws;
  g.L = L;
  g.M = M;
  // embed Conv1d(512->768, k7, pad 3)
  g.A = sc.feats; g.lda = CIN; g.cin = CIN; g.taps = 7;
  g.W = w.embed_w; g.ldw = 7 * CIN; g.K = 7 * CIN; g.N = CD;
  g.C = x; g.ldc = CD; g.bias = w.embed_b;
  gemm_w<TW, A_CONV, E_BIAS>(g, 1, s);

  auto resnet = [&](int i) {  // models.py:58-78
    hipLaunchKernelGGL((gn_apply_kernel<true>), dim3(GN_G, B), dim3(256), 0, s, x, L, w.rn_n1w[i], w.rn_n1b[i], gn);
    GemmArgs c{};
    c.ws = sc.ws;
    c.L = L; c.M = M; c.cin = CD; c.taps = 3; c.K = 3 * CD; c.N = CD; c.ldw = 3 * CD;
    c.A = gn; c.lda = CD;
    c.W = w.rn_c1w[i]; c.bias = w.rn_c1b[i]; c.C = t1; c.ldc = CD;
    gemm_w<TW, A_CONV, E_BIAS>(c, 1, s);
    hipLaunchKernelGGL((gn_apply_kernel<true>), dim3(GN_G, B), dim3(256), 0, s, t1, L, w.rn_n2w[i], w.rn_n2b[i], gn);
    c.W = w.rn_c2w[i]; c.bias = w.rn_c2b[i]; c.C = x; c.res = x; c.ldr = CD;
    gemm_w<TW, A_CONV, E_BIAS_RES>(c, 1, s);
  };
  resnet(0);
  resnet(1);
  {  // AttnBlock (models.py:107-127)
    hipLaunchKernelGGL((gn_apply_kernel<false>), dim3(GN_G, B), dim3(256), 0, s, x, L, w.at_nw, w.at_nb, gn);
    GemmArgs c{};
    c.ws = sc.ws;
    c.L = L; c.M = M; c.K = CD; c.N = 3 * CD; c.ldw = CD;
    c.A = gn; c.lda = CD;
    c.W = w.at_qkv_w; c.bias = w.at_qkv_b; c.C = t1; c.ldc = CFF;
    gemm_w<TW, A_PLAIN, E_BIAS>(c, 1, s);
    const int ldS = (L + 3) & ~3;
    float* S = sc.att;            // [B][L][ldS]
    float* Vt = t2;               // [B][768][ldS]
    hipLaunchKernelGGL(v_transpose_kernel, dim3((ldS + 31) / 32, CD / 32, B), dim3(256), 0, s, t1, L, ldS, Vt);
    // scores = q k^T * 768^-0.5, batched over streams
    GemmArgs a{};
    a.ws = sc.ws;
    a.M = L; a.N = L; a.K = CD; a.L = L;
    a.A = t1; a.lda = CFF; a.sA = (long long)L * CFF;
    a.W = t1 + CD; a.ldw = CFF; a.sW = (long long)L * CFF;
    a.C = S; a.ldc = ldS; a.sC = (long long)L * ldS;
    a.alpha = 0.036084391824351615f;  // 768 ** -0.5
    gemm_act<TW, E_SCALE>(a, B, s);
    hipLaunchKernelGGL(softmax_rows_kernel, dim3(M), dim3(256), 0, s, S, L, ldS);
    // h = P V  (A = P [L][L], W = Vt [768][L])
    GemmArgs p{};
    p.ws = sc.ws;
    p.M = L; p.N = CD; p.K = L; p.L = L;
    p.A = S; p.lda = ldS; p.sA = (long long)L * ldS;
    p.W = Vt; p.ldw = ldS; p.sW = (long long)CD * ldS;
    p.C = t1; p.ldc = CFF; p.sC = (long long)L * CFF;  // h overwrites the (consumed) q columns
    gemm_act<TW, E_BIAS>(p, B, s);
    // proj_out + residual
    GemmArgs o{};
    o.ws = sc.ws;
    o.M = M; o.N = CD; o.K = CD; o.L = L;
    o.A = t1; o.lda = CFF; o.W = w.at_proj_w; o.ldw = CD; o.bias = w.at_proj_b;
    o.C = x; o.ldc = CD; o.res = x; o.ldr = CD;
    gemm_w<TW, A_PLAIN, E_BIAS_RES>(o, 1, s);
  }
  resnet(2);
  resnet(3);
  // pos_net[5] GroupNorm + backbone AdaLN
  hipLaunchKernelGGL(gn_stats_kernel, dim3(GN_G, B), dim3(256), 0, s, x, L, sc.stats);
  hipLaunchKernelGGL(gn_adaln_kernel, dim3(M), dim3(256), 0, s, x, L, sc.stats, w.pn_w, w.pn_b,
                     w.ada_scale + (size_t)bw * CD, w.ada_shift + (size_t)bw * CD, x);
  for (int i = 0; i < 12; ++i) {  // ConvNeXt blocks (modules.py:43-60)
    hipLaunchKernelGGL(dwconv_adaln_kernel, dim3(M), dim3(256), 0, s, x, L, w.dw_w[i], w.dw_b[i],
                       w.cn_scale[i] + (size_t)bw * CD, w.cn_shift[i] + (size_t)bw * CD, t2);
    GemmArgs c{};
    c.ws = sc.ws;
    c.M = M; c.L = L; c.N = CFF; c.K = CD; c.ldw = CD;
    c.A = t2; c.lda = CD; c.W = w.pw1_w[i]; c.bias = w.pw1_b[i]; c.C = t1; c.ldc = CFF;
    gemm_w<TW, A_PLAIN, E_BIAS_GELU>(c, 1, s);
    GemmArgs d{};
    d.ws = sc.ws;
    d.M = M; d.L = L; d.N = CD; d.K = CFF; d.ldw = CFF;
    d.A = t1; d.lda = CFF; d.W = w.pw2_w[i]; d.bias = w.pw2_b[i]; d.gamma = w.gamma[i];
    d.C = x; d.ldc = CD; d.res = x; d.ldr = CD;
    gemm_w<TW, A_PLAIN, E_BIAS_GAMMA_RES>(d, 1, s);
  }
  hipLaunchKernelGGL(ln_affine_kernel, dim3(M), dim3(256), 0, s, x, w.fln_w, w.fln_b, t2);
  {  // ISTFTHead.out Linear(768 -> 1282)
    GemmArgs h{};
    h.ws = sc.ws;
    h.M = M; h.L = L; h.N = 2 * NB; h.K = CD; h.ldw = CD;
    h.A = t2; h.lda = CD; h.W = w.head_w; h.bias = w.head_b; h.C = sc.spec; h.ldc = 2 * NB;
    gemm_w<TW, A_PLAIN, E_BIAS>(h, 1, s);
  }
  hipLaunchKernelGGL(istft_frames_kernel, dim3(M), dim3(256), 0, s, sc.spec,
                     reinterpret_cast<const float2*>(w.twiddle), w.window, sc.frames);
  hipLaunchKernelGGL(istft_ola_kernel, dim3((HOPL * L + 255) / 256, B), dim3(256), 0, s, sc.frames, w.window, L, pcm);
}

void codec_launch_decode(const CodecWeights& w, const CodecScratch& sc, int wdtype, const float* feats_in,
                         const int32_t* codes, int B, int L, int bw, float* pcm, hipStream_t s) {
  if (wdtype == LVX_DTYPE_BF16) decode_impl<bf16_t>(w, sc, feats_in, codes, B, L, bw, pcm, s);
  else decode_impl<float>(w, sc, feats_in, codes, B, L, bw, pcm, s);
}

}  // namespace lvx
