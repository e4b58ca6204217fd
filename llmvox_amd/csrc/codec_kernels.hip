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
#include <type_traits>

#include "lvx_internal.h"

// no implicit a*b+c contraction: rows / frames computed by different unrolled copies round alike
#pragma clang fp contract(off)

namespace lvx {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int CD = 768, CFF = 2304, CIN = 512, NFFT = 1280, HOPL = 320, NB = 641, GN_G = 32;

enum { A_PLAIN = 0, A_CONV = 1 };
enum { E_BIAS = 0, E_BIAS_GELU = 1, E_BIAS_GAMMA_RES = 2, E_BIAS_RES = 3, E_SCALE = 4 };

typedef __attribute__((address_space(1))) unsigned gu32;

struct GemmArgs {
  const void* A; int lda;    // fp32 or bf16 activations (kernel template TA)
  const void* W; int ldw;
  void* C; int ldc;          // fp32 or bf16 output (kernel template TC)
  const float* bias; const float* gamma; const float* res; int ldr;
  int M, N, K;
  long long sA, sW, sC, sR;  // per-batch strides (elements)
  int L;                     // frames per stream (rows per stream)
  int cin, taps;
  float alpha;
  int ksplit;                // >1: deterministic split-K through the fp32 workspace `ws`
  int xcd_remap;             // gemm_bf16_kernel: XCD-aware tile order (option codec_xcd)
  const float* wscale;       // fp8 weights: per-output-column scale (w = q * s), else null
  float* ws;
  uint32_t* tick;            // gemm_mfma_kernel split-K: per-tile arrival counters of the in-launch
                             // combine (zero between launches: the last arriver resets its own), or
                             // null for the separate reduce kernel
  int asplit;                // fp32 parity mode, bf16x3 GEMM: A is a split image (split_store), not fp32
  int csplit;                // fp32 parity mode, bf16x3 GEMM (bias + GELU): C written as a split image
  const float* ascale;       // fp8 activations (codec_dtype FP8, gemm_glds_kernel<fp8_t>): per-row scale, a = q * s
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
constexpr int KS_INLAUNCH = 16;    // most K splits of an in-launch combined GEMM
constexpr int M_INLAUNCH = 16;     // in-launch split-K combine for M <= this (the first dumps)
constexpr int LDF = BK + 1;  // fp32 LDS row (conflict-free b32 column reads)
constexpr int LDH = BK + 8;  // bf16 LDS row (80 B)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2n __attribute__((ext_vector_type(2)));
typedef float f32x4n __attribute__((ext_vector_type(4)));
// one 16-B A chunk from global, replaced by zeros when !ok (conv padding) with a select
__device__ __forceinline__ void g2_ld(u32x4& v, const bf16_t* src, bool ok) {
  const u32x4 t = *reinterpret_cast<const u32x4*>(src);
  v = ok ? t : u32x4{0u, 0u, 0u, 0u};
}
__device__ __forceinline__ void g2_ld(f32x4n& v, const float* src, bool ok) {
  const f32x4n t = *reinterpret_cast<const f32x4n*>(src);
  v = ok ? t : f32x4n{0.f, 0.f, 0.f, 0.f};
}
// one A chunk into the bf16 LDS tile: 8 bf16 as they are, or 4 fp32 rounded to bf16
__device__ __forceinline__ void g2_st(bf16_t* d, u32x4 v) { *reinterpret_cast<u32x4*>(d) = v; }
__device__ __forceinline__ void g2_st(bf16_t* d, f32x4n f) {
  *reinterpret_cast<uint2*>(d) = make_uint2((uint32_t)f32_to_bf16(f.x) | ((uint32_t)f32_to_bf16(f.y) << 16),
                                            (uint32_t)f32_to_bf16(f.z) | ((uint32_t)f32_to_bf16(f.w) << 16));
}

template <typename TC>
__device__ __forceinline__ void store_out(TC* p, float v);
template <> __device__ __forceinline__ void store_out<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void store_out<bf16_t>(bf16_t* p, float v) { *p = f32_to_bf16(v); }
template <> __device__ __forceinline__ void store_out<fp8_t>(fp8_t* p, float v) { *p = f32_to_fp8(v); }

template <bool BF, typename TA, typename TB, int AMODE, int EPI, typename TC, bool KF>
__global__ __launch_bounds__(256) void gemm_mfma_kernel(GemmArgs g) {
  constexpr int LDSZ = BF ? (BM * LDH / 2) : (BM * LDF);  // in floats
  __shared__ __attribute__((aligned(16))) float As_[LDSZ];
  __shared__ __attribute__((aligned(16))) float Bs_[LDSZ];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int zb = blockIdx.z / g.ksplit, ks = blockIdx.z - zb * g.ksplit;
  const TA* A = reinterpret_cast<const TA*>(g.A) + zb * g.sA;
  const TB* W = reinterpret_cast<const TB*>(g.W) + zb * g.sW;
  const int lrow = tid >> 2, lseg = (tid & 3) * 8;
  const int am = m0 + lrow, bn = n0 + lrow;
  int ab = 0, at = 0;
  if (AMODE == A_CONV && am < g.M) { ab = am / g.L; at = am - ab * g.L; }
  const int nkt = (g.K + BK - 1) / BK;
  const int kt_per = (nkt + g.ksplit - 1) / g.ksplit;
  const int kt0 = ks * kt_per, kt1 = min(nkt, kt0 + kt_per);

  // KF (K a multiple of BK: every weight GEMM): branch-free loads — clamped row / tap, the load
  // always issued, zeros selected afterwards (a load under a branch made the compiler wait for
  // every outstanding load: the k-tile's loads ran one round trip each)
  const int amc = min(am, g.M - 1), bnc = min(bn, g.N - 1);
  auto load_tile_kf = [&](int kt, float* av, float* bv) {
    const int k = kt * BK + lseg;
    bool aok = am < g.M;
    if (AMODE == A_PLAIN) {
      load8<TA>(A + (size_t)amc * g.lda + k, av);
    } else {
      const int tap = k / g.cin, c = k - tap * g.cin;
      const int tt = at + tap - (g.taps - 1) / 2;
      aok = aok && tt >= 0 && tt < g.L;
      load8<TA>(A + ((size_t)ab * g.L + min(max(tt, 0), g.L - 1)) * g.cin + c, av);
    }
    load8<TB>(W + (size_t)bnc * g.ldw + k, bv);
    const bool bok = bn < g.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      av[i] = aok ? av[i] : 0.f;
      bv[i] = bok ? bv[i] : 0.f;
    }
  };
  auto load_tile = [&](int kt, float* av, float* bv) {
    if constexpr (KF) {
      load_tile_kf(kt, av, bv);
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) { av[i] = 0.f; bv[i] = 0.f; }
    const int k = kt * BK + lseg;
    if (am < g.M) {
      if (AMODE == A_PLAIN) {
        const TA* ap = A + (size_t)am * g.lda + k;
        if (k + 8 <= g.K) load8<TA>(ap, av);
        else {
#pragma unroll
          for (int i = 0; i < 8; ++i) av[i] = (k + i < g.K) ? Ld<TA>::load1(ap + i) : 0.f;
        }
      } else {
        const int tap = k / g.cin, c = k - tap * g.cin;
        const int tt = at + tap - (g.taps - 1) / 2;
        if (tt >= 0 && tt < g.L) load8<TA>(A + ((size_t)ab * g.L + tt) * g.cin + c, av);
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
  // stage a k-tile's registers into LDS, then its MFMAs (both waves of a pair of k-tiles share the
  // LDS tiles: barrier before overwriting, barrier before reading)
  auto stage = [&](const float* av, const float* bv) {
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
  };
  auto mma = [&]() {
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
  };
  if (KF) {
    // two k-tiles in flight: tile kt + 2 is loaded into the register set tile kt just left (its
    // index clamped to the split's last tile: the load is always issued, no branch around it)
    float av0[8], bv0[8], av1[8], bv1[8];
    if (kt0 < kt1) {
      load_tile(kt0, av0, bv0);
      load_tile(min(kt0 + 1, kt1 - 1), av1, bv1);
    }
    for (int kt = kt0; kt < kt1; kt += 2) {
      stage(av0, bv0);
      load_tile(min(kt + 2, kt1 - 1), av0, bv0);
      mma();
      if (kt + 1 >= kt1) break;
      stage(av1, bv1);
      load_tile(min(kt + 3, kt1 - 1), av1, bv1);
      mma();
    }
  } else {
    float av[8], bv[8];
    if (kt0 < kt1) load_tile(kt0, av, bv);
    for (int kt = kt0; kt < kt1; ++kt) {
      stage(av, bv);
      if (kt + 1 < kt1) load_tile(kt + 1, av, bv);  // in flight during the MFMAs below
      mma();
    }
  }
  const int col = n0 + wn * 32 + (lane & 31), colc = min(col, g.N - 1);
  // epilogue operands loaded unconditionally (clamped row / column) before any branch
  const float* R = g.res ? g.res + zb * g.sR : nullptr;
  const float bias = (EPI != E_SCALE && g.bias) ? g.bias[colc] : 0.f;
  const float gam = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[colc] : 0.f;
  float rv[16];
  if (EPI == E_BIAS_GAMMA_RES || EPI == E_BIAS_RES) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = min(m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), g.M - 1);
      rv[r] = (g.ksplit > 1) ? 0.f : R[(size_t)row * g.ldr + colc];
    }
  }
  if (g.ksplit > 1) {  // raw partial tile -> ws[ks][zb][M][N]
    const int batch = gridDim.z / g.ksplit;
    float* P = g.ws + ((size_t)ks * batch + zb) * (size_t)g.M * g.N;
    if (!g.tick) {  // reduced by gemm_splitk_reduce
      if (col >= g.N) return;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < g.M) P[(size_t)row * g.N + col] = acc[r];
      }
      return;
    }
    // In-launch combine (cdna_hip_programming.md G16, counter form with write-through slabs): every
    // wave stores its partial with sc1 stores and drains them, one relaxed agent ticket per block;
    // the tile's last arriving slice reads every slab with sc1 loads (no fences), sums them in
    // split order and applies the epilogue -- the same arithmetic as gemm_splitk_reduce, one
    // launch fewer per GEMM.
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < g.M && col < g.N)
        __hip_atomic_store((gu32*)(P + (size_t)row * g.N + col), __float_as_uint(acc[r]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int tile = (zb * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (tid == 0) {
      const unsigned tk = __hip_atomic_fetch_add((gu32*)(g.tick + tile), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = tk == (unsigned)g.ksplit - 1;
      if (last) __hip_atomic_store((gu32*)(g.tick + tile), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      As_[0] = last ? 1.f : 0.f;
    }
    __syncthreads();
    if (As_[0] == 0.f) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below here
    const size_t MN = (size_t)g.M * g.N;
    TC* C = reinterpret_cast<TC*>(g.C) + zb * g.sC;
    const int rows = min(BM, g.M - m0), cols = min(BN, g.N - n0);  // launched for M <= 16: <= 4 per thread
    for (int e = tid; e < rows * cols; e += 256) {
      const int row = m0 + e / cols, cc = n0 + e % cols;
      const size_t off = (size_t)zb * MN + (size_t)row * g.N + cc;
      float p[KS_INLAUNCH];  // every slab load in flight at once (index clamped, no load under a branch)
#pragma unroll
      for (int k = 0; k < KS_INLAUNCH; ++k)
        p[k] = __uint_as_float(__hip_atomic_load((gu32*)(g.ws + (size_t)min(k, g.ksplit - 1) * batch * MN + off),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < KS_INLAUNCH; ++k) v = k < g.ksplit ? v + p[k] : v;  // split order, as the reduce kernel
      const float bb = (EPI != E_SCALE && g.bias) ? g.bias[cc] : 0.f;
      const float gm = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[cc] : 0.f;
      store_out<TC>(C + (size_t)row * g.ldc + cc, gemm_epi<EPI>(g, R, row, cc, v, bb, gm));
    }
    return;
  }
  if (col >= g.N) return;
  TC* C = reinterpret_cast<TC*>(g.C) + zb * g.sC;
  // outputs computed before any row guard: the empty asm takes them as inputs, so the waits for
  // the epilogue loads happen once here. Computed inside each guarded store, every store block
  // re-waited vmcnt(0) (the skip edge leaves the loads "pending") and the 16 stores ran one
  // write acknowledgement apart.
  float o[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (EPI == E_BIAS_GAMMA_RES) o[r] = rv[r] + gam * (acc[r] + bias);
    else if (EPI == E_BIAS_RES) o[r] = rv[r] + (acc[r] + bias);
    else o[r] = gemm_epi<EPI>(g, R, row, col, acc[r], bias, gam);
    asm volatile("" : "+v"(o[r]));
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (row < g.M) store_out<TC>(C + (size_t)row * g.ldc + col, o[r]);
  }
}

// sum the ksplit partials in split order, then the epilogue
template <int EPI, typename TC>
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
    store_out<TC>(reinterpret_cast<TC*>(g.C) + zb * g.sC + (size_t)row * g.ldc + col, gemm_epi<EPI>(g, R, row, col, v, bias, gam));
  }
}

// capacity of the split-K workspace and the per-tile counters of the in-launch combine, set from
// the context's scratch at the start of each codec_launch_decode and read by the launch helpers it
// calls on the same host thread: thread_local, so two contexts decoding from two threads (two
// devices) never see each other's workspace or tickets
static thread_local size_t g_ws_floats = 0;
static thread_local uint32_t* g_tick = nullptr;

template <bool BF, typename TA, typename TB, int AMODE, int EPI, typename TC>
static void gemm_launch(GemmArgs g, int batch, hipStream_t s) {
  const int tiles = ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM) * batch;
  const int nkt = (g.K + BK - 1) / BK;
  int ks = 1;
  // split K until the grid covers the chip (>= ~256 blocks), >= 4 k-tiles per split,
  // and the partials fit the workspace
  // (measured, tools/codec_probe.py, 1 x 10 / 1 x 256 frames: no split 1.05 / 1.15 ms, at most 2
  // splits 0.75 / 0.85, at most 4 0.56 / 0.74, this rule 0.51 / 0.70; a 160-block target the same,
  // 640 slower at 32 x 256 frames)
  while (tiles * ks * 2 <= 320 && nkt / (ks * 2) >= 4 && (size_t)(ks * 2) * g.M * g.N * batch <= g_ws_floats) ks *= 2;
  // in-launch combine for the first dumps (1 x 10 frames: 0.502 -> 0.442 ms)
  const bool inl = g_tick && batch == 1 && g.M <= M_INLAUNCH && tiles <= 4096;
  if (inl) ks = std::min(ks, KS_INLAUNCH);
  g.ksplit = ks;
  g.tick = (inl && ks > 1) ? g_tick : nullptr;
  dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, batch * ks);
  if (g.K % BK == 0) hipLaunchKernelGGL((gemm_mfma_kernel<BF, TA, TB, AMODE, EPI, TC, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((gemm_mfma_kernel<BF, TA, TB, AMODE, EPI, TC, false>), grid, dim3(256), 0, s, g);
  if (ks > 1 && !g.tick) {
    const size_t total = (size_t)g.M * g.N * batch;
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 2048);
    hipLaunchKernelGGL((gemm_splitk_reduce<EPI, TC>), dim3(blocks), dim3(256), 0, s, g, batch);
  }
}
// ---------------------------------------------------------------------------------
// bf16 weight GEMM for large M (bf16 mode): 128 x 128 block tile, BK 64, 4 waves in 2 x 2, each
// a 64 x 64 tile of four v_mfma_f32_32x32x16_bf16 accumulators. Operands are bf16 in LDS (double
// buffered: one barrier per k-tile); the next k-tile's global loads are in flight in registers
// while the current one is multiplied, and up to two blocks share a CU (73 KB LDS each), so one
// block's loads overlap the other's MFMAs. A is bf16 (TA = bf16_t: activations written in bf16 by
// their producer, identical to rounding them here) or fp32 (rounded on the way into LDS), plain
// or implicit-Conv1d. TC = output type of the plain epilogue (bf16 for the GELU output that only
// feeds the next GEMM). Rows of every tile are whole 128-B runs: coalesced loads and stores.
// ---------------------------------------------------------------------------------
constexpr int G2_BN = 128, G2_BK = 64, G2_LDK = G2_BK + 8;  // bf16 row stride 144 B

template <typename TB> struct BLoad;
template <> struct BLoad<bf16_t> {  // 4 x 8 bf16 per thread per tile
  u32x4 v[4];
};
template <> struct BLoad<fp8_t> {  // 4 x 8 e4m3 per thread per tile
  u32x2n v[4];
};
// 8 weights into the bf16 LDS tile: as they are, or e4m3 -> bf16 (exact: 3 mantissa bits fit)
__device__ __forceinline__ void g2_stb(bf16_t* d, u32x4 v) { *reinterpret_cast<u32x4*>(d) = v; }
__device__ __forceinline__ void g2_stb(bf16_t* d, u32x2n v) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  u32x4 o;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f2 a = __builtin_amdgcn_cvt_pk_f32_fp8(v[h], false), b = __builtin_amdgcn_cvt_pk_f32_fp8(v[h], true);
    o[2 * h] = (__float_as_uint(a.x) >> 16) | (__float_as_uint(a.y) & 0xffff0000u);
    o[2 * h + 1] = (__float_as_uint(b.x) >> 16) | (__float_as_uint(b.y) & 0xffff0000u);
  }
  *reinterpret_cast<u32x4*>(d) = o;
}
__device__ __forceinline__ void g2_ldb(u32x4& v, const bf16_t* p) { v = *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void g2_ldb(u32x2n& v, const fp8_t* p) { v = *reinterpret_cast<const u32x2n*>(p); }

template <typename TA> struct ALoad;
template <> struct ALoad<bf16_t> {  // 4 x 16 B per thread per tile (native vectors: register-resident)
  u32x4 v[4];
};
template <> struct ALoad<float> {  // 8 x 16 B per thread per tile
  f32x4n v[8];
};


// BMt = 128: 4 waves of 64 x 64 (2 x 2 MFMA tiles), 2 blocks per CU. BMt = 256: 4 waves of 128 x 64
// (4 x 2), one block per CU: 0.75 LDS fragment reads per MFMA instead of 1 (the LDS read rate of a
// 64 x 64 wave tile equals the MFMA rate).
template <typename TA, typename TB, int AMODE, int EPI, typename TC, int BMt>
__global__ __launch_bounds__(256, BMt == 128 ? 2 : 1) void gemm_bf16_kernel(GemmArgs g) {
  constexpr int WMt = BMt / 2, MI = WMt / 32;  // rows per wave, 32-row MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) bf16_t As[2][BMt * G2_LDK];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][G2_BN * G2_LDK];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs (id % 8), so XCD x gets
  // the contiguous logical range [x * T/8, (x+1) * T/8); logical tiles walk G2_GM M-tiles down one
  // N column before moving right, so the ~64 tiles in flight on an XCD share 8 A row-blocks and
  // 8 weight row-blocks in that XCD's L2 instead of touching all of them.
  const int ntn = gridDim.x, ntm = gridDim.y, T = ntn * ntm;
  const int pid = blockIdx.x + ntn * blockIdx.y;
  int q = pid;
  if (g.xcd_remap && (T & 7) == 0) q = (pid & 7) * (T >> 3) + (pid >> 3);
  const int G2_GM = g.xcd_remap ? 8 : 1;
  const int gsz = G2_GM * ntn, grp = q / gsz, within = q - grp * gsz;
  const int gm = min(G2_GM, ntm - grp * G2_GM);
  const int tm = grp * G2_GM + within % gm, tn = within / gm;
  const int m0 = tm * BMt, n0 = tn * G2_BN;
  const int ks = blockIdx.z;
  const TA* __restrict__ A = reinterpret_cast<const TA*>(g.A);
  const TB* __restrict__ W = reinterpret_cast<const TB*>(g.W);
  const int nkt = g.K / G2_BK;  // K % 64 == 0 (checked by the launcher)
  const int kt_per = (nkt + g.ksplit - 1) / g.ksplit;
  const int kt0 = ks * kt_per, kt1 = min(nkt, kt0 + kt_per);
  // loader geometry: chunk c = tid + 256 i covers row c / ACH, 16-B segment c % ACH
  constexpr int ACH = sizeof(TA) == 2 ? 8 : 16;  // 16-B chunks per A row of the tile
  constexpr int AN = BMt * ACH / 256;             // chunks per thread
  constexpr int AROWS = 256 / ACH;                // rows covered per i step
  const int arow0 = tid / ACH, aseg = (tid % ACH) * (16 / (int)sizeof(TA));
  // implicit conv: (stream, frame) of this thread's first row; later rows are +AROWS frames
  int cb0 = 0, ct0 = 0;
  if (AMODE == A_CONV) { cb0 = (m0 + arow0) / g.L; ct0 = (m0 + arow0) - cb0 * g.L; }
  ALoad<TA> ar0, ar1;
  BLoad<TB> br0, br1;
#define G2_LOAD(kt, ar, br)                                                                                \
  {                                                                                                        \
    const int kb = (kt) * G2_BK;                                                                           \
    _Pragma("unroll") for (int i = 0; i < AN; ++i) {                                                       \
      /* unconditional loads from a clamped row (rows past M are never stored; conv padding is */         \
      /* zeroed by a select): no branches, so the waitcnt of each register set stays exact */              \
      const int m = min(m0 + arow0 + AROWS * i, g.M - 1);                                                  \
      const TA* src;                                                                                       \
      bool ok = true;                                                                                      \
      if (AMODE == A_PLAIN) {                                                                              \
        src = A + (size_t)m * g.lda + kb + aseg;                                                           \
      } else {                                                                                             \
        int b = cb0, t = ct0 + AROWS * i;                                                                  \
        while (t >= g.L) { t -= g.L; ++b; }                                                                \
        const int tap = kb / g.cin, c = kb + aseg - tap * g.cin; /* a 64-wide k-tile lies in one tap */   \
        const int tt = t + tap - (g.taps - 1) / 2;                                                         \
        ok = tt >= 0 && tt < g.L && b * g.L + t < g.M;                                                     \
        src = A + ((size_t)b * g.L + min(max(tt, 0), g.L - 1)) * g.cin + c;                                \
        if (b * g.L + t >= g.M) src = A + (size_t)m * g.cin + c;                                           \
      }                                                                                                    \
      g2_ld(ar.v[i], src, ok);                                                                             \
    }                                                                                                      \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                        \
      const int c = tid + 256 * i, r = c >> 3, seg = (c & 7) * 8;                                          \
      const int n = min(n0 + r, g.N - 1); /* rows past N duplicate row N-1 (never stored) */              \
      g2_ldb(br.v[i], W + (size_t)n * g.ldw + kb + seg);                                                   \
    }                                                                                                      \
  }
#define G2_STORE(buf, ar, br)                                                                                      \
  {                                                                                                        \
    bf16_t* as = As[buf];                                                                                  \
    bf16_t* bs = Bs[buf];                                                                                  \
    _Pragma("unroll") for (int i = 0; i < AN; ++i) {                                                       \
      g2_st(as + (arow0 + AROWS * i) * G2_LDK + aseg, ar.v[i]);                                            \
    }                                                                                                      \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                        \
      const int c = tid + 256 * i, r = c >> 3, seg = (c & 7) * 8;                                          \
      g2_stb(bs + r * G2_LDK + seg, br.v[i]);                                                              \
    }                                                                                                      \
  }

  f32x16 acc[MI][2];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // two k-tiles in flight: tile kt+2 is loaded into one register set while tile kt is multiplied
  // from LDS and tile kt+1 (the other set, issued one step earlier) goes to the other LDS buffer
#define G2_COMPUTE(buf)                                                                                    \
  {                                                                                                        \
    const bf16_t* as = As[buf];                                                                            \
    const bf16_t* bs = Bs[buf];                                                                            \
    _Pragma("unroll") for (int kk = 0; kk < G2_BK; kk += 16) {                                             \
      bf16x8 fa[MI], fb[2];                                                                                \
      _Pragma("unroll") for (int i = 0; i < MI; ++i)                                                       \
        fa[i] = *reinterpret_cast<const bf16x8*>(as + (wm * WMt + i * 32 + (lane & 31)) * G2_LDK + kk + 8 * (lane >> 5)); \
      _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                        \
        fb[i] = *reinterpret_cast<const bf16x8*>(bs + (wn * 64 + i * 32 + (lane & 31)) * G2_LDK + kk + 8 * (lane >> 5)); \
      _Pragma("unroll") for (int i = 0; i < MI; ++i)                                                       \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                        \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);              \
    }                                                                                                      \
  }
  // Loads are issued unconditionally (tile index clamped to the last one: a few redundant loads at
  // the end) so that no load sits under a branch: the compiler's vmcnt for "set 1 has landed" then
  // leaves set 0's loads in flight instead of draining everything.
  if (kt0 < kt1) {
    const int kl = kt1 - 1;
    G2_LOAD(kt0, ar0, br0);
    G2_LOAD(min(kt0 + 1, kl), ar1, br1);
    G2_STORE(0, ar0, br0);
    __syncthreads();
    for (int kt = kt0; kt < kt1; kt += 2) {
      // even step: tile kt in LDS 0, set 1 holds kt+1 (in flight), set 0 is free
      G2_LOAD(min(kt + 2, kl), ar0, br0);
      G2_COMPUTE(0);
      if (kt + 1 >= kt1) break;
      G2_STORE(1, ar1, br1);
      __syncthreads();
      // odd step: tile kt+1 in LDS 1, set 0 holds kt+2, set 1 is free
      G2_LOAD(min(kt + 3, kl), ar1, br1);
      G2_COMPUTE(1);
      if (kt + 2 >= kt1) break;
      G2_STORE(0, ar0, br0);
      __syncthreads();
    }
  }
#undef G2_COMPUTE
#undef G2_LOAD
#undef G2_STORE
  // epilogue: acc[i][j][r] = C[row][col], col = n0 + wn*64 + j*32 + (lane & 31),
  // row = m0 + wm*64 + i*32 + (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + j * 32 + (lane & 31);
    if (col >= g.N) continue;
    if constexpr (sizeof(TB) == 1) {  // fp8 weights: per-row dequantisation scale
      const float sc = g.wscale[col];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] *= sc;
    }
    if (g.ksplit > 1) {
      float* P = g.ws + (size_t)ks * g.M * g.N;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * WMt + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < g.M) P[(size_t)row * g.N + col] = acc[i][j][r];
        }
      continue;
    }
    TC* C = reinterpret_cast<TC*>(g.C);
    const float bias = (EPI != E_SCALE && g.bias) ? g.bias[col] : 0.f;
    const float gam = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[col] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      // residual operands first, all 16 in flight (rows clamped: loads never sit under a branch)
      float rv[16];
      if constexpr (EPI == E_BIAS_GAMMA_RES || EPI == E_BIAS_RES) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = min(m0 + wm * WMt + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), g.M - 1);
          rv[r] = g.res[(size_t)row * g.ldr + col];
        }
      }
      // outputs in place, before the row guards (the empty asm keeps them here): computed inside
      // a guarded store, each store block re-waited for the bias / residual loads, one write
      // acknowledgement after the previous store
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[i][j][r] + bias;
        float o;
        if constexpr (EPI == E_BIAS) o = v;
        else if constexpr (EPI == E_BIAS_GELU) o = sizeof(TC) == 2 ? gelu_erf_bf16out(v) : gelu_erf(v);
        else if constexpr (EPI == E_BIAS_GAMMA_RES) o = rv[r] + gam * v;
        else if constexpr (EPI == E_BIAS_RES) o = rv[r] + v;
        else o = acc[i][j][r] * g.alpha;
        acc[i][j][r] = o;
        asm volatile("" : "+v"(acc[i][j][r]));
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WMt + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < g.M) store_out<TC>(C + (size_t)row * g.ldc + col, acc[i][j][r]);
      }
    }
  }
}

// split-K partials of gemm_bf16_kernel summed in split order, then the epilogue (output TC)
template <int EPI, typename TC>
__global__ __launch_bounds__(256) void gemm2_splitk_reduce(GemmArgs g) {
  const size_t MN = (size_t)g.M * g.N;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < MN; e += (size_t)gridDim.x * 256) {
    const int row = (int)(e / g.N), col = (int)(e - (size_t)row * g.N);
    float v = 0.f;
    for (int ks = 0; ks < g.ksplit; ++ks) v += g.ws[(size_t)ks * MN + e];
    const float bias = (EPI != E_SCALE && g.bias) ? g.bias[col] : 0.f;
    const float gam = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[col] : 0.f;
    store_out<TC>(reinterpret_cast<TC*>(g.C) + (size_t)row * g.ldc + col, gemm_epi<EPI>(g, g.res, row, col, v, bias, gam));
  }
}

// option codec_g2 (default 1, Opts in lvx_internal.h): 1: large-M bf16 GEMMs on gemm_bf16_kernel; 0: on gemm_mfma (cross-check)
// smallest M that takes gemm_bf16_kernel (measured: M = 256 0.86 vs 1.04 ms, M = 10 0.64 vs 0.59).
// 256-row tiles (one block per CU) measured slower (32 x 256 frames: 3.51 vs 2.99 ms; 64 x 256: 7.04
// vs 5.16): one resident block per CU exposes the load latency that two 128-row blocks hide for each other.
constexpr int CODEC_G2_MIN_M = 128;

template <typename TA, typename TB, int AMODE, int EPI, typename TC>
static void gemm2_launch(GemmArgs g, hipStream_t s) {
  const int tiles = ((g.N + G2_BN - 1) / G2_BN) * ((g.M + 127) / 128);
  const int nkt = g.K / G2_BK;
  int ks = 1;
  while (tiles * ks * 2 <= 512 && nkt / (ks * 2) >= 4 && (size_t)(ks * 2) * g.M * g.N <= g_ws_floats) ks *= 2;
  g.ksplit = ks;
  g.xcd_remap = 1;
  dim3 grid((g.N + G2_BN - 1) / G2_BN, (g.M + 127) / 128, ks);
  hipLaunchKernelGGL((gemm_bf16_kernel<TA, TB, AMODE, EPI, TC, 128>), grid, dim3(256), 0, s, g);
  if (ks > 1) {
    const int blocks = (int)std::min<size_t>(((size_t)g.M * g.N + 255) / 256, 2048);
    hipLaunchKernelGGL((gemm2_splitk_reduce<EPI, TC>), dim3(blocks), dim3(256), 0, s, g);
  }
}

// ---------------------------------------------------------------------------------
// bf16 weight GEMM for the batched chunk decodes (M >= ~2,048 frames, bf16 operands and weights):
// operands staged by LDS-DMA (global_load_lds_dwordx4: no register staging, no ds_write pass) into
// two LDS stages (the DMA of k-tile kt+1 in flight while kt is multiplied; raw s_barrier, a
// __syncthreads() would drain the DMAs), one barrier per k-tile, both k32 sub-steps' fragments
// read before the first MFMA. Block tile 128 x 192, BK 64, 8 waves in 2 (M) x 4 (N), each 64 x 48 =
// 4 x 3 v_mfma_f32_16x16x32_bf16 accumulators. With >= 2 tiles per CU: 2 stages = 80 KB of LDS,
// two blocks per CU (the other block's
// MFMAs cover a block's barrier / fragment-read / epilogue phases: tools/gemm_ubench.hip measured the
// fragment reads and barriers of one lock-stepped block, not the MFMAs or the DMA, as its time);
// with fewer tiles, 3 stages (120 KB, the DMA of k-tile kt+2 in flight) and one block per CU.
// 128 x 192 divides the codec's shapes at 8,192 frames evenly over the 256 CUs: N = 768 -> 256
// tiles, N = 2,304 -> 768. LDS image: [row][64 k] bf16 (128-B rows, one DMA instruction = 8 rows),
// 16-B segment s of row r stored in slot s ^ (r & 7) (swizzled through the per-lane SOURCE address;
// each ds_read_b128 lane group then hits 16 distinct 4-bank groups: conflict-free). Conv padding
// rows are DMA'd from a zero granule. Rows past M / N are clamped (never stored).
// ---------------------------------------------------------------------------------
constexpr int G3_BM = 128, G3_BN = 192, G3_BK = 64;
constexpr int G3_ABYTES = G3_BM * G3_BK * 2, G3_BBYTES = G3_BN * G3_BK * 2, G3_STAGE = G3_ABYTES + G3_BBYTES;
constexpr int G3_AP = G3_BM / 8 / 8, G3_BP = G3_BN / 8 / 8;  // 1-KB DMA pieces per wave per k-tile (A, B)
static_assert(2 * 2 * G3_STAGE <= 160 * 1024 && 3 * G3_STAGE <= 160 * 1024, "LDS stages");
__device__ __attribute__((aligned(16))) uint32_t g3_zero[4];
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef int i32x8f __attribute__((ext_vector_type(8)));  // 32 fp8 (e4m3fn) MFMA operand

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// fp32 -> bf16x3 operand split (SPLIT form of gemm_glds_kernel<float>): x = hi + lo + r with
// hi = bf16_rn(x), lo = bf16_rn(x - hi) (x - hi is exact in fp32), |r| <= 2^-17 |x|. The 8 elements are
// the two 16-B fragments of one row (k 4 g + e of the k-tile's two 16-k halves, g = lane >> 4); the
// weights' split image (upload_cw in lvx_api.cpp) holds the same k order, precomputed
__device__ __forceinline__ void split_bf16x3(const f32x4v& x0, const f32x4v& x1, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h0 = (__bf16)x0[e], h1 = (__bf16)x1[e];
    hi[e] = h0;
    hi[4 + e] = h1;
    lo[e] = (__bf16)(x0[e] - (float)h0);
    lo[4 + e] = (__bf16)(x1[e] - (float)h1);
  }
}

// the split image of an fp32 row [K] (K % 32 == 0), as the bf16x3 GEMM's operands are read: per 32-k
// block, 16-B segment g < 4 holds bf16 hi of k = 4 g + e and 16 + 4 g + e (e < 4), segment 4 + g the lo
// parts; same size as the fp32 row. Element c of a row: hi at bf16 index split_pos(c), lo 32 later
__device__ __forceinline__ int split_pos(int c) {
  const int r = c & 31;
  return 2 * (c & ~31) + ((r >> 2) & 3) * 8 + (r >> 4) * 4 + (r & 3);
}
__device__ __forceinline__ void split_store(float* row, int c, float v) {
  bf16_t* o = reinterpret_cast<bf16_t*>(row) + split_pos(c);
  const bf16_t hi = f32_to_bf16(v);
  o[0] = hi;
  o[32] = f32_to_bf16(v - bf16_to_f32(hi));
}

// SPLIT bits (TA = float): 1 bf16x3 products, 2 A is a split image (no in-register split), 4 C written
// as a split image (the next GEMM's A; E_BIAS_GELU, N % 32 == 0)
template <int AMODE, int EPI, typename TC, int NS, typename TA = bf16_t, int SPLIT = 0>
__global__ __launch_bounds__(512, NS == 2 ? 2 : 1) void gemm_glds_kernel(GemmArgs g) {
  // TA = bf16: 64-deep k-tiles, v_mfma_f32_16x16x32_bf16. TA = float (the fp32 parity mode): the same
  // 128-B LDS rows hold 32 k of fp32, and each 16-B fragment (4 consecutive k of one row) feeds four
  // exact-fp32 v_mfma_f32_16x16x4_f32, MFMA e taking element e from every lane group (A and B
  // permuted alike: the k order inside a 16-k block is 4 g + e). TA = float, SPLIT: the k-tile's two
  // fragments of a row are split into bf16 hi / lo (split_bf16x3) and multiplied as
  // hi.hi + lo.hi + hi.lo by three v_mfma_f32_16x16x32_bf16 (fp32 accumulation; the lo.lo term,
  // <= 2^-16 of a product, dropped): 3 MFMAs of 16 cycles per 32 k and 16 x 16 tile instead of 8 of
  // 32. The weights come as their split image (stored right behind the fp32 matrix, g.N rows of
  // g.ldw: upload_cw), whose 128-B rows the DMA stages like fp32 rows: segment g = hi, 4 + g = lo
  static_assert(!SPLIT || sizeof(TA) == 4, "the split is of fp32 operands");
  static_assert(!(SPLIT & 4) || (EPI == E_BIAS_GELU && sizeof(TC) == 4), "split output: fp32 GELU epilogue");
  constexpr int EPS = 16 / (int)sizeof(TA);  // elements per 16-B segment
  constexpr int BKE = 8 * EPS;               // elements per k-tile (64 bf16 / 32 fp32)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * G3_STAGE];  // the only LDS object
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  // XCD-aware tile order (as gemm_bf16_kernel): an XCD's blocks walk 8 M-tiles down an N column
  const int ntn = gridDim.x, ntm = gridDim.y, T = ntn * ntm;
  const int pid = blockIdx.x + ntn * blockIdx.y;
  const int q = (T & 7) == 0 ? (pid & 7) * (T >> 3) + (pid >> 3) : pid;
  const int gsz = 8 * ntn, grp = q / gsz, within = q - grp * gsz;
  const int gm = min(8, ntm - grp * 8);
  const int m0 = (grp * 8 + within % gm) * G3_BM, n0 = (within / gm) * G3_BN;
  const TA* __restrict__ A = reinterpret_cast<const TA*>(g.A);
  const TA* __restrict__ W = reinterpret_cast<const TA*>(g.W) + (SPLIT ? (size_t)g.N * g.ldw : 0);
  const int nkt = g.K / BKE;  // K % BKE == 0 (checked by the launcher)
  // DMA geometry: lane -> row lane / 8 of a 1-KB piece, LDS slot lane % 8 <- global segment gseg
  const int lrow = lane >> 3, gseg = (lane & 7) ^ lrow;
  const TA* bsrc[G3_BP];
#pragma unroll
  for (int i = 0; i < G3_BP; ++i) {
    const int n = min(n0 + (wave * G3_BP + i) * 8 + lrow, g.N - 1);  // rows past N: never stored
    bsrc[i] = W + (size_t)n * g.ldw + gseg * EPS;
  }
  const TA* asrc[G3_AP];
  int cb[G3_AP], ct[G3_AP];
#pragma unroll
  for (int i = 0; i < G3_AP; ++i) {
    const int m = min(m0 + (wave * G3_AP + i) * 8 + lrow, g.M - 1);  // rows past M: never stored
    asrc[i] = A + (size_t)m * g.lda + gseg * EPS;
    cb[i] = AMODE == A_CONV ? m / g.L : 0;
    ct[i] = m - cb[i] * g.L;
  }
  auto issue = [&](int kt, int st) {
    unsigned char* sa = smem + st * G3_STAGE;
    unsigned char* sb = sa + G3_ABYTES;
    const int kb = kt * BKE;
#pragma unroll
    for (int i = 0; i < G3_AP; ++i) {
      const void* src;
      if (AMODE == A_PLAIN) {
        src = asrc[i] + kb;
      } else {  // implicit conv: a 64-wide k-tile lies in one tap; padding rows from the zero granule
        const int tap = kb / g.cin, c = kb - tap * g.cin + gseg * EPS;
        const int tt = ct[i] + tap - (g.taps - 1) / 2;
        src = (tt >= 0 && tt < g.L) ? (const void*)(A + ((size_t)cb[i] * g.L + tt) * g.cin + c) : (const void*)g3_zero;
      }
      glds16(src, sa + (wave * G3_AP + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < G3_BP; ++i) glds16(bsrc[i] + kb, sb + (wave * G3_BP + i) * 1024);
  };

  f32x4v acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
  // fragment addresses: lane l reads row (l & 15) of a 16-row sub-tile, segment kk / 8 + (l >> 4)
  const int frow = lane & 15, fseg = lane >> 4, fsw = lane & 7;
  const int kl = nkt - 1;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p) issue(min(p, kl), p);
  if constexpr (sizeof(TA) == 1) {
    // fp8 x fp8 (codec_dtype FP8): a 128-B row holds 128 k; lane l's fragment is k 32 (l >> 4) .. + 31 of
    // its row (the two 16-B segments 2 (l >> 4), 2 (l >> 4) + 1), one v_mfma_scale_f32_16x16x128_f8f6f4 per
    // (i, j) and k-tile with unit E8M0 scales (127): the weights' per-row and the activations' per-frame
    // fp32 scales are applied in the epilogue (tools/mx_fp8_probe.hip checks the lane maps and scales)
    for (int kt = 0; kt < nkt; ++kt) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (G3_AP + G3_BP)) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(min(kt + NS - 1, kl), (kt + NS - 1) % NS);
      const unsigned char* sa = smem + (kt % NS) * G3_STAGE;
      const unsigned char* sb = sa + G3_ABYTES;
      const int s0 = ((2 * fseg) ^ fsw) * 16, s1 = ((2 * fseg + 1) ^ fsw) * 16;
      i32x8f fa8[4], fb8[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned char* r = sa + (wm * 64 + i * 16 + frow) * 128;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(r + s0), hi = *reinterpret_cast<const u32x4*>(r + s1);
        fa8[i] = i32x8f{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const unsigned char* r = sb + (wn * 48 + j * 16 + frow) * 128;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(r + s0), hi = *reinterpret_cast<const u32x4*>(r + s1);
        fb8[j] = i32x8f{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb8[j], fa8[i], acc[i][j], 0, 0, 0, 127, 0, 127);
    }
    // the scales: acc[i][j][e] belongs to row m0 + wm*64 + i*16 + (lane & 15), column n0 + wn*48 + j*16 + cq + e
    f32x4v wsc[3];
    float asc[4];
#pragma unroll
    for (int j = 0; j < 3; ++j)
      wsc[j] = *reinterpret_cast<const f32x4v*>(g.wscale + min(n0 + wn * 48 + j * 16 + 4 * (lane >> 4), g.N - 4));
#pragma unroll
    for (int i = 0; i < 4; ++i) asc[i] = g.ascale[min(m0 + wm * 64 + i * 16 + frow, g.M - 1)];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] = acc[i][j][e] * wsc[j][e] * asc[i];
  } else
  for (int kt = 0; kt < nkt; ++kt) {
    // this wave's DMAs of tile kt have landed (the NS - 2 later tiles' stay in flight); after the
    // barrier every wave's have, and every wave is done reading the stage (tile kt - 1) that tile
    // kt + NS - 1 now goes to (clamped: the tail re-loads the last tile, never read)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (G3_AP + G3_BP)) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(min(kt + NS - 1, kl), (kt + NS - 1) % NS);
    const unsigned char* sa = smem + (kt % NS) * G3_STAGE;
    const unsigned char* sb = sa + G3_ABYTES;
    // both k32 sub-steps' fragments issued before the first MFMA
    typedef typename std::conditional<sizeof(TA) == 2, bf16x8, f32x4v>::type Frag;
    Frag fa[2][4], fb[2][3];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int slot = ((kk * 4 + fseg) ^ fsw) * 16;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[kk][i] = *reinterpret_cast<const Frag*>(sa + (wm * 64 + i * 16 + frow) * 128 + slot);
#pragma unroll
      for (int j = 0; j < 3; ++j)
        fb[kk][j] = *reinterpret_cast<const Frag*>(sb + (wn * 48 + j * 16 + frow) * 128 + slot);
    }
    if constexpr (SPLIT) {
      bf16x8 bh[3], bl[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        bh[j] = __builtin_bit_cast(bf16x8, fb[0][j]);
        bl[j] = __builtin_bit_cast(bf16x8, fb[1][j]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf16x8 ah, al;
        if constexpr ((SPLIT & 2) != 0) {
          ah = __builtin_bit_cast(bf16x8, fa[0][i]);
          al = __builtin_bit_cast(bf16x8, fa[1][i]);
        } else {
          split_bf16x3(fa[0][i], fa[1][i], ah, al);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], ah, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], ah, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], al, acc[i][j], 0, 0, 0);
        }
      }
      continue;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          // weights as the MFMA's A operand: the accumulator is the transposed tile, so each lane
          // holds 4 consecutive output columns of one row (same products, same k order: same bits)
          if constexpr (sizeof(TA) == 2) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][j], fa[kk][i], acc[i][j], 0, 0, 0);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[kk][j][e], fa[kk][i][e], acc[i][j], 0, 0, 0);
          }
        }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail DMAs
  // epilogue: acc[i][j][e] = C[m0 + wm*64 + i*16 + (lane & 15)][n0 + wn*48 + j*16 + 4*(lane >> 4) + e]:
  // bias / gamma / residual as 16-B loads and the outputs as one 16-B (fp32) or 8-B (bf16) store per
  // (i, j), 4x fewer memory instructions than one element per lane; every operand in flight at once
  // (one round trip; rows / columns clamped, no branch). N % 4 != 0 (the head's 1,282 columns) takes
  // the per-element form.
  TC* C = reinterpret_cast<TC*>(g.C);
  constexpr bool RES = EPI == E_BIAS_GAMMA_RES || EPI == E_BIAS_RES;
  const int cq = 4 * (lane >> 4);
  if ((g.N & 3) == 0 && (g.ldc & 3) == 0 && (!RES || (g.ldr & 3) == 0)) {
    f32x4v bias[3], gam[3], rv[3][4];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c4 = min(n0 + wn * 48 + j * 16 + cq, g.N - 4);
      bias[j] = g.bias ? *reinterpret_cast<const f32x4v*>(g.bias + c4) : f32x4v{0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == E_BIAS_GAMMA_RES) gam[j] = *reinterpret_cast<const f32x4v*>(g.gamma + c4);
      if constexpr (RES) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          rv[j][i] = *reinterpret_cast<const f32x4v*>(g.res + (size_t)min(m0 + wm * 64 + i * 16 + frow, g.M - 1) * g.ldr + c4);
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = n0 + wn * 48 + j * 16 + cq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = acc[i][j][e] + bias[j][e];
          float o;
          if constexpr (EPI == E_BIAS) o = v;
          else if constexpr (EPI == E_BIAS_GELU) o = sizeof(TC) == 2 ? gelu_erf_bf16out(v) : gelu_erf(v);
          else if constexpr (EPI == E_BIAS_GAMMA_RES) o = rv[j][i][e] + gam[j][e] * v;
          else o = rv[j][i][e] + v;
          acc[i][j][e] = o;
        }
        asm volatile("" : "+v"(acc[i][j]));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + wm * 64 + i * 16 + frow;
        if (col < g.N && row < g.M) {
          TC* p = C + (size_t)row * g.ldc + col;
          if constexpr ((SPLIT & 4) != 0) {  // 4 consecutive k of the split image: 8-B hi, 8-B lo
            uint32_t h[4], l[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bf16_t hb = f32_to_bf16(acc[i][j][e]);
              h[e] = hb;
              l[e] = f32_to_bf16(acc[i][j][e] - bf16_to_f32(hb));
            }
            bf16_t* o = reinterpret_cast<bf16_t*>(C + (size_t)row * g.ldc) + split_pos(col);
            *reinterpret_cast<uint2*>(o) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
            *reinterpret_cast<uint2*>(o + 32) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
          } else if constexpr (sizeof(TC) == 2) {
            *reinterpret_cast<uint2*>(p) =
                make_uint2((uint32_t)f32_to_bf16(acc[i][j][0]) | ((uint32_t)f32_to_bf16(acc[i][j][1]) << 16),
                           (uint32_t)f32_to_bf16(acc[i][j][2]) | ((uint32_t)f32_to_bf16(acc[i][j][3]) << 16));
          } else {
            *reinterpret_cast<f32x4v*>(p) = acc[i][j];
          }
        }
      }
    }
    return;
  }
  float bias[3][4], gam[3][4], rv[3][4][4];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int colc = min(n0 + wn * 48 + j * 16 + cq + e, g.N - 1);
      bias[j][e] = g.bias ? g.bias[colc] : 0.f;
      gam[j][e] = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[colc] : 0.f;
      if constexpr (RES) {
#pragma unroll
        for (int i = 0; i < 4; ++i) rv[j][i][e] = g.res[(size_t)min(m0 + wm * 64 + i * 16 + frow, g.M - 1) * g.ldr + colc];
      }
    }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + wm * 64 + i * 16 + frow;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = acc[i][j][e] + bias[j][e];
        float o;
        if constexpr (EPI == E_BIAS) o = v;
        else if constexpr (EPI == E_BIAS_GELU) o = sizeof(TC) == 2 ? gelu_erf_bf16out(v) : gelu_erf(v);
        else if constexpr (EPI == E_BIAS_GAMMA_RES) o = rv[j][i][e] + gam[j][e] * v;
        else o = rv[j][i][e] + v;
        acc[i][j][e] = o;
      }
      asm volatile("" : "+v"(acc[i][j]));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = n0 + wn * 48 + j * 16 + cq + e;
        if (col < g.N && row < g.M) store_out<TC>(C + (size_t)row * g.ldc + col, acc[i][j][e]);
      }
    }
  }
}

// option codec_g3 (default 1, Opts in lvx_internal.h): 1: large-M bf16 GEMMs on gemm_glds_kernel; 0: off (cross-check)
// option codec_g3f (default 2, Opts in lvx_internal.h): large-M fp32 (parity mode) GEMMs on gemm_glds_kernel<float>,
// 2: bf16x3 split products, 1: exact fp32 products (cross-check); 0: gemm_mfma (exact fp32, cross-check)
// the LDS-DMA kernel needs enough 128 x 192 tiles to fill the chip
template <typename TA = bf16_t>
static bool g3_ok(const GemmArgs& g) {
  return opts().codec_g3 && g.K % (128 / (int)sizeof(TA)) == 0 && ((g.M + G3_BM - 1) / G3_BM) * ((g.N + G3_BN - 1) / G3_BN) >= 192;
}
// the fp32 parity mode's bf16x3 form of gemm_glds_kernel (option codec_g3f = 2)
static bool g3_split(const GemmArgs& g) { return opts().codec_g3f == 2 && g3_ok<float>(g); }
// its operand given as a split image by the producer kernel (codec_exp bit 16: every bf16x3 GEMM splits
// its fp32 operand in registers instead; the same hi / lo bits either way)
static bool g3_split_in(const GemmArgs& g) { return g3_split(g) && !(opts().codec_exp & 16); }
template <int AMODE, int EPI, typename TC, typename TA = bf16_t, int SPLIT = 0>
static void g3_launch(GemmArgs g, hipStream_t s) {
  static_assert(EPI != E_SCALE, "weight GEMMs only");
  dim3 grid((g.N + G3_BN - 1) / G3_BN, (g.M + G3_BM - 1) / G3_BM);
  // more tiles than CUs: two blocks per CU (2 stages, 80 KB each), else one (3 stages, 120 KB).
  // Kernel traces of the 32 x 256-frame decode: N = 2,304 (768 tiles) 52.5 vs 61 us, N = 768 (256
  // tiles) 40.4 vs 47 us; 16 x 256 frames (N = 2,304: 384 tiles) 1.57 vs 1.70 ms per decode
  // (round 5: one block per CU at any tile count, leaving 40 KB of LDS to the decode kernels beside the
  // codec, measured the same: configs[2] 235.0 / 235.5 / 235.7k vs 235.1 / 234.4 / 235.2k tok/s)
  if (grid.x * grid.y > 256) hipLaunchKernelGGL((gemm_glds_kernel<AMODE, EPI, TC, 2, TA, SPLIT>), grid, dim3(512), 0, s, g);
  else hipLaunchKernelGGL((gemm_glds_kernel<AMODE, EPI, TC, 3, TA, SPLIT>), grid, dim3(512), 0, s, g);
}

// ---------------------------------------------------------------------------------
// Skinny weight GEMM for the small decodes (bf16 mode, M <= SKINNY_MAX_M frames: the first dumps
// and short single-stream chunks). C[M][N] = epi(A[M][K] . W[N][K]^T). One block owns 16 x NJ
// weight rows and 16 x MI frames; its NWV waves take K in NWV slices, so a block's whole operand
// volume is in flight at once instead of a k-loop of dependent round trips (the 64 x 64 tile ran
// 3 k-tiles per split + a split-K combine). Operands go global -> registers directly in
// v_mfma_f32_16x16x32_bf16 layout (A-operand = 16 weight rows, B-operand = 16 frames; lane l: row
// l & 15, k + 8 (l >> 4)); KC 32-wide k-steps per register set, two sets in flight. The k-steps
// per wave (S) are a template constant: the pipeline unrolls completely, no load is issued past
// the slice and no load sits under a branch. The NWV wave partials are summed through LDS in wave
// order (deterministic), then the epilogue.
// ---------------------------------------------------------------------------------
constexpr int SKINNY_MAX_M = 384;
typedef float f32x4s __attribute__((ext_vector_type(4)));
template <int AMODE, int EPI, typename TC, int MI, int NJ, int S, int NWV>
__global__ __launch_bounds__(NWV * 64) void gemm_skinny_kernel(GemmArgs g) {
  constexpr int KC = MI + NJ <= 2 ? 6 : 4;  // k-steps per register set (2 sets: <= 96 VGPRs of operands)
  __shared__ float red[NWV][MI][16][16 * NJ + 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n0 = blockIdx.x * 16 * NJ, m0 = blockIdx.y * 16 * MI;
  const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(g.A);
  const bf16_t* __restrict__ W = reinterpret_cast<const bf16_t*>(g.W);
  const int kw0 = wave * S * 32;                 // first k of this wave's slice
  const int kl = kw0 + 8 * (lane >> 4);          // + this lane's 8-element chunk
  // this lane's weight rows and frames (clamped: rows past N / M are computed, never stored)
  const bf16_t* wrow[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) wrow[j] = W + (size_t)min(n0 + j * 16 + (lane & 15), g.N - 1) * g.ldw + kl;
  int fb[MI], ft[MI];  // A_CONV: (stream, frame) of the lane's frames; A_PLAIN: row
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mc = min(m0 + i * 16 + (lane & 15), g.M - 1);
    if (AMODE == A_CONV) { fb[i] = mc / g.L; ft[i] = mc - fb[i] * g.L; }
    else { fb[i] = mc; ft[i] = 0; }
  }
  u32x4 wv[2][KC][NJ], av[2][KC][MI];
  auto issue = [&](int set, int s0) {
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int st = s0 + c;
      if (st >= S) break;  // compile-time after unrolling
#pragma unroll
      for (int j = 0; j < NJ; ++j) g2_ldb(wv[set][c][j], wrow[j] + st * 32);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (AMODE == A_PLAIN) {
          g2_ld(av[set][c][i], A + (size_t)fb[i] * g.lda + kl + st * 32, true);
        } else {
          const int kb = kw0 + st * 32;  // k of this step (uniform); a 32-wide step lies in one tap
          const int tap = kb / g.cin, cc = kb - tap * g.cin + 8 * (lane >> 4);
          const int tt = ft[i] + tap - (g.taps - 1) / 2;
          g2_ld(av[set][c][i], A + ((size_t)fb[i] * g.L + min(max(tt, 0), g.L - 1)) * g.cin + cc, tt >= 0 && tt < g.L);
        }
      }
    }
  };
  f32x4s acc[NJ][MI];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < MI; ++i) acc[j][i] = f32x4s{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int set, int s0) {
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if (s0 + c >= S) break;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < MI; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv[set][c][j]),
                                                              __builtin_bit_cast(bf16x8, av[set][c][i]), acc[j][i], 0, 0, 0);
    }
  };
  issue(0, 0);
  issue(1, KC);
#pragma unroll
  for (int s0 = 0; s0 < S; s0 += 2 * KC) {
    mma(0, s0);
    issue(0, s0 + 2 * KC);
    mma(1, s0 + KC);
    issue(1, s0 + 3 * KC);
  }
  // wave partials -> LDS: lane holds weight rows 4 (lane >> 4) + r of tile j, frame lane & 15
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][i][lane & 15][j * 16 + 4 * (lane >> 4) + r] = acc[j][i][r];
  __syncthreads();
  constexpr int NW = 16 * NJ;  // output columns per block
#pragma unroll
  for (int e0 = 0; e0 < MI * 16 * NW; e0 += NWV * 64) {
    const int e = e0 + tid;
    if (MI * 16 * NW % (NWV * 64) != 0 && e >= MI * 16 * NW) break;
    const int i = e / (16 * NW), rm = (e / NW) % 16, cn = e % NW;
    const int row = m0 + i * 16 + rm, col = n0 + cn;
    const int rowc = min(row, g.M - 1), colc = min(col, g.N - 1);
    float v = red[0][i][rm][cn];
#pragma unroll
    for (int w = 1; w < NWV; ++w) v += red[w][i][rm][cn];
    const float bias = (EPI != E_SCALE && g.bias) ? g.bias[colc] : 0.f;
    const float gam = (EPI == E_BIAS_GAMMA_RES) ? g.gamma[colc] : 0.f;
    const float o = gemm_epi<EPI>(g, g.res, rowc, colc, v, bias, gam);
    if (row < g.M && col < g.N) store_out<TC>(reinterpret_cast<TC*>(g.C) + (size_t)row * g.ldc + col, o);
  }
}

template <int AMODE, int EPI, typename TC, int MI, int NJ, int NWV>
static bool skinny_go(const GemmArgs& g, hipStream_t s) {
  const dim3 grid((g.N + 16 * NJ - 1) / (16 * NJ), (g.M + 16 * MI - 1) / (16 * MI));
  const int S = g.K / (32 * NWV);
  if (g.K % (32 * NWV)) return false;
  switch (S) {  // the codec's K: 768 (1x1 convs, head), 2,304 (pwconv2, k3 convs), 3,584 (embed k7)
    case 3: hipLaunchKernelGGL((gemm_skinny_kernel<AMODE, EPI, TC, MI, NJ, 3, NWV>), grid, dim3(NWV * 64), 0, s, g); return true;
    case 6: hipLaunchKernelGGL((gemm_skinny_kernel<AMODE, EPI, TC, MI, NJ, 6, NWV>), grid, dim3(NWV * 64), 0, s, g); return true;
    case 9: hipLaunchKernelGGL((gemm_skinny_kernel<AMODE, EPI, TC, MI, NJ, 9, NWV>), grid, dim3(NWV * 64), 0, s, g); return true;
    case 14: hipLaunchKernelGGL((gemm_skinny_kernel<AMODE, EPI, TC, MI, NJ, 14, NWV>), grid, dim3(NWV * 64), 0, s, g); return true;
    case 18: hipLaunchKernelGGL((gemm_skinny_kernel<AMODE, EPI, TC, MI, NJ, 18, NWV>), grid, dim3(NWV * 64), 0, s, g); return true;
    case 28: hipLaunchKernelGGL((gemm_skinny_kernel<AMODE, EPI, TC, MI, NJ, 28, NWV>), grid, dim3(NWV * 64), 0, s, g); return true;
  }
  return false;
}
// Tile shape by M, waves by K (tools/codec_probe.py, decode ms, skinny vs the 64 x 64 split-K /
// 128 x 128 kernels it replaces): 1 x 10 frames 0.29 vs 0.45, 1 x 30 0.37 vs 0.53, 1 x 90 0.41 vs
// 0.58, 1 x 256 0.56 vs 0.71, 2 x 160 0.57 vs 0.74; 1 x 480 0.87 vs 0.84 (the limit below).
// 8 waves for K > 1,024 (a shorter chain per wave), 4 otherwise; 16 x 16 tiles at M <= 16, 32 x 16
// up to 128, 32 x 32 above (measured at 90 and 256 against the other two and 64 x 32 / 32 x 64).
template <int AMODE, int EPI, typename TC>
static bool skinny_launch(const GemmArgs& g, hipStream_t s) {
  const bool w8 = g.K > 1024;
  if (g.M <= 16) return w8 ? skinny_go<AMODE, EPI, TC, 1, 1, 8>(g, s) : skinny_go<AMODE, EPI, TC, 1, 1, 4>(g, s);
  if (g.M <= 128) return w8 ? skinny_go<AMODE, EPI, TC, 2, 1, 8>(g, s) : skinny_go<AMODE, EPI, TC, 2, 1, 4>(g, s);
  return w8 ? skinny_go<AMODE, EPI, TC, 2, 2, 8>(g, s) : skinny_go<AMODE, EPI, TC, 2, 2, 4>(g, s);
}
// option codec_skinny (default 1, Opts in lvx_internal.h): 1: bf16 weight GEMMs with M <= SKINNY_MAX_M on gemm_skinny_kernel; 0: off (cross-check)

// weight GEMMs: bf16 weights -> bf16 MFMA (gemm_bf16_kernel for large M); fp32 weights -> exact
// fp32 MFMA (parity mode). TA / TC: activation types of the operand / output (bf16 only in bf16 mode)
template <typename TW, typename TA, int AMODE, int EPI, typename TC = float>
static void gemm_w(const GemmArgs& g, hipStream_t s) {
  if constexpr (sizeof(TW) == 2) {
    if (g.ascale) {  // fp8 activations x fp8 weights on the block-scaled fp8 MFMA (the decode's large-M pwconv1)
      if constexpr (AMODE == A_PLAIN && EPI != E_SCALE) g3_launch<AMODE, EPI, TC, fp8_t>(g, s);
    } else if (g.wscale) gemm2_launch<TA, fp8_t, AMODE, EPI, TC>(g, s);  // fp8 codec weights: any M
    else if (sizeof(TA) == 2 && opts().codec_skinny && g.M <= SKINNY_MAX_M && skinny_launch<AMODE, EPI, TC>(g, s))
      return;
    else if (sizeof(TA) == 2 && EPI != E_SCALE && g3_ok(g)) g3_launch<AMODE, (EPI == E_SCALE ? E_BIAS : EPI), TC>(g, s);
    else if (opts().codec_g2 && g.M >= CODEC_G2_MIN_M) gemm2_launch<TA, bf16_t, AMODE, EPI, TC>(g, s);
    else gemm_launch<true, TA, bf16_t, AMODE, EPI, TC>(g, 1, s);
  } else {
    static_assert(sizeof(TA) == 4 && sizeof(TC) == 4, "parity mode keeps fp32 activations");
    constexpr int EW = EPI == E_SCALE ? E_BIAS : EPI;
    if (EPI != E_SCALE && g3_split(g)) {
      // A / C as split images only where the orchestration asked for them (decode_impl's ConvNeXt loop)
      if constexpr (AMODE == A_PLAIN && EW == E_BIAS_GELU) {
        // the split-image store lives in the vectorised epilogue only (4 consecutive columns per lane):
        // N or ldc not a multiple of 32 would take the per-element store and write plain fp32, which
        // the next GEMM would read as a split image -- such a C is never split
        const bool cs = g.csplit && (g.N % 32) == 0 && (g.ldc % 32) == 0;
        if (g.asplit && cs) return g3_launch<AMODE, EW, float, float, 7>(g, s);
        if (cs) return g3_launch<AMODE, EW, float, float, 5>(g, s);
      }
      if (g.asplit) return g3_launch<AMODE, EW, float, float, 3>(g, s);
      g3_launch<AMODE, EW, float, float, 1>(g, s);
    } else if (EPI != E_SCALE && opts().codec_g3f == 1 && g3_ok<float>(g)) g3_launch<AMODE, EW, float, float>(g, s);
    else gemm_launch<false, float, float, AMODE, EPI, float>(g, 1, s);
  }
}
// activation x activation GEMMs (AttnBlock scores / P.V): operands are fp32 in memory
template <typename TW, int EPI, typename TC = float>
static void gemm_act(const GemmArgs& g, int batch, hipStream_t s) {
  if constexpr (sizeof(TW) == 2) gemm_launch<true, float, float, A_PLAIN, EPI, TC>(g, batch, s);
  else gemm_launch<false, float, float, A_PLAIN, EPI, float>(g, batch, s);
}

// ---------------------------------------------------------------------------------
// GroupNorm (32 groups, eps 1e-6, affine) [+ swish] applied once per (stream, group): statistics
// (two-pass fp32) and the transformed output in one kernel, so the following conv / 1x1 GEMM
// reads a ready operand (decoder/models.py:15-16, 59-68, 109).
// ---------------------------------------------------------------------------------
// One (stream, group) of GroupNorm (32 groups x 24 channels, eps 1e-6) over L frames, 256
// threads, two-pass fp32: 16-byte loads (6 per frame), eight in flight per thread (unconditional:
// a load under a branch makes the compiler drain all outstanding loads), the group's
// values kept in LDS when L <= GN_LDS_FRAMES for the second pass and the apply.
constexpr int GN_LDS_FRAMES = 512;  // 48 KB of LDS
__device__ __forceinline__ float4 gn_ld(const float* base, int e) {
  const int t = e / 6, q = e - t * 6;
  return *reinterpret_cast<const float4*>(base + (size_t)t * CD + q * 4);
}
__device__ __forceinline__ float sum4(float4 v) { return (v.x + v.y) + (v.z + v.w); }
__device__ __forceinline__ float sqd4(float4 v, float m) {
  const float a = v.x - m, b = v.y - m, c = v.z - m, d = v.w - m;
  return (a * a + b * b) + (c * c + d * d);
}
__device__ __forceinline__ void gn_group_stats(const float* base, int L, float* red, float4* cache, float& mean,
                                               float& rstd) {
  const int n4 = L * 6, tid = threadIdx.x;
  const bool lds = L <= GN_LDS_FRAMES;
  // 8 loads in flight per thread per round: clamped index, unconditional load, masked use
  float s = 0.f;
  for (int e0 = tid; e0 < n4; e0 += 8 * 256) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = gn_ld(base, min(e0 + u * 256, n4 - 1));
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (e0 + u * 256 < n4) {
        if (lds) cache[e0 + u * 256] = v[u];
        s += sum4(v[u]);
      }
  }
  mean = block_sum<256>(s, red) / (float)(L * 24);  // its barriers also publish the LDS copy
  float q = 0.f;
  if (lds) {
    for (int e = tid; e < n4; e += 256) q += sqd4(cache[e], mean);
  } else {
    for (int e0 = tid; e0 < n4; e0 += 8 * 256) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = gn_ld(base, min(e0 + u * 256, n4 - 1));
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u * 256 < n4) q += sqd4(v[u], mean);
    }
  }
  rstd = 1.0f / sqrtf(block_sum<256>(q, red) / (float)(L * 24) + 1e-6f);
}

__device__ __forceinline__ void store4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void store4(bf16_t* p, float4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16),
                                            (uint32_t)f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16));
}

// 4 consecutive channels c..c+3 (c % 4 == 0) of row `row`: plain, or (SPO, fp32 parity mode) into the
// row's split image for a bf16x3 conv / 1x1 GEMM (split_store's layout: 8-B hi, 8-B lo)
template <bool SPO, typename TO>
__device__ __forceinline__ void gn_store(TO* row, int c, float4 o) {
  if constexpr (SPO) {
    const float v[4] = {o.x, o.y, o.z, o.w};
    uint32_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bf16_t hb = f32_to_bf16(v[e]);
      h[e] = hb;
      l[e] = f32_to_bf16(v[e] - bf16_to_f32(hb));
    }
    bf16_t* p = reinterpret_cast<bf16_t*>(row) + split_pos(c);
    *reinterpret_cast<uint2*>(p) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    *reinterpret_cast<uint2*>(p + 32) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
  } else {
    store4(row + c, o);
  }
}

// GroupNorm (+ swish) of one (stream, group), decoder/models.py:15-16,58-78 (ResnetBlock norms)
// and :107-127 (AttnBlock norm): y = swish?((x - mean) * rstd * w + b)
template <bool SWISH, typename TO, bool SPO = false>
__global__ __launch_bounds__(256) void gn_apply_kernel(const float* __restrict__ x, int L, const float* __restrict__ gw,
                                                       const float* __restrict__ gb, TO* __restrict__ y) {
  __shared__ float red[4];
  __shared__ float4 cache[GN_LDS_FRAMES * 6];
  const int gi = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  constexpr int CG = CD / GN_G;  // 24 channels
  const size_t off = (size_t)b * L * CD + gi * CG;
  // gamma / beta of this thread's apply elements, loaded up front (in the loop they were one
  // dependent round trip per iteration): element e = tid + 256 k has chunk (tid + 4 k) mod 6, a
  // cycle of three chunks
  const int q0 = tid % 6, q1 = (q0 + 4) % 6, q2 = (q0 + 2) % 6;
  const float4* gw4 = reinterpret_cast<const float4*>(gw + gi * CG);
  const float4* gb4 = reinterpret_cast<const float4*>(gb + gi * CG);
  const float4 wq0 = gw4[q0], wq1 = gw4[q1], wq2 = gw4[q2], bq0 = gb4[q0], bq1 = gb4[q1], bq2 = gb4[q2];
  float mean, rstd;
  gn_group_stats(x + off, L, red, cache, mean, rstd);
  const bool lds = L <= GN_LDS_FRAMES;
  int ph = 0;
  for (int e = tid; e < L * 6; e += 256, ph = ph == 2 ? 0 : ph + 1) {
    const int t = e / 6, q = e - t * 6;
    const float4 v = lds ? cache[e] : gn_ld(x + off, e);
    const float4 w = ph == 0 ? wq0 : ph == 1 ? wq1 : wq2, bb = ph == 0 ? bq0 : ph == 1 ? bq1 : bq2;
    float4 o = make_float4((v.x - mean) * rstd * w.x + bb.x, (v.y - mean) * rstd * w.y + bb.y,
                           (v.z - mean) * rstd * w.z + bb.z, (v.w - mean) * rstd * w.w + bb.w);
    if (SWISH) o = make_float4(swishf(o.x), swishf(o.y), swishf(o.z), swishf(o.w));
    gn_store<SPO>(y + ((size_t)b * L + t) * CD, gi * CG + q * 4, o);
  }
}

// gn_apply for L * 6 <= 2,048 (L <= 341: every chunk decode): the group in one round of 8 loads per
// thread, issued before the affine operands (gn_apply_kernel waited for those at its loop head: one
// more round trip ahead of the data), values kept in registers (no LDS copy: 4 blocks per CU). Same
// sums in the same order as gn_apply_kernel: same bits.
template <bool SWISH, typename TO, bool SPO = false>
__global__ __launch_bounds__(256) void gn_apply1_kernel(const float* __restrict__ x, int L, const float* __restrict__ gw,
                                                        const float* __restrict__ gb, TO* __restrict__ y) {
  __shared__ float red[4];
  const int gi = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  constexpr int CG = CD / GN_G;
  const size_t off = (size_t)b * L * CD + gi * CG;
  const int q0 = tid % 6, q1 = (q0 + 4) % 6, q2 = (q0 + 2) % 6;
  const float4* gw4 = reinterpret_cast<const float4*>(gw + gi * CG);
  const float4* gb4 = reinterpret_cast<const float4*>(gb + gi * CG);
  const int n4 = L * 6;
  float4 v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = gn_ld(x + off, min(tid + u * 256, n4 - 1));
  const float4 wq0 = gw4[q0], wq1 = gw4[q1], wq2 = gw4[q2], bq0 = gb4[q0], bq1 = gb4[q1], bq2 = gb4[q2];
  __builtin_amdgcn_sched_barrier(0);
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (tid + u * 256 < n4) s += sum4(v[u]);
  const float mean = block_sum<256>(s, red) / (float)(L * 24);
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (tid + u * 256 < n4) q += sqd4(v[u], mean);
  const float rstd = 1.0f / sqrtf(block_sum<256>(q, red) / (float)(L * 24) + 1e-6f);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + u * 256;
    if (e >= n4) break;
    const int t = e / 6, qq = e - t * 6, ph = u % 3;  // chunk (tid + 4 u) mod 6
    const float4 w = ph == 0 ? wq0 : ph == 1 ? wq1 : wq2, bb = ph == 0 ? bq0 : ph == 1 ? bq1 : bq2;
    float4 o = make_float4((v[u].x - mean) * rstd * w.x + bb.x, (v[u].y - mean) * rstd * w.y + bb.y,
                           (v[u].z - mean) * rstd * w.z + bb.z, (v[u].w - mean) * rstd * w.w + bb.w);
    if (SWISH) o = make_float4(swishf(o.x), swishf(o.y), swishf(o.z), swishf(o.w));
    gn_store<SPO>(y + ((size_t)b * L + t) * CD, gi * CG + qq * 4, o);
  }
}
// codec A/B bits (development): 1 the general gn_apply at every L; 6: dwconv FT at >= 2,048 frames
// (0: 4, 2: 16, 4: 32, 6: 8); 8: library exp / sin / cos in the bf16 iSTFT; 16: fp32 bf16x3 GEMMs
// split their operands in registers (no split-image producers; same bits)
// option codec_exp (default 0, Opts in lvx_internal.h):
template <bool SWISH, typename TO>
static void gn_apply_launch(const float* x, int B, int L, const float* gw, const float* gb, TO* y, hipStream_t s,
                            bool spo = false) {  // spo: y as split images (fp32, the consumer GEMM's asplit)
  if constexpr (sizeof(TO) == 4) {
    if (spo) {
      if (L * 6 <= 8 * 256 && !(opts().codec_exp & 1)) hipLaunchKernelGGL((gn_apply1_kernel<SWISH, TO, true>), dim3(GN_G, B), dim3(256), 0, s, x, L, gw, gb, y);
      else hipLaunchKernelGGL((gn_apply_kernel<SWISH, TO, true>), dim3(GN_G, B), dim3(256), 0, s, x, L, gw, gb, y);
      return;
    }
  }
  if (L * 6 <= 8 * 256 && !(opts().codec_exp & 1)) hipLaunchKernelGGL((gn_apply1_kernel<SWISH, TO>), dim3(GN_G, B), dim3(256), 0, s, x, L, gw, gb, y);
  else hipLaunchKernelGGL((gn_apply_kernel<SWISH, TO>), dim3(GN_G, B), dim3(256), 0, s, x, L, gw, gb, y);
}

// ---------------------------------------------------------------------------------
// GroupNorm statistics (decoder/models.py:15-16: 32 groups, eps 1e-6): per (stream, group)
// mean and 1/sqrt(var + eps) over L frames x 24 channels, two-pass fp32.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gn_stats_kernel(const float* __restrict__ x, int L, float* __restrict__ stats) {
  __shared__ float red[4];
  __shared__ float4 cache[GN_LDS_FRAMES * 6];
  const int gi = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  constexpr int CG = CD / GN_G;  // 24
  float mean, rstd;
  gn_group_stats(x + (size_t)b * L * CD + gi * CG, L, red, cache, mean, rstd);
  if (tid == 0) {
    stats[((size_t)b * GN_G + gi) * 2] = mean;
    stats[((size_t)b * GN_G + gi) * 2 + 1] = rstd;
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
  float sc[3], sh[3];  // the closing affine's operands with the inputs (not behind the reductions)
#pragma unroll
  for (int j = 0; j < 3; ++j) { sc[j] = scale[tid + 256 * j]; sh[j] = shift[tid + 256 * j]; }
  float v[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j, gi = c / (CD / GN_G);
    v[j] = (x[(size_t)m * CD + c] - stats[((size_t)b * GN_G + gi) * 2]) * stats[((size_t)b * GN_G + gi) * 2 + 1] * gw[c] + gb[c];
  }
  __builtin_amdgcn_sched_barrier(0);
  row_ln(v, 1e-6f, red);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
    y[(size_t)m * CD + c] = v[j] * sc[j] + sh[j];
  }
}

// ConvNeXt prologue (modules.py:45-50): depthwise conv k7 pad 3 (+bias, tap-major weights [7][768]
// repacked at upload) then AdaLN, over a tile of FT consecutive frames of one stream per block:
// each thread owns 3 channels and slides the 7-tap window along the tile, so x is read
// (FT + 6) / FT times instead of 7 and the tap weights once per tile instead of once per frame (the
// round-1 one-frame-per-block form moved 43 KB through L2 per 1.5 KB written: 19.6 us at 8,192
// frames = 1.9 TB/s). Taps outside [0, L) read a clamped frame and are dropped by a select, in the
// guarded sum's order; the LayerNorm reductions follow row_ln's order (same bits as that form).
// FT = 16 for large M, 4 when there are few frames.
// SPO (fp32 parity mode): y written as the split image of its rows (split_store) for pwconv1's bf16x3 GEMM
// TO = fp8_t (codec_dtype FP8, pwconv1 on the block-scaled fp8 MFMA): y as e4m3fn with one fp32 scale per
// frame in ys (y = q * ys[frame], ys = max |y| / 448 over the frame's 768 channels, RNE)
template <typename TO, int FT, bool SPO = false>
__global__ __launch_bounds__(256) void dwconv_adaln_tile_kernel(const float* __restrict__ x, int L,
                                                                const float* __restrict__ dwt,
                                                                const float* __restrict__ dwb,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift, TO* __restrict__ y,
                                                                float* __restrict__ ys = nullptr) {
  __shared__ float red[3][4][FT];
  const int b = blockIdx.y, t0 = blockIdx.x * FT, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  float v[3][FT], sc[3], sh[3];
  // every load of the block issued before the first use, the small operands first (the compiler had
  // interleaved the three channel passes: three dependent round trips ahead of the main 66 loads);
  // the sched_barrier keeps the FMAs behind them
  float w[3][7], xs[3][FT + 6], bb[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
#pragma unroll
    for (int k = 0; k < 7; ++k) w[j][k] = dwt[k * CD + c];
    bb[j] = dwb[c];
    sc[j] = scale[c];
    sh[j] = shift[c];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
#pragma unroll
    for (int i = 0; i < FT + 6; ++i) xs[j][i] = x[((size_t)b * L + min(max(t0 + i - 3, 0), L - 1)) * CD + c];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
#pragma unroll
    for (int f = 0; f < FT; ++f) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const int tt = t0 + f + k - 3;
        const float na = a + w[j][k] * xs[j][f + k];
        a = (tt >= 0 && tt < L) ? na : a;
      }
      v[j][f] = a + bb[j];
    }
  }
  // AdaLayerNorm (modules.py:81-86) per frame: block_sum's order (wave DPP sum, then waves 0..3)
  float mean[FT];
#pragma unroll
  for (int f = 0; f < FT; ++f) {
    const float s = wave_sum(v[0][f] + v[1][f] + v[2][f]);
    if (lane == 0) red[0][wave][f] = s;
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < FT; ++f) {
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += red[0][i][f];
    mean[f] = r * (1.0f / CD);
  }
#pragma unroll
  for (int f = 0; f < FT; ++f) {
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) { v[j][f] -= mean[f]; q += v[j][f] * v[j][f]; }
    q = wave_sum(q);
    if (lane == 0) red[1][wave][f] = q;
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < FT; ++f) {
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += red[1][i][f];
    const float rstd = 1.0f / sqrtf(r * (1.0f / CD) + 1e-6f);
    if constexpr (sizeof(TO) == 1) {  // fp8: the frame's max |y| first (block max), then q = y / s
      float o[3], m = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        o[j] = v[j][f] * rstd * sc[j] + sh[j];
        m = fmaxf(m, fabsf(o[j]));
      }
      m = wave_max(m);
      if (lane == 0) red[2][wave][f] = m;
      __syncthreads();
      m = fmaxf(fmaxf(red[2][0][f], red[2][1][f]), fmaxf(red[2][2][f], red[2][3][f]));
      const float sf = m > 0.f ? m * (1.0f / 448.f) : 1.f, inv = 1.0f / sf;
      if (t0 + f < L) {
#pragma unroll
        for (int j = 0; j < 3; ++j) y[((size_t)b * L + t0 + f) * CD + tid + 256 * j] = f32_to_fp8(o[j] * inv);
        if (tid == 0) ys[(size_t)b * L + t0 + f] = sf;
      }
      continue;
    }
    if (t0 + f < L) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float o = v[j][f] * rstd * sc[j] + sh[j];
        if constexpr (SPO) split_store(reinterpret_cast<float*>(y + ((size_t)b * L + t0 + f) * CD), tid + 256 * j, o);
        else store_out<TO>(y + ((size_t)b * L + t0 + f) * CD + tid + 256 * j, o);
      }
    }
  }
}

// final_layer_norm (affine, eps 1e-6); SPO: y as split images (fp32 parity mode, bf16x3 head GEMM)
template <typename TO, bool SPO = false>
__global__ __launch_bounds__(256) void ln_affine_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bb, TO* __restrict__ y) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  float v[3], wv[3], bv[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    v[j] = x[(size_t)m * CD + tid + 256 * j];
    wv[j] = w[tid + 256 * j];
    bv[j] = bb[tid + 256 * j];
  }
  __builtin_amdgcn_sched_barrier(0);  // the affine's operands with the row, not behind the reductions
  row_ln(v, 1e-6f, red);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = tid + 256 * j;
    if constexpr (SPO) split_store(reinterpret_cast<float*>(y + (size_t)m * CD), c, v[j] * wv[j] + bv[j]);
    else store_out<TO>(y + (size_t)m * CD + c, v[j] * wv[j] + bv[j]);
  }
}

// features [B][512][L] -> [B*L][512]
template <typename TO>
__global__ void feats_transpose_kernel(const float* __restrict__ f, int L, TO* __restrict__ out) {
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
    if (t < L) store_out<TO>(out + ((size_t)b * L + t) * CIN + c, tile[tx][i]);
  }
}

// codes [B*L] -> [B*L][512]
// SPO (fp32 parity mode): the rows as split images for the embed conv's bf16x3 GEMM (gn_store)
template <bool SPO = false>
__global__ void codes_gather_kernel(const float* __restrict__ cb, const int32_t* __restrict__ codes, float* __restrict__ out, int32_t* __restrict__ err) {
  const int m = blockIdx.x;
  const int raw = codes[m];
  const int code = min(max(raw, 0), 4095);  // clamped for the load; flagged (lvx_check_errors -> LVX_E_INDEX)
  if (threadIdx.x == 0 && raw != code) atomicOr(err, 4);
  const float4 v = reinterpret_cast<const float4*>(cb + (size_t)code * CIN)[threadIdx.x];
  gn_store<SPO>(out + (size_t)m * CIN, 4 * threadIdx.x, v);
}
// bf16 mode: the rows as the embed conv's bf16 operand
__global__ void codes_gather_bf16_kernel(const float* __restrict__ cb, const int32_t* __restrict__ codes,
                                         bf16_t* __restrict__ out, int32_t* __restrict__ err) {
  const int m = blockIdx.x;
  const int raw = codes[m];
  const int code = min(max(raw, 0), 4095);  // clamped for the load; flagged (lvx_check_errors -> LVX_E_INDEX)
  if (threadIdx.x == 0 && raw != code) atomicOr(err, 4);
  const float4 v = reinterpret_cast<const float4*>(cb + (size_t)code * CIN)[threadIdx.x];
  reinterpret_cast<uint2*>(out + (size_t)m * CIN)[threadIdx.x] =
      make_uint2((uint32_t)f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16),
                 (uint32_t)f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16));
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

// One radix-R Stockham pass over the 640-point transform in LDS. The twiddles a thread needs
// (e^{+2 pi i k r / (Ns R)} = tw[2 (640 / (Ns R)) k r], for its j = tid + 256 it) are loaded into
// registers by stockham_tw at the top of the kernel, with the spectrum: the passes then run on LDS
// alone (a twiddle load inside each pass had been one L2 round trip per pass).
template <int R, int NJ>
struct StockTw {
  float2 t[NJ][R - 1];
};
template <int R, int NJ>
__device__ __forceinline__ void stockham_tw(int Ns, const float2* __restrict__ tw, StockTw<R, NJ>& w) {
  const int step = FM / (Ns * R);
#pragma unroll
  for (int it = 0; it < NJ; ++it) {
    const int j = min((int)threadIdx.x + 256 * it, FM / R - 1), k = j % Ns;
#pragma unroll
    for (int r = 1; r < R; ++r) w.t[it][r - 1] = tw[(2 * step * k * r) % (2 * FM)];
  }
}
template <int R, int NJ>
__device__ __forceinline__ void stockham_pass(const float2* __restrict__ src, float2* __restrict__ dst, int Ns,
                                              const StockTw<R, NJ>& w, const float2 (&c5)[5]) {
#pragma unroll
  for (int it = 0; it < NJ; ++it) {
    const int j = threadIdx.x + 256 * it;
    if (j >= FM / R) break;
    const int k = j % Ns;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float2 x = src[j + r * (FM / R)];
      v[r] = (r == 0) ? x : cmul(x, w.t[it][r - 1]);
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
    } else {  // R == 5: direct 5-point DFT with e^{+2 pi i rq/5} = tw[256 * ((r q) mod 5)] = c5[(r q) mod 5]
#pragma unroll
      for (int q = 0; q < R; ++q) {
        float2 accv = v[0];
#pragma unroll
        for (int r = 1; r < R; ++r) {
          const float2 c = cmul(v[r], c5[(r * q) % 5]);
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

// FAST (bf16 codec modes, whose PCM is held to 2 % relative RMS of fp32): exp / sin / cos of the head's
// magnitudes and phases on the native v_exp / v_sin / v_cos (~1e-6 relative for |phase| of order 10)
// instead of the range-reduced library forms; the fp32 parity mode keeps expf / cosf / sinf.
template <bool FAST>
__global__ __launch_bounds__(256) void istft_frames_kernel(const float* __restrict__ spec, const float2* __restrict__ tw,
                                                           const float* __restrict__ window, float* __restrict__ frames) {
  __shared__ float2 bufA[FM], bufB[FM];
  __shared__ float2 X[NB];
  const int f = blockIdx.x, tid = threadIdx.x;
  const float* row = spec + (size_t)f * (2 * NB);
  // every global load of the block first (clamped indices, no load under a branch): the frame's
  // magnitudes / phases, the twiddles of the Z step and of each pass, the window
  float lm[3], lp[3];
  float2 tz[3], wv[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int k = min(tid + 256 * u, NB - 1);
    lm[u] = row[k];
    lp[u] = row[NB + k];
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) tz[u] = tw[min(tid + 256 * u, FM - 1)];
  StockTw<4, 1> w1, w2, w3;
  StockTw<2, 2> w4;
  StockTw<5, 1> w5;
  stockham_tw(1, tw, w1);
  stockham_tw(4, tw, w2);
  stockham_tw(16, tw, w3);
  stockham_tw(64, tw, w4);
  stockham_tw(128, tw, w5);
  float2 c5[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) c5[m] = tw[256 * m];
#pragma unroll
  for (int u = 0; u < 3; ++u) wv[u] = reinterpret_cast<const float2*>(window)[min(tid + 256 * u, FM - 1)];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int k = tid + 256 * u;
    if (k < NB) {
      const float mag = fminf(FAST ? __expf(lm[u]) : expf(lm[u]), 100.0f);
      const float ph = lp[u];
      float2 x = FAST ? make_float2(mag * __cosf(ph), mag * __sinf(ph)) : make_float2(mag * cosf(ph), mag * sinf(ph));
      if (k == 0 || k == NB - 1) x.y = 0.f;  // C2R ignores imag of DC and Nyquist
      X[k] = x;
    }
  }
  __syncthreads();
  // Z[k] = Xe[k] + i Xo[k];  Xe = (X[k] + conj X[M-k]) / 2,  Xo = (X[k] - conj X[M-k]) e^{+2 pi i k/N} / 2
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int k = tid + 256 * u;
    if (k < FM) {
      const float2 a = X[k];
      const float2 bc = make_float2(X[FM - k].x, -X[FM - k].y);
      const float2 xe = make_float2(0.5f * (a.x + bc.x), 0.5f * (a.y + bc.y));
      const float2 xo = cmul(make_float2(0.5f * (a.x - bc.x), 0.5f * (a.y - bc.y)), tz[u]);
      bufA[k] = make_float2(xe.x - xo.y, xe.y + xo.x);
    }
  }
  __syncthreads();
  stockham_pass(bufA, bufB, 1, w1, c5);
  stockham_pass(bufB, bufA, 4, w2, c5);
  stockham_pass(bufA, bufB, 16, w3, c5);
  stockham_pass(bufB, bufA, 64, w4, c5);
  stockham_pass(bufA, bufB, 128, w5, c5);
  float* out = frames + (size_t)f * NFFT;
  const float sc = 1.0f / FM;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int m = tid + 256 * u;
    if (m < FM) {
      const float2 zz = bufB[m];
      reinterpret_cast<float2*>(out)[m] = make_float2(zz.x * sc * wv[u].x, zz.y * sc * wv[u].y);
    }
  }
}

// overlap-add (fold, hop 320) + trim 480 + divide by the window-square envelope
__global__ void istft_ola_kernel(const float* __restrict__ frames, const float* __restrict__ window, int L,
                                 float* __restrict__ pcm, int32_t* __restrict__ err) {
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
  if (!(env > 1e-11f)) atomicOr(err, 8);  // spectral_ops.py:72 `assert (window_envelope > 1e-11).all()`
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
  // operands that only feed a weight GEMM are stored in the GEMM's input precision (bf16 in bf16
  // mode: the GEMM would round them on the way into LDS anyway, so results are unchanged)
  typedef TW TAct;
  TAct* gn = reinterpret_cast<TAct*>(sc.gn);  // [M][768] normalised operand of the next conv / 1x1
  TAct* t2a = reinterpret_cast<TAct*>(t2);    // dwconv+AdaLN / final LN output (pwconv1 / head operand)
  TAct* t1a = reinterpret_cast<TAct*>(t1);    // GELU(pwconv1) (pwconv2 operand)
  // a3: features, time-major [M][512]
  TAct* feats = reinterpret_cast<TAct*>(sc.feats);
  g_ws_floats = sc.ws_floats;
  g_tick = sc.tick;
  // fp32 parity mode: a producer whose output feeds a bf16x3 GEMM writes it as split images (the
  // GEMM's operand has no other reader)
  auto spl = [&](GemmArgs& c) {
    if constexpr (sizeof(TW) == 4) c.asplit = g3_split_in(c);
    return c.asplit != 0;
  };
  GemmArgs g{};
  g.ws = sc.ws;
  g.L = L;
  g.M = M;
  // embed Conv1d(512->768, k7, pad 3)
  g.A = feats; g.lda = CIN; g.cin = CIN; g.taps = 7;
  g.W = w.embed_w; g.wscale = w.embed_s; g.ldw = 7 * CIN; g.K = 7 * CIN; g.N = CD;
  g.C = x; g.ldc = CD; g.bias = w.embed_b;
  spl(g);
  if (codes) {
    if constexpr (sizeof(TAct) == 2) hipLaunchKernelGGL(codes_gather_bf16_kernel, dim3(M), dim3(CIN / 4), 0, s, w.codebook, codes, feats, sc.err);
    else if (g.asplit) hipLaunchKernelGGL(codes_gather_kernel<true>, dim3(M), dim3(CIN / 4), 0, s, w.codebook, codes, feats, sc.err);
    else hipLaunchKernelGGL(codes_gather_kernel<>, dim3(M), dim3(CIN / 4), 0, s, w.codebook, codes, feats, sc.err);
  } else {
    g.asplit = 0;  // features handed in: transposed as plain rows
    hipLaunchKernelGGL(feats_transpose_kernel<TAct>, dim3((L + 31) / 32, CIN / 32, B), dim3(256), 0, s, feats_in, L, feats);
  }
  gemm_w<TW, TAct, A_CONV, E_BIAS>(g, s);

  auto resnet = [&](int i) {  // models.py:58-78
    GemmArgs c{};
    c.ws = sc.ws;
    c.L = L; c.M = M; c.cin = CD; c.taps = 3; c.K = 3 * CD; c.N = CD; c.ldw = 3 * CD;
    c.A = gn; c.lda = CD;
    c.W = w.rn_c1w[i]; c.wscale = w.rn_c1s[i]; c.bias = w.rn_c1b[i]; c.C = t1; c.ldc = CD;
    gn_apply_launch<true, TAct>(x, B, L, w.rn_n1w[i], w.rn_n1b[i], gn, s, spl(c));
    gemm_w<TW, TAct, A_CONV, E_BIAS>(c, s);
    gn_apply_launch<true, TAct>(t1, B, L, w.rn_n2w[i], w.rn_n2b[i], gn, s, c.asplit != 0);
    c.W = w.rn_c2w[i]; c.wscale = w.rn_c2s[i]; c.bias = w.rn_c2b[i]; c.C = x; c.res = x; c.ldr = CD;
    gemm_w<TW, TAct, A_CONV, E_BIAS_RES>(c, s);
  };
  resnet(0);
  resnet(1);
  {  // AttnBlock (models.py:107-127)
    GemmArgs c{};
    c.ws = sc.ws;
    c.L = L; c.M = M; c.K = CD; c.N = 3 * CD; c.ldw = CD;
    c.A = gn; c.lda = CD;
    c.W = w.at_qkv_w; c.wscale = w.at_qkv_s; c.bias = w.at_qkv_b; c.C = t1; c.ldc = CFF;
    gn_apply_launch<false, TAct>(x, B, L, w.at_nw, w.at_nb, gn, s, spl(c));
    gemm_w<TW, TAct, A_PLAIN, E_BIAS>(c, s);
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
    if constexpr (sizeof(TAct) == 2) {  // h (bf16) into gn: it only feeds proj_out
      p.C = gn; p.ldc = CD; p.sC = (long long)L * CD;
    } else {  // h overwrites the (consumed) q columns
      p.C = t1; p.ldc = CFF; p.sC = (long long)L * CFF;
    }
    gemm_act<TW, E_BIAS, TAct>(p, B, s);
    // proj_out + residual
    GemmArgs o{};
    o.ws = sc.ws;
    o.M = M; o.N = CD; o.K = CD; o.L = L;
    o.A = p.C; o.lda = p.ldc; o.W = w.at_proj_w; o.wscale = w.at_proj_s; o.ldw = CD; o.bias = w.at_proj_b;
    o.C = x; o.ldc = CD; o.res = x; o.ldr = CD;
    gemm_w<TW, TAct, A_PLAIN, E_BIAS_RES>(o, s);
  }
  resnet(2);
  resnet(3);
  // pos_net[5] GroupNorm + backbone AdaLN
  hipLaunchKernelGGL(gn_stats_kernel, dim3(GN_G, B), dim3(256), 0, s, x, L, sc.stats);
  hipLaunchKernelGGL(gn_adaln_kernel, dim3(M), dim3(256), 0, s, x, L, sc.stats, w.pn_w, w.pn_b,
                     w.ada_scale + (size_t)bw * CD, w.ada_shift + (size_t)bw * CD, x);
  for (int i = 0; i < 12; ++i) {  // ConvNeXt blocks (modules.py:43-60)
    const int dwft = (opts().codec_exp >> 1) & 3;
    GemmArgs c{};
    c.ws = sc.ws;
    c.M = M; c.L = L; c.N = CFF; c.K = CD; c.ldw = CD;
    c.A = t2a; c.lda = CD; c.W = w.pw1_w[i]; c.wscale = w.pw1_s[i]; c.bias = w.pw1_b[i]; c.C = t1a; c.ldc = CFF;
    GemmArgs d{};
    d.ws = sc.ws;
    d.M = M; d.L = L; d.N = CD; d.K = CFF; d.ldw = CFF;
    d.A = t1a; d.lda = CFF; d.W = w.pw2_w[i]; d.wscale = w.pw2_s[i]; d.bias = w.pw2_b[i]; d.gamma = w.gamma[i];
    d.C = x; d.ldc = CD; d.res = x; d.ldr = CD;
    // fp32 parity mode with both GEMMs on the bf16x3 kernel: the dwconv output and pwconv1's output
    // go to HBM as split images (hi / lo bf16 of each element, split_store: the same bits the GEMMs'
    // in-register split makes, computed once per element instead of once per reading block)
    if constexpr (sizeof(TW) == 4) {
      const bool s1 = g3_split_in(c) && dwft == 0, s2 = g3_split_in(d);
      const bool cs = s1 && s2 && (c.N % 32) == 0 && (c.ldc % 32) == 0;  // (gemm_w's split-store condition)
      c.asplit = s1;
      c.csplit = cs;
      d.asplit = cs;
    }
    // codec_dtype FP8 at large M: pwconv1 as fp8 x fp8 on the block-scaled MFMA, its operand written in
    // e4m3fn with per-frame scales by the dwconv + AdaLN kernel (option codec_exp bit 32: off, the
    // fp8-weight bf16 GEMM)
    const bool q8 = sizeof(TW) == 2 && c.wscale && sc.rowscale && !(opts().codec_exp & 32) && g3_ok<fp8_t>(c);
    if (q8) {
      c.A = t2; c.ascale = sc.rowscale;  // (t2 as bytes: [M][768] e4m3fn)
      hipLaunchKernelGGL((dwconv_adaln_tile_kernel<fp8_t, 4>), dim3((L + 3) / 4, B), dim3(256), 0, s, x, L, w.dw_w[i],
                         w.dw_b[i], w.cn_scale[i] + (size_t)bw * CD, w.cn_shift[i] + (size_t)bw * CD,
                         reinterpret_cast<fp8_t*>(t2), sc.rowscale);
    } else if (c.asplit)
      hipLaunchKernelGGL((dwconv_adaln_tile_kernel<TAct, 4, true>), dim3((L + 3) / 4, B), dim3(256), 0, s, x, L, w.dw_w[i],
                         w.dw_b[i], w.cn_scale[i] + (size_t)bw * CD, w.cn_shift[i] + (size_t)bw * CD, t2a);
    else if (M >= 2048 && dwft == 3)
      hipLaunchKernelGGL((dwconv_adaln_tile_kernel<TAct, 8>), dim3((L + 7) / 8, B), dim3(256), 0, s, x, L, w.dw_w[i],
                         w.dw_b[i], w.cn_scale[i] + (size_t)bw * CD, w.cn_shift[i] + (size_t)bw * CD, t2a);
    else if (M >= 2048 && dwft == 2)
      hipLaunchKernelGGL((dwconv_adaln_tile_kernel<TAct, 32>), dim3((L + 31) / 32, B), dim3(256), 0, s, x, L, w.dw_w[i],
                         w.dw_b[i], w.cn_scale[i] + (size_t)bw * CD, w.cn_shift[i] + (size_t)bw * CD, t2a);
    else if (M >= 2048 && dwft == 1)
      hipLaunchKernelGGL((dwconv_adaln_tile_kernel<TAct, 16>), dim3((L + 15) / 16, B), dim3(256), 0, s, x, L, w.dw_w[i],
                         w.dw_b[i], w.cn_scale[i] + (size_t)bw * CD, w.cn_shift[i] + (size_t)bw * CD, t2a);
    else
      hipLaunchKernelGGL((dwconv_adaln_tile_kernel<TAct, 4>), dim3((L + 3) / 4, B), dim3(256), 0, s, x, L, w.dw_w[i],
                         w.dw_b[i], w.cn_scale[i] + (size_t)bw * CD, w.cn_shift[i] + (size_t)bw * CD, t2a);
    gemm_w<TW, TAct, A_PLAIN, E_BIAS_GELU, TAct>(c, s);
    gemm_w<TW, TAct, A_PLAIN, E_BIAS_GAMMA_RES>(d, s);
  }
  {  // final LayerNorm, ISTFTHead.out Linear(768 -> 1282)
    GemmArgs h{};
    h.ws = sc.ws;
    h.M = M; h.L = L; h.N = 2 * NB; h.K = CD; h.ldw = CD;
    h.A = t2a; h.lda = CD; h.W = w.head_w; h.wscale = w.head_s; h.bias = w.head_b; h.C = sc.spec; h.ldc = 2 * NB;
    if (spl(h)) hipLaunchKernelGGL((ln_affine_kernel<TAct, true>), dim3(M), dim3(256), 0, s, x, w.fln_w, w.fln_b, t2a);
    else hipLaunchKernelGGL(ln_affine_kernel<TAct>, dim3(M), dim3(256), 0, s, x, w.fln_w, w.fln_b, t2a);
    gemm_w<TW, TAct, A_PLAIN, E_BIAS>(h, s);
  }
  if (sizeof(TAct) == 2 && !(opts().codec_exp & 8))
    hipLaunchKernelGGL(istft_frames_kernel<true>, dim3(M), dim3(256), 0, s, sc.spec,
                       reinterpret_cast<const float2*>(w.twiddle), w.window, sc.frames);
  else
    hipLaunchKernelGGL(istft_frames_kernel<false>, dim3(M), dim3(256), 0, s, sc.spec,
                     reinterpret_cast<const float2*>(w.twiddle), w.window, sc.frames);
  hipLaunchKernelGGL(istft_ola_kernel, dim3((HOPL * L + 255) / 256, B), dim3(256), 0, s, sc.frames, w.window, L, pcm, sc.err);
}

void codec_launch_decode(const CodecWeights& w, const CodecScratch& sc, int wdtype, const float* feats_in,
                         const int32_t* codes, int B, int L, int bw, float* pcm, hipStream_t s) {
  if (wdtype == LVX_DTYPE_BF16) decode_impl<bf16_t>(w, sc, feats_in, codes, B, L, bw, pcm, s);
  else decode_impl<float>(w, sc, feats_in, codes, B, L, bw, pcm, s);
}

}  // namespace lvx
