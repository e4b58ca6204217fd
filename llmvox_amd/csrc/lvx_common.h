// Shared device helpers for the LLMVoX MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LVX_WAVE 64

typedef uint16_t bf16_t;  // raw bf16 bits
typedef uint8_t fp8_t;    // raw OCP e4m3fn bits (KV cache)

// ---- dtype plumbing -------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// round-to-nearest-even; NaN stays NaN (quiet). On the device this is gfx950's v_cvt_pk_bf16_f32
// (same rounding, branch-free); the host form is the bit-exact software equivalent.
__host__ __device__ __forceinline__ bf16_t f32_to_bf16(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(bf16_t, (__bf16)f);
#else
  uint32_t u; __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
#endif
}

// f32 -> e4m3fn, round to nearest even, saturated to the finite range (+-448)
__device__ __forceinline__ fp8_t f32_to_fp8(float f) {
  f = fminf(fmaxf(f, -448.f), 448.f);
  return (fp8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(f, f, 0, false) & 0xff);
}

// a + w.x x.x + w.y x.y + w.z x.z + w.w x.w as an explicit fma chain: the rounding does not
// depend on how the compiler contracts each unrolled copy, so equal batch rows stay bit-equal
__device__ __forceinline__ float dot4_fma(float a, float4 w, float4 x) {
  return fmaf(w.w, x.w, fmaf(w.z, x.z, fmaf(w.y, x.y, fmaf(w.x, x.x, a))));
}

template <typename T> struct Ld;
template <> struct Ld<float> {
  // load 4 consecutive elements as floats
  __device__ __forceinline__ static float4 load4(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ __forceinline__ static float load1(const float* p) { return *p; }
  __device__ __forceinline__ static void store1(float* p, float v) { *p = v; }
};
template <> struct Ld<bf16_t> {
  __device__ __forceinline__ static float4 load4(const bf16_t* p) {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
  __device__ __forceinline__ static float load1(const bf16_t* p) { return bf16_to_f32(*p); }
  __device__ __forceinline__ static void store1(bf16_t* p, float v) { *p = f32_to_bf16(v); }
};

// ---- wave / block reductions ---------------------------------------------
// Full-wave reductions (every lane active): DPP within each 16-lane row (quad_perm xor 1 / xor 2,
// then row_ror 8 / row_ror 4: VALU-latency steps), then the four row results read into SGPRs
// (v_readlane) and combined in a fixed order, so the result is wave-uniform. Rotating by 8 before
// 4 adds the same two pair sums on every lane of a row (only operand order differs), so row16_sum
// is bit-identical across the row, like a butterfly. A ds_bpermute butterfly (__shfl_xor) costs an
// LDS round trip per step, six in a chain.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float lane_f32(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ float quad_sum(float v) {  // sum over the 4 lanes of a quad (xor 1, 2)
  v += dpp_f32<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  v = quad_sum(v);
  v += dpp_f32<0x128>(v);  // row_ror 8
  v += dpp_f32<0x124>(v);  // row_ror 4
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(v));
  v = fmaxf(v, dpp_f32<0x4E>(v));
  v = fmaxf(v, dpp_f32<0x128>(v));
  v = fmaxf(v, dpp_f32<0x124>(v));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  return (lane_f32(v, 0) + lane_f32(v, 16)) + (lane_f32(v, 32) + lane_f32(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_f32(v, 0), lane_f32(v, 16)), fmaxf(lane_f32(v, 32), lane_f32(v, 48)));
}

// block of NT threads; scratch must hold NT/64 floats; result broadcast to all threads
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  return r;
}

__device__ __forceinline__ float gelu_tanh(float x) {  // src/model.py:21-26
  const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
  return 0.5f * x * (1.0f + tanhf(k0 * (x + 0.044715f * x * x * x)));
}
__device__ __forceinline__ float gelu_erf(float x) {  // nn.GELU() default
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
// GELU (erf form) for outputs stored in bf16 (2^-9 relative rounding): erfc from Abramowitz & Stegun
// 7.1.26 (|error| <= 1.5e-7 absolute), branch-free on the native v_rcp_f32 / v_exp_f32, about a third
// of erff's instructions. x >= 0: x (1 - erfc(z) / 2); x < 0: x erfc(z) / 2 (no cancellation in the
// negative tail); z = |x| / sqrt(2).
__device__ __forceinline__ float gelu_erf_bf16out(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float h = 0.5f * (p * t) * __builtin_amdgcn_exp2f(-(z * z) * 1.4426950408889634f);
  return x * (x >= 0.f ? 1.0f - h : h);
}
__device__ __forceinline__ float swishf(float x) { return x / (1.0f + expf(-x)); }

#define LVX_CHECK_LAUNCH() (void)0
