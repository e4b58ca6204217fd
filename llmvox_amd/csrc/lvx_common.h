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
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
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
__device__ __forceinline__ float swishf(float x) { return x / (1.0f + expf(-x)); }

#define LVX_CHECK_LAUNCH() (void)0
