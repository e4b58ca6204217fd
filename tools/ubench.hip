// Micro-benchmarks of kernel-chain latency on gfx950 (development tool).
// hipcc -O3 --offload-arch=gfx950 tools/ubench.hip -o tools/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty(float* p) { if (threadIdx.x == 999999) p[0] = 1; }

// every block reads one value written by the previous kernel, writes one value
__global__ void k_dep(float* p) {
  float v = p[(blockIdx.x * 7) & 1023];
  if (threadIdx.x == 0) p[blockIdx.x & 1023] = v + 1.f;
}

// GEMV-shaped: each wave streams RPW rows x K bf16 (8 B / lane / load), x[768] from global
template <int K, int RPW>
__global__ __launch_bounds__(256) void k_gemv(const uint2* __restrict__ W, float* x, float* y, int N) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + wave) * RPW;
  uint2 w[RPW][K / 256];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int i = 0; i < K / 256; ++i) w[r][i] = W[((size_t)(row0 + r) * K + i * 256 + lane * 4) / 4];
  float acc[RPW] = {};
#pragma unroll
  for (int i = 0; i < K / 256; ++i) {
    const float4 xv = *reinterpret_cast<const float4*>(x + i * 256 + lane * 4);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      acc[r] += __uint_as_float(w[r][i].x << 16) * xv.x + __uint_as_float(w[r][i].x & 0xffff0000u) * xv.y +
                __uint_as_float(w[r][i].y << 16) * xv.z + __uint_as_float(w[r][i].y & 0xffff0000u) * xv.w;
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    float v = acc[r];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0 && row0 + r < N) y[row0 + r] = v;
  }
}

// same, 16-byte loads (8 bf16 per lane per load)
template <int K, int RPW>
__global__ __launch_bounds__(256) void k_gemv16(const uint4* __restrict__ W, float* x, float* y, int N) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + wave) * RPW;
  constexpr int NI = K / 512;
  uint4 w[RPW][NI];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int i = 0; i < NI; ++i) w[r][i] = W[((size_t)(row0 + r) * K + i * 512 + lane * 8) / 8];
  float acc[RPW] = {};
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const float4 xa = *reinterpret_cast<const float4*>(x + i * 512 + lane * 8);
    const float4 xb = *reinterpret_cast<const float4*>(x + i * 512 + lane * 8 + 4);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const uint4 u = w[r][i];
      acc[r] += __uint_as_float(u.x << 16) * xa.x + __uint_as_float(u.x & 0xffff0000u) * xa.y +
                __uint_as_float(u.y << 16) * xa.z + __uint_as_float(u.y & 0xffff0000u) * xa.w +
                __uint_as_float(u.z << 16) * xb.x + __uint_as_float(u.z & 0xffff0000u) * xb.y +
                __uint_as_float(u.w << 16) * xb.z + __uint_as_float(u.w & 0xffff0000u) * xb.w;
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    float v = acc[r];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0 && row0 + r < N) y[row0 + r] = v;
  }
}

template <typename F>
static float time_graph(hipStream_t s, int n, F launch) {
  hipGraph_t g;
  hipGraphExec_t ex;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < n; ++i) launch(i);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  hipGraphLaunch(ex, s);
  hipStreamSynchronize(s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, s);
  for (int r = 0; r < 5; ++r) hipGraphLaunch(ex, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ex);
  hipGraphDestroy(g);
  return ms * 1000.f / (5 * n);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* buf;
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMemset(buf, 0, 64 << 20));
  void* W;
  const size_t wbytes = 8 * 4096 * 3072 * 2;  // 8 distinct 25 MB matrices... (200 MB) to rotate
  CK(hipMalloc(&W, wbytes));
  CK(hipMemset(W, 0, wbytes));
  float *x, *y;
  CK(hipMalloc(&x, 1 << 20));
  CK(hipMalloc(&y, 1 << 20));
  CK(hipMemset(x, 0, 1 << 20));
  const int n = 200;
  for (int grid : {1, 64, 256, 512, 1024}) {
    float us = time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, buf); });
    printf("empty kernel grid=%4d: %6.2f us/kernel\n", grid, us);
  }
  for (int grid : {1, 256, 512}) {
    float us = time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_dep, dim3(grid), dim3(256), 0, s, buf); });
    printf("dependent-load kernel grid=%4d: %6.2f us/kernel\n", grid, us);
  }
  // GEMV c_fc shape: N=3072 K=768 (4.7 MB bf16); rotate over 8 matrices so the stream is not L2-hot
  const size_t mat = (size_t)3072 * 768;  // elements
  {
    float us = time_graph(s, n, [&](int i) {
      const uint2* Wi = reinterpret_cast<const uint2*>((const uint16_t*)W + (i % 8) * mat);
      hipLaunchKernelGGL((k_gemv<768, 2>), dim3(3072 / 8), dim3(256), 0, s, Wi, x, y, 3072);
    });
    printf("gemv 3072x768 bf16 8B loads RPW2 (384 blk): %6.2f us  (%.0f GB/s)\n", us, mat * 2 / us / 1e3);
  }
  {
    float us = time_graph(s, n, [&](int i) {
      const uint2* Wi = reinterpret_cast<const uint2*>((const uint16_t*)W + (i % 8) * mat);
      hipLaunchKernelGGL((k_gemv<768, 4>), dim3(3072 / 16), dim3(256), 0, s, Wi, x, y, 3072);
    });
    printf("gemv 3072x768 bf16 8B loads RPW4 (192 blk): %6.2f us  (%.0f GB/s)\n", us, mat * 2 / us / 1e3);
  }
  {
    float us = time_graph(s, n, [&](int i) {
      const uint2* Wi = reinterpret_cast<const uint2*>((const uint16_t*)W + (i % 8) * mat);
      hipLaunchKernelGGL((k_gemv<768, 1>), dim3(3072 / 4), dim3(256), 0, s, Wi, x, y, 3072);
    });
    printf("gemv 3072x768 bf16 8B loads RPW1 (768 blk): %6.2f us  (%.0f GB/s)\n", us, mat * 2 / us / 1e3);
  }
  {
    float us = time_graph(s, n, [&](int i) {
      const uint4* Wi = reinterpret_cast<const uint4*>((const uint16_t*)W + (i % 8) * mat);
      hipLaunchKernelGGL((k_gemv16<1024, 2>), dim3(3072 * 768 / 1024 / 8), dim3(256), 0, s, Wi, x, y, 3072);
    });
    printf("gemv 2304x1024 bf16 16B loads RPW2 : %6.2f us  (%.0f GB/s)\n", us, mat * 2 / us / 1e3);
  }
  // the same weights every time (MALL/L2-resident)
  {
    float us = time_graph(s, n, [&](int i) {
      hipLaunchKernelGGL((k_gemv<768, 2>), dim3(3072 / 8), dim3(256), 0, s, (const uint2*)W, x, y, 3072);
    });
    printf("gemv 3072x768 same W each time: %6.2f us\n", us);
  }
  // whole step shape: 21 GEMV-like kernels rotating through 63 MB
  {
    float us = time_graph(s, 21 * 10, [&](int i) {
      const uint2* Wi = reinterpret_cast<const uint2*>((const uint16_t*)W + (i % 21) * (mat * 2 / 3));
      hipLaunchKernelGGL((k_gemv<768, 2>), dim3(2048 / 8), dim3(256), 0, s, Wi, x, y, 2048);
    });
    printf("21-kernel step of 2048x768 GEMVs over 66 MB: %6.2f us/kernel -> %.1f us/step\n", us, us * 21);
  }
  return 0;
}
