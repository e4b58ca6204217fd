// Micro-benchmarks for fusing GEMV seams on gfx950 (development tool):
//  cost of G blocks x 768 float atomicAdds into one 768-vector (split-K residual add),
//  cost of a "last block reduces the partials" tail, vs a plain kernel boundary.
// hipcc -O3 --offload-arch=gfx950 tools/ubench_atomic.hip -o tools/ubench_atomic
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_dep(float* p) {
  float v = p[(blockIdx.x * 7) & 1023];
  if (threadIdx.x == 0) p[blockIdx.x & 1023] = v + 1.f;
}

// every block adds 768 values into x (all blocks the same 768 addresses)
__global__ __launch_bounds__(256) void k_atomic_same(float* x, const float* src) {
  const int t = threadIdx.x;
  const float v = src[(blockIdx.x * 256 + t) & 4095];
#pragma unroll
  for (int j = 0; j < 3; ++j) atomicAdd(x + t + 256 * j, v);
}
// unsafe (no-return) fp32 atomics via the builtin
__global__ __launch_bounds__(256) void k_atomic_same_nr(float* x, const float* src) {
  const int t = threadIdx.x;
  const float v = src[(blockIdx.x * 256 + t) & 4095];
#pragma unroll
  for (int j = 0; j < 3; ++j) __hip_atomic_fetch_add(x + t + 256 * j, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 4 float atomics per thread packed as consecutive addresses (192 threads x 4)
__global__ __launch_bounds__(256) void k_atomic_pk(float* x, const float* src) {
  const int t = threadIdx.x;
  if (t >= 192) return;
  const float v = src[(blockIdx.x * 256 + t) & 4095];
#pragma unroll
  for (int j = 0; j < 4; ++j) __hip_atomic_fetch_add(x + t * 4 + j, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same adds into per-block private copies (no contention) - plain stores
__global__ __launch_bounds__(256) void k_store_private(float* x, const float* src) {
  const int t = threadIdx.x;
  const float v = src[(blockIdx.x * 256 + t) & 4095];
#pragma unroll
  for (int j = 0; j < 3; ++j) x[(size_t)blockIdx.x * 768 + t + 256 * j] = v;
}
// partials + last-block reduction (ticket counter), deterministic
__global__ __launch_bounds__(256) void k_lastblock(float* part, float* x, unsigned* counter, const float* src) {
  __shared__ bool last;
  const int t = threadIdx.x;
  const float v = src[(blockIdx.x * 256 + t) & 4095];
#pragma unroll
  for (int j = 0; j < 3; ++j) part[(size_t)blockIdx.x * 768 + t + 256 * j] = v;
  __threadfence();
  __syncthreads();
  if (t == 0) {
    const unsigned tk = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (tk == gridDim.x - 1);
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  float acc[3] = {0.f, 0.f, 0.f};
  for (int b = 0; b < (int)gridDim.x; ++b)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] += __builtin_nontemporal_load(part + (size_t)b * 768 + t + 256 * j);
#pragma unroll
  for (int j = 0; j < 3; ++j) x[t + 256 * j] += acc[j];
  if (t == 0) *counter = 0;
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
  float *buf, *x, *src, *part;
  unsigned* counter;
  CK(hipMalloc(&buf, 1 << 20));
  CK(hipMalloc(&x, 1 << 20));
  CK(hipMalloc(&src, 1 << 20));
  CK(hipMalloc(&part, 4 << 20));
  CK(hipMalloc(&counter, 256));
  CK(hipMemset(buf, 0, 1 << 20));
  CK(hipMemset(x, 0, 1 << 20));
  CK(hipMemset(src, 0, 1 << 20));
  CK(hipMemset(counter, 0, 256));
  const int n = 200;
  printf("dep kernel grid 256: %6.2f us\n",
         time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_dep, dim3(256), dim3(256), 0, s, buf); }));
  for (int G : {48, 96, 192, 384}) {
    printf("G=%3d atomicAdd same 768 addr : %6.2f us\n", G,
           time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_atomic_same, dim3(G), dim3(256), 0, s, x, src); }));
    printf("G=%3d agent-scope no-ret adds : %6.2f us\n", G,
           time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_atomic_same_nr, dim3(G), dim3(256), 0, s, x, src); }));
    printf("G=%3d packed 4/thread adds    : %6.2f us\n", G,
           time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_atomic_pk, dim3(G), dim3(256), 0, s, x, src); }));
    printf("G=%3d private stores          : %6.2f us\n", G,
           time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_store_private, dim3(G), dim3(256), 0, s, part, src); }));
    printf("G=%3d partials + last block   : %6.2f us\n", G,
           time_graph(s, n, [&](int) { hipLaunchKernelGGL(k_lastblock, dim3(G), dim3(256), 0, s, part, x, counter, src); }));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
