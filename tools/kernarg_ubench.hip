// Development micro-benchmark: dependent kernel chain cost by kernel-argument form on gfx950.
// Each kernel reads a value its predecessor wrote through a pointer argument and writes one back
// (256 blocks). Forms: a 320-byte struct argument (like GemvArgs), or three scalar arguments,
// built with and without -mllvm -amdgpu-kernarg-preload-count=16 (kernarg words in SGPRs at launch).
// hipcc -O3 --offload-arch=gfx950 [-mllvm -amdgpu-kernarg-preload-count=16] tools/kernarg_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Big {
  const float* in;
  float* out;
  int n;
  int pad;
  const void* more[36];
};

__global__ void k_struct(Big a) {
  const float v = a.in[(blockIdx.x * 7) & 1023];
  if (threadIdx.x == 0) a.out[blockIdx.x & 1023] = v + 1.f;
}
__global__ void k_scalar(const float* in, float* out, int n) {
  const float v = in[(blockIdx.x * 7) & 1023];
  if (threadIdx.x == 0) out[blockIdx.x & (n - 1)] = v + 1.f;
}

int main() {
  float *a, *b;
  CK(hipMalloc(&a, 4096 * 4));
  CK(hipMalloc(&b, 4096 * 4));
  CK(hipMemset(a, 0, 4096 * 4));
  CK(hipMemset(b, 0, 4096 * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int N = 2000;
  for (int form = 0; form < 4; ++form) {  // 0/1 launched, 2/3 replayed as one captured graph
    hipGraphExec_t gx = nullptr;
    if (form >= 2) {
      hipGraph_t gr;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      Big g{};
      for (int i = 0; i < N; ++i) {
        float* in = (i & 1) ? b : a;
        float* out = (i & 1) ? a : b;
        if (form == 2) {
          g.in = in; g.out = out; g.n = 1024;
          hipLaunchKernelGGL(k_struct, dim3(256), dim3(256), 0, s, g);
        } else {
          hipLaunchKernelGGL(k_scalar, dim3(256), dim3(256), 0, s, in, out, 1024);
        }
      }
      CK(hipStreamEndCapture(s, &gr));
      CK(hipGraphInstantiate(&gx, gr, nullptr, nullptr, 0));
    }
    for (int rep = 0; rep < 2; ++rep) {
      Big g{};
      CK(hipEventRecord(e0, s));
      if (gx) CK(hipGraphLaunch(gx, s));
      else for (int i = 0; i < N; ++i) {
        float* in = (i & 1) ? b : a;
        float* out = (i & 1) ? a : b;
        if (form == 0) {
          g.in = in; g.out = out; g.n = 1024;
          hipLaunchKernelGGL(k_struct, dim3(256), dim3(256), 0, s, g);
        } else {
          hipLaunchKernelGGL(k_scalar, dim3(256), dim3(256), 0, s, in, out, 1024);
        }
      }
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) printf("%s args, %s: %.3f us per dependent kernel\n", (form & 1) == 0 ? "struct (320 B)" : "scalar",
                      form >= 2 ? "graph" : "launched", ms * 1e3 / N);
    }
  }
  return 0;
}
