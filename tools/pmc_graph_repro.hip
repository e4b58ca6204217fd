// Library-free check of the rocprofv3 --pmc fault seen under HIP-graph replay (VERDICT r03 item 4,
// profiles/r03/pmc_segv_graph_replay.log: SIGSEGV at 0xfffe000003e8 in a non-Python thread while the
// main thread was in hipGraphLaunch of the library's captured 16-step decode graph).
//
// Mirrors the shape of that launch path without the library: a chain of dependent kernels that take
// a 320-byte kernel-argument struct (as GemvArgs), captured with hipStreamCaptureModeThreadLocal on a
// non-blocking side stream, instantiated once and replayed many times on that stream.
//   usage: pmc_graph_repro [mode] [kernels per graph] [replays] [small kernargs 0/1]
//   mode 0: graph replay on the side stream (the bench's default path)
//        1: the same kernels launched one by one on the side stream (no graph)
//        2: graph replay on the legacy null stream
//        3: the kernels launched one by one on the legacy null stream
// Exit 0 and one line "ok ..." when the chain ran and its result checks out.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      return 3;                                                                                 \
    }                                                                                           \
  } while (0)

struct Args {  // 320 bytes, like the decode step's GemvArgs
  float* x;
  int n;
  int k;
  int pad[76];
};
static_assert(sizeof(Args) == 320, "kernarg size");

__global__ __launch_bounds__(256) void chain_step(Args a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) a.x[i] = a.x[i] * 0.5f + (float)(a.k & 3);
}
__global__ __launch_bounds__(256) void chain_step_small(float* x, int n, int k) {  // 16 B of kernargs
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * 0.5f + (float)(k & 3);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int nk = argc > 2 ? std::atoi(argv[2]) : 416;   // 16 decode steps x 26 kernels
  const int reps = argc > 3 ? std::atoi(argv[3]) : 320;  // 20 bench steps x 256 / 16
  const bool small = argc > 4 && std::atoi(argv[4]) != 0;
  const int n = 256 * 256;
  float* x = nullptr;
  CK(hipMalloc(&x, n * sizeof(float)));
  CK(hipMemset(x, 0, n * sizeof(float)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Args a{};
  a.x = x;
  a.n = n;
  auto enqueue = [&](hipStream_t q) -> hipError_t {
    for (int k = 0; k < nk; ++k) {
      a.k = k;
      if (small) hipLaunchKernelGGL(chain_step_small, dim3(n / 256), dim3(256), 0, q, x, n, k);
      else hipLaunchKernelGGL(chain_step, dim3(n / 256), dim3(256), 0, q, a);
    }
    return hipGetLastError();
  };
  if (mode == 1 || mode == 3) {
    hipStream_t q = mode == 3 ? nullptr : s;
    for (int r = 0; r < reps; ++r) CK(enqueue(q));
    CK(hipStreamSynchronize(q));
  } else {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const hipError_t le = enqueue(s);
    CK(hipStreamEndCapture(s, &g));
    CK(le);
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipStream_t q = mode == 2 ? nullptr : s;
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, q));
    CK(hipStreamSynchronize(q));
    CK(hipDeviceSynchronize());
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // x converges to the fixed point of the last kernels' map: check a few values are finite and equal
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), x, n * sizeof(float), hipMemcpyDeviceToHost));
  for (int i = 1; i < n; ++i)
    if (h[i] != h[0] || !std::isfinite(h[i])) {
      std::fprintf(stderr, "mismatch at %d: %g vs %g\n", i, h[i], h[0]);
      return 4;
    }
  std::printf("ok mode %d kernels/graph %d replays %d small-kernargs %d x[0] %.6f\n", mode, nk, reps, (int)small, h[0]);
  CK(hipStreamDestroy(s));
  CK(hipFree(x));
  return 0;
}
