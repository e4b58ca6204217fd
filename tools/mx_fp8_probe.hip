// Probe of gfx950's block-scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) before the codec uses it:
// the A / B lane -> k map (lane l: row / column l & 15, k = 32 (l >> 4) + byte j of its 8 dwords), the
// C / D map (column l & 15, row 4 (l >> 4) + e) and the E8M0 scale operand (127 = 1.0; every lane's
// scale applies to its 32 k). Exact small-integer data: the products and sums are exact in fp32.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mx_fp8_probe.hip -o tools/mx_fp8_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static unsigned char e4m3(float v) {  // exact for the small integers used here (|v| <= 8)
  if (v == 0.f) return 0;
  unsigned char s = v < 0 ? 0x80 : 0;
  float a = std::fabs(v);
  int e = (int)std::floor(std::log2(a));
  int m = (int)std::lround((a / std::ldexp(1.f, e) - 1.f) * 8.f);
  return s | (unsigned char)(((e + 7) & 15) << 3) | (unsigned char)(m & 7);
}

__global__ void probe(const unsigned char* A, const unsigned char* B, float* D, int sa, int sb) {
  const int l = threadIdx.x;
  i32x8 a, b;
  // A [16][128] row-major, B stored as Bt [16][128] (column-major B): lane l holds row / column l & 15,
  // k = 32 (l >> 4) .. + 31
  const int* pa = reinterpret_cast<const int*>(A + (l & 15) * 128 + 32 * (l >> 4));
  const int* pb = reinterpret_cast<const int*>(B + (l & 15) * 128 + 32 * (l >> 4));
  for (int i = 0; i < 8; ++i) { a[i] = pa[i]; b[i] = pb[i]; }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
  for (int e = 0; e < 4; ++e) D[(4 * (l >> 4) + e) * 16 + (l & 15)] = c[e];
}

int main() {
  float A[16][128], Bt[16][128];
  unsigned char qa[16 * 128], qb[16 * 128];
  srand(7);
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) {
      A[i][k] = (float)(rand() % 9 - 4);
      Bt[i][k] = (float)(rand() % 7 - 3) * ((k % 5) == 0 ? 2.f : 1.f);  // asymmetric in k
      qa[i * 128 + k] = e4m3(A[i][k]);
      qb[i * 128 + k] = e4m3(Bt[i][k]);
    }
  unsigned char *dA, *dB;
  float* dD;
  hipMalloc(&dA, sizeof qa);
  hipMalloc(&dB, sizeof qb);
  hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, qa, sizeof qa, hipMemcpyHostToDevice);
  hipMemcpy(dB, qb, sizeof qb, hipMemcpyHostToDevice);
  const int scales[3][2] = {{127, 127}, {128, 127}, {127, 125}};
  const float mult[3] = {1.f, 2.f, 0.25f};
  int bad = 0;
  for (int t = 0; t < 3; ++t) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, scales[t][0], scales[t][1]);
    float D[256];
    hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double r = 0;
        for (int k = 0; k < 128; ++k) r += (double)A[i][k] * Bt[j][k];
        maxerr = std::fmax(maxerr, std::fabs(D[i * 16 + j] - r * mult[t]));
      }
    printf("scale_a %d scale_b %d: max |D - %g A.B| = %g\n", scales[t][0], scales[t][1], mult[t], maxerr);
    bad += maxerr != 0;
  }
  printf(bad ? "MX fp8 probe: MISMATCH\n" : "MX fp8 probe: lane maps and E8M0 scales as assumed\n");
  return bad ? 1 : 0;
}
