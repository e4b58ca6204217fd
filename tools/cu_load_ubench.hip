// Development micro-benchmark: how fast can one CU load the bytes a batched
// B = 32 decode GEMM block needs -- the operand rows every block shares (written by the previous
// kernel, so no L2 holds them at launch) plus the block's own weight slice (Infinity-Cache resident,
// a different 64 MB region's slice each launch, as the step's 17 GEMMs cycle through 63 MB) -- with
// 1 / 2 / 4 / 8 loader waves, loaded into registers (global_load_dwordx4) or by LDS-DMA
// (global_load_lds_dwordx4). Timed in-kernel (s_memrealtime, 100 MHz) from block entry to every
// byte landed (s_waitcnt vmcnt(0) + barrier), per block; a small producer kernel rewrites the rows
// before every consumer launch, as the previous GEMM / rows kernel does in the step.
// hipcc -O3 --offload-arch=gfx950 tools/cu_load_ubench.hip -o tools/cu_load_ubench && tools/cu_load_ubench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__global__ void produce(uint4* rows, int chunks, int it) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += gridDim.x * blockDim.x)
    rows[c] = make_uint4(c + it, c ^ it, it, c);
}

// RC / WC: 16-B row / weight chunks per thread; NWV waves per block; LDS: 1 = LDS-DMA, 0 = registers.
// Only the first LW waves load (the other waves idle, as consumers would).
// ROT: block b issues its row loads starting at 1-KB piece (b * 7) mod (pieces): the CUs of an XCD
// then ask for different lines of the shared rows at any moment instead of all for the same one.
template <int NWV, int LW, int RC, int WC, int LDS, int ROT = 0>
__global__ __launch_bounds__(NWV * 64) void consume(const uint4* __restrict__ rows, const uint4* __restrict__ w,
                                                    size_t w_off, uint64_t* ts, unsigned* sink) {
  constexpr int NT = LW * 64;
  __shared__ __attribute__((aligned(16))) uint4 lds[LDS ? NT * (RC + WC) : 1];  // (at most 72 KB)
  const int tid = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint4* wb = w + w_off + (size_t)blockIdx.x * (NT * WC);
  unsigned x = 0;
  // piece k of this thread -> chunk (k' * NT + tid), k' = (k + rot) % RC
  const int rot = ROT ? (blockIdx.x * 7) % (RC > 0 ? RC : 1) : 0;
  if (tid < NT) {
    const int wave = tid >> 6;
    if constexpr (LDS) {
#pragma unroll
      for (int k = 0; k < RC; ++k) {
        const int kr = ROT ? (k + rot) % RC : k;
        glds16(rows + tid + kr * NT, lds + (kr * NT + wave * 64));
      }
#pragma unroll
      for (int k = 0; k < WC; ++k) glds16(wb + tid + k * NT, lds + ((RC + k) * NT + wave * 64));
      __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) (and the rest): every DMA landed in LDS
    } else {
      uint4 r[RC > 0 ? RC : 1], v[WC > 0 ? WC : 1];
#pragma unroll
      for (int k = 0; k < RC; ++k) r[k] = rows[tid + (ROT ? (k + rot) % RC : k) * NT];
#pragma unroll
      for (int k = 0; k < WC; ++k) v[k] = wb[tid + k * NT];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < RC; ++k) x ^= r[k].x ^ r[k].w;
#pragma unroll
      for (int k = 0; k < WC; ++k) x ^= v[k].y ^ v[k].z;
    }
  }
  __syncthreads();
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if constexpr (LDS) x = lds[tid % (NT * (RC + WC) > 0 ? NT * (RC + WC) : 1)].x;
  if (x == 0x9e3779b9u) sink[blockIdx.x] = x;  // (keeps the loads live)
  if (tid == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15;
    ts[blockIdx.x * 3 + 0] = t0;
    ts[blockIdx.x * 3 + 1] = t1;
    ts[blockIdx.x * 3 + 2] = xcc;
  }
}

static int g_prod_blocks = 8;

template <int NWV, int LW, int RC, int WC, int LDS, int ROT = 0>
static void run(const char* name, int G, uint4* rows, uint4* w, size_t w_total_chunks, uint64_t* ts, unsigned* sink) {
  constexpr int NT = LW * 64;
  const size_t per_launch = (size_t)G * NT * WC;
  const int rows_chunks = NT * RC;
  const int iters = 40;
  std::vector<double> dts, spans, entry;
  std::vector<uint64_t> h(G * 3);
  for (int it = 0; it < iters; ++it) {
    if (rows_chunks && g_prod_blocks) hipLaunchKernelGGL(produce, dim3(g_prod_blocks), dim3(64), 0, 0, rows, rows_chunks, it);
    const size_t off = per_launch ? (size_t)(it % std::max<size_t>(1, w_total_chunks / per_launch)) * per_launch : 0;
    hipLaunchKernelGGL((consume<NWV, LW, RC, WC, LDS, ROT>), dim3(G), dim3(NWV * 64), 0, 0, rows, w, off, ts, sink);
    CK(hipDeviceSynchronize());
    if (it < 5) continue;  // warm-up
    CK(hipMemcpy(h.data(), ts, G * 3 * 8, hipMemcpyDeviceToHost));
    uint64_t mn = ~0ull, mx = 0, mxe = 0;
    for (int b = 0; b < G; ++b) {
      dts.push_back((h[b * 3 + 1] - h[b * 3]) * 0.01);  // us
      mn = std::min(mn, h[b * 3]);
      mx = std::max(mx, h[b * 3 + 1]);
      mxe = std::max(mxe, h[b * 3]);
    }
    spans.push_back((mx - mn) * 0.01);
    entry.push_back((mxe - mn) * 0.01);
  }
  std::sort(dts.begin(), dts.end());
  std::sort(spans.begin(), spans.end());
  std::sort(entry.begin(), entry.end());
  const double bytes = 16.0 * NT * (RC + WC);
  const double med = dts[dts.size() / 2], p90 = dts[dts.size() * 9 / 10];
  printf("%-40s G %3d waves %d loaders %d  %5.1f KB/block (rows %4.1f + w %4.1f)  entry->landed p50 %5.2f us p90 %5.2f"
         "  => %5.1f GB/s per CU (p50)  launch span p50 %5.2f us, entry skew %4.2f\n",
         name, G, NWV, LW, bytes / 1024, 16.0 * NT * RC / 1024, 16.0 * NT * WC / 1024, med, p90, bytes / med * 1e-3,
         spans[spans.size() / 2], entry[entry.size() / 2]);
}

int main() {
  uint4 *rows, *w;
  uint64_t* ts;
  unsigned* sink;
  const size_t w_total = (64ull << 20) / 16;  // 64 MB of weights, cycled
  CK(hipMalloc(&rows, 1 << 20));
  CK(hipMalloc(&w, w_total * 16));
  CK(hipMemset(w, 1, w_total * 16));
  CK(hipMalloc(&ts, 4096 * 3 * 8));
  CK(hipMalloc(&sink, 4096 * 4));
  // c_fc / lm_head-like block at B = 32: 48 KB of shared rows + 24 KB of weights (18 KB per wave over 4 waves)
  run<4, 4, 12, 6, 0>("regs 4 loaders (as ar_mfma2)", 192, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 0>("regs 4 loaders (as ar_mfma2)", 256, rows, w, w_total, ts, sink);
  run<8, 8, 6, 3, 0>("regs 8 loaders", 192, rows, w, w_total, ts, sink);
  run<8, 8, 6, 3, 0>("regs 8 loaders", 256, rows, w, w_total, ts, sink);
  run<16, 16, 3, 3, 0>("regs 16 loaders (rows 48, w 48)", 256, rows, w, w_total, ts, sink);
  run<4, 2, 24, 12, 0>("regs 2 loaders of 4 waves", 256, rows, w, w_total, ts, sink);
  run<4, 1, 48, 24, 1>("ldsdma 1 loader of 4 waves", 256, rows, w, w_total, ts, sink);
  run<4, 2, 24, 12, 1>("ldsdma 2 loaders of 4 waves", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 1>("ldsdma 4 loaders", 192, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 1>("ldsdma 4 loaders", 256, rows, w, w_total, ts, sink);
  run<8, 8, 6, 3, 1>("ldsdma 8 loaders", 256, rows, w, w_total, ts, sink);
  // the parts alone
  run<4, 4, 12, 0, 0>("regs rows only (48 KB)", 256, rows, w, w_total, ts, sink);
  run<4, 4, 0, 6, 0>("regs weights only (24 KB)", 256, rows, w, w_total, ts, sink);
  run<4, 4, 3, 6, 0>("regs 12 KB rows + 24 KB w (qkv_ksplit)", 256, rows, w, w_total, ts, sink);
  run<8, 8, 0, 3, 0>("regs weights only, 8 loaders", 256, rows, w, w_total, ts, sink);
  run<4, 4, 0, 0, 0>("nothing", 256, rows, w, w_total, ts, sink);
  // c_proj at B = 32 as launched (96 blocks: 16-row batch tiles, 24 KB rows + 24 KB w)
  run<4, 4, 6, 6, 0>("regs c_proj tile (24 + 24 KB)", 96, rows, w, w_total, ts, sink);
  run<4, 4, 6, 6, 0>("regs c_proj tile (24 + 24 KB)", 256, rows, w, w_total, ts, sink);
  // latency floors: 4 KB of shared rows / of own weights
  run<4, 4, 1, 0, 0>("regs rows only (4 KB)", 256, rows, w, w_total, ts, sink);
  run<4, 4, 0, 1, 0>("regs weights only (4 KB)", 256, rows, w, w_total, ts, sink);
  run<4, 4, 3, 0, 0>("regs rows only (12 KB)", 256, rows, w, w_total, ts, sink);
  run<4, 4, 6, 0, 0>("regs rows only (24 KB)", 256, rows, w, w_total, ts, sink);
  // row-load order rotated per block
  run<4, 4, 12, 0, 0, 1>("regs rows only (48 KB) rotated", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 0, 1>("regs 4 loaders rotated", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 1, 1>("ldsdma 4 loaders rotated", 256, rows, w, w_total, ts, sink);
  run<8, 8, 6, 3, 1, 1>("ldsdma 8 loaders rotated", 256, rows, w, w_total, ts, sink);
  // rows written by 256 producer blocks (spread over every XCD, as a GEMM epilogue writes them)
  g_prod_blocks = 256;
  run<4, 4, 12, 0, 0>("P256 regs rows only (48 KB)", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 0>("P256 regs 4 loaders", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 1>("P256 ldsdma 4 loaders", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 1, 1>("P256 ldsdma 4 loaders rotated", 256, rows, w, w_total, ts, sink);
  // rows not rewritten at all between launches (read-only: the L2 / MALL copy stays valid)
  g_prod_blocks = 0;
  run<4, 4, 12, 0, 0>("P0 regs rows only (48 KB)", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 0>("P0 regs 4 loaders", 256, rows, w, w_total, ts, sink);
  run<4, 4, 12, 6, 1>("P0 ldsdma 4 loaders", 256, rows, w, w_total, ts, sink);
  return 0;
}
