// Weight-stream probe for wn_layer_bf16_kernel (wavenet.hip): is 19-25 us per launch the
// L2 -> CU port or the kernel?  Every block streams exactly the fused layer's 1.3 MB of
// fragment-ordered bf16 weights (GEMM1: gate + filter tiles, 64 k-steps x 1 KiB per wave and
// tile; GEMM2: residual + skip, 16 k-steps) through the same register ring (WD k-steps deep),
// with no math ("stream"), or with the layer's 160 MFMAs per wave fed from registers
// ("stream+mfma"), at the grids the C3 (216 blocks) and C2-like (54) layers launch, plus 256
// and 512.  8 waves per block, 1 block per CU as the real kernel.  Diagnostic only.
//   build: make -C tools wn_stream_probe      run: tools/bin/wn_stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int KS1 = 64, KS2 = 16;

template <int WD, bool MFMA>
__global__ __launch_bounds__(512) void stream_kernel(const bf16x8* __restrict__ W1f, const bf16x8* __restrict__ W2f,
                                                     float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bf16x8* wg = W1f + (long long)wave * KS1 * 64 + lane;
  const bf16x8* wf = W1f + (long long)(8 + wave) * KS1 * 64 + lane;
  const bf16x8* wr = W2f + (long long)wave * KS2 * 64 + lane;
  const bf16x8* wsk = W2f + (long long)(8 + wave) * KS2 * 64 + lane;
  bf16x8 rg[WD], rf[WD];
#pragma unroll
  for (int i = 0; i < WD; ++i) { rg[i] = wg[i * 64]; rf[i] = wf[i * 64]; }
  f32x16 ag = {}, af = {};
  bf16x8 a = {};
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)(0.001f * (lane + i));
  unsigned acc = 0;
#pragma unroll
  for (int ks = 0; ks < KS1; ++ks) {
    const bf16x8 bg = rg[ks % WD], bfv = rf[ks % WD];
    if (ks + WD < KS1) {
      rg[ks % WD] = wg[(ks + WD) * 64];
      rf[ks % WD] = wf[(ks + WD) * 64];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (MFMA) {
      ag = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bg, ag, 0, 0, 0);
      af = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bfv, af, 0, 0, 0);
    } else {
      acc ^= __builtin_bit_cast(unsigned, __builtin_shufflevector(bg, bg, 0, 1)) ^
             __builtin_bit_cast(unsigned, __builtin_shufflevector(bfv, bfv, 2, 3));
    }
  }
  bf16x8 r2a[8], r2b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { r2a[i] = wr[i * 64]; r2b[i] = wsk[i * 64]; }
#pragma unroll
  for (int ks = 0; ks < KS2; ++ks) {
    const bf16x8 b0 = r2a[ks % 8], b1 = r2b[ks % 8];
    if (ks + 8 < KS2) {
      r2a[ks % 8] = wr[(ks + 8) * 64];
      r2b[ks % 8] = wsk[(ks + 8) * 64];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (MFMA) {
      ag = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, ag, 0, 0, 0);
      af = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, af, 0, 0, 0);
    } else {
      acc ^= __builtin_bit_cast(unsigned, __builtin_shufflevector(b0, b0, 0, 1)) ^
             __builtin_bit_cast(unsigned, __builtin_shufflevector(b1, b1, 2, 3));
    }
  }
  float s = (float)acc;
  for (int r = 0; r < 16; ++r) s += ag[r] + af[r];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int WD, bool MFMA> int run(const bf16x8* w1, const bf16x8* w2, float* out, int grid, const char* name) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((stream_kernel<WD, MFMA>), dim3(grid), dim3(512), 0, 0, w1, w2, out);
  CK(hipDeviceSynchronize());
  const int reps = 50;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((stream_kernel<WD, MFMA>), dim3(grid), dim3(512), 0, 0, w1, w2, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, per_block = (2.0 * 8 * KS1 + 2.0 * 8 * KS2) * 1024;
  printf("%-14s WD=%2d grid=%3d  %7.2f us   %.2f MB per block, %6.1f GB/s per block, %5.2f TB/s chip\n", name, WD,
         grid, us, per_block / 1e6, per_block / us * 1e-3, per_block * grid / us * 1e-6);
  return 0;
}

int main() {
  bf16x8 *w1, *w2;
  float* out;
  CK(hipMalloc((void**)&w1, 16 * KS1 * 64 * sizeof(bf16x8)));
  CK(hipMalloc((void**)&w2, 16 * KS2 * 64 * sizeof(bf16x8)));
  CK(hipMalloc((void**)&out, 1024 * 512 * sizeof(float)));
  CK(hipMemset(w1, 0, 16 * KS1 * 64 * sizeof(bf16x8)));
  CK(hipMemset(w2, 0, 16 * KS2 * 64 * sizeof(bf16x8)));
  int e = 0;
  for (int grid : {54, 216, 256, 512}) {
    e |= run<12, false>(w1, w2, out, grid, "stream");
    e |= run<24, false>(w1, w2, out, grid, "stream");
    e |= run<12, true>(w1, w2, out, grid, "stream+mfma");
  }
  return e;
}
