// Store-shape probe for the kernel-predictor output (kp_kernel_bf16_kernel): how fast does
// the chip take 339 MB of 16-B-per-lane stores when one wave-instruction (1 KiB) covers
//   S = 128 B in 8 rows, 256 B in 4 rows, 512 B in 2 rows, or 1 KiB in one row
// of a [27552 rows][12288 B] table (4 layers x 6888 frames x 6144 bf16, the C3 K tensor),
// and when a wave's whole 96 KiB region is contiguous (seq).  Every wave owns 32 rows x
// 3 KiB and sweeps them column-chunk by column-chunk, as kp_kernel's waves do; 8 waves per
// block, 2 blocks per CU.  Plain and non-temporal stores.  Diagnostic only.
//   build: make -C tools store_probe      run: tools/bin/store_probe
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr long long ROWS = 27552, ROWB = 12288, WAVE_COLB = 3072;
constexpr int WAVES_PER_BLOCK = 8;

template <int S, bool NT, bool SEQ>
__global__ __launch_bounds__(512, 2) void store_kernel(char* __restrict__ out, int nwaves) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
  if (w >= nwaves) return;
  const long long colblocks = ROWB / WAVE_COLB;
  const long long rb = w / colblocks, cb = w - rb * colblocks;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7FFFFFFF, 0x00020000);
  (void)rsrc;
  constexpr int RPI = 1024 / S;                 // rows per instruction
  constexpr int LPR = S / 16;                   // lanes per row
  const u32x4 v = {(unsigned)w, (unsigned)lane, 7u, 9u};
  for (int c = 0; c < WAVE_COLB / S; ++c) {
#pragma unroll 4
    for (int rg = 0; rg < 32 / RPI; ++rg) {
      long long off;
      if (SEQ) {
        off = (long long)w * 32 * WAVE_COLB + ((long long)c * (32 / RPI) + rg) * 1024 + lane * 16;
      } else {
        const long long row = rb * 32 + rg * RPI + lane / LPR;
        off = row * ROWB + cb * WAVE_COLB + (long long)c * S + (lane % LPR) * 16;
      }
      u32x4* p = reinterpret_cast<u32x4*>(out + off);
      if (NT)
        __builtin_nontemporal_store(v, p);
      else
        *p = v;
    }
  }
}

template <int S, bool NT, bool SEQ> int run(char* buf, const char* name) {
  const int nwaves = (int)(ROWS / 32 * (ROWB / WAVE_COLB));
  const int nblocks = (nwaves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((store_kernel<S, NT, SEQ>), dim3(nblocks), dim3(512), 0, 0, buf, nwaves);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((store_kernel<S, NT, SEQ>), dim3(nblocks), dim3(512), 0, 0, buf, nwaves);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, bytes = (double)ROWS * ROWB;
  printf("%-28s %8.1f us  %6.2f TB/s\n", name, us, bytes / us * 1e-6);
  return 0;
}

// r05: the same 8-rows-x-128-B pattern from exactly W waves per CU (one W-wave block per CU, held
// there by 100 KB of dynamic LDS; each wave takes every (256 W)-th 32-row job): does the store rate
// depend on the waves per CU?  (kp_kernel_bf16_kernel runs 8 per CU at ~4 TB/s with its MFMAs)
template <int W>
__global__ __launch_bounds__(64 * W, 1) void store_occ_kernel(char* __restrict__ out, int njobs) {
  extern __shared__ char occ_pad[];
  const int lane = threadIdx.x & 63;
  const int w0 = blockIdx.x * W + (threadIdx.x >> 6);
  if (threadIdx.x == 0) occ_pad[0] = 0;
  const long long colblocks = ROWB / WAVE_COLB;
  const u32x4 v = {(unsigned)w0, (unsigned)lane, 7u, 9u};
  for (int w = w0; w < njobs; w += gridDim.x * W) {
    const long long rb = w / colblocks, cb = w - rb * colblocks;
    for (int c = 0; c < WAVE_COLB / 128; ++c) {
#pragma unroll 4
      for (int rg = 0; rg < 4; ++rg) {
        const long long row = rb * 32 + rg * 8 + lane / 8;
        *reinterpret_cast<u32x4*>(out + row * ROWB + cb * WAVE_COLB + (long long)c * 128 + (lane % 8) * 16) = v;
      }
    }
  }
}

template <int W> int run_occ(char* buf) {
  const int njobs = (int)(ROWS / 32 * (ROWB / WAVE_COLB));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&store_occ_kernel<W>), hipFuncAttributeMaxDynamicSharedMemorySize,
                         100 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(store_occ_kernel<W>, dim3(256), dim3(64 * W), 100 * 1024, 0, buf, njobs);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(store_occ_kernel<W>, dim3(256), dim3(64 * W), 100 * 1024, 0, buf, njobs);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, bytes = (double)ROWS * ROWB;
  printf("%2d waves per CU, 8 rows x 128 B  %8.1f us  %6.2f TB/s\n", W, us, bytes / us * 1e-6);
  return 0;
}

int main() {
  char* buf;
  if (hipMalloc((void**)&buf, ROWS * ROWB) != hipSuccess) return 1;
  int e = 0;
  e |= run<128, false, false>(buf, "8 rows x 128 B, plain");
  e |= run<128, true, false>(buf, "8 rows x 128 B, nt");
  e |= run<256, false, false>(buf, "4 rows x 256 B, plain");
  e |= run<256, true, false>(buf, "4 rows x 256 B, nt");
  e |= run<512, false, false>(buf, "2 rows x 512 B, plain");
  e |= run<512, true, false>(buf, "2 rows x 512 B, nt");
  e |= run<1024, false, false>(buf, "1 row x 1 KiB, plain");
  e |= run<1024, true, false>(buf, "1 row x 1 KiB, nt");
  e |= run<1024, false, true>(buf, "seq 96 KiB per wave, plain");
  e |= run<1024, true, true>(buf, "seq 96 KiB per wave, nt");
  e |= run_occ<4>(buf);
  e |= run_occ<8>(buf);
  e |= run_occ<12>(buf);
  e |= run_occ<16>(buf);
  (void)hipFree(buf);
  return e;
}
