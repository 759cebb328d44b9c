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

// r05: the kp_kernel rhythm without its data: per 32-frame tile a wave runs NM MFMAs (two
// independent 32x32x16 bf16 chains, as kp's 24) and then its 4 stores of 1 KiB; 8 waves per CU.
// Does the chip overlap the MFMA phases with the store stream?
typedef float f32x16p __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8p __attribute__((ext_vector_type(8)));
template <int NM>
__global__ __launch_bounds__(512, 1) void store_mfma_kernel(char* __restrict__ out, int njobs, float* sink) {
  extern __shared__ char occ_pad2[];
  const int lane = threadIdx.x & 63;
  const int w0 = blockIdx.x * 8 + (threadIdx.x >> 6);
  if (threadIdx.x == 0) occ_pad2[0] = 0;
  const long long colblocks = ROWB / WAVE_COLB;
  bf16x8p a, bb;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.001f * (lane + i)); bb[i] = (__bf16)(0.002f * (lane - i)); }
  f32x16p c0 = {}, c1 = {};
  for (int w = w0; w < njobs; w += gridDim.x * 8) {
    const long long rb = w / colblocks, cb = w - rb * colblocks;
    for (int c = 0; c < WAVE_COLB / 128; ++c) {
#pragma unroll
      for (int m = 0; m < NM / 2; ++m) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bb, a, c1, 0, 0, 0);
      }
      const u32x4 v = {__float_as_uint(c0[0]), __float_as_uint(c1[1]), (unsigned)w, (unsigned)lane};
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const long long row = rb * 32 + rg * 8 + lane / 8;
        *reinterpret_cast<u32x4*>(out + row * ROWB + cb * WAVE_COLB + (long long)c * 128 + (lane % 8) * 16) = v;
      }
    }
  }
  if (c0[3] == 1234.5f) sink[0] = c1[2];
}

template <int NM> int run_mfma(char* buf, float* sink) {
  const int njobs = (int)(ROWS / 32 * (ROWB / WAVE_COLB));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&store_mfma_kernel<NM>), hipFuncAttributeMaxDynamicSharedMemorySize,
                         100 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(store_mfma_kernel<NM>, dim3(256), dim3(512), 100 * 1024, 0, buf, njobs, sink);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(store_mfma_kernel<NM>, dim3(256), dim3(512), 100 * 1024, 0, buf, njobs, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, bytes = (double)ROWS * ROWB;
  // MFMA-only time of the same launch: NM MFMAs x 32 cycles per tile, 2 waves per SIMD, 2.4 GHz
  const double tiles = (double)njobs * (WAVE_COLB / 128) / (256.0 * 8), mfma_us = tiles * NM * 32 * 2 / 2.4e3;
  printf("8 waves/CU, %2d MFMAs + 4 stores per tile  %8.1f us  %6.2f TB/s  (MFMA alone ~%.1f us)\n", NM, us,
         bytes / us * 1e-6, mfma_us);
  return 0;
}

// r05: kp_kernel's stores straight from the MFMA C layout (no LDS transpose): per tile 8 stores of 8 B
// per lane, lane -> frame row lane & 31, 8-B chunk 2 j4 + (lane >> 5) -- 32 rows x 16 B per
// instruction, the 8 instructions of a tile covering the same 32 rows x 128 B as kp's 4 x 1 KiB.
typedef unsigned int u32x2p __attribute__((ext_vector_type(2)));
template <int NM>
__global__ __launch_bounds__(512, 1) void store_cl_kernel(char* __restrict__ out, int njobs, float* sink) {
  extern __shared__ char occ_pad3[];
  const int lane = threadIdx.x & 63;
  const int w0 = blockIdx.x * 8 + (threadIdx.x >> 6);
  if (threadIdx.x == 0) occ_pad3[0] = 0;
  const long long colblocks = ROWB / WAVE_COLB;
  bf16x8p a, bb;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.001f * (lane + i)); bb[i] = (__bf16)(0.002f * (lane - i)); }
  f32x16p c0 = {}, c1 = {};
  for (int w = w0; w < njobs; w += gridDim.x * 8) {
    const long long rb = w / colblocks, cb = w - rb * colblocks;
    for (int c = 0; c < WAVE_COLB / 128; ++c) {
#pragma unroll
      for (int m = 0; m < NM / 2; ++m) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bb, a, c1, 0, 0, 0);
      }
      const long long row = rb * 32 + (lane & 31);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x2p v = {__float_as_uint(c0[q]), __float_as_uint(c1[q])};
        *reinterpret_cast<u32x2p*>(out + row * ROWB + cb * WAVE_COLB + (long long)c * 128 + (2 * q + (lane >> 5)) * 8) = v;
      }
    }
  }
  if (c0[3] == 1234.5f) sink[0] = c1[2];
}

template <int NM> int run_cl(char* buf, float* sink) {
  const int njobs = (int)(ROWS / 32 * (ROWB / WAVE_COLB));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&store_cl_kernel<NM>), hipFuncAttributeMaxDynamicSharedMemorySize,
                         100 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(store_cl_kernel<NM>, dim3(256), dim3(512), 100 * 1024, 0, buf, njobs, sink);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(store_cl_kernel<NM>, dim3(256), dim3(512), 100 * 1024, 0, buf, njobs, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, bytes = (double)ROWS * ROWB;
  printf("8 waves/CU, %2d MFMAs + 8 C-layout stores (32 rows x 16 B) per tile  %8.1f us  %6.2f TB/s\n", NM, us,
         bytes / us * 1e-6);
  return 0;
}

// r05: kp's whole epilogue without its data: per tile NM MFMAs, the bf16 conversion into a
// wave-private 32 x (64 + 8) LDS tile (8 ds_write_b64), lgkmcnt wait, 4 ds_read_b128, 4 stores of
// 1 KiB (8 rows x 128 B) -- kp_kernel_bf16_kernel's epi() with its wave barriers.
typedef __bf16 bf16x4p __attribute__((ext_vector_type(4)));
template <int NM>
__global__ __launch_bounds__(512, 1) void store_tr_kernel(char* __restrict__ out, int njobs, float* sink) {
  __shared__ __attribute__((aligned(16))) __bf16 Ot[8][32 * 72];
  const int lane = threadIdx.x & 63, r32 = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int w0 = blockIdx.x * 8 + wave;
  const long long colblocks = ROWB / WAVE_COLB;
  bf16x8p a, bb;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.001f * (lane + i)); bb[i] = (__bf16)(0.002f * (lane - i)); }
  __bf16* ot = Ot[wave];
  for (int w = w0; w < njobs; w += gridDim.x * 8) {
    const long long rb = w / colblocks, cb = w - rb * colblocks;
    for (int c = 0; c < WAVE_COLB / 128; ++c) {
      f32x16p acc[2];
      for (int r = 0; r < 16; ++r) { acc[0][r] = 0.f; acc[1][r] = (float)c; }
#pragma unroll
      for (int m = 0; m < NM / 2; ++m) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bb, a, acc[1], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4p*>(&ot[r32 * 72 + 4 * (8 * j + 2 * g + h)]) =
              bf16x4p{(__bf16)acc[j][4 * g], (__bf16)acc[j][4 * g + 1], (__bf16)acc[j][4 * g + 2], (__bf16)acc[j][4 * g + 3]};
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int fl = i * 8 + (lane >> 3);
        const uint4 v = *reinterpret_cast<const uint4*>(&ot[fl * 72 + 8 * (lane & 7)]);
        const long long row = rb * 32 + fl;
        *reinterpret_cast<uint4*>(out + row * ROWB + cb * WAVE_COLB + (long long)c * 128 + (lane & 7) * 16) = v;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  (void)sink;
}

template <int NM> int run_tr(char* buf, float* sink) {
  const int njobs = (int)(ROWS / 32 * (ROWB / WAVE_COLB));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(store_tr_kernel<NM>, dim3(256), dim3(512), 0, 0, buf, njobs, sink);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(store_tr_kernel<NM>, dim3(256), dim3(512), 0, 0, buf, njobs, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps, bytes = (double)ROWS * ROWB;
  printf("8 waves/CU, %2d MFMAs + kp's LDS-transpose epilogue + 4 stores per tile  %8.1f us  %6.2f TB/s\n", NM, us,
         bytes / us * 1e-6);
  return 0;
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
  float* sink;
  if (hipMalloc((void**)&sink, 64) != hipSuccess) return 1;
  e |= run_mfma<0>(buf, sink);
  e |= run_mfma<8>(buf, sink);
  e |= run_mfma<16>(buf, sink);
  e |= run_mfma<24>(buf, sink);
  e |= run_mfma<48>(buf, sink);
  e |= run_cl<0>(buf, sink);
  e |= run_cl<24>(buf, sink);
  e |= run_tr<0>(buf, sink);
  e |= run_tr<24>(buf, sink);
  (void)hipFree(sink);
  (void)hipFree(buf);
  return e;
}
