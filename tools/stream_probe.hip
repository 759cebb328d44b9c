// Standalone probe for lvc_stream_bf16_kernel<true, true, 4> (the sampler's last LVC block):
// times the kernel alone on C3-sized synthetic inputs and prints, per wave, where a step
// of workgroup (5, 0) goes (s_memtime stamps, steps 100..107).  Diagnostic only (random
// inputs, no parity check).   build: make -C tools stream_probe   run: tools/build/stream_probe
#define LB_TRACE 1
#include "../prodiff_amd/csrc/fastdiff.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static unsigned long long rng = 88172645463325252ull;
static float frand() {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return (float)((rng >> 40) & 0xFFFFFF) / 8388608.f - 1.f;
}
template <typename T> static T* upload(size_t n, float scale) {
  std::vector<T> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (T)(scale * frand());
  T* d;
  CK(hipMalloc((void**)&d, n * sizeof(T)));
  CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int B = 8, Tc = 861, hop = 256, r = 4;
  const long long Lh = (long long)Tc * hop, rows = B * Lh;
  LvcBlockArgs la{};
  la.xin = upload<float>(rows / r * CI, 1.f);
  for (int l = 0; l < NLY; ++l) {
    la.Kf[l] = upload<__bf16>((size_t)B * Tc * KPERLAYER, 0.1f);
    la.Wc[l] = upload<__bf16>(CI * 96, 0.2f);
    la.bc[l] = upload<float>(CI, 0.05f);
  }
  la.Bf = upload<float>((size_t)B * Tc * 2 * CI * NLY, 0.1f);
  la.Tc = Tc; la.hop = hop;
  la.Wup = upload<__bf16>((size_t)r * CI * 64, 0.2f);
  la.bup = upload<float>(CI, 0.05f);
  la.r = r; la.p = r / 2 + r % 2;
  la.audio = upload<float>(rows, 1.f);
  la.fw = upload<float>(CI * 7, 0.3f);
  la.fb = upload<float>(CI, 0.05f);
  la.wfin = upload<float>(7 * CI, 0.1f);
  la.bfin = upload<float>(1, 0.05f);
  CK(hipMalloc((void**)&la.audio_out, rows * sizeof(float)));
  la.ce = 0.3f; la.den = 0.9f; la.sig = 0.1f; la.seed = 7; la.stream = 1;
  CK(hipMalloc((void**)&la.trace, 8 * 8 * 8 * 8));
  CK(hipMemset(la.trace, 0, 8 * 8 * 8 * 8));
  const int seg = argc > 1 ? atoi(argv[1]) : lvc_stream_seg((int)Lh, B);
  const dim3 grid(cdiv(Lh, seg), B);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((lvc_stream_bf16_kernel<true, true, 4>), grid, dim3(512), 0, 0, la, seg);
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((lvc_stream_bf16_kernel<true, true, 4>), grid, dim3(512), 0, 0, la, seg);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  printf("seg=%d grid=%dx%d CUs=%d  %.1f us/launch  (%d steps per workgroup)\n", seg, grid.x, grid.y, ncu,
         ms * 1000.0 / reps, (seg + 31) / 32 + 4 + 22);
  std::vector<unsigned long long> tr(8 * 8 * 8);
  CK(hipMemcpy(tr.data(), la.trace, tr.size() * 8, hipMemcpyDeviceToHost));
  for (int s = 0; s < 8; ++s) {
    unsigned long long t0 = ~0ull;
    for (int w = 0; w < 8; ++w) if (tr[(s * 8 + w) * 8] && tr[(s * 8 + w) * 8] < t0) t0 = tr[(s * 8 + w) * 8];
    printf("step %d:", 100 + s);
    for (int w = 0; w < 8; ++w) {
      printf("  w%d[", w);
      for (int i = 0; i < 8; ++i) {
        const unsigned long long v = tr[(s * 8 + w) * 8 + i];
        if (v) printf("%d:%lld ", i, (long long)(v - t0));
      }
      printf("]");
    }
    printf("\n");
  }
  return 0;
}
