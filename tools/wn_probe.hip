// Phase probe for wn_layer_bf16_kernel<1024, 1> (wavenet.hip) at C3's shape (B*T = 8 x 861
// rows, C = H = 256, 216 blocks): times the kernel alone and prints where a wave's life goes
// (s_memtime stamps, WN_TRACE): ring prime + staging, staging barrier, GEMM1, gate epilogue,
// gate barrier, GEMM2, final epilogue.  Random inputs (not a parity check).
//   build: make -C tools wn_probe      run: tools/bin/wn_probe
#define WN_TRACE 1
#include "../prodiff_amd/csrc/wavenet.hip"

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
  // argv[1] = distinct layer weight sets cycled through (1: the same weights every launch, warm
  // in L2; 20: the sampler's layer sequence, each launch's weights cold in L2)
  const int NL = argc > 1 ? atoi(argv[1]) : 1;
  const int PF = argc > 2 ? atoi(argv[2]) : 0;   // argv[2] = 1: each launch prefetches the next set into L2
  const int B = 8, T = 861, C = 256, H = 256, rows = B * T;
  WnLayerArgs P{};
  P.xin = upload<float>((size_t)rows * C, 1.f);
  CK(hipMalloc((void**)&P.xout, (size_t)rows * C * 4));
  P.skip = upload<float>((size_t)rows * C, 1.f);
  P.cond = upload<float>((size_t)rows * H, 1.f);
  P.dp = upload<float>((size_t)B * C, 0.1f);
  P.dp_ld = C;
  std::vector<const __bf16*> W1s(NL), W2s(NL);
  for (int i = 0; i < NL; ++i) {
    W1s[i] = upload<__bf16>((size_t)2 * C * 1024, 0.03f);
    W2s[i] = upload<__bf16>((size_t)2 * C * C, 0.05f);
  }
  P.W1f = W1s[0];
  P.b1 = upload<float>(2 * C, 0.05f);
  P.W2f = W2s[0];
  P.b2 = upload<float>(2 * C, 0.05f);
  P.B = B; P.T = T; P.H = H; P.dil = 1; P.first = 0;
  const int grid = (rows + 31) / 32, nblk = (grid + 6) / 7;
  CK(hipMalloc((void**)&P.trace, (size_t)nblk * 8 * 8 * 8));
  CK(hipMemset(P.trace, 0, (size_t)nblk * 8 * 8 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  P.pfw[0] = W1s[0]; P.pfw[1] = W2s[0];
  P.pf_lines[0] = 2 * C * 1024 * 2 / 128; P.pf_lines[1] = 2 * C * C * 2 / 128;
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((wn_layer_bf16_kernel<1024, 1>), dim3(grid), dim3(512), 0, 0, P);
  const int reps = 50;
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) {
    P.W1f = W1s[i % NL];
    P.W2f = W2s[i % NL];
    const int ip = PF ? (i + 1) % NL : i % NL;   // the kernel always prefetches: itself when off
    P.pfw[0] = W1s[ip]; P.pfw[1] = W2s[ip];
    P.pf_lines[0] = 2 * C * 1024 * 2 / 128; P.pf_lines[1] = 2 * C * C * 2 / 128;
    hipLaunchKernelGGL((wn_layer_bf16_kernel<1024, 1>), dim3(grid), dim3(512), 0, 0, P);
  }
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("wn_layer<1024,1>: grid %d, %d weight sets, prefetch %d, %.2f us/launch\n", grid, NL, PF, ms * 1000.0 / reps);
  std::vector<unsigned long long> tr((size_t)nblk * 8 * 8);
  CK(hipMemcpy(tr.data(), P.trace, tr.size() * 8, hipMemcpyDeviceToHost));
  const char* names[7] = {"prime+stage", "stage barrier", "GEMM1", "gate epilogue", "gate barrier", "GEMM2",
                          "final epilogue"};
  std::vector<double> sum(7, 0.0);
  double life = 0;
  int n = 0;
  for (int b = 0; b < nblk; ++b)
    for (int w = 0; w < 8; ++w) {
      const unsigned long long* t = &tr[((size_t)b * 8 + w) * 8];
      bool ok = true;
      for (int k = 0; k < 7; ++k) ok = ok && t[k] && t[k + 1] >= t[k];
      if (!ok) continue;
      for (int k = 0; k < 7; ++k) sum[k] += (double)(t[k + 1] - t[k]);
      life += (double)(t[7] - t[0]);
      ++n;
    }
  printf("  mean wave life %.0f cycles (%d waves)\n", n ? life / n : 0.0, n);
  for (int k = 0; k < 7; ++k)
    printf("    %-15s %7.0f cyc  %5.1f%%\n", names[k], n ? sum[k] / n : 0.0, n && life ? 100.0 * sum[k] / life : 0.0);
  return 0;
}
