// Standalone probe for lvc_skew_bf16_kernel (the sampler's last block: upsample r=4 + first
// conv + final update fused): times the kernel alone on C3-sized synthetic inputs and prints
// where one workgroup's steps go (s_memtime stamps per phase, LB_TRACE).  Diagnostic only
// (random inputs, not a parity check).   build: make -C tools skew_probe
#define LB_TRACE 1
#include "../prodiff_amd/csrc/fastdiff.hip"

#include <algorithm>
#include <cstdio>
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

int main() {
  const int B = 8, Tc = 861, hop = 256, r = 4;
  const long long Lh = (long long)Tc * hop, rows = B * Lh;
  LvcBlockArgs la{};
  for (int l = 0; l < NLY; ++l) {
    la.Kf[l] = upload<__bf16>((size_t)B * Tc * KPERLAYER, 0.1f);
    la.Wc[l] = upload<__bf16>(CI * 96, 0.2f);
    la.bc[l] = upload<float>(CI, 0.05f);
  }
  la.Bf = upload<float>((size_t)B * Tc * 2 * CI * NLY, 0.1f);
  la.Tc = Tc; la.hop = hop;
  la.xin = upload<float>(rows / r * CI, 1.f);
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
  int nseg, seg_tiles;
  lvc_skew_segments((int)(Lh / 32), B, 256, 0, &nseg, &seg_tiles);
  const dim3 grid(B * nseg);
  constexpr int NSTEP = 8, NS = 20;
  CK(hipMalloc((void**)&la.trace, (size_t)NSTEP * lsw::NWV * NS * 8));
  CK(hipMemset(la.trace, 0, (size_t)NSTEP * lsw::NWV * NS * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((lvc_skew_bf16_kernel<true, true>), grid, dim3(lsw::NTH), 0, 0, la, nseg, seg_tiles);
  const int reps = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((lvc_skew_bf16_kernel<true, true>), grid, dim3(lsw::NTH), 0, 0, la, nseg, seg_tiles);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("skew final block: grid %d (nseg %d, %d tiles), %.1f us/launch\n", grid.x, nseg, seg_tiles, ms * 1000.0 / reps);
  std::vector<unsigned long long> tr((size_t)NSTEP * lsw::NWV * NS);
  CK(hipMemcpy(tr.data(), la.trace, tr.size() * 8, hipMemcpyDeviceToHost));
  const char* names[NS] = {"A1", "A1 bar", "A2", "A2 bar", "B0", "B0 bar", "C0", "C0 bar", "B1", "B1 bar", "C1",
                           "C1 bar", "B2", "B2 bar", "C2", "C2 bar", "B3", "B3 bar", "C3", "C3 bar"};
  // per phase: mean over (step, wave) of stamp[idx + 1] - stamp[idx]; the last wraps to the next step's A1
  std::vector<double> sum(NS, 0.0);
  std::vector<int> cnt(NS, 0);
  double step_sum = 0; int step_cnt = 0;
  for (int s = 0; s + 1 < NSTEP; ++s)
    for (int w = 0; w < lsw::NWV; ++w) {
      const unsigned long long* t = &tr[((size_t)s * lsw::NWV + w) * NS];
      const unsigned long long* tn = &tr[((size_t)(s + 1) * lsw::NWV + w) * NS];
      for (int k = 0; k < NS; ++k) {
        const unsigned long long a = t[k], bnext = k + 1 < NS ? t[k + 1] : tn[0];
        if (a && bnext > a && bnext - a < 10000000ull) { sum[k] += (double)(bnext - a); cnt[k]++; }
      }
      if (t[0] && tn[0] > t[0]) { step_sum += (double)(tn[0] - t[0]); step_cnt++; }
    }
  const double st = step_cnt ? step_sum / step_cnt : 0;
  printf("  mean step %.0f cycles (%d samples)\n", st, step_cnt);
  for (int k = 0; k < NS; ++k)
    printf("    %-7s %7.0f cyc  %5.1f%%\n", names[k], cnt[k] ? sum[k] / cnt[k] : 0.0, cnt[k] && st ? 100.0 * sum[k] / cnt[k] / st : 0.0);
  return 0;
}
