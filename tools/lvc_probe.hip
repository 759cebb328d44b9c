// Standalone probe for lvc_block_bf16_kernel: times the kernel alone on C3-sized
// synthetic inputs and prints where a block spends its time (s_memtime stamps per
// phase, LB_TRACE).  Diagnostic only (not a parity check: inputs are random).
//   build: make -C tools lvc_probe      run: tools/bin/lvc_probe [hop] [TS] [final=1]
#define LB_TRACE 1
#include "../prodiff_amd/csrc/fastdiff.hip"

// (kernels.hip's pd_build_config names every translation unit's flags; the probe links only this one)
namespace pd {
const char* nsf_build_flags() { return ""; }
const char* wavenet_build_flags() { return ""; }
}  // namespace pd

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
static float frand() {   // xorshift, uniform [-1, 1)
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

// FINAL: the sampler's last block as bench.py runs it (upsample r=4 + first conv + final
// update fused, next-layer kernel prefetch): lvc_block_bf16_kernel<TS, true, true, true, true>.
template <int TS, bool FINAL = false, bool PS = false> static void run(int hop) {
  using G = LbGeo<TS>;
  constexpr bool UPS = FINAL, AUD = FINAL, FIN = FINAL, PF = FINAL;
  const int B = 8, Tc = 861;
  const long long Lh = (long long)Tc * hop, rows = B * Lh;
  LvcBlockArgs la{};
  la.xin = upload<float>(rows * CI, 1.f);
  la.a = upload<float>(rows * CI, 1.f);
  CK(hipMalloc((void**)&la.xout, rows * CI * sizeof(float)));
  for (int l = 0; l < NLY; ++l) {
    la.Kf[l] = upload<__bf16>((size_t)B * Tc * KPERLAYER, 0.1f);
    la.Wc[l] = upload<__bf16>(CI * 96, 0.2f);
    la.bc[l] = upload<float>(CI, 0.05f);
  }
  la.Bf = upload<float>((size_t)B * Tc * 2 * CI * NLY, 0.1f);
  la.Tc = Tc; la.hop = hop;
  if (FINAL) {
    const int r = 4;
    la.xin = upload<float>(rows / r * CI, 1.f);
    la.Wup = upload<__bf16>((size_t)r * CI * 64, 0.2f);
    la.bup = upload<float>(CI, 0.05f);
    la.r = r; la.p = r / 2 + r % 2;
    la.a = nullptr;
    la.audio = upload<float>(rows, 1.f);
    la.fw = upload<float>(CI * 7, 0.3f);
    la.fb = upload<float>(CI, 0.05f);
    la.wfin = upload<float>(7 * CI, 0.1f);
    la.bfin = upload<float>(1, 0.05f);
    CK(hipMalloc((void**)&la.audio_out, rows * sizeof(float)));
    la.ce = 0.3f; la.den = 0.9f; la.sig = 0.1f; la.seed = 7; la.stream = 1;
  }
  if (PS) {   // the persistent final block (r06): iteration-5 stamps of every 4th block
    const int ntx = cdiv(Lh, TS), ntiles = ntx * B, nblk = 256;
    constexpr int NS = 24;
    const int nsamp = nblk / 4;
    CK(hipMalloc((void**)&la.trace, (size_t)nsamp * G::NW * NS * 8));
    CK(hipMemset(la.trace, 0, (size_t)nsamp * G::NW * NS * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(lvc_ps_kernel<true>, dim3(nblk), dim3(512), 0, 0, la, ntx, ntiles);
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(lvc_ps_kernel<true>, dim3(nblk), dim3(512), 0, 0, la, ntx, ntiles);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("PS TS=%d hop=%d tiles=%d blocks=%d  %.1f us/launch\n", TS, hop, ntiles, nblk, ms * 1000.0 / reps);
    std::vector<unsigned long long> tr((size_t)nsamp * G::NW * NS);
    CK(hipMemcpy(tr.data(), la.trace, tr.size() * 8, hipMemcpyDeviceToHost));
    const char* names[18] = {"top", "dma wait", "XP fill", "phase GEMM", "x/a regs", "L0 stage", "L0 preconv",
                             "L0 lvc", "L1 stage", "L1 preconv", "L1 lvc", "L2 stage", "L2 preconv", "L2 lvc",
                             "L3 stage", "L3 preconv", "L3 lvc", "FIN"};
    std::vector<std::vector<double>> ph(18);
    std::vector<double> life;
    for (int w = 0; w < nsamp * G::NW; ++w) {
      const unsigned long long* t = &tr[(size_t)w * NS];
      bool ok = t[0] != 0;
      for (int q = 1; q < 18 && ok; ++q) ok = t[q] >= t[q - 1] && t[q] - t[q - 1] < 100000000ull;
      if (!ok) continue;
      for (int q = 1; q < 18; ++q) ph[q].push_back((double)(t[q] - t[q - 1]));
      life.push_back((double)(t[17] - t[0]));
    }
    auto med = [](std::vector<double> v) {
      if (v.empty()) return 0.0;
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    const double L = med(life);
    printf("  %zu sampled waves, median tile time %.0f cycles\n", life.size(), L);
    for (int q = 1; q < 18; ++q) printf("    %-11s %8.0f cyc  %5.1f%%\n", names[q], med(ph[q]), 100.0 * med(ph[q]) / L);
    // layer 0's LVC phase split by stamps 18 (after its MFMAs) and 19 (after the next tile's DMA / fragment loads)
    std::vector<double> s0, s1, s2;
    for (int w = 0; w < nsamp * G::NW; ++w) {
      const unsigned long long* t = &tr[(size_t)w * NS];
      if (t[0] == 0 || t[18] < t[6] || t[19] < t[18] || t[7] < t[19]) continue;
      s0.push_back((double)(t[18] - t[6])); s1.push_back((double)(t[19] - t[18])); s2.push_back((double)(t[7] - t[19]));
    }
    printf("    L0 lvc = MFMAs %.0f + next tile's DMA / loads %.0f + gate %.0f cyc\n", med(s0), med(s1), med(s2));
    return;
  }
  const dim3 grid(cdiv(Lh, TS), B);
  const int nsamp = (grid.x * grid.y) / 61 + 1;
  constexpr int NS = 24;   // stamp slots per wave (LB_STAMP)
  CK(hipMalloc((void**)&la.trace, (size_t)nsamp * G::NW * NS * 8));
  CK(hipMemset(la.trace, 0, (size_t)nsamp * G::NW * NS * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((lvc_block_bf16_kernel<TS, UPS, AUD, FIN, PF>), grid, dim3(G::NT), 0, 0, la);
  const int reps = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((lvc_block_bf16_kernel<TS, UPS, AUD, FIN, PF>), grid, dim3(G::NT), 0, 0, la);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1000.0 / reps;
  const double bytes = (double)rows * 3 * 128 + (double)B * Tc * NLY * (KPERLAYER * 2 + 256);
  printf("TS=%d hop=%d grid=%dx%d  %.1f us/launch  %.2f TB/s (x,a in + x out + kernels)\n", TS, hop, grid.x,
         grid.y, us, bytes / us * 1e-6);
  std::vector<unsigned long long> tr((size_t)nsamp * G::NW * NS);
  CK(hipMemcpy(tr.data(), la.trace, tr.size() * 8, hipMemcpyDeviceToHost));
  // stamps in time order (0 = start, 15 = end); 16..20 only in the fused prologue
  std::vector<int> seq = {0};
  if (FINAL) seq.insert(seq.end(), {16, 17, 18, 19, 20});
  for (int i = 1; i <= 12; ++i) seq.push_back(i);
  seq.push_back(14);
  seq.push_back(15);
  const char* names[NS] = {"start", "kload+sync", "L0 stage", "L0 preconv", "L0 lvc", "L1 stage", "L1 preconv",
                           "L1 lvc", "L2 stage", "L2 preconv", "L2 lvc", "L3 stage", "L3 preconv", "-",
                           "L3 lvc", "store", "staging", "XP fill", "phase GEMM", "x/a regs", "zero U/Y"};
  // median per-phase duration over sampled waves whose stamps are monotone
  std::vector<std::vector<double>> ph(NS);
  std::vector<double> life;
  for (int s = 0; s < nsamp * G::NW; ++s) {
    const unsigned long long* t = &tr[(size_t)s * NS];
    bool ok = t[0] != 0;
    for (size_t q = 1; q < seq.size() && ok; ++q)
      ok = t[seq[q]] >= t[seq[q - 1]] && t[seq[q]] - t[seq[q - 1]] < 100000000ull;
    if (!ok) continue;
    for (size_t q = 1; q < seq.size(); ++q) ph[seq[q]].push_back((double)(t[seq[q]] - t[seq[q - 1]]));
    life.push_back((double)(t[15] - t[0]));
  }
  auto med = [](std::vector<double> v) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const double L = med(life);
  printf("  %zu sampled waves, median lifetime %.0f cycles\n", life.size(), L);
  for (size_t q = 1; q < seq.size(); ++q)
    printf("    %-11s %8.0f cyc  %5.1f%%\n", names[seq[q]], med(ph[seq[q]]), 100.0 * med(ph[seq[q]]) / L);
}

int main(int argc, char** argv) {
  const int hop = argc > 1 ? atoi(argv[1]) : 256;
  const int ts = argc > 2 ? atoi(argv[2]) : 128;
  if (argc > 3 && atoi(argv[3]) == 2) run<384, true, true>(hop);
  else if (argc > 3 && atoi(argv[3]) == 1) run<384, true>(hop);
  else if (ts == 256) run<256>(hop);
  else run<128>(hop);
  return 0;
}
