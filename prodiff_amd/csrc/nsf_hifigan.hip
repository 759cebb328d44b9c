// NSF-HiFiGAN generator on gfx950.
//
// Reference: modules/nsf_hifigan/models.py:222-283 (Generator), :100-219 (SineGen,
// SourceModuleHnNSF), :36-97 (ResBlock1/2); called by NsfHifiGAN.spec2wav_torch
// (component/vocoder/nsf_hifigan.py:29-56).
//
// Layout: every activation is time-major [B][t][c] (the ProDiff/FastDiff convention),
// so the mel the acoustic model produces feeds conv_pre with no transpose.
//  * harmonic source: the reference cumsums the per-sample phase increment in float64
//    over the whole upsampled signal (models.py:136-161).  The increment is constant
//    inside a frame (nearest upsampling), so sample t = f*upp + j has phase
//    upp * P[f] + (j+1) * rad[f] with P the per-frame prefix: one short double scan per
//    (utterance, harmonic), then every sample is independent.  The reference's
//    "cumsum_shift" only adds whole cycles and leaves sin(2*pi*phase) unchanged.
//  * Conv1d / ConvTranspose1d run on the implicit-GEMM engine (gemm.h, fp32 MFMA):
//    a conv is one segment per tap; a ConvTranspose1d with stride u is u phase GEMMs
//    (output rows t = q*u + o_phi, k/u taps each) whose epilogue also adds the
//    noise_convs output (x = ups(x) + noise_conv(har), models.py:272-274).
//  * ResBlock pre-activations (leaky_relu 0.1) and the 1/num_kernels average are
//    applied on load by the consuming GEMM, so no elementwise pass materialises them.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "../../include/prodiff_hip.h"
#include "gemm.h"
#include "kernels.h"

using namespace pd;

struct NsfConv {
  const float* w = nullptr;   // packed [cout][taps * kpad]
  const float* b = nullptr;
  int taps = 0, dil = 1, cin = 0, cout = 0, kpad = 0;
  int w256 = 1;               // NSF_OPT_C256 (r06): the 256-channel windowed conv's block shape
  // ResBlock convs with at most this many channels use nsf_conv_small_kernel (NSF_OPT_SMALL_MAX;
  // measured: 32 channels run faster on the bf16 GEMM)
  int small_max = 16;
  bool wconv = true;          // NSF_OPT_WCONV: bf16 ResBlock convs on nsf_wconv_kernel
};

struct NsfUps {
  int u = 0, k = 0, cin = 0, cout = 0, ntap = 0, kpad = 0;
  std::vector<const float*> w;   // per phase: packed [cout][ntap * kpad]
  std::vector<int> qmin;         // per phase: first input row offset
  const float* b = nullptr;
  const float* nc_w = nullptr;   // noise conv [cout][nc_k]
  const float* nc_b = nullptr;
  int nc_k = 0, nc_stride = 1, nc_pad = 0;
};

struct nsf_model {
  nsf_dims d{};
  int dim = 9, C0 = 0, upp = 1;
  float* pool = nullptr;
  __bf16* pool_bf = nullptr;     // PD_DTYPE_BF16: bf16 mirror, registered with launch_gemm
  size_t pool_n = 0;
  const float* lin_w = nullptr;
  const float* lin_b = nullptr;
  NsfConv pre, post;
  std::vector<NsfUps> ups;
  std::vector<NsfConv> res;      // [stage][kernel][conv] flattened in state-dict order
  bool ups_window = true;        // NSF_OPT_WCONV also selects the windowed ConvTranspose
  bool pair = true;              // NSF_OPT_PAIR: a ResBlock1 conv pair in one launch (nsf_pair_kernel)
  int rb16 = 1;                  // NSF_OPT_RB16 (r06): a whole 16-channel ResBlock1 per launch (nsf_rb16_kernel)
  // NSF_OPT_RB32 / RB64 (r06): the same at 32 / 64 channels, per kernel-size bit.  Measured (C5, one job,
  // profiles/r06_ab/nsf_resblock_fused_ab.txt): only the 32-channel taps-3 ResBlock gains (343 vs 3 x 130 us);
  // with taps 7 / 11 or 64 channels the 2 x 12 (k - 1) halo rows and one 8-wave block per CU cost more
  // than the two fp32 round trips saved (545 vs 465, 764 vs 572, 557 vs 471, 624 vs 650, 941 vs 805 us)
  int rb32 = 1, rb64 = 0;
  int nc_mfma = 2;               // NSF_OPT_NC_MFMA (r06): the K = 128 and K = 16 source convs on the f32 MFMA
  bool pair16 = true;            // NSF_OPT_PAIR16: the C = 16 pairs too (nsf_pair16_kernel), with pair
  bool ups_nc = true;            // NSF_OPT_UPS_NC: the windowed upsample computes short noise convs itself
  int convs_per_block = 0;
};

namespace {

constexpr float NSF_LRELU = 0.1f;
constexpr float NSF_SINE_AMP = 0.1f;     // SineGen defaults (models.py:118-119)
constexpr float NSF_NOISE_STD = 0.003f;
constexpr unsigned NSF_STREAM_INI = 0x4e534600u, NSF_STREAM_NOISE = 0x4e534601u;

// Ragged batch (nsf_forward's lens): utterance b's rows at a stage of `rate` rows per mel frame end
// at lens[b] * rate <= Tl; every conv reads zero past that end.  lens == null: every row is Tl.
struct NsfRag {
  const int* lens = nullptr;
  int rate = 1;
};
__device__ __forceinline__ int nsf_tv(const NsfRag& rg, int b, int Tl) {
  return rg.lens ? min(rg.lens[b] * rg.rate, Tl) : Tl;
}

// rad_values of SineGen._f02sine (models.py:137-141), bit-for-bit in fp32:
// fn = f0 * (h+1); rad = fmod(fn / sr, 1); frame 0 adds rand_ini[h] (rand_ini[0] = 0).
__device__ __forceinline__ float nsf_rad(float f0, int h, int f, float sr, const float* rand_ini,
                                         unsigned long long seed, const int* uid, int b) {
  float fn = __fmul_rn(f0, (float)(h + 1));
  float r = fmodf(__fdiv_rn(fn, sr), 1.0f);
  if (f == 0 && h > 0) {
    float ini = rand_ini ? rand_ini[h] : philox_uniform_u(seed, utt_id(uid, b), (unsigned)h, NSF_STREAM_INI);
    r = __fadd_rn(r, ini);
  }
  return r;
}

// P[b][f][h] = sum_{f' < f} rad[b][f'][h] in double, and Rd[b][f][h] = rad[b][f][h] (fp32, the
// source kernel reads it instead of recomputing fmod/div per sample).  One block per (b, h):
// each thread sums a contiguous run of frames, a block-wide exclusive scan of the run sums
// (double, in LDS) gives every run its offset.  (r02: one serial thread per (b, h) took 181 us.)
constexpr int NSF_PP_THREADS = 256;
__global__ __launch_bounds__(NSF_PP_THREADS) void nsf_phase_prefix_kernel(const float* __restrict__ f0, int B, int T,
                                                                        int dim, float sr,
                                                                        const float* __restrict__ rand_ini,
                                                                        unsigned long long seed,
                                                                        const int* __restrict__ uid,
                                                                        double* __restrict__ P,
                                                                        float* __restrict__ Rd) {
  __shared__ double part[NSF_PP_THREADS];
  const int i = blockIdx.x, b = i / dim, h = i - b * dim, tid = threadIdx.x;
  const int run = (T + NSF_PP_THREADS - 1) / NSF_PP_THREADS, fa = tid * run, fb = min(fa + run, T);
  double acc = 0.0;
  for (int f = fa; f < fb; ++f) {
    const float r = nsf_rad(f0[(long long)b * T + f], h, f, sr, rand_ini, seed, uid, b);
    Rd[((long long)b * T + f) * dim + h] = r;
    acc += (double)r;
  }
  part[tid] = acc;
  __syncthreads();
  // Hillis-Steele inclusive scan over the 256 run sums
  for (int o = 1; o < NSF_PP_THREADS; o <<= 1) {
    const double v = tid >= o ? part[tid - o] : 0.0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  double run_off = tid > 0 ? part[tid - 1] : 0.0;
  for (int f = fa; f < fb; ++f) {
    const long long e = ((long long)b * T + f) * dim + h;
    P[e] = run_off;
    run_off += (double)Rd[e];
  }
}

// har[b][t] = tanh(l_linear(sine_waves)) (models.py:168-219), one thread per sample.
__global__ __launch_bounds__(256) void nsf_source_kernel(const float* __restrict__ f0, const double* __restrict__ P,
                                                         const float* __restrict__ Rd,
                                                         int B, int T, int upp, int dim, float sr,
                                                         const float* __restrict__ rand_ini,
                                                         const float* __restrict__ noise, unsigned long long seed,
                                                         const int* __restrict__ uid, const float* __restrict__ lw, const float* __restrict__ lb,
                                                         float* __restrict__ har) {
  const long long L = (long long)T * upp;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * L) return;
  const int b = (int)(i / L);
  const long long t = i - (long long)b * L;
  const int f = (int)(t / upp), j = (int)(t - (long long)f * upp);
  const float fv = f0[(long long)b * T + f];
  const float uv = fv > 0.f ? 1.f : 0.f;
  const float namp = uv * NSF_NOISE_STD + (1.f - uv) * NSF_SINE_AMP / 3.f;
  float acc = 0.f;
  for (int h = 0; h < dim; ++h) {
    const long long e = ((long long)b * T + f) * dim + h;
    double ph = (double)upp * P[e] + (double)(j + 1) * (double)Rd[e];
    ph -= floor(ph);
    float s = (float)sin(ph * 6.283185307179586) * NSF_SINE_AMP;
    long long ni = i * dim + h;
    float z = noise ? noise[ni] : philox_normal_u(seed, utt_id(uid, b), (unsigned)(t * dim + h), NSF_STREAM_NOISE);
    acc = fmaf(lw[h], s * uv + namp * z, acc);
  }
  har[i] = tanhf(acc + lb[0]);
}

// noise_convs[i] (models.py:241-245): Conv1d(1, C, K, stride, pad) over har [B][L]
// -> out [B][Tout][C] time-major.  A block stages one window of har in LDS and
// computes NC_ROWS rows per thread group; weights are stored tap-major [K][C] so a
// tap's weights are one coalesced load, reused for NC_ROWS outputs.
constexpr int NC_ROWS = 8;
__global__ __launch_bounds__(256) void nsf_noise_conv_kernel(const float* __restrict__ har, long long L,
                                                             const float* __restrict__ wt,
                                                             const float* __restrict__ bias, int C, int K,
                                                             int stride, int pad, long long Tout,
                                                             float* __restrict__ out, NsfRag rag_) {
  extern __shared__ float s_har[];
  const int CT = C < 256 ? C : 256, G = 256 / CT;
  const int tid = threadIdx.x;
  const int o = blockIdx.y * CT + tid % CT, rg = tid / CT;
  const int b = blockIdx.z;
  const long long row0 = (long long)blockIdx.x * G * NC_ROWS;
  const int win = (G * NC_ROWS - 1) * stride + K;
  const float* hb = har + (long long)b * L;
  const long long s0 = row0 * stride - pad;
  const long long Lv = rag_.lens ? min((long long)rag_.lens[b] * rag_.rate, L) : L;   // the utterance's own end
  for (int i = tid; i < win; i += 256) {
    long long sidx = s0 + i;
    s_har[i] = (sidx >= 0 && sidx < Lv) ? hb[sidx] : 0.f;
  }
  __syncthreads();
  float acc[NC_ROWS];
  const float bo = bias[o];
#pragma unroll
  for (int i = 0; i < NC_ROWS; ++i) acc[i] = bo;
  // (r05: taps' weights loaded in batches of 8: 87 vs 82 us; four taps per 16-B LDS read: 105 us either way, noise_conv_lds4_ab.txt)
  for (int j = 0; j < K; ++j) {
    const float w = wt[(long long)j * C + o];
#pragma unroll
    for (int i = 0; i < NC_ROWS; ++i) acc[i] = fmaf(w, s_har[(rg + G * i) * stride + j], acc[i]);
  }
#pragma unroll
  for (int i = 0; i < NC_ROWS; ++i) {
    long long r = row0 + rg + G * i;
    if (r < Tout) out[((long long)b * Tout + r) * C + o] = acc[i];
  }
}

// noise conv weight [C][1][K] -> tap-major [K][C]
// The two long source convs (the first two stages: Conv1d(1, C, K = 2 s, stride s), s = 64 / 8; models.py:255-262)
// on the f32 MFMA (r06): out^T[o][r] = b[o] + sum_k w[k][o] har[r s - pad + k] as v_mfma_f32_32x32x2_f32
// chains started from the bias, k ascending -- the VALU kernel's fmaf chain (MI355X_MICROARCH.md: the f32-input
// MFMA is exact f32, bitwise an fmaf chain).  Block = 4 waves x 32 rows, 32 channels: the block's source
// window and its channels' weights in LDS; lane (row, k half) holds 4 consecutive channels per register
// group, so results leave as float4 stores.  The VALU kernel ran 100-106 us per launch at C5 (3.6 and 1.8
// GFLOP): fp32 VALU-bound.
template <int K>
__global__ __launch_bounds__(256) void nsf_noise_mfma_kernel(const float* __restrict__ har, long long L,
                                                             const float* __restrict__ wt,
                                                             const float* __restrict__ bias, int C, int pad,
                                                             long long Tout, float* __restrict__ out, NsfRag rag_) {
  constexpr int S = K / 2, RB = 128, WIN = (RB - 1) * S + K;
  __shared__ float s_har[WIN];
  __shared__ float s_w[K * 32];                 // [k][channel within the block's 32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = lane & 31, kh = lane >> 5;
  const int b = blockIdx.z, o0 = blockIdx.y * 32;
  const long long row0 = (long long)blockIdx.x * RB;
  const float* hb = har + (long long)b * L;
  const long long s0 = row0 * S - pad;
  const long long Lv = rag_.lens ? min((long long)rag_.lens[b] * rag_.rate, L) : L;   // the utterance's own end
  // staging: every load of the window and the weights issued before any LDS store (a load-store loop
  // waited one round trip per item: 33 of them per thread at K = 128)
  constexpr int NH = (WIN + 255) / 256, NWV = K * 32 / 256;
  float hv[NH], wv[NWV];
#pragma unroll
  for (int u = 0; u < NH; ++u) {
    const long long sidx = s0 + tid + 256 * u;
    const long long sc = sidx < 0 ? 0 : sidx >= L ? L - 1 : sidx;      // unconditional load, masked value
    hv[u] = hb[sc];
  }
#pragma unroll
  for (int u = 0; u < NWV; ++u) {
    const int i = tid + 256 * u;
    wv[u] = wt[(long long)(i >> 5) * C + o0 + (i & 31)];
  }
#pragma unroll
  for (int u = 0; u < NH; ++u) {
    const int i = tid + 256 * u;
    const long long sidx = s0 + i;
    if (i < WIN) s_har[i] = (sidx >= 0 && sidx < Lv) ? hv[u] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < NWV; ++u) s_w[tid + 256 * u] = wv[u];
  f32x16 acc;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) acc[reg] = bias[o0 + (reg & 3) + 8 * (reg >> 2) + 4 * kh];
  __syncthreads();
  const float* hr = s_har + (wave * 32 + j) * S + kh;
#pragma unroll 8
  for (int k0 = 0; k0 < K; k0 += 2)
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(s_w[(k0 + kh) * 32 + j], hr[k0], acc, 0, 0, 0);
  const long long r = row0 + wave * 32 + j;
  if (r < Tout) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<float4*>(out + ((long long)b * Tout + r) * C + o0 + 8 * g + 4 * kh) =
          make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
  }
}

__global__ void nsf_pack_noise_kernel(float* __restrict__ dst, const float* __restrict__ src, int C, int K) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * K) return;
  int o = i / K, j = i - o * K;
  dst[j * C + o] = src[i];
}

// Small-channel Conv1d (C in {4, 8, 16, 32}: the last ResBlock stages, where a 64-wide
// GEMM tile would be 1/2 .. 1/16 empty and every tap re-reads the rows).  One block
// stages TR + halo input rows (leaky_relu * scale applied once, on load) and the layer's
// weights in LDS, then each thread accumulates RR rows x OC channels on the VALU in
// fp32.  Rows are interleaved across threads (row = rg + i * NRG) and the LDS row pitch
// is C + 1, so a wave's reads hit 32 distinct banks.
template <int C>
__global__ __launch_bounds__(256) void nsf_conv_small_kernel(const float* __restrict__ in, const float* __restrict__ wp,
                                                             int ldw, int kpad, const float* __restrict__ bias,
                                                             int taps, int dil, float alpha, float scale, int Tl,
                                                             const float* __restrict__ res, float* __restrict__ out,
                                                             NsfRag rag_) {
  constexpr int OC = C < 8 ? C : 8, NG = C / OC, NRG = 256 / NG, RR = 4, TR = NRG * RR, P = C + 1;
  extern __shared__ float lds[];
  const int pad = (taps - 1) * dil / 2;
  const int win = TR + (taps - 1) * dil;
  float* s_w = lds;                          // [tap][ci][co]
  float* s_x = lds + taps * C * C;           // [win][P]
  const int tid = threadIdx.x, b = blockIdx.y;
  const int t0 = blockIdx.x * TR, Tv = nsf_tv(rag_, b, Tl);
  const float* ib = in + (long long)b * Tl * C;
  for (int i = tid; i < taps * C * C; i += 256) {
    int co = i % C, r = i / C, ci = r % C, k = r / C;
    s_w[i] = wp[(long long)co * ldw + k * kpad + ci];
  }
  for (int i = tid; i < win * C; i += 256) {
    int row = i / C, c = i - row * C;
    int t = t0 - pad + row;
    float v = 0.f;
    if (t >= 0 && t < Tv) {
      v = ib[(long long)t * C + c];
      v = (v >= 0.f ? v : alpha * v) * scale;
    }
    s_x[row * P + c] = v;
  }
  __syncthreads();
  const int og = tid % NG, rg = tid / NG;
  float acc[RR][OC];
#pragma unroll
  for (int i = 0; i < RR; ++i)
#pragma unroll
    for (int c = 0; c < OC; ++c) acc[i][c] = bias[og * OC + c];
  for (int k = 0; k < taps; ++k) {
    const float* xk = s_x + (rg + k * dil) * P;
    const float* wk = s_w + k * C * C + og * OC;
#pragma unroll 4
    for (int ci = 0; ci < C; ++ci) {
      float w[OC];
#pragma unroll
      for (int c = 0; c < OC; ++c) w[c] = wk[ci * C + c];
#pragma unroll
      for (int i = 0; i < RR; ++i) {
        const float x = xk[i * NRG * P + ci];
#pragma unroll
        for (int c = 0; c < OC; ++c) acc[i][c] = fmaf(w[c], x, acc[i][c]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < RR; ++i) {
    const int t = t0 + rg + i * NRG;
    if (t >= Tl) continue;
    const long long o = ((long long)b * Tl + t) * C + og * OC;
#pragma unroll
    for (int c = 0; c < OC; ++c) out[o + c] = acc[i][c] + (res ? res[o + c] : 0.f);
  }
}

template <int C>
int launch_conv_small(const NsfConv& c, const float* in, float alpha, float scale, int B, int Tl, float* out,
                      const float* res, hipStream_t st, NsfRag rag_) {
  constexpr int OC = C < 8 ? C : 8, NG = C / OC, TR = 256 / NG * 4;
  const size_t lds = ((size_t)c.taps * C * C + (size_t)(TR + (c.taps - 1) * c.dil) * (C + 1)) * sizeof(float);
  if (lds > 160 * 1024) { set_error("nsf conv: LDS window too large"); return PD_ERR_UNSUPPORTED; }
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&nsf_conv_small_kernel<C>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) { set_error("nsf conv: cannot raise the dynamic LDS limit"); return PD_ERR_HIP; }
  ProfScope ps("nsf_res_small", st);
  hipLaunchKernelGGL(nsf_conv_small_kernel<C>, dim3(cdiv(Tl, TR), B), dim3(256), lds, st, in, c.w, c.taps * c.kpad,
                     c.kpad, c.b, c.taps, c.dil, alpha, scale, Tl, res, out, rag_);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- windowed MFMA conv (bf16)
// ResBlock conv y[t] = b + sum_tap W_tap . lrelu(x[t + tap*d - pad]) (+ res) on the bf16 MFMA
// path.  The implicit-GEMM engine streams one K segment per tap, so each tap re-reads the
// activations from L2/HBM and every 32-deep K chunk waits on a global load.  Here a block
// stages its input window ONCE -- TM rows plus the (k-1)*d halo, all C channels,
// leaky-ReLU'd, scaled and rounded to bf16 -- into LDS; every tap's A fragments are
// row-shifted reads of that window.  Weights (the pool's bf16 copy, packed
// [cout][tap*kpad + ci]) stream from L2 into registers one 16-deep k-step ahead.
// Block = 256 threads = WM x WN waves, wave tile (32 FM rows) x (32 FN channels):
// TM = 32 FM WM = 128 rows, TN = 32 FN WN output channels (grid.y covers C / TN),
// grid.z = utterance.  LDS row stride C + 8 bf16: lanes r and r+1 of a b128 fragment read
// sit 4 banks apart for every C used here, so a wave's fragment read is conflict-free.
// Stage rows [r0, r0 + W) of utterance b (zero outside [0, Tl)) of a time-major [B][Tl][C]
// tensor into LDS as bf16 (row pitch lda), leaky_relu(alpha) * scale applied: the input window
// of the windowed convs.  Each thread keeps NSF_WB 16-byte items in flight: all loads of a batch
// are issued before any is converted (r02: C5 21.6 -> 21.0 ms/step).
constexpr int NSF_WB = 4;
// Epilogue stores without a row-range branch (r04: with `if (t < Tl)` around each store the waitcnt
// pass put a full vmcnt(0) before every one, so a lane's 16 stores ran one round trip apart): a
// buffer resource spanning exactly one utterance's rows of `out`; stores past its last row are
// dropped by the hardware range check.
// The range and the byte offsets are unsigned 32-bit: the host guards (nsf_check_rows) keep one
// utterance's Tl * C * sizeof(out) below 2^32.
template <bool OUT_BF>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t nsf_utt_rsrc(void* out, int rowb, int Tl, int C) {
  const unsigned es = OUT_BF ? 2u : 4u;
  char* base = reinterpret_cast<char*>(out) + (long long)rowb * C * es;
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (unsigned)Tl * (unsigned)C * es, 0x00020000);
}
template <bool OUT_BF>
__device__ __forceinline__ void nsf_store_utt(__amdgpu_buffer_rsrc_t r, int elem, float v) {
  if constexpr (OUT_BF) {
    const __bf16 hv = (__bf16)v;
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, hv), r, (unsigned)elem * 2u, 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, (unsigned)elem * 4u, 0, 0);
  }
}

// Stages window rows r0 .. r0 + W - 1 of `in` (lrelu(alpha) * scale, bf16) into win; rows outside
// [0, Tv) are zero (Tv <= Tl: the utterance's own end in a ragged batch; rows are laid out at Tl).  r04: loads unconditional (clamped row), zero rows by a multiply, and every LDS
// store unconditional -- items past the window go to row W, one spare row the callers allocate
// (or that the next stage overwrites): with `if (ok)` loads / `if (i < nitems)` stores hipcc sank
// the loads into the branches and waited for each one, a round trip per item instead of per batch.
template <int C, bool IN_BF, int NT = 256>
__device__ __forceinline__ void stage_window(const void* __restrict__ in, int b, int Tl, int Tv, int r0, int W,
                                             float alpha, float scale, __bf16* __restrict__ win, int lda, int tid) {
  constexpr int C8 = C / 8;
  const int nitems = W * C8;
  for (int base = tid; base < nitems; base += NT * NSF_WB) {
    float f[NSF_WB][8];
#pragma unroll
    for (int u = 0; u < NSF_WB; ++u) {
      const int i = base + NT * u;
      const int row = i / C8, c8 = i - row * C8;
      const int t = r0 + row;
      const bool ok = i < nitems && t >= 0 && t < Tv;
      const float m = ok ? 1.f : 0.f;
      const long long e = ((long long)b * Tl + (ok ? t : 0)) * C + 8 * c8;
      if constexpr (IN_BF) {
        const bf16x8 x = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(in) + e);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[u][j] = (float)x[j] * m;
      } else {
        const float4 x0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(in) + e);
        const float4 x1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(in) + e + 4);
        f[u][0] = x0.x * m; f[u][1] = x0.y * m; f[u][2] = x0.z * m; f[u][3] = x0.w * m;
        f[u][4] = x1.x * m; f[u][5] = x1.y * m; f[u][6] = x1.z * m; f[u][7] = x1.w * m;
      }
    }
#pragma unroll
    for (int u = 0; u < NSF_WB; ++u) {
      const int i = base + NT * u;
      const bool in_w = i < nitems;
      const int row = in_w ? i / C8 : W, c8 = in_w ? i - (i / C8) * C8 : 0;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)((f[u][j] >= 0.f ? f[u][j] : alpha * f[u][j]) * scale);
      *reinterpret_cast<bf16x8*>(win + row * lda + 8 * c8) = v;
    }
  }
}

// weight-fragment prefetch depth (k-steps).  Measured (r02, C5 B=8): ring 4 without a
// sched_barrier 386 us for the 128-channel k=11 conv; pinning the ring with sched_barrier
// raised VGPRs to 2 waves/SIMD and ran slower (459 us at depth 4, 486 us at depth 8).
#ifndef NSF_PF_DEPTH
#define NSF_PF_DEPTH 4
#endif
#ifndef NSF_RING_PIN
#define NSF_RING_PIN 0
#endif
constexpr int NSF_PF = NSF_PF_DEPTH;
#ifndef NSF_PAIR_PF
#define NSF_PAIR_PF NSF_PF_DEPTH   // the pair kernel's weight ring depth (k-steps)
#endif

// WM x WN = 4 waves, or 8 (r06, C = 256: one block covers all 256 output channels, so the window is
// staged once per row tile instead of once per 128-channel half, two waves per SIMD)
template <int C, int FM, int FN, int WM, int WN, bool IN_BF, bool OUT_BF>
__global__ __launch_bounds__(64 * WM * WN, WM * WN == 4 ? 3 : 1) void nsf_wconv_kernel(const void* __restrict__ in, const __bf16* __restrict__ w,
                                                        int ldw, int kpad, const float* __restrict__ bias, int taps,
                                                        int dil, float alpha, float scale, int Tl,
                                                        const float* __restrict__ res, void* __restrict__ out,
                                                        int accum, NsfRag rag_) {
  static_assert(WM * WN == 4 || WM * WN == 8, "4 or 8 waves");
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = 32 * FM * WM, TN = 32 * FN * WN, LDA = C + 8, KS = C / 16;
  static_assert(C % TN == 0, "channel tiling");
  extern __shared__ __attribute__((aligned(16))) __bf16 nsf_win[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int b = blockIdx.z, t0 = blockIdx.x * TM, n0 = blockIdx.y * TN;
  const int pad = (taps - 1) * dil / 2;
  const int W = TM + (taps - 1) * dil;
  // 1. the input window, 8 channels (16 B of bf16) per item, NSF_WB items per thread in flight
  //    together (a load-convert-store loop waits one HBM round trip per item)
  stage_window<C, IN_BF, NT>(in, b, Tl, nsf_tv(rag_, b, Tl), t0 - pad, W, alpha, scale, nsf_win, LDA, tid);
  __syncthreads();
  // 2. taps x 16-deep k-steps; B fragments prefetched one step ahead
  const int r32 = lane & 31, h = lane >> 5;
  const __bf16* wr[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) wr[j] = w + (long long)(n0 + (wn * FN + j) * 32 + r32) * ldw + 8 * h;
  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // B fragments run PF k-steps ahead in a register ring (one L2 round trip is ~2k cycles, one
  // k-step of MFMAs ~100-200).  PF divides the k-steps per tap, so S = taps * KS is a multiple
  // of PF and the loop body -- unrolled by PF, every slot index static -- has no branch; the
  // last prefetches re-load the final step instead of testing the bound.
  constexpr int PF = KS >= NSF_PF ? NSF_PF : KS;
  static_assert(KS % PF == 0, "ring depth divides the k-steps per tap");
  const int S = taps * KS;
  bf16x8 bq[PF][FN];
  auto bload = [&](int st, bf16x8* dst) {
    const int tn = st / KS, kn = st - tn * KS;
#pragma unroll
    for (int j = 0; j < FN; ++j) dst[j] = *reinterpret_cast<const bf16x8*>(wr[j] + tn * kpad + 16 * kn);
  };
#pragma unroll
  for (int q = 0; q < PF - 1; ++q) bload(q, bq[q]);
  const __bf16* arow = nsf_win + (wm * FM * 32 + r32) * LDA + 8 * h;
  for (int s0 = 0; s0 < S; s0 += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int s = s0 + q;
      bload(min(s + PF - 1, S - 1), bq[(q + PF - 1) % PF]);
#if NSF_RING_PIN
      __builtin_amdgcn_sched_barrier(0);   // keep the load PF - 1 steps ahead of its use
#endif
      const int tap = s / KS, kc = s - tap * KS;
      bf16x8 af[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(arow + (i * 32 + tap * dil) * LDA + 16 * kc);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bq[q][j], acc[i][j], 0, 0, 0);
    }
  }
  // 3. epilogue: + bias (+ res) (+ out when accumulating), C/D map col = lane&31,
  // row = (reg&3) + 8(reg>>2) + 4(lane>>5).  In two batches of 8 rows per fragment, the
  // residual / accumulator loads of EVERY fragment are in flight together (rows past the end
  // clamp to the last row), then the predicated stores: two memory round trips per block
  // instead of two per fragment (r02: the residual convs ran ~1.5x their plain twins).
  // 32-bit element offsets (the host checks B*Tl*C < 2^31) keep one VGPR per address
  const int rowb = b * Tl;
  const __amdgpu_buffer_rsrc_t ors = nsf_utt_rsrc<OUT_BF>(out, rowb, Tl, C);
  float bn[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bn[j] = bias[n0 + (wn * FN + j) * 32 + r32];
#pragma unroll
  for (int hb = 0; hb < 16; hb += 8) {   // two batches of 8 rows: fewer live registers
    float rv[FM][FN][8];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int reg = hb + q, n = n0 + (wn * FN + j) * 32 + r32;
          const int t = min(t0 + wm * FM * 32 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, Tl - 1);
          const int o = (rowb + t) * C + n;
          // branch-free (r04): a load under `res ?` / `if (accum)` made the waitcnt pass wait for
          // each one in turn (16 round trips per lane); an fp32 output always has a residual
          float v = 0.f;
          if constexpr (!OUT_BF) {
            const float a = reinterpret_cast<const float*>(out)[o];
            v = res[o];
            v = accum ? v + a : v;
          }
          rv[i][j][q] = v;
        }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int reg = hb + q, n = n0 + (wn * FN + j) * 32 + r32;
          const int t = t0 + wm * FM * 32 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
          const float v = acc[i][j][reg] + bn[j] + rv[i][j][q];
          nsf_store_utt<OUT_BF>(ors, t * C + n, v);   // rows t >= Tl fall outside ors and are dropped
        }
  }
}

// ResBlock1 conv pair in ONE launch (models.py:57-63, one q of ResBlock1.forward):
//   xt = c1(lrelu(x)) (dilation d), out = c2(lrelu(xt)) (dilation 1) + x [+ out when accumulating]
// Block = TM = 32 FMO output rows of one utterance, 4 waves.  The x window (rows t0 - p2 - p1 ..
// t0 + TM + p2 + p1, lrelu'd, bf16) is staged once; c1 runs on the 32 (FMO + 1) rows of xt that
// c2 reads (TM + 2 p2 <= 32 (FMO + 1) for k <= 33), rounds them to bf16 exactly as the two-launch
// path's bf16 intermediate, applies lrelu and keeps them in LDS; c2 reads that window.  Per
// output row this drops the intermediate's HBM write and read and the second staging of x.
// Waves: column tile ct = wave % NCT (NCT = C / 32) of both convs; with NCT = 2 the row tiles are
// split between two wave pairs by parity, with NCT = 1 (C = 32, r04) between all four waves (FMO = 15:
// 16 c1 row tiles and 15 c2 row tiles over 4 waves).
// TAPS / DIL > 0 (r05): the ResBlock's kernel size and c1's dilation as compile-time constants --
// every LDS / weight address of the fully unrolled tap loops folds into an immediate offset (the
// runtime-taps build spent ~60 VALU instructions per MFMA at C = 32, mostly address arithmetic,
// and ran VALU-bound: 0.90 VALU busy, profiles/r04_final/c5_sq.json).  0 = runtime (other shapes).
template <int C, int FMO, int TAPS = 0, int DIL = 0>
__global__ __launch_bounds__(256, 2) void nsf_pair_kernel(const float* __restrict__ x, const __bf16* __restrict__ w1,
                                                      const __bf16* __restrict__ w2, int ldw_, int kpad_,
                                                      const float* __restrict__ b1, const float* __restrict__ b2,
                                                      int taps_, int dil_, int Tl, float* __restrict__ out, int accum,
                                                      NsfRag rag_) {
  // (compile-time shapes: the packed weights' K chunk is C, the host checks kpad == C)
  const int taps = TAPS ? TAPS : taps_, dil = DIL ? DIL : dil_;
  const int kpad = TAPS ? C : kpad_, ldw = TAPS ? TAPS * C : ldw_;
  constexpr int NCT = C / 32, RG = 4 / NCT, LDA = C + 8, KS = C / 16;
  constexpr int TM = 32 * FMO, RT1 = FMO + 1;            // output rows; c1 row tiles
  constexpr int MF1 = (RT1 + RG - 1) / RG, MF2 = (FMO + RG - 1) / RG;   // row tiles per wave
  static_assert(NCT == 1 || NCT == 2 || NCT == 4, "C = 32, 64 or 128");
  extern __shared__ __attribute__((aligned(16))) __bf16 nsf_win[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int ct = wave % NCT, rg = wave / NCT;
  const int b = blockIdx.z, t0 = blockIdx.x * TM;
  const int p2 = (taps - 1) / 2, p1 = (taps - 1) * dil / 2;
  const int WX = 32 * RT1 + (taps - 1) * dil;            // x window rows
  __bf16* xwin = nsf_win;                                // [WX][LDA]: lrelu(x), time t0 - p2 - p1 + j
  // [32 RT1][LDA]: lrelu(xt), time t0 - p2 + i.  It takes x's window rows (32 RT1 <= WX) once every
  // wave's c1 is done (a barrier between c1's MFMAs and its epilogue): one window per block, so 2
  // blocks share a CU at C = 128 (r04: x and xt side by side, 88-101 KB, left room for one)
  __bf16* xtw = nsf_win;
  const int Tv = nsf_tv(rag_, b, Tl);
  stage_window<C, false>(x, b, Tl, Tv, t0 - p2 - p1, WX, NSF_LRELU, 1.f, xwin, LDA, tid);
  __syncthreads();
  const int S = taps * KS;
  constexpr int PF = KS >= NSF_PAIR_PF ? NSF_PAIR_PF : KS;
  static_assert(KS % PF == 0, "ring depth divides the k-steps per tap");
  const int n = ct * 32 + r32;                           // this lane's output channel (C layout column)
  // ---- c1 on row tiles rt = rg + RG m (xt rows 32 rt ..)
  {
    const __bf16* wr = w1 + (long long)n * ldw + 8 * h;
    f32x16 acc[MF1];
#pragma unroll
    for (int m = 0; m < MF1; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
    bf16x8 bq[PF];
    auto bload = [&](int st) {
      const int tn = st / KS, kn = st - tn * KS;
      return *reinterpret_cast<const bf16x8*>(wr + tn * kpad + 16 * kn);
    };
#pragma unroll
    for (int q = 0; q < PF - 1; ++q) bq[q] = bload(q);
#pragma unroll
    for (int s0 = 0; s0 < S; s0 += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int s = s0 + q;
        bq[(q + PF - 1) % PF] = bload(min(s + PF - 1, S - 1));
        const int tap = s / KS, kc = s - tap * KS;
#pragma unroll
        for (int m = 0; m < MF1; ++m) {
          const int rt = rg + RG * m;
          if (rt < RT1) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(xwin + (rt * 32 + r32 + tap * dil) * LDA + 16 * kc + 8 * h);
            acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bq[q], acc[m], 0, 0, 0);
          }
        }
      }
    }
    // xt = bf16(acc + b1) (the two-launch path's bf16 intermediate), then c2's input lrelu(xt)
    // rounded to bf16 again; rows outside the utterance are c2's zero padding
    const float bn = b1[n];
    __syncthreads();   // x's window is dead: xt overwrites it
#pragma unroll
    for (int m = 0; m < MF1; ++m) {
      const int rt = rg + RG * m;
      if (rt < RT1) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int i = rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, t = t0 - p2 + i;
          const float v = (float)(__bf16)(acc[m][reg] + bn);
          const float u = (t >= 0 && t < Tv) ? (v >= 0.f ? v : NSF_LRELU * v) : 0.f;
          xtw[i * LDA + n] = (__bf16)u;
        }
      }
    }
  }
  __syncthreads();
  // ---- c2 on output row tiles rt = rg + RG m, + bias + residual x (+ out)
  {
    const __bf16* wr = w2 + (long long)n * ldw + 8 * h;
    f32x16 acc[MF2];
#pragma unroll
    for (int m = 0; m < MF2; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
    bf16x8 bq[PF];
    auto bload = [&](int st) {
      const int tn = st / KS, kn = st - tn * KS;
      return *reinterpret_cast<const bf16x8*>(wr + tn * kpad + 16 * kn);
    };
#pragma unroll
    for (int q = 0; q < PF - 1; ++q) bq[q] = bload(q);
#pragma unroll
    for (int s0 = 0; s0 < S; s0 += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int s = s0 + q;
        bq[(q + PF - 1) % PF] = bload(min(s + PF - 1, S - 1));
        const int tap = s / KS, kc = s - tap * KS;
#pragma unroll
        for (int m = 0; m < MF2; ++m) {
          const int rt = rg + RG * m;
          if (rt < FMO) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(xtw + (rt * 32 + r32 + tap) * LDA + 16 * kc + 8 * h);
            acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bq[q], acc[m], 0, 0, 0);
          }
        }
      }
    }
    const float bn = b2[n];
    const int rowb = b * Tl;
#pragma unroll
    for (int m = 0; m < MF2; ++m) {
      const int rt = rg + RG * m;
      if (rt < FMO) {
        float rv[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {   // residual (and accumulator) loads in flight together
          const int t = min(t0 + rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, Tl - 1);
          const int o = (rowb + t) * C + n;
          rv[reg] = x[o] + (accum ? out[o] : 0.f);
        }
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int t = t0 + rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
          if (t < Tl) out[(rowb + t) * C + n] = acc[m][reg] + bn + rv[reg];
        }
      }
    }
  }
}

#ifndef NSF_PAIR_FMO32
#define NSF_PAIR_FMO32 15   // C = 32 output row tiles per block (r04: 7 -> 15, C5 -3%)
#endif
#ifndef NSF_PAIR_FMO64
#define NSF_PAIR_FMO64 8   // C = 64 output row tiles per block (r04: 4 -> 8, C5 -4%)
#endif
#ifndef NSF_PAIR_FMO128
#define NSF_PAIR_FMO128 4  // C = 128 output row tiles per block
#endif
template <int C, int TAPS, int DIL>
int launch_pair_ct(const NsfConv& c1, const NsfConv& c2, const float* x, int B, int Tl, float* out, int accum,
                   hipStream_t st, NsfRag rag_) {
  constexpr int FMO = C == 32 ? NSF_PAIR_FMO32 : C == 64 ? NSF_PAIR_FMO64 : NSF_PAIR_FMO128, TM = 32 * FMO;
  // x / xt window + stage_window's spare row
  const size_t lds = (size_t)(32 * (FMO + 1) + (c1.taps - 1) * c1.dil + 1) * (C + 8) * sizeof(__bf16);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&nsf_pair_kernel<C, FMO, TAPS, DIL>), hipFuncAttributeMaxDynamicSharedMemorySize,
      160 * 1024);
  if (attr != hipSuccess) { set_error("nsf pair: cannot raise the dynamic LDS limit"); return PD_ERR_HIP; }
  ProfScope ps("nsf_pair", st);
  hipLaunchKernelGGL((nsf_pair_kernel<C, FMO, TAPS, DIL>), dim3(cdiv(Tl, TM), 1, B), dim3(256), lds, st, x,
                     lookup_bf16(c1.w), lookup_bf16(c2.w), c1.taps * c1.kpad, c1.kpad, c1.b, c2.b, c1.taps, c1.dil, Tl,
                     out, accum, rag_);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// compile-time (taps, dilation) for the shipped ResBlock1 shapes (kernel sizes 3, 7, 11 x dilations
// 1, 3, 5; handler/base_config.yaml), the runtime kernel otherwise
template <int C>
int launch_pair_c(const NsfConv& c1, const NsfConv& c2, const float* x, int B, int Tl, float* out, int accum,
                  hipStream_t st, NsfRag rag_) {
#define PD_PAIR_CASE(K, D) \
  if (c1.taps == K && c1.dil == D && c1.kpad == C) return launch_pair_ct<C, K, D>(c1, c2, x, B, Tl, out, accum, st, rag_)
  PD_PAIR_CASE(3, 1); PD_PAIR_CASE(3, 3); PD_PAIR_CASE(3, 5);
  PD_PAIR_CASE(7, 1); PD_PAIR_CASE(7, 3); PD_PAIR_CASE(7, 5);
  PD_PAIR_CASE(11, 1); PD_PAIR_CASE(11, 3); PD_PAIR_CASE(11, 5);
#undef PD_PAIR_CASE
  return launch_pair_ct<C, 0, 0>(c1, c2, x, B, Tl, out, accum, st, rag_);
}

bool wconv_ok(const NsfConv& c);
// The fused pair for these convs, if it has one: both windowed (bf16), 32, 64 or 128 channels, equal
// taps and packing, c2 undilated.
// C = 16 (nsf_pair16_kernel): the shipped shapes only -- taps 3 / 7 / 11, c1 dilation 1 / 3 / 5.
// The whole 16-channel ResBlock1 in one launch (nsf_rb16_kernel): three bf16 windowed pairs of one
// shipped kernel size with c1 dilations 1, 3, 5 and c2 undilated.
bool rb_ok(const nsf_model* m, const NsfConv* c1, const NsfConv* c2, int C) {
  const int k = c1[0].taps, bit = k == 3 ? 1 : k == 7 ? 2 : k == 11 ? 4 : 0;
  if (C == 16 ? !m->rb16 : C == 32 ? !(m->rb32 & bit) : C == 64 ? !(m->rb64 & bit) : true) return false;
  for (int q = 0; q < 3; ++q) {
    const NsfConv &a = c1[q], &b = c2[q];
    if (!wconv_ok(a) || !wconv_ok(b) || a.cout != C || b.cout != C || a.kpad != (C == 16 ? 32 : C) || b.kpad != a.kpad ||
        a.taps != c1[0].taps || b.taps != a.taps || a.dil != (q == 0 ? 1 : q == 1 ? 3 : 5) || b.dil != 1)
      return false;
  }
  return c1[0].taps == 3 || c1[0].taps == 7 || c1[0].taps == 11;
}
bool pair_ok(const nsf_model* m, const NsfConv& c1, const NsfConv& c2) {
  const bool c16 = c1.cout == 16 && c1.kpad == 32 && (c1.taps == 3 || c1.taps == 7 || c1.taps == 11) &&
                   (c1.dil == 1 || c1.dil == 3 || c1.dil == 5);
  return m->pair && wconv_ok(c1) && wconv_ok(c2) && c1.cout == c2.cout &&
         (c1.cout == 32 || c1.cout == 64 || c1.cout == 128 || (c16 && m->pair16)) &&
         c1.taps == c2.taps && c1.kpad == c2.kpad && c2.dil == 1 && c1.taps <= 33;
}
int launch_pair16(const NsfConv& c1, const NsfConv& c2, const float* x, int B, int Tl, float* out, int accum,
                  hipStream_t st, NsfRag rag_);

int launch_pair(const NsfConv& c1, const NsfConv& c2, const float* x, int B, int Tl, float* out, int accum,
                hipStream_t st, NsfRag rag_) {
  if ((long long)B * Tl * c1.cout >= (1ll << 31)) {
    set_error("nsf pair: B * T * C >= 2^31 elements (32-bit epilogue offsets)");
    return PD_ERR_UNSUPPORTED;
  }
  if (c1.cout == 16) return launch_pair16(c1, c2, x, B, Tl, out, accum, st, rag_);
  if (c1.cout == 128) return launch_pair_c<128>(c1, c2, x, B, Tl, out, accum, st, rag_);
  if (c1.cout == 32) return launch_pair_c<32>(c1, c2, x, B, Tl, out, accum, st, rag_);
  return launch_pair_c<64>(c1, c2, x, B, Tl, out, accum, st, rag_);
}

// 16-channel variant (the last upsample stage, 512 samples per frame) on
// v_mfma_f32_16x16x32_bf16: one MFMA's 32-deep K covers TWO taps x 16 channels (lane group
// g = lane>>4 holds channels 8(g&1).. of tap 2p + (g>>1)); an odd tap count pads the last
// pair with zero weights and zero activations.  All taps' weights fit in registers (<= 6
// fragments), loaded once.  Block = 4 waves x 64 rows (4 M fragments of 16) = 256 rows.
// MFMA 16x16x32 layouts: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15],
// D[row 4(l>>4)+r][col l&15].
// TAPS / DIL > 0 (r05): compile-time kernel size and dilation (see nsf_pair_kernel); kpad is then 32.
template <bool IN_BF, bool OUT_BF, int TAPS = 0, int DIL = 0>
__global__ __launch_bounds__(256) void nsf_wconv16_kernel(const void* __restrict__ in, const __bf16* __restrict__ w,
                                                          int kpad_, const float* __restrict__ bias, int taps_,
                                                          int dil_, float alpha, float scale, int Tl,
                                                          const float* __restrict__ res, void* __restrict__ out,
                                                          int accum, NsfRag rag_) {
  constexpr int C = 16, TM = 256, LDA = 24, MAXP = 6;
  const int taps = TAPS ? TAPS : taps_, dil = DIL ? DIL : dil_, kpad = TAPS ? 32 : kpad_;
  extern __shared__ __attribute__((aligned(16))) __bf16 nsf_win16[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.y, t0 = blockIdx.x * TM;
  const int pad = (taps - 1) * dil / 2;
  const int W = TM + (taps - 1) * dil;
  // the window (W rows x 2 items) in batches of NSF_WB items per thread, every load of a batch
  // issued before any is converted (one round trip per batch, not one per item)
  stage_window<C, IN_BF>(in, b, Tl, nsf_tv(rag_, b, Tl), t0 - pad, W, alpha, scale, nsf_win16, LDA, tid);
  const int r16 = lane & 15, g = lane >> 4, kg = g & 1, tg = g >> 1;
  const int npair = (taps + 1) >> 1;
  // every pair's fragment loaded unconditionally (clamped tap) and zeroed by a bit mask: a load
  // under `if (tap < taps)` was waited for on its own, six L2 round trips in a row (r04)
  bf16x8 bw[MAXP];
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int tap = 2 * p + tg, tc = min(tap, taps - 1);
    const uint4 raw = *reinterpret_cast<const uint4*>(w + (long long)r16 * (taps * kpad) + tc * kpad + 8 * kg);
    const unsigned mk = (p < npair && tap < taps) ? 0xffffffffu : 0u;
    bw[p] = __builtin_bit_cast(bf16x8, make_uint4(raw.x & mk, raw.y & mk, raw.z & mk, raw.w & mk));
  }
  // the epilogue's residual / accumulator operands, loaded now so they land under the MFMAs
  float rv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = min(t0 + wave * 64 + i * 16 + 4 * g + r, Tl - 1);
      const long long o = ((long long)b * Tl + t) * C + r16;
      float v = 0.f;   // branch-free, as nsf_wconv_kernel's epilogue
      if constexpr (!OUT_BF) {
        const float a = reinterpret_cast<const float*>(out)[o];
        v = res[o];
        v = accum ? v + a : v;
      }
      rv[i][r] = v;
    }
  __syncthreads();
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    if (p < npair) {
      const int tap = 2 * p + tg;
      const bool live = tap < taps;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf16x8 af;
        if (live) {
          af = *reinterpret_cast<const bf16x8*>(nsf_win16 + (wave * 64 + i * 16 + r16 + tap * dil) * LDA + 8 * kg);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) af[j] = (__bf16)0.f;
        }
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[p], acc[i], 0, 0, 0);
      }
    }
  }
  const float bn = bias[r16];
  const __amdgpu_buffer_rsrc_t ors = nsf_utt_rsrc<OUT_BF>(out, b * Tl, Tl, C);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = t0 + wave * 64 + i * 16 + 4 * g + r;
      const float v = acc[i][r] + bn + rv[i][r];
      nsf_store_utt<OUT_BF>(ors, t * C + r16, v);   // rows t >= Tl dropped by the range check
    }
  }
}

// ResBlock1 conv pair at C = 16 in ONE launch (r05; models.py:57-63): nsf_pair_kernel's structure on
// nsf_wconv16_kernel's 16x16x32 MFMA layout, for the shipped (taps, dilation) shapes.  Block = 256
// output rows, 4 waves.  The x window (rows t0 - p2 - p1 .., lrelu'd, bf16) is staged once; c1 runs
// on the 17 16-row tiles of xt that c2 reads (times t0 - p2 + i, i < 272 >= 256 + 2 p2), rounds them
// to bf16 as the two-launch path's bf16 intermediate, applies lrelu, zeroes rows outside the
// utterance and keeps them in their own LDS window; c2 adds bias and the residual x (+ out).  Same
// roundings and the same MFMA order as two nsf_wconv16 launches: bit-identical, without the bf16
// intermediate's HBM write and read (the C = 16 stage is the step's largest activation: 64 B per
// row at 441k rows per utterance) and the second window staging.
template <int TAPS, int DIL>
__global__ __launch_bounds__(256, 3) void nsf_pair16_kernel(const float* __restrict__ x, const __bf16* __restrict__ w1,
                                                         const __bf16* __restrict__ w2, const float* __restrict__ b1,
                                                         const float* __restrict__ b2, int Tl, float* __restrict__ out,
                                                         int accum, NsfRag rag_) {
  constexpr int C = 16, TM = 256, LDA = 24, NP = (TAPS + 1) / 2, KP = 32;
  constexpr int P2 = (TAPS - 1) / 2, P1 = (TAPS - 1) * DIL / 2;
  constexpr int RT1 = 17, XR = 16 * RT1, WX = XR + (TAPS - 1) * DIL, MF1 = (RT1 + 3) / 4;
  static_assert(TM + 2 * P2 <= XR, "c1's tiles cover c2's reach");
  __shared__ __attribute__((aligned(16))) __bf16 xwin[(WX + 1) * LDA];   // + stage_window's spare row
  __shared__ __attribute__((aligned(16))) __bf16 xtw[XR * LDA];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.y, t0 = blockIdx.x * TM;
  const int Tv = nsf_tv(rag_, b, Tl);
  stage_window<C, false>(x, b, Tl, Tv, t0 - P2 - P1, WX, NSF_LRELU, 1.f, xwin, LDA, tid);
  const int r16 = lane & 15, g = lane >> 4, kg = g & 1, tg = g >> 1;
  // a conv's tap-pair fragments, unconditional loads at a clamped tap, zeroed by a bit mask (c2's
  // are loaded after c1's MFMAs: 24 fewer live registers through c1)
  auto wload = [&](const __bf16* w, bf16x8 (&wf)[NP]) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int tap = 2 * p + tg, tc = min(tap, TAPS - 1);
      const unsigned mk = tap < TAPS ? 0xffffffffu : 0u;
      const uint4 r = *reinterpret_cast<const uint4*>(w + (long long)r16 * (TAPS * KP) + tc * KP + 8 * kg);
      wf[p] = __builtin_bit_cast(bf16x8, make_uint4(r.x & mk, r.y & mk, r.z & mk, r.w & mk));
    }
  };
  bf16x8 wf1[NP], wf2[NP];
  wload(w1, wf1);
  // c2's residual / accumulator operands, in flight under the MFMAs (nsf_wconv16_kernel's order)
  float rv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = min(t0 + wave * 64 + i * 16 + 4 * g + r, Tl - 1);
      const long long o = ((long long)b * Tl + t) * C + r16;
      const float a = out[o];
      const float v = x[o];
      rv[i][r] = accum ? v + a : v;
    }
  const float bn1 = b1[r16], bn2 = b2[r16];
  __syncthreads();
  const bf16x8 z8 = {};
  // ---- c1 on xt tiles rt = wave + 4 m
  {
    f32x4 acc[MF1];
#pragma unroll
    for (int m = 0; m < MF1; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int tap = 2 * p + tg;
#pragma unroll
      for (int m = 0; m < MF1; ++m) {
        const int rt = wave + 4 * m;
        if (rt < RT1) {   // (wave-uniform)
          bf16x8 af = *reinterpret_cast<const bf16x8*>(xwin + (rt * 16 + r16 + min(tap, TAPS - 1) * DIL) * LDA + 8 * kg);
          if (TAPS % 2 == 1 && p == NP - 1) af = tap < TAPS ? af : z8;
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf1[p], acc[m], 0, 0, 0);
        }
      }
    }
    wload(w2, wf2);
    // xt = bf16(acc + b1) (the two-launch path's bf16 intermediate), then c2's input lrelu(xt)
    // rounded to bf16 again; rows outside the utterance are c2's zero padding
#pragma unroll
    for (int m = 0; m < MF1; ++m) {
      const int rt = wave + 4 * m;
      if (rt < RT1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = rt * 16 + 4 * g + r, t = t0 - P2 + i;
          const float v = (float)(__bf16)(acc[m][r] + bn1);
          const float u = (t >= 0 && t < Tv) ? (v >= 0.f ? v : NSF_LRELU * v) : 0.f;
          xtw[i * LDA + r16] = (__bf16)u;
        }
      }
    }
  }
  __syncthreads();
  // ---- c2 on output tiles wave * 4 + i, + bias + residual (+ out)
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int tap = 2 * p + tg;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8 af = *reinterpret_cast<const bf16x8*>(xtw + (wave * 64 + i * 16 + r16 + min(tap, TAPS - 1)) * LDA + 8 * kg);
      if (TAPS % 2 == 1 && p == NP - 1) af = tap < TAPS ? af : z8;
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf2[p], acc[i], 0, 0, 0);
    }
  }
  const __amdgpu_buffer_rsrc_t ors = nsf_utt_rsrc<false>(out, b * Tl, Tl, C);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = t0 + wave * 64 + i * 16 + 4 * g + r;
      nsf_store_utt<false>(ors, t * C + r16, acc[i][r] + bn2 + rv[i][r]);   // rows t >= Tl dropped
    }
}

int launch_pair16(const NsfConv& c1, const NsfConv& c2, const float* x, int B, int Tl, float* out, int accum,
                  hipStream_t st, NsfRag rag_) {
  const dim3 grid(cdiv(Tl, 256), B);
  ProfScope ps("nsf_pair16", st);
#define PD_PAIR16(K, D)                                                                                            \
  if (c1.taps == K && c1.dil == D)                                                                                 \
    hipLaunchKernelGGL((nsf_pair16_kernel<K, D>), grid, dim3(256), 0, st, x, lookup_bf16(c1.w), lookup_bf16(c2.w), \
                       c1.b, c2.b, Tl, out, accum, rag_)
  PD_PAIR16(3, 1); else PD_PAIR16(3, 3); else PD_PAIR16(3, 5);
  else PD_PAIR16(7, 1); else PD_PAIR16(7, 3); else PD_PAIR16(7, 5);
  else PD_PAIR16(11, 1); else PD_PAIR16(11, 3); else PD_PAIR16(11, 5);
  else { set_error("nsf pair16: not a shipped (taps, dilation) shape"); return PD_ERR_UNSUPPORTED; }
#undef PD_PAIR16
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- whole ResBlock1 at C = 16 (r06)
// One launch per ResBlock1 of the 16-channel stage (models.py:57-63: the three (c1, c2) pairs with c1
// dilations 1 / 3 / 5): x_{q+1} = x_q + c2(lrelu(c1(lrelu(x_q)))), the last pair adding into the ResBlock
// sum xs (models.py:275-279).  That stage is the step's largest activation (16 fp32 channels at 512
// samples per mel frame): the three pair launches read and wrote it three times per ResBlock (HBM-bound:
// 131-167 us each at C5).  Here a block keeps its rows' residual x_q in registers across the three pairs
// and reads x / writes (or adds into) xs once.
// Window: NTW 16-row tiles, W = 16 NTW rows at times tw + i (tw = t0 - H); the ResBlock's reach on each
// side is H = sum over the pairs of p1 + p2 = 12 (TAPS - 1) / 2 rows, so TM = W - 2 H rows are output.
// x_q is exact on rows [V_q, W - V_q), V_{q+1} = V_q + p1 + p2; each conv runs on the 16-row tiles its
// consumers read (rows outside the exact range only ever feed rows outside it).
// Layout: transposed MFMA D[co][t] = W . act on v_mfma_f32_16x16x32_bf16 (A = the weights exactly as
// nsf_pair16_kernel's B operand, B = the activation window as its A operand): lane (t = lane & 15,
// g = lane >> 4) holds channels 4g .. 4g + 3 of one row, so a row's bf16 activation goes to LDS as one
// 8-B write and the residual is 4 registers per tile.  Same products, same k order per MFMA, same
// epilogue roundings and additions as the pair launches: bit-identical (tests/test_gpu_nsf.py).
// One LDS window rewritten in place: a conv reads it, a barrier, the conv's output activation replaces
// it, a barrier.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct NsfRb16Args {
  const __bf16* w1[3];
  const __bf16* w2[3];
  const float* b1[3];
  const float* b2[3];
};
template <int TAPS, int NTW, int NW>
__global__ __launch_bounds__(NW * 64) void nsf_rb16_kernel(const float* __restrict__ x, const NsfRb16Args A, int Tl,
                                                           float* __restrict__ out, int accum, NsfRag rag_) {
  constexpr int C = 16, LDA = 24, NP = (TAPS + 1) / 2, KP = 32, P2 = (TAPS - 1) / 2;
  constexpr int H = 12 * P2, W = 16 * NTW, TM = W - 2 * H, IPW = NTW / NW, PADR = 16;
  static_assert(NTW % NW == 0 && TM > 0, "window tiles per wave");
  // (a conv on tiles [kf, kl] clipped to its exact rows [e, W - e) reads rows [e - r - 15, W - e + r + 14) of an
  // input exact on [e - r, W - e + r): never more than 15 rows outside the window, whatever its reach r)
  __shared__ __attribute__((aligned(16))) __bf16 buf[(W + 2 * PADR) * LDA];
  __bf16* bw = buf + PADR * LDA;               // window row i at bw + i LDA, i in [-16, W + 16)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4, kg = g & 1, tg = g >> 1;
  const int b = blockIdx.y, t0 = blockIdx.x * TM, tw = t0 - H;
  const int Tv = nsf_tv(rag_, b, Tl);
  const long long rowb = (long long)b * Tl;
  const bf16x8 z8 = {};
  auto wload = [&](const __bf16* w, bf16x8 (&wf)[NP]) {   // nsf_pair16_kernel's fragments
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int tap = 2 * p + tg, tc = min(tap, TAPS - 1);
      const unsigned mk = tap < TAPS ? 0xffffffffu : 0u;
      const uint4 r = *reinterpret_cast<const uint4*>(w + (long long)r16 * (TAPS * KP) + tc * KP + 8 * kg);
      wf[p] = __builtin_bit_cast(bf16x8, make_uint4(r.x & mk, r.y & mk, r.z & mk, r.w & mk));
    }
  };
  // lrelu(v) rounded to bf16, zero outside the utterance (the conv's zero padding): one 8-B LDS write
  auto put = [&](int m, const float* v) {
    const int i = 16 * (wave + NW * m) + r16, t = tw + i;
    const bool in = t >= 0 && t < Tv;
    bf16x4 u;
#pragma unroll
    for (int e = 0; e < 4; ++e) u[e] = (__bf16)(in ? (v[e] >= 0.f ? v[e] : NSF_LRELU * v[e]) : 0.f);
    *reinterpret_cast<bf16x4*>(bw + i * LDA + 4 * g) = u;
  };
  // registers: a conv's weight fragments are loaded once the previous conv's MFMAs are issued (one set
  // live at a time), the ResBlock sum's rows only after the last conv's (r06: loaded up front, k = 11
  // took 240 VGPRs, two blocks per CU)
  bf16x8 wf[NP];
  wload(A.w1[0], wf);
  float xr[IPW][4];                            // residual x_q of rows 16 (wave + NW m) + r16, channels 4g ..
#pragma unroll
  for (int m = 0; m < IPW; ++m) {             // unconditional loads at clamped rows
    const int t = min(max(tw + 16 * (wave + NW * m) + r16, 0), Tl - 1);
    const float4 v = *reinterpret_cast<const float4*>(x + (rowb + t) * C + 4 * g);
    xr[m][0] = v.x; xr[m][1] = v.y; xr[m][2] = v.z; xr[m][3] = v.w;
  }
#pragma unroll
  for (int m = 0; m < IPW; ++m) put(m, xr[m]);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int d = q == 0 ? 1 : q == 1 ? 3 : 5, p1 = P2 * d;
    const int V = q == 0 ? 0 : q == 1 ? 2 * P2 : 6 * P2;           // x_q exact on [V, W - V)
    const int kf1 = (V + p1) / 16, kl1 = (W - V - p1 - 1) / 16;   // xt tiles c2 reads
    const int kf2 = (V + p1 + P2) / 16, kl2 = (W - V - p1 - P2 - 1) / 16;
    const float4 bn1 = *reinterpret_cast<const float4*>(A.b1[q] + 4 * g);
    // ---- c1 (dilation d) on the xt tiles, then xt = bf16(c1 + b1) -> lrelu -> bf16 over x_q's rows
    f32x4 acc[IPW];
#pragma unroll
    for (int m = 0; m < IPW; ++m) {
      const int k = wave + NW * m;
      acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k >= kf1 && k <= kl1) {   // (wave-uniform)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const int tap = 2 * p + tg;
          bf16x8 af = *reinterpret_cast<const bf16x8*>(bw + (16 * k + r16 + min(tap, TAPS - 1) * d - p1) * LDA + 8 * kg);
          if (TAPS % 2 == 1 && p == NP - 1) af = tap < TAPS ? af : z8;
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[p], af, acc[m], 0, 0, 0);
        }
      }
    }
    wload(A.w2[q], wf);
    const float4 bn2 = *reinterpret_cast<const float4*>(A.b2[q] + 4 * g);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < IPW; ++m) {
      const int k = wave + NW * m;
      if (k >= kf1 && k <= kl1) {
        const float v[4] = {(float)(__bf16)(acc[m][0] + bn1.x), (float)(__bf16)(acc[m][1] + bn1.y),
                            (float)(__bf16)(acc[m][2] + bn1.z), (float)(__bf16)(acc[m][3] + bn1.w)};
        put(m, v);
      }
    }
    __syncthreads();
    // ---- c2 (dilation 1) + b2 + x_q (+ xs after the last pair)
#pragma unroll
    for (int m = 0; m < IPW; ++m) {
      const int k = wave + NW * m;
      acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k >= kf2 && k <= kl2) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const int tap = 2 * p + tg;
          bf16x8 af = *reinterpret_cast<const bf16x8*>(bw + (16 * k + r16 + min(tap, TAPS - 1) - P2) * LDA + 8 * kg);
          if (TAPS % 2 == 1 && p == NP - 1) af = tap < TAPS ? af : z8;
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[p], af, acc[m], 0, 0, 0);
        }
      }
    }
    if (q < 2) {
      wload(A.w1[q + 1], wf);
      __syncthreads();
#pragma unroll
      for (int m = 0; m < IPW; ++m) {
        const int k = wave + NW * m;
        if (k >= kf2 && k <= kl2) {
          xr[m][0] = acc[m][0] + bn2.x + xr[m][0];
          xr[m][1] = acc[m][1] + bn2.y + xr[m][1];
          xr[m][2] = acc[m][2] + bn2.z + xr[m][2];
          xr[m][3] = acc[m][3] + bn2.w + xr[m][3];
          put(m, xr[m]);
        }
      }
      __syncthreads();
    } else {
      // output rows [H, W - H) = times [t0, t0 + TM), through a buffer resource spanning the
      // utterance: rows past Tl (and the halo rows, given an offset past the range) are dropped
      const __amdgpu_buffer_rsrc_t ors = nsf_utt_rsrc<false>(out, b * Tl, Tl, C);
      float xs[IPW][4];                        // the ResBlock sum's rows so far (accum)
#pragma unroll
      for (int m = 0; m < IPW; ++m) {
        const int t = min(max(tw + 16 * (wave + NW * m) + r16, 0), Tl - 1);
        const float4 v = *reinterpret_cast<const float4*>(out + (rowb + t) * C + 4 * g);
        xs[m][0] = v.x; xs[m][1] = v.y; xs[m][2] = v.z; xs[m][3] = v.w;
      }
#pragma unroll
      for (int m = 0; m < IPW; ++m) {
        const int k = wave + NW * m;
        if (k >= kf2 && k <= kl2) {
          const int i = 16 * k + r16, t = tw + i;
          const bool ok = i >= H && i < W - H;
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float rv = accum ? xr[m][e] + xs[m][e] : xr[m][e];
            o[e] = acc[m][e] + (e == 0 ? bn2.x : e == 1 ? bn2.y : e == 2 ? bn2.z : bn2.w) + rv;
          }
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4, make_float4(o[0], o[1], o[2], o[3])), ors,
              ok ? (unsigned)(t * C + 4 * g) * 4u : 0xfffffff0u, 0, 0);
        }
      }
    }
  }
}

// Whole ResBlock1 at C = 32 / 64 (r06): nsf_rb16_kernel's structure on 32x32x16 MFMAs (nsf_pair_kernel's
// fragments, transposed: A = its weight fragments, B = its window reads).  Item = (32-row tile k, 32-channel
// column tile ct); a wave keeps one ct and tiles k = kw + (NW / NCT) m, so lane (t = lane & 31, h = lane >> 5)
// holds channels 32 ct + 8 g + 4 h + e (g, e < 4) of one row: 16 residual registers per item, and a row's
// activation goes to LDS as four 8-B writes.  Weights stream from L2 through an NSF_PAIR_PF-deep register
// ring, each fragment serving the wave's IPW items.  Bit-identical to the pair launches (same products
// and k order per MFMA, same epilogue roundings).
template <int C, int TAPS, int NTW, int NW>
__global__ __launch_bounds__(NW * 64) void nsf_rb_kernel(const float* __restrict__ x, const NsfRb16Args A, int Tl,
                                                         float* __restrict__ out, int accum, NsfRag rag_) {
  constexpr int NCT = C / 32, LDA = C + 8, KS = C / 16, P2 = (TAPS - 1) / 2, S = TAPS * KS;
  constexpr int H = 12 * P2, W = 32 * NTW, TM = W - 2 * H, PADR = 32, KST = NW / NCT, IPW = NTW / KST;
  static_assert(NW % NCT == 0 && NTW % KST == 0 && TM > 0, "item tiling");
  constexpr int PF = KS >= NSF_PAIR_PF ? NSF_PAIR_PF : KS;
  static_assert(KS % PF == 0, "ring depth divides the k-steps per tap");
  extern __shared__ __attribute__((aligned(16))) __bf16 nsf_win[];
  __bf16* bw = nsf_win + PADR * LDA;           // window row i at bw + i LDA, i in [-32, W + 32)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int ct = wave % NCT, kw = wave / NCT;
  const int b = blockIdx.y, t0 = blockIdx.x * TM, tw = t0 - H;
  const int Tv = nsf_tv(rag_, b, Tl);
  const long long rowb = (long long)b * Tl;
  const int n = ct * 32 + r32;                 // the lane's weight row (output channel)
  auto put = [&](int m, const float* v) {      // lrelu -> bf16, zero outside the utterance
    const int i = 32 * (kw + KST * m) + r32, t = tw + i;
    const bool in = t >= 0 && t < Tv;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = v[4 * gq + e];
        u[e] = (__bf16)(in ? (a >= 0.f ? a : NSF_LRELU * a) : 0.f);
      }
      *reinterpret_cast<bf16x4*>(bw + i * LDA + 32 * ct + 8 * gq + 4 * h) = u;
    }
  };
  // one conv over the items of tiles [kf, kl]: acc[m] = sum over k-steps of W . window rows shifted
  auto conv = [&](const __bf16* w, int dil, int pad, int kf, int kl, f32x16 (&acc)[IPW]) {
    const __bf16* wr = w + (long long)n * (TAPS * C) + 8 * h;
#pragma unroll
    for (int m = 0; m < IPW; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][r] = 0.f;
    bf16x8 bq[PF];
    auto bload = [&](int st) {
      const int tn = st / KS, kn = st - tn * KS;
      return *reinterpret_cast<const bf16x8*>(wr + tn * C + 16 * kn);
    };
#pragma unroll
    for (int q = 0; q < PF - 1; ++q) bq[q] = bload(q);
#pragma unroll
    for (int s0 = 0; s0 < S; s0 += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int st = s0 + q;
        bq[(q + PF - 1) % PF] = bload(min(st + PF - 1, S - 1));
        const int tap = st / KS, kc = st - tap * KS;
#pragma unroll
        for (int m = 0; m < IPW; ++m) {
          const int k = kw + KST * m;
          if (k >= kf && k <= kl) {   // (wave-uniform)
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(bw + (32 * k + r32 + tap * dil - pad) * LDA + 16 * kc + 8 * h);
            acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bq[q], af, acc[m], 0, 0, 0);
          }
        }
      }
    }
  };
  float xr[IPW][16];                           // residual x_q
#pragma unroll
  for (int m = 0; m < IPW; ++m) {
    const int t = min(max(tw + 32 * (kw + KST * m) + r32, 0), Tl - 1);
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const float4 v = *reinterpret_cast<const float4*>(x + (rowb + t) * C + 32 * ct + 8 * gq + 4 * h);
      xr[m][4 * gq] = v.x; xr[m][4 * gq + 1] = v.y; xr[m][4 * gq + 2] = v.z; xr[m][4 * gq + 3] = v.w;
    }
  }
#pragma unroll
  for (int m = 0; m < IPW; ++m) put(m, xr[m]);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int d = q == 0 ? 1 : q == 1 ? 3 : 5, p1 = P2 * d;
    const int V = q == 0 ? 0 : q == 1 ? 2 * P2 : 6 * P2;
    const int kf1 = (V + p1) / 32, kl1 = (W - V - p1 - 1) / 32;
    const int kf2 = (V + p1 + P2) / 32, kl2 = (W - V - p1 - P2 - 1) / 32;
    f32x16 acc[IPW];
    conv(A.w1[q], d, p1, kf1, kl1, acc);
    __syncthreads();
    {
      float bn[16];
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const float4 v = *reinterpret_cast<const float4*>(A.b1[q] + 32 * ct + 8 * gq + 4 * h);
        bn[4 * gq] = v.x; bn[4 * gq + 1] = v.y; bn[4 * gq + 2] = v.z; bn[4 * gq + 3] = v.w;
      }
#pragma unroll
      for (int m = 0; m < IPW; ++m) {
        const int k = kw + KST * m;
        if (k >= kf1 && k <= kl1) {
          float v[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = (float)(__bf16)(acc[m][r] + bn[r]);
          put(m, v);
        }
      }
    }
    __syncthreads();
    conv(A.w2[q], 1, P2, kf2, kl2, acc);
    float bn[16];
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const float4 v = *reinterpret_cast<const float4*>(A.b2[q] + 32 * ct + 8 * gq + 4 * h);
      bn[4 * gq] = v.x; bn[4 * gq + 1] = v.y; bn[4 * gq + 2] = v.z; bn[4 * gq + 3] = v.w;
    }
    if (q < 2) {
      __syncthreads();
#pragma unroll
      for (int m = 0; m < IPW; ++m) {
        const int k = kw + KST * m;
        if (k >= kf2 && k <= kl2) {
#pragma unroll
          for (int r = 0; r < 16; ++r) xr[m][r] = acc[m][r] + bn[r] + xr[m][r];
          put(m, xr[m]);
        }
      }
      __syncthreads();
    } else {
      const __amdgpu_buffer_rsrc_t ors = nsf_utt_rsrc<false>(out, b * Tl, Tl, C);
#pragma unroll
      for (int m = 0; m < IPW; ++m) {
        const int k = kw + KST * m;
        if (k >= kf2 && k <= kl2) {
          const int i = 32 * k + r32, t = tw + i, tc = min(max(t, 0), Tl - 1);
          const bool ok = i >= H && i < W - H;
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const int col = 32 * ct + 8 * gq + 4 * h;
            const float4 a = *reinterpret_cast<const float4*>(out + (rowb + tc) * C + col);   // the sum so far
            const float av[4] = {a.x, a.y, a.z, a.w};
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float rv = accum ? xr[m][4 * gq + e] + av[e] : xr[m][4 * gq + e];
              o[e] = acc[m][4 * gq + e] + bn[4 * gq + e] + rv;
            }
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_float4(o[0], o[1], o[2], o[3])), ors,
                                                   ok ? (unsigned)(t * C + col) * 4u : 0xfffffff0u, 0, 0);
          }
        }
      }
    }
  }
}

template <int C, int TAPS, int NTW, int NW>
int launch_rb_ct(const NsfRb16Args& a, const float* x, int B, int Tl, float* out, int accum, hipStream_t st,
                 NsfRag rag_) {
  constexpr int LDS = (32 * NTW + 64) * (C + 8) * 2;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&nsf_rb_kernel<C, TAPS, NTW, NW>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  if (attr != hipSuccess) { set_error("nsf rb: cannot raise the dynamic LDS limit"); return PD_ERR_HIP; }
  hipLaunchKernelGGL((nsf_rb_kernel<C, TAPS, NTW, NW>), dim3(cdiv(Tl, 32 * NTW - 12 * (TAPS - 1)), B), dim3(64 * NW),
                     LDS, st, x, a, Tl, out, accum, rag_);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// NSF_OPT_RB32 / RB64: the 32- / 64-channel ResBlock1s as one launch each, for the kernel sizes whose bit
// (1: taps 3, 2: taps 7, 4: taps 11) is set
int launch_rb(const NsfConv* c1, const NsfConv* c2, const float* x, int B, int Tl, float* out, int accum,
              hipStream_t st, NsfRag rag_) {
  NsfRb16Args a{};
  for (int q = 0; q < 3; ++q) {
    a.w1[q] = lookup_bf16(c1[q].w); a.w2[q] = lookup_bf16(c2[q].w);
    a.b1[q] = c1[q].b; a.b2[q] = c2[q].b;
  }
  ProfScope ps(c1[0].cout == 32 ? "nsf_rb32" : "nsf_rb64", st);
  const int k = c1[0].taps;
  if (c1[0].cout == 32) {
    if (k == 3) return launch_rb_ct<32, 3, 16, 8>(a, x, B, Tl, out, accum, st, rag_);
    if (k == 7) return launch_rb_ct<32, 7, 16, 8>(a, x, B, Tl, out, accum, st, rag_);
    return launch_rb_ct<32, 11, 16, 8>(a, x, B, Tl, out, accum, st, rag_);
  }
  if (k == 3) return launch_rb_ct<64, 3, 8, 8>(a, x, B, Tl, out, accum, st, rag_);
  if (k == 7) return launch_rb_ct<64, 7, 16, 8>(a, x, B, Tl, out, accum, st, rag_);
  return launch_rb_ct<64, 11, 16, 8>(a, x, B, Tl, out, accum, st, rag_);
}

// NSF_OPT_RB16: the 16-channel ResBlock1s of the shipped shapes as one launch each (nsf_rb16_kernel)
int launch_rb16(const NsfConv* c1, const NsfConv* c2, const float* x, int B, int Tl, float* out, int accum,
                hipStream_t st, NsfRag rag_, int geo) {
  NsfRb16Args a{};
  for (int q = 0; q < 3; ++q) {
    a.w1[q] = lookup_bf16(c1[q].w); a.w2[q] = lookup_bf16(c2[q].w);
    a.b1[q] = c1[q].b; a.b2[q] = c2[q].b;
  }
  ProfScope ps("nsf_rb16", st);
  // geometry (NSF_OPT_RB16): 1 = 32-tile windows of 4 waves (3 blocks per CU), 2 = 64-tile windows of 8
  // waves (half the halo share, one block per CU)
#define PD_RB16(K, NTW, NW)                                                                                 \
  hipLaunchKernelGGL((nsf_rb16_kernel<K, NTW, NW>), dim3(cdiv(Tl, 16 * NTW - 12 * (K - 1)), B), dim3(64 * NW), 0, \
                     st, x, a, Tl, out, accum, rag_)
  if (geo == 2) {
    if (c1[0].taps == 3) PD_RB16(3, 64, 8);
    else if (c1[0].taps == 7) PD_RB16(7, 64, 8);
    else PD_RB16(11, 64, 8);
  } else {
    if (c1[0].taps == 3) PD_RB16(3, 32, 4);
    else if (c1[0].taps == 7) PD_RB16(7, 32, 4);
    else PD_RB16(11, 32, 4);
  }
#undef PD_RB16
  PD_LAUNCH_CHECK();
  return PD_OK;
}

int launch_wconv16(const NsfConv& c, const __bf16* wb, const void* in, bool in_bf, float alpha, float scale, int B,
                   int Tl, void* out, bool out_bf, const float* res, hipStream_t st, int accum, NsfRag rag_) {
  if (c.taps > 12) { set_error("nsf wconv16: at most 12 taps"); return PD_ERR_UNSUPPORTED; }
  const size_t lds = (size_t)(256 + (c.taps - 1) * c.dil + 1) * 24 * sizeof(__bf16);   // + stage_window's spare row
  dim3 grid(cdiv(Tl, 256), B);
  ProfScope ps("nsf_res_small", st);
#define PD_WCONV16T(IB, OB, K, D)                                                                                 \
  hipLaunchKernelGGL((nsf_wconv16_kernel<IB, OB, K, D>), grid, dim3(256), lds, st, in, wb, c.kpad, c.b, c.taps,   \
                     c.dil, alpha, scale, Tl, res, out, accum, rag_)
  // compile-time (taps, dilation) for the shipped ResBlock shapes, the runtime kernel otherwise
#define PD_WCONV16(IB, OB)                                                                                        \
  do {                                                                                                            \
    const int K_ = c.kpad == 32 ? c.taps : 0, D_ = c.dil;                                                         \
    if (K_ == 3 && D_ == 1) PD_WCONV16T(IB, OB, 3, 1);                                                            \
    else if (K_ == 3 && D_ == 3) PD_WCONV16T(IB, OB, 3, 3);                                                       \
    else if (K_ == 3 && D_ == 5) PD_WCONV16T(IB, OB, 3, 5);                                                       \
    else if (K_ == 7 && D_ == 1) PD_WCONV16T(IB, OB, 7, 1);                                                       \
    else if (K_ == 7 && D_ == 3) PD_WCONV16T(IB, OB, 7, 3);                                                       \
    else if (K_ == 7 && D_ == 5) PD_WCONV16T(IB, OB, 7, 5);                                                       \
    else if (K_ == 11 && D_ == 1) PD_WCONV16T(IB, OB, 11, 1);                                                     \
    else if (K_ == 11 && D_ == 3) PD_WCONV16T(IB, OB, 11, 3);                                                     \
    else if (K_ == 11 && D_ == 5) PD_WCONV16T(IB, OB, 11, 5);                                                     \
    else PD_WCONV16T(IB, OB, 0, 0);                                                                               \
  } while (0)
  if (in_bf && out_bf) PD_WCONV16(true, true);
  else if (in_bf) PD_WCONV16(true, false);
  else if (out_bf) PD_WCONV16(false, true);
  else PD_WCONV16(false, false);
#undef PD_WCONV16
#undef PD_WCONV16T
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// conv_post (models.py:280-282): wav = tanh(conv7(leaky_relu(x, 0.01) * scale)) with ONE output
// channel -- a GEMM with N = 1 would leave 31/32 of every MFMA tile empty.  fp32 VALU: each
// block stages 256 + 6 rows of the C-channel input (activation applied once) and the C x 7
// weights in LDS; one thread per output sample.
template <int C>
__global__ __launch_bounds__(256) void nsf_post_kernel(const float* __restrict__ in, const float* __restrict__ wp,
                                                       int kpad, const float* __restrict__ bias, float alpha,
                                                       float scale, int Tl, float* __restrict__ out, NsfRag rag_) {
  constexpr int TR = 256, K = 7, P = C + 1;
  __shared__ float s_x[(TR + K - 1) * P];
  __shared__ float s_w[K * C];
  const int tid = threadIdx.x, b = blockIdx.y, t0 = blockIdx.x * TR, Tv = nsf_tv(rag_, b, Tl);
  for (int i = tid; i < K * C; i += 256) s_w[i] = wp[(i / C) * kpad + i % C];
  const float* ib = in + (long long)b * Tl * C;
  for (int i = tid; i < (TR + K - 1) * C; i += 256) {
    const int row = i / C, c = i - row * C;
    const int t = t0 - (K - 1) / 2 + row;
    float v = 0.f;
    if (t >= 0 && t < Tv) {
      v = ib[(long long)t * C + c];
      v = (v >= 0.f ? v : alpha * v) * scale;
    }
    s_x[row * P + c] = v;
  }
  __syncthreads();
  const int t = t0 + tid;
  if (t >= Tl) return;
  float acc = bias[0];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int c = 0; c < C; ++c) acc = fmaf(s_w[k * C + c], s_x[(tid + k) * P + c], acc);
  out[(long long)b * Tl + t] = tanhf(acc);
}

// ConvTranspose1d(k = ntap*u, stride u, padding p) + noise-conv add (models.py:270-274) on the
// bf16 MFMA path, windowed like nsf_wconv_kernel.  Output row o_phi + q*u (phase phi, input row
// q) = b + sum_mt W_phi,mt . lrelu(x[q + q0_phi - mt]) + res; q0_phi = ceil((p - phi)/u) if
// p > phi else 0, o_phi = q0_phi*u + phi - p (the host's NsfUps::qmin).  A block stages TQ + halo
// input rows ONCE and runs every phase from that window (the phase-GEMM path re-reads the
// input 2u times); weights of all phases are contiguous [phi][cout][ntap*kpad] (bf16 mirror),
// streamed in a PF-deep register ring across the phase boundaries.  NPAD: cout < 32 channels
// on a 32-wide tile (weight rows clamped, extra columns dropped).
// The noise conv (models.py:271-272: Conv1d(1, cout, k = 2s, stride s, padding s / 2) of the
// harmonic source) fused into the upsample's epilogue (r05, NC): the block stages its rows' source
// samples in LDS after the input window and adds b + sum_j w[j] har[R s - pad + j] -- the order of
// nsf_noise_conv_kernel -- where the unfused path reads that kernel's fp32 output back.
struct NsfNoise {
  const float* har = nullptr;   // [B][L] harmonic source
  long long L = 0;
  const float* w = nullptr;     // tap-major [k][cout]
  const float* b = nullptr;
  int k = 0, stride = 1, pad = 0;
  NsfRag rag;                   // the source's ragged ends (rate = samples per frame)
};
constexpr int NSF_NC_KMAX = 8;   // fused for k <= 8 (the last three stages: LDS of the source window)
template <int CIN, int FM, int FN, int WM, int WN, bool NPAD, bool NC = false>
__global__ __launch_bounds__(256, 2) void nsf_ups_kernel(const float* __restrict__ in, const __bf16* __restrict__ w,
                                                      long long wstride, int kpad, int ntap, int u, int p, int dlo,
                                                      int cout, const float* __restrict__ bias, float alpha,
                                                      float scale, int Tin, const float* __restrict__ res,
                                                      float* __restrict__ out, NsfRag rag_, NsfNoise nz) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TQ = 32 * FM * WM, TN = 32 * FN * WN, LDA = CIN + 8, KS = CIN / 16;
  constexpr int PF = KS >= NSF_PF ? NSF_PF : KS;
  extern __shared__ __attribute__((aligned(16))) __bf16 nsf_uwin[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int b = blockIdx.z, i0 = blockIdx.x * TQ, n0 = blockIdx.y * TN;
  const int W = TQ + ntap;                 // rows i0 + dlo ... (dlo = 1 - ntap, top offset q0 <= 1)
  // NC: source samples [s0, s0 + nwin) of output rows [i0 u, (i0 + TQ) u), after the input window
  float* s_har = reinterpret_cast<float*>(nsf_uwin + ((W + 1) * LDA + 7) / 8 * 8);
  const long long s0 = (long long)i0 * u * nz.stride - nz.pad;
  const int nwin = NC ? TQ * u * nz.stride + nz.k : 0;
  if constexpr (NC) {
    const float* hb = nz.har + (long long)b * nz.L;
    const long long Lv = nz.rag.lens ? min((long long)nz.rag.lens[b] * nz.rag.rate, nz.L) : nz.L;
    for (int base = tid; base < nwin; base += 256 * 8) {   // 8 loads per thread in flight together
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const long long si = s0 + base + 256 * e;
        v[e] = hb[si < 0 ? 0 : si >= nz.L ? nz.L - 1 : si];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = base + 256 * e;
        const long long si = s0 + i;
        s_har[min(i, nwin)] = (si >= 0 && si < Lv && i < nwin) ? v[e] : 0.f;   // (slot nwin: spare)
      }
    }
  }
  stage_window<CIN, false>(in, b, Tin, nsf_tv(rag_, b, Tin), i0 + dlo, W, alpha, scale, nsf_uwin, LDA, tid);
  __syncthreads();
  const int r32 = lane & 31, h = lane >> 5;
  const int ldw = ntap * kpad;
  const __bf16* wr[FN];
  bool ncol[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + (wn * FN + j) * 32 + r32;
    ncol[j] = !NPAD || n < cout;
    wr[j] = w + (long long)(NPAD ? min(n, cout - 1) : n) * ldw + 8 * h;
  }
  const int Sph = ntap * KS, S = u * Sph;
  bf16x8 bq[PF][FN];
  auto bload = [&](int st, bf16x8* dst) {
    const int ph = st / Sph, rem = st - ph * Sph, mt = rem / KS, kn = rem - mt * KS;
#pragma unroll
    for (int j = 0; j < FN; ++j)
      dst[j] = *reinterpret_cast<const bf16x8*>(wr[j] + ph * wstride + mt * kpad + 16 * kn);
  };
#pragma unroll
  for (int q = 0; q < PF - 1; ++q) bload(q, bq[q]);
  float bv[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bv[j] = ncol[j] ? bias[n0 + (wn * FN + j) * 32 + r32] : 0.f;
  const __bf16* arow = nsf_uwin + (wm * FM * 32 + r32) * LDA + 8 * h;
#pragma unroll 1
  for (int phi = 0; phi < u; ++phi) {
    const int q0 = p - phi > 0 ? (p - phi + u - 1) / u : 0;
    const int o = q0 * u + phi - p;
    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll 1
    for (int s0 = 0; s0 < Sph; s0 += PF) {
#pragma unroll
      for (int qq = 0; qq < PF; ++qq) {
        const int sl = s0 + qq, sg = phi * Sph + sl;
        bload(min(sg + PF - 1, S - 1), bq[(qq + PF - 1) % PF]);
        const int mt = sl / KS, kc = sl - mt * KS;
        const int roff = q0 - mt - dlo;
        bf16x8 af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(arow + (i * 32 + roff) * LDA + 16 * kc);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bq[qq][j], acc[i][j], 0, 0, 0);
      }
    }
    // epilogue of this phase: rows o + q*u (q < Tin), + bias + noise-conv output; the 16
    // residual loads of one fragment are issued together (clamped rows, predicated stores)
    const int Lc = Tin * u;
    // stores through a buffer resource spanning this utterance's rows: rows q >= Tin fall past its
    // end and columns past cout are sent there, so no store sits under a branch (r05: the waitcnt
    // pass waited before every predicated store)
    const __amdgpu_buffer_rsrc_t ors = nsf_utt_rsrc<false>(out, b * Lc, Lc, cout);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + (wn * FN + j) * 32 + r32;
        const int nc = NPAD ? min(n, cout - 1) : n;
        float rv[16];
        if constexpr (NC) {   // the noise conv of output row o + q u, nsf_noise_conv_kernel's order
          float wv[NSF_NC_KMAX];
#pragma unroll
          for (int jj = 0; jj < NSF_NC_KMAX; ++jj) wv[jj] = nz.w[(long long)min(jj, nz.k - 1) * cout + nc];
          const float bo = nz.b[nc];
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            const int q = min(i0 + wm * FM * 32 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, Tin - 1);
            const float* sh = s_har + (o + (q - i0) * u) * nz.stride;
            float acc = bo;
#pragma unroll
            for (int jj = 0; jj < NSF_NC_KMAX; ++jj)
              if (jj < nz.k) acc = fmaf(wv[jj], sh[jj], acc);   // (uniform)
            rv[reg] = acc;
          }
        } else {
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) {
            const int q = min(i0 + wm * FM * 32 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, Tin - 1);
            rv[reg] = res[((long long)b * Lc + o + (long long)q * u) * cout + nc];
          }
        }
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int q = i0 + wm * FM * 32 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
          const unsigned off = ncol[j] ? (unsigned)((o + q * u) * cout + n) * 4u : 0xfffffff0u;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][reg] + bv[j] + rv[reg]), ors, off, 0, 0);
        }
      }
    }
  }
}

template <int CIN, int FM, int FN, int WM, int WN, bool NPAD>
int launch_ups_c(const NsfUps& U, const __bf16* wb, const float* in, float scale, int B, int Tin, const float* res,
                 float* out, hipStream_t st, NsfRag rag_, const NsfNoise& nz) {
  constexpr int TQ = 32 * FM * WM, TN = 32 * FN * WN;
  const int p = (U.k - U.u) / 2;
  // input window + stage_window's spare row (+ NC: the source window and its spare slot)
  const size_t win = (size_t)((U.ntap + TQ + 1) * (CIN + 8) + 7) / 8 * 8 * sizeof(__bf16);
  const size_t lds = win + (nz.har ? (size_t)(TQ * U.u * nz.stride + nz.k + 1) * sizeof(float) : 0);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&nsf_ups_kernel<CIN, FM, FN, WM, WN, NPAD>),
      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  static const hipError_t attr_nc = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&nsf_ups_kernel<CIN, FM, FN, WM, WN, NPAD, true>),
      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess || attr_nc != hipSuccess) { set_error("nsf ups: cannot raise the dynamic LDS limit"); return PD_ERR_HIP; }
  if (lds > 160 * 1024) { set_error("nsf ups: LDS window too large"); return PD_ERR_UNSUPPORTED; }
  dim3 grid(cdiv(Tin, TQ), NPAD ? 1 : U.cout / TN, B);
  ProfScope ps("nsf_ups", st);
  if (nz.har)
    hipLaunchKernelGGL((nsf_ups_kernel<CIN, FM, FN, WM, WN, NPAD, true>), grid, dim3(256), lds, st, in, wb,
                       (long long)(U.w[1] - U.w[0]), U.kpad, U.ntap, U.u, p, 1 - U.ntap, U.cout, U.b, NSF_LRELU,
                       scale, Tin, res, out, rag_, nz);
  else
    hipLaunchKernelGGL((nsf_ups_kernel<CIN, FM, FN, WM, WN, NPAD>), grid, dim3(256), lds, st, in, wb,
                       (long long)(U.w[1] - U.w[0]), U.kpad, U.ntap, U.u, p, 1 - U.ntap, U.cout, U.b, NSF_LRELU,
                       scale, Tin, res, out, rag_, nz);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// The windowed ConvTranspose for this upsample, if it has one: bf16 weights, phases packed
// back to back, k = 2u with the phase offsets the kernel derives, a channel pair it is built for.
bool ups_window_ok(const NsfUps& U, bool wconv) {
  if (!wconv || U.u < 2 || U.ntap != 2 || U.k != 2 * U.u || U.w.size() != (size_t)U.u || !lookup_bf16(U.w[0]))
    return false;
  const long long stride = U.w[1] - U.w[0];
  if (stride != (long long)U.cout * U.ntap * U.kpad) return false;
  for (int phi = 1; phi < U.u; ++phi)
    if (U.w[phi] - U.w[phi - 1] != stride) return false;
  const int p = (U.k - U.u) / 2;
  for (int phi = 0; phi < U.u; ++phi) {
    const int q0 = p - phi > 0 ? (p - phi + U.u - 1) / U.u : 0;
    if (q0 != U.qmin[phi] || q0 > 1) return false;
  }
  return (U.cin == 512 && U.cout == 256) || (U.cin == 256 && U.cout == 128) || (U.cin == 128 && U.cout == 64) ||
         (U.cin == 64 && U.cout == 32) || (U.cin == 32 && U.cout == 16);
}

int launch_ups_window(const NsfUps& U, const float* in, float scale, int B, int Tin, const float* res, float* out,
                      hipStream_t st, NsfRag rag_, const NsfNoise& nz) {
  const __bf16* wb = lookup_bf16(U.w[0]);
  // (r02: one row-wave per column tile, <512,2,1,1,4> / <256,4,1,1,4>, measured slower: 188 vs 178 us avg)
  if (U.cin == 512) return launch_ups_c<512, 1, 2, 2, 2, false>(U, wb, in, scale, B, Tin, res, out, st, rag_, nz);
  if (U.cin == 256) return launch_ups_c<256, 2, 1, 2, 2, false>(U, wb, in, scale, B, Tin, res, out, st, rag_, nz);
  if (U.cin == 128) return launch_ups_c<128, 2, 1, 2, 2, false>(U, wb, in, scale, B, Tin, res, out, st, rag_, nz);
  if (U.cin == 64) return launch_ups_c<64, 1, 1, 4, 1, false>(U, wb, in, scale, B, Tin, res, out, st, rag_, nz);
  return launch_ups_c<32, 1, 1, 4, 1, true>(U, wb, in, scale, B, Tin, res, out, st, rag_, nz);
}

template <int C, int FM, int FN, int WM, int WN>
int launch_wconv_c(const NsfConv& c, const __bf16* wb, const void* in, bool in_bf, float alpha, float scale, int B,
                   int Tl, void* out, bool out_bf, const float* res, hipStream_t st, int accum, NsfRag rag_) {
  constexpr int TM = 32 * FM * WM, TN = 32 * FN * WN;
  const size_t lds = (size_t)(TM + (c.taps - 1) * c.dil + 1) * (C + 8) * sizeof(__bf16);   // + stage_window's spare row
  if (lds > 160 * 1024) { set_error("nsf conv: LDS window too large"); return PD_ERR_UNSUPPORTED; }
  dim3 grid(cdiv(Tl, TM), C / TN, B);
  const int ldw = c.taps * c.kpad;
#define PD_WCONV(IB, OB)                                                                                          \
  do {                                                                                                            \
    static const hipError_t attr = hipFuncSetAttribute(                                                           \
        reinterpret_cast<const void*>(&nsf_wconv_kernel<C, FM, FN, WM, WN, IB, OB>),                              \
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                                                  \
    if (attr != hipSuccess) { set_error("nsf conv: cannot raise the dynamic LDS limit"); return PD_ERR_HIP; }    \
    hipLaunchKernelGGL((nsf_wconv_kernel<C, FM, FN, WM, WN, IB, OB>), grid, dim3(64 * WM * WN), lds, st, in, wb, ldw, \
                       c.kpad, c.b, c.taps, c.dil, alpha, scale, Tl, res, out, accum, rag_);                        \
  } while (0)
  ProfScope ps("nsf_res", st);
  if (in_bf && out_bf) PD_WCONV(true, true);
  else if (in_bf) PD_WCONV(true, false);
  else if (out_bf) PD_WCONV(false, true);
  else PD_WCONV(false, false);
#undef PD_WCONV
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// The windowed conv for this ResBlock conv, if it has one (bf16 weights, C in {16..256}); on the
// bf16 path it takes precedence over NSF_OPT_SMALL_MAX, which then only routes the fp32 path.
bool wconv_ok(const NsfConv& c) {
  return c.wconv && c.cin == c.cout && c.taps <= 11 && lookup_bf16(c.w) != nullptr &&
         (c.cout == 16 || c.cout == 32 || c.cout == 64 || c.cout == 128 || c.cout == 256);
}

// accum = 1: out (fp32) += conv + res -- the ResBlock sum xs += resblock_j(x) (models.py:275-279)
// fused into the block's last conv instead of a separate pass.
int launch_wconv(const NsfConv& c, const void* in, bool in_bf, float alpha, float scale, int B, int Tl, void* out,
                 bool out_bf, const float* res, hipStream_t st, int accum, NsfRag rag_) {
  const __bf16* wb = lookup_bf16(c.w);
  // 32-bit element offsets, and one utterance's bytes inside the unsigned buffer-resource range
  if ((long long)B * Tl * c.cout >= (1ll << 31) || (long long)Tl * c.cout * 4 >= (1ll << 32)) {
    set_error("nsf wconv: B * T * C >= 2^31 elements or T * C * 4 >= 2^32 bytes (32-bit epilogue offsets)");
    return PD_ERR_UNSUPPORTED;
  }
  if (out_bf == (res != nullptr)) {   // the kernels' epilogue: fp32 outputs add a residual, bf16 ones none
    set_error("nsf wconv: an fp32 output needs a residual and a bf16 output takes none");
    return PD_ERR_ARG;
  }
  switch (c.cout) {
    // Tilings: a wave owns all TM rows of its 32-channel column tiles (WM = 1), so each weight
    // fragment crosses the L2 -> CU port once per block instead of once per row-wave (r02:
    // 2 x 2 wave grids at C = 128/256 read every fragment twice; C5 21.07 -> 19.19 ms/step,
    // ResBlock convs 187 -> 159 us avg).  C = 32: 128, 256 or 512 rows per block measured
    // equal or slower than 128 rows with four row-waves.
    case 256:
      if (c.w256 == 1)   // NSF_OPT_C256 (r06): 8 waves, all 256 output channels per block (95 -> 83 us)
        return launch_wconv_c<256, 4, 1, 1, 8>(c, wb, in, in_bf, alpha, scale, B, Tl, out, out_bf, res, st, accum, rag_);
      return launch_wconv_c<256, 4, 1, 1, 4>(c, wb, in, in_bf, alpha, scale, B, Tl, out, out_bf, res, st, accum, rag_);
    case 128: return launch_wconv_c<128, 4, 1, 1, 4>(c, wb, in, in_bf, alpha, scale, B, Tl, out, out_bf, res, st, accum, rag_);
    case 64: return launch_wconv_c<64, 4, 1, 2, 2>(c, wb, in, in_bf, alpha, scale, B, Tl, out, out_bf, res, st, accum, rag_);
    case 32: return launch_wconv_c<32, 1, 1, 4, 1>(c, wb, in, in_bf, alpha, scale, B, Tl, out, out_bf, res, st, accum, rag_);
    case 16: return launch_wconv16(c, wb, in, in_bf, alpha, scale, B, Tl, out, out_bf, res, st, accum, rag_);
    default: set_error("nsf wconv: unsupported channel count"); return PD_ERR_UNSUPPORTED;
  }
}

// ConvTranspose1d weight [Cin][Cout][K] -> phase phi: dst[co][m*cpad + ci] = W[ci][co][phi + m*u]
__global__ void nsf_pack_ups_kernel(float* __restrict__ dst, const float* __restrict__ src, int Cin, int Cout,
                                    int K, int u, int phi, int ntap, int cpad) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)Cout * ntap * Cin) return;
  int ci = (int)(i % Cin);
  long long r = i / Cin;
  int m = (int)(r % ntap);
  int co = (int)(r / ntap);
  dst[(long long)co * ntap * cpad + m * cpad + ci] = src[((long long)ci * Cout + co) * K + phi + m * u];
}

// xs = v (assign) or xs += v
__global__ __launch_bounds__(256) void nsf_accum_kernel(float4* __restrict__ xs, const float4* __restrict__ v,
                                                        long long n4, int assign) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 a = v[i];
  if (!assign) {
    float4 x = xs[i];
    a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
  }
  xs[i] = a;
}

struct NsfWs {
  size_t P = 0, Rd = 0, har = 0, X = 0, T1 = 0, R = 0, XS = 0, src = 0, total = 0;   // float offsets
};

NsfWs nsf_layout(const nsf_model* m, int B, int T) {
  NsfWs W;
  auto al = [](size_t n) { return (n + 63) / 64 * 64; };
  long long per_frame = m->C0;
  long long len = 1;
  for (const NsfUps& u : m->ups) {
    len *= u.u;
    per_frame = std::max(per_frame, len * u.cout);
  }
  size_t act = al((size_t)B * T * per_frame);
  size_t off = 0;
  W.P = off; off += al((size_t)B * T * m->dim * 2);
  W.Rd = off; off += al((size_t)B * T * m->dim);
  W.har = off; off += al((size_t)B * T * m->upp);
  W.X = off; off += act;
  W.T1 = off; off += act;
  W.R = off; off += act;
  W.XS = off; off += act;
  W.src = off; off += act;
  W.total = off * sizeof(float);
  return W;
}

// conv over time-major `in` [B][Tl][cin] (taps with dilation, zero padding (taps-1)*dil/2),
// pre-activation leaky_relu(alpha) * in_scale on load; out = act(conv + b) (+ res).
int nsf_conv(const NsfConv& c, const float* in, float in_alpha, float in_scale, int B, int Tl, float* out,
             const float* res, int act, hipStream_t st, int use, NsfRag rag_) {
  if (use == U_NSF_RES && c.cin == c.cout && c.cout <= c.small_max && in_alpha >= 0.f) {
    switch (c.cout) {
      case 4: return launch_conv_small<4>(c, in, in_alpha, in_scale, B, Tl, out, res, st, rag_);
      case 8: return launch_conv_small<8>(c, in, in_alpha, in_scale, B, Tl, out, res, st, rag_);
      case 16: return launch_conv_small<16>(c, in, in_alpha, in_scale, B, Tl, out, res, st, rag_);
      case 32: return launch_conv_small<32>(c, in, in_alpha, in_scale, B, Tl, out, res, st, rag_);
      default: break;
    }
  }
  const int pad = (c.taps - 1) * c.dil / 2;
  GemmArgs a = make_gemm(B, Tl, c.cout, c.w, c.taps * c.kpad, c.b, out, (long long)Tl * c.cout, c.cout);
  for (int k = 0; k < c.taps; ++k) {
    Seg s = make_seg(in, (long long)Tl * c.cin, c.cin, c.cin, k * c.dil - pad);
    s.kpad = c.kpad;
    if (in_alpha >= 0.f) { s.act = ACT_LRELU; s.alpha = in_alpha; }
    s.scale = in_scale;
    add_seg(a, s);
  }
  a.act = act;
  a.lens = rag_.lens; a.lens_mul = rag_.rate;
  if (res) { a.res = res; a.res_bs = (long long)Tl * c.cout; a.res_ld = c.cout; }
  if (use == U_NSF_POST) return launch_gemm<1, 1, 4, 1, EPI_STORE, U_NSF_POST>(a, st, "nsf_post");
  if (use == U_NSF_CONV_PRE) return launch_gemm<1, 2, 4, 1, EPI_STORE, U_NSF_CONV_PRE>(a, st, "nsf_conv_pre");
  // (a 256 x 32 tile for the 32-channel stage measured slower: 11.9 vs 9.9 ms per step)
  return launch_gemm<1, 2, 4, 1, EPI_STORE, U_NSF_RES>(a, st, "nsf_res");
}

}  // namespace

extern "C" {

int nsf_num_params(const nsf_dims* d) {
  if (!d || d->num_upsamples < 1 || d->num_upsamples > 6 || d->num_kernels < 1 || d->num_kernels > 4 ||
      d->num_dilations < 1 || d->num_dilations > 4 || (d->resblock != 1 && d->resblock != 2))
    return -1;
  int per_block = (d->resblock == 1 ? 2 : 1) * d->num_dilations;
  return 2 + 2 * d->num_upsamples + 2 + 2 * d->num_upsamples + 2 * per_block * d->num_kernels * d->num_upsamples + 2;
}

int nsf_create(const nsf_dims* dims, const float* const* params, int dtype, void* stream, nsf_model** out) {
  PD_CHECK_ARG(dims && params && out, "null argument");
  const int np = nsf_num_params(dims);
  PD_CHECK_ARG(np > 0, "nsf_dims: bad counts");
  PD_CHECK_ARG(dtype == PD_DTYPE_F32 || dtype == PD_DTYPE_BF16, "dtype");
  for (int i = 0; i < np; ++i) PD_CHECK_ARG(params[i] != nullptr, "null parameter " + std::to_string(i));
  const nsf_dims& d = *dims;
  PD_CHECK_ARG(d.num_mels > 0 && d.num_mels % 4 == 0, "num_mels must be a multiple of 4");
  PD_CHECK_ARG(d.harmonic_num >= 0 && d.sampling_rate > 0, "harmonic_num / sampling_rate");
  PD_CHECK_ARG(d.upsample_initial_channel % (4 << d.num_upsamples) == 0,
               "upsample_initial_channel / 2^num_upsamples must be a multiple of 4");
  for (int j = 0; j < d.num_kernels; ++j)
    PD_CHECK_ARG(d.resblock_kernel_sizes[j] % 2 == 1 && d.resblock_kernel_sizes[j] <= MAX_SEGS,
                 "resblock kernel sizes must be odd and <= 11");
  for (int i = 0; i < d.num_upsamples; ++i) {
    int u = d.upsample_rates[i], k = d.upsample_kernel_sizes[i];
    PD_CHECK_ARG(u >= 1 && k >= u && k % u == 0 && (k - u) % 2 == 0 && k / u <= MAX_SEGS,
                 "upsample kernel must be a multiple of the rate with k - u even");
    const int co = d.upsample_initial_channel >> (i + 1);
    PD_CHECK_ARG(co >= 256 ? co % 256 == 0 : 256 % co == 0, "stage channels must divide 256 or be a multiple of it");
  }
  hipStream_t st = (hipStream_t)stream;
  nsf_model* m = new nsf_model();
  m->d = d;
  m->dim = d.harmonic_num + 1;
  m->C0 = d.upsample_initial_channel;
  m->upp = 1;
  for (int i = 0; i < d.num_upsamples; ++i) m->upp *= d.upsample_rates[i];
  m->convs_per_block = (d.resblock == 1 ? 2 : 1) * d.num_dilations;

  // --- pool layout (floats)
  size_t off = 0;
  auto take = [&](size_t n) { size_t o = off; off += (n + 63) / 64 * 64; return o; };
  const int dim = m->dim;
  size_t o_lin_w = take(dim), o_lin_b = take(1);
  std::vector<size_t> o_nc_w, o_nc_b, o_ups_b;
  std::vector<std::vector<size_t>> o_ups_w;
  m->ups.resize(d.num_upsamples);
  for (int i = 0; i < d.num_upsamples; ++i) {
    NsfUps& U = m->ups[i];
    U.u = d.upsample_rates[i];
    U.k = d.upsample_kernel_sizes[i];
    U.cin = m->C0 >> i;
    U.cout = m->C0 >> (i + 1);
    U.ntap = U.k / U.u;
    U.kpad = round_up(U.cin, GEMM_BK);
    if (i + 1 < d.num_upsamples) {
      int sf = 1;
      for (int r = i + 1; r < d.num_upsamples; ++r) sf *= d.upsample_rates[r];
      U.nc_k = 2 * sf; U.nc_stride = sf; U.nc_pad = sf / 2;
    } else {
      U.nc_k = 1; U.nc_stride = 1; U.nc_pad = 0;
    }
    o_nc_w.push_back(take((size_t)U.cout * U.nc_k));
    o_nc_b.push_back(take(U.cout));
    const int p = (U.k - U.u) / 2;
    std::vector<size_t> ph;
    U.qmin.resize(U.u);
    for (int phi = 0; phi < U.u; ++phi) {
      ph.push_back(take((size_t)U.cout * U.ntap * U.kpad));
      const int num = p - phi;              // first q with q*u + phi - p >= 0
      U.qmin[phi] = num > 0 ? (num + U.u - 1) / U.u : 0;
    }
    o_ups_w.push_back(ph);
    o_ups_b.push_back(take(U.cout));
  }
  auto conv_init = [&](NsfConv& c, int cin, int cout, int taps, int dil, size_t& ow, size_t& ob) {
    c.cin = cin; c.cout = cout; c.taps = taps; c.dil = dil; c.kpad = round_up(cin, GEMM_BK);
    ow = take((size_t)cout * taps * c.kpad);
    ob = take(cout);
  };
  size_t o_pre_w, o_pre_b, o_post_w, o_post_b;
  conv_init(m->pre, d.num_mels, m->C0, 7, 1, o_pre_w, o_pre_b);
  std::vector<size_t> o_res_w, o_res_b;
  for (int i = 0; i < d.num_upsamples; ++i) {
    const int c = m->C0 >> (i + 1);
    for (int j = 0; j < d.num_kernels; ++j) {
      const int k = d.resblock_kernel_sizes[j];
      for (int q = 0; q < m->convs_per_block; ++q) {
        // ResBlock1: convs1.{0..D-1} (dilated) then convs2.{0..D-1} (dilation 1); ResBlock2: convs.{0..D-1}
        int dil = (d.resblock == 1 && q >= d.num_dilations) ? 1 : d.resblock_dilation_sizes[j][q % d.num_dilations];
        NsfConv cv;
        size_t ow, ob;
        conv_init(cv, c, c, k, dil, ow, ob);
        m->res.push_back(cv);
        o_res_w.push_back(ow);
        o_res_b.push_back(ob);
      }
    }
  }
  conv_init(m->post, m->C0 >> d.num_upsamples, 1, 7, 1, o_post_w, o_post_b);

  auto run = [&]() -> int {
    PD_HIP(hipMalloc((void**)&m->pool, off * sizeof(float)));
    PD_HIP(hipMemsetAsync(m->pool, 0, off * sizeof(float), st));
    float* P = m->pool;
    auto cp = [&](size_t o, const float* src, size_t n) -> int {
      PD_HIP(hipMemcpyAsync(P + o, src, n * sizeof(float), hipMemcpyDeviceToDevice, st));
      return PD_OK;
    };
    int p = 0;
    PD_TRY(cp(o_lin_w, params[p++], dim));
    PD_TRY(cp(o_lin_b, params[p++], 1));
    m->lin_w = P + o_lin_w;
    m->lin_b = P + o_lin_b;
    for (int i = 0; i < d.num_upsamples; ++i) {
      NsfUps& U = m->ups[i];
      hipLaunchKernelGGL(nsf_pack_noise_kernel, dim3(cdiv((long long)U.cout * U.nc_k, 256)), dim3(256), 0, st,
                         P + o_nc_w[i], params[p++], U.cout, U.nc_k);
      PD_LAUNCH_CHECK();
      PD_TRY(cp(o_nc_b[i], params[p++], U.cout));
      U.nc_w = P + o_nc_w[i];
      U.nc_b = P + o_nc_b[i];
    }
    PD_TRY(pack_conv(P + o_pre_w, 7 * m->pre.kpad, 0, 0, m->pre.kpad, params[p++], m->C0, d.num_mels, 7, st));
    PD_TRY(cp(o_pre_b, params[p++], m->C0));
    m->pre.w = P + o_pre_w;
    m->pre.b = P + o_pre_b;
    for (int i = 0; i < d.num_upsamples; ++i) {
      NsfUps& U = m->ups[i];
      const float* w = params[p++];
      for (int phi = 0; phi < U.u; ++phi) {
        long long n = (long long)U.cout * U.ntap * U.cin;
        hipLaunchKernelGGL(nsf_pack_ups_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, P + o_ups_w[i][phi], w, U.cin,
                           U.cout, U.k, U.u, phi, U.ntap, U.kpad);
        PD_LAUNCH_CHECK();
        U.w.push_back(P + o_ups_w[i][phi]);
      }
      PD_TRY(cp(o_ups_b[i], params[p++], U.cout));
      U.b = P + o_ups_b[i];
    }
    for (size_t r = 0; r < m->res.size(); ++r) {
      NsfConv& c = m->res[r];
      PD_TRY(pack_conv(P + o_res_w[r], c.taps * c.kpad, 0, 0, c.kpad, params[p++], c.cout, c.cin, c.taps, st));
      PD_TRY(cp(o_res_b[r], params[p++], c.cout));
      c.w = P + o_res_w[r];
      c.b = P + o_res_b[r];
    }
    PD_TRY(pack_conv(P + o_post_w, 7 * m->post.kpad, 0, 0, m->post.kpad, params[p++], 1, m->post.cin, 7, st));
    PD_TRY(cp(o_post_b, params[p++], 1));
    m->post.w = P + o_post_w;
    m->post.b = P + o_post_b;
    if (p != np) { set_error("nsf_create: parameter count mismatch"); return PD_ERR_ARG; }
    m->pool_n = off;
    if (dtype == PD_DTYPE_BF16) {
      // every GEMM weight then streams as bf16 (v_mfma_f32_32x32x16_bf16, fp32 accumulate)
      PD_HIP(hipMalloc((void**)&m->pool_bf, off * sizeof(__bf16)));
      PD_TRY(convert_f32_bf16(m->pool, m->pool_bf, (long long)off, st));
      register_bf16_pool(m->pool, off, m->pool_bf);
    }
    return PD_OK;
  };
  int rc = run();
  if (rc != PD_OK) {
    if (m->pool) (void)hipFree(m->pool);
    if (m->pool_bf) (void)hipFree(m->pool_bf);
    delete m;
    return rc;
  }
  *out = m;
  return PD_OK;
}

void nsf_destroy(nsf_model* m) {
  if (!m) return;
  if (m->pool_bf) {
    unregister_bf16_pool(m->pool);
    (void)hipFree(m->pool_bf);
  }
  (void)hipFree(m->pool);
  delete m;
}

int nsf_hop(const nsf_model* m) { return m ? m->upp : 0; }

int nsf_set_option(nsf_model* m, int option, int value) {
  PD_CHECK_ARG(m, "null pointer");
  if (option == NSF_OPT_SMALL_MAX) {
    PD_CHECK_ARG(value >= 0, "NSF_OPT_SMALL_MAX >= 0");
    for (auto& c : m->res) c.small_max = value;
    return PD_OK;
  }
  if (option == NSF_OPT_WCONV) {
    PD_CHECK_ARG(value == 0 || value == 1, "NSF_OPT_WCONV is 0 or 1");
    for (auto& c : m->res) c.wconv = value != 0;
    m->ups_window = value != 0;
    return PD_OK;
  }
  if (option == NSF_OPT_PAIR) {
    PD_CHECK_ARG(value == 0 || value == 1, "NSF_OPT_PAIR is 0 or 1");
    m->pair = value != 0;
    return PD_OK;
  }
  if (option == NSF_OPT_UPS_NC) {
    PD_CHECK_ARG(value == 0 || value == 1, "NSF_OPT_UPS_NC is 0 or 1");
    m->ups_nc = value != 0;
    return PD_OK;
  }
  if (option == NSF_OPT_NC_MFMA) {
    PD_CHECK_ARG(value >= 0 && value <= 2, "NSF_OPT_NC_MFMA is 0, 1 or 2");
    m->nc_mfma = value;
    return PD_OK;
  }
  if (option == NSF_OPT_C256) {
    PD_CHECK_ARG(value == 0 || value == 1, "NSF_OPT_C256 is 0 or 1");
    for (auto& c : m->res) c.w256 = value;
    return PD_OK;
  }
  if (option == NSF_OPT_RB32 || option == NSF_OPT_RB64) {
    PD_CHECK_ARG(value >= 0 && value <= 7, "NSF_OPT_RB32 / RB64: a kernel-size bit mask (1: 3, 2: 7, 4: 11)");
    (option == NSF_OPT_RB32 ? m->rb32 : m->rb64) = value;
    return PD_OK;
  }
  if (option == NSF_OPT_RB16) {
    PD_CHECK_ARG(value >= 0 && value <= 2, "NSF_OPT_RB16 is 0, 1 or 2");
    m->rb16 = value;
    return PD_OK;
  }
  if (option == NSF_OPT_PAIR16) {
    PD_CHECK_ARG(value == 0 || value == 1, "NSF_OPT_PAIR16 is 0 or 1");
    m->pair16 = value != 0;
    return PD_OK;
  }
  set_error("nsf_set_option: unknown option " + std::to_string(option));
  return PD_ERR_ARG;
}

size_t nsf_workspace_size(const nsf_model* m, int B, int T) {
  if (!m || B < 0 || T < 0) return 0;
  return nsf_layout(m, B, T).total;
}

int nsf_forward(const nsf_model* m, const float* mel, float mel_scale, const float* f0, const float* rand_ini, const float* noise,
                unsigned long long seed, const int* utt_ids, const int* lens, float* wav, int B, int T, void* workspace,
                size_t ws_bytes, void* stream) {
  PD_CHECK_ARG(m && mel && f0 && wav && B >= 0 && T >= 0, "null argument");
  if (B == 0 || T == 0) return PD_OK;
  const NsfWs W = nsf_layout(m, B, T);
  if (!workspace || ws_bytes < W.total) { set_error("workspace too small"); return PD_ERR_WORKSPACE; }
  PD_CHECK_ARG((reinterpret_cast<uintptr_t>(mel) & 15) == 0, "mel must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  float* ws = static_cast<float*>(workspace);
  const nsf_dims& d = m->d;
  const int dim = m->dim, nk = d.num_kernels;
  const long long L = (long long)T * m->upp;
  double* P = reinterpret_cast<double*>(ws + W.P);
  float* har = ws + W.har;
  float *X = ws + W.X, *T1 = ws + W.T1, *R = ws + W.R, *XS = ws + W.XS, *XSRC = ws + W.src;
  const float sr = (float)d.sampling_rate;
  {
    ProfScope ps("nsf_source", st);
    float* Rd = ws + W.Rd;
    hipLaunchKernelGGL(nsf_phase_prefix_kernel, dim3(B * dim), dim3(NSF_PP_THREADS), 0, st, f0, B, T, dim, sr,
                       rand_ini, seed, utt_ids, P, Rd);
    hipLaunchKernelGGL(nsf_source_kernel, dim3(cdiv((long long)B * L, 256)), dim3(256), 0, st, f0, P, Rd, B, T, m->upp,
                       dim, sr, rand_ini, noise, seed, utt_ids, m->lin_w, m->lin_b, har);
  }
  PD_LAUNCH_CHECK();
  // ragged batch: stage s of `rate` samples per frame reads zero past lens[b] * rate (the phase
  // prefix and the source are causal per utterance, so frames past an utterance's end change nothing
  // before it)
  auto rag = [&](int rate) { NsfRag g; g.lens = lens; g.rate = rate; return g; };
  // conv_pre(mel_scale * mel^T) (nsf_hifigan.py:53, models.py:267)
  {
    const NsfConv& c = m->pre;
    GemmArgs a = make_gemm(B, T, c.cout, c.w, 7 * c.kpad, c.b, XS, (long long)T * c.cout, c.cout);
    for (int k = 0; k < 7; ++k) {
      Seg s = make_seg(mel, (long long)T * d.num_mels, d.num_mels, d.num_mels, k - 3);
      s.kpad = c.kpad;
      s.scale = mel_scale;
      add_seg(a, s);
    }
    a.lens = lens; a.lens_mul = 1;
    PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_NSF_CONV_PRE>(a, st, "nsf_conv_pre")));
  }
  int Tin = T;
  float in_scale = 1.f;
  size_t r = 0;
  for (int i = 0; i < d.num_upsamples; ++i) {
    const NsfUps& U = m->ups[i];
    const int Lc = Tin * U.u;
    const bool upsw = ups_window_ok(U, m->ups_window);
    // NSF_OPT_UPS_NC: the windowed upsample computes the noise conv itself (short source kernels:
    // the last three stages); otherwise nsf_noise_conv_kernel writes it for the upsample to add
    NsfNoise nz;
    if (upsw && m->ups_nc && U.nc_k <= NSF_NC_KMAX) {
      nz.har = har; nz.L = L; nz.w = U.nc_w; nz.b = U.nc_b;
      nz.k = U.nc_k; nz.stride = U.nc_stride; nz.pad = U.nc_pad; nz.rag = rag(m->upp);
    }
    // (NSF_OPT_NC_MFMA 1: the K = 128 conv only; 2 (default): the K = 16 one too.  C5: 104-105 -> 91-93 us per
    // launch, profiles/r06_ab/nsf_c256_noise_ab.txt)
    if (!nz.har && m->nc_mfma && U.nc_stride * 2 == U.nc_k && (U.nc_k == 128 || (U.nc_k == 16 && m->nc_mfma == 2)) &&
        U.cout % 32 == 0) {
      ProfScope ps("nsf_noise_conv", st);
      const dim3 grid(cdiv(Lc, 128), U.cout / 32, B);
      if (U.nc_k == 128)
        hipLaunchKernelGGL(nsf_noise_mfma_kernel<128>, grid, dim3(256), 0, st, har, L, U.nc_w, U.nc_b, U.cout,
                           U.nc_pad, (long long)Lc, XSRC, rag(m->upp));
      else
        hipLaunchKernelGGL(nsf_noise_mfma_kernel<16>, grid, dim3(256), 0, st, har, L, U.nc_w, U.nc_b, U.cout,
                           U.nc_pad, (long long)Lc, XSRC, rag(m->upp));
      PD_LAUNCH_CHECK();
    } else if (!nz.har) {
      const int CT = U.cout < 256 ? U.cout : 256, G = 256 / CT;
      const size_t lds = (size_t)((G * NC_ROWS - 1) * U.nc_stride + U.nc_k) * sizeof(float);
      ProfScope ps("nsf_noise_conv", st);
      hipLaunchKernelGGL(nsf_noise_conv_kernel, dim3(cdiv(Lc, G * NC_ROWS), U.cout / CT, B), dim3(256), lds, st, har,
                         L, U.nc_w, U.nc_b, U.cout, U.nc_k, U.nc_stride, U.nc_pad, (long long)Lc, XSRC, rag(m->upp));
      PD_LAUNCH_CHECK();
    }
    // x = ups(leaky_relu(x, 0.1)) + noise_conv(har)  (models.py:270-274): the windowed bf16
    // kernel, or one GEMM per phase
    const int p = (U.k - U.u) / 2;
    if (upsw) PD_TRY(launch_ups_window(U, XS, in_scale, B, Tin, XSRC, X, st, rag(Tin / T), nz));
    for (int phi = 0; phi < (upsw ? 0 : U.u); ++phi) {
      const int q0 = U.qmin[phi];
      const int o = q0 * U.u + phi - p;        // first output row of this phase, in [0, u)
      GemmArgs a = make_gemm(B, Tin, U.cout, U.w[phi], U.ntap * U.kpad, U.b, X + (long long)o * U.cout,
                             (long long)Lc * U.cout, U.u * U.cout);
      for (int mt = 0; mt < U.ntap; ++mt) {
        Seg s = make_seg(XS, (long long)Tin * U.cin, U.cin, U.cin, q0 - mt);
        s.kpad = U.kpad;
        s.act = ACT_LRELU;
        s.alpha = NSF_LRELU;
        s.scale = in_scale;
        add_seg(a, s);
      }
      a.res = XSRC + (long long)o * U.cout;
      a.res_bs = (long long)Lc * U.cout;
      a.res_ld = U.u * U.cout;
      a.lens = lens; a.lens_mul = Tin / T;
      PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_NSF_UPS>(a, st, "nsf_ups")));
    }
    // xs = sum_j resblock_j(x); x = xs / num_kernels (models.py:275-281); the division is
    // folded into the next consumer's load scale.
    const long long n4 = (long long)B * Lc * U.cout / 4;
    const NsfRag rag_ = rag(Lc / T);
    for (int j = 0; j < nk; ++j) {
      float* target = j == 0 ? XS : R;
      const float* cur = X;
      bool summed = false;   // resblock_j(x) already added into XS by its last conv
      const int D = d.num_dilations;
      if (d.resblock == 1 && D == 3) {
        NsfConv c1s[3], c2s[3];
        for (int q = 0; q < 3; ++q) { c1s[q] = m->res[r + q]; c2s[q] = m->res[r + D + q]; }
        const int Cr = c1s[0].cout;
        if ((Cr == 16 || Cr == 32 || Cr == 64) && rb_ok(m, c1s, c2s, Cr)) {
          // r06: the whole ResBlock in one launch, x read once, xs written / added once
          if ((long long)B * Lc * Cr >= (1ll << 31)) { set_error("nsf rb: B * T * C >= 2^31"); return PD_ERR_UNSUPPORTED; }
          if (Cr == 16) PD_TRY(launch_rb16(c1s, c2s, X, B, Lc, XS, j > 0 ? 1 : 0, st, rag_, m->rb16));
          else PD_TRY(launch_rb(c1s, c2s, X, B, Lc, XS, j > 0 ? 1 : 0, st, rag_));
          r += m->convs_per_block;
          continue;
        }
      }
      for (int q = 0; q < D; ++q) {
        if (d.resblock == 1) {
          const NsfConv& c1 = m->res[r + q];
          const NsfConv& c2 = m->res[r + D + q];
          if (pair_ok(m, c1, c2)) {
            // one launch per pair; it reads neighbouring blocks' rows of cur, so it never writes
            // cur: the pairs alternate between T1 (fp32 here) and target (XS / R), the last one
            // landing in target -- or accumulating into XS for resblock j >= 1
            const bool last_acc = j > 0 && q == D - 1;
            float* dst = q == D - 1 ? (last_acc ? XS : target) : ((D - 2 - q) % 2 == 0 ? T1 : target);
            PD_TRY(launch_pair(c1, c2, cur, B, Lc, dst, last_acc ? 1 : 0, st, rag_));
            if (last_acc) { summed = true; continue; }
            cur = dst;
            continue;
          }
          if (wconv_ok(c1) && wconv_ok(c2)) {
            // windowed bf16 convs; the inner activation xt = c1(lrelu(x)) travels as bf16; the
            // last pair of resblock j >= 1 accumulates straight into XS
            const bool last_acc = j > 0 && q == d.num_dilations - 1;
            PD_TRY(launch_wconv(c1, cur, false, NSF_LRELU, 1.f, B, Lc, T1, true, nullptr, st, 0, rag_));
            PD_TRY(launch_wconv(c2, T1, true, NSF_LRELU, 1.f, B, Lc, last_acc ? XS : target, false, cur, st,
                                last_acc ? 1 : 0, rag_));
            if (last_acc) { summed = true; continue; }
          } else {
            PD_TRY(nsf_conv(c1, cur, NSF_LRELU, 1.f, B, Lc, T1, nullptr, ACT_NONE, st, U_NSF_RES, rag_));
            PD_TRY(nsf_conv(c2, T1, NSF_LRELU, 1.f, B, Lc, target, cur, ACT_NONE, st, U_NSF_RES, rag_));
          }
          cur = target;
        } else {
          // out must not alias the taps being read: ping-pong target <-> T1
          float* dst = (cur == target) ? T1 : target;
          if (wconv_ok(m->res[r + q]))
            PD_TRY(launch_wconv(m->res[r + q], cur, false, NSF_LRELU, 1.f, B, Lc, dst, false, cur, st, 0, rag_));
          else
            PD_TRY(nsf_conv(m->res[r + q], cur, NSF_LRELU, 1.f, B, Lc, dst, cur, ACT_NONE, st, U_NSF_RES, rag_));
          cur = dst;
        }
      }
      r += m->convs_per_block;
      if (summed) continue;
      if (j == 0 && cur == XS) continue;
      ProfScope ps("nsf_accum", st);
      hipLaunchKernelGGL(nsf_accum_kernel, dim3(cdiv(n4, 256)), dim3(256), 0, st, reinterpret_cast<float4*>(XS),
                         reinterpret_cast<const float4*>(cur), n4, j == 0 ? 1 : 0);
      PD_LAUNCH_CHECK();
    }
    Tin = Lc;
    in_scale = 1.f / (float)nk;
  }
  // tanh(conv_post(leaky_relu(x, 0.01)))  (models.py:280-282)
  if (m->post.taps == 7 && m->post.cout == 1 && (m->post.cin == 16 || m->post.cin == 32)) {
    ProfScope ps("nsf_post", st);
    if (m->post.cin == 16)
      hipLaunchKernelGGL(nsf_post_kernel<16>, dim3(cdiv(Tin, 256), B), dim3(256), 0, st, XS, m->post.w, m->post.kpad,
                         m->post.b, 0.01f, in_scale, Tin, wav, rag(Tin / T));
    else
      hipLaunchKernelGGL(nsf_post_kernel<32>, dim3(cdiv(Tin, 256), B), dim3(256), 0, st, XS, m->post.w, m->post.kpad,
                         m->post.b, 0.01f, in_scale, Tin, wav, rag(Tin / T));
    PD_LAUNCH_CHECK();
  } else {
    PD_TRY(nsf_conv(m->post, XS, 0.01f, in_scale, B, Tin, wav, nullptr, ACT_TANH, st, U_NSF_POST, rag(Tin / T)));
  }
  return PD_OK;
}

}  // extern "C"

// Non-default compile-time knobs of this file (pd_build_config): "" for the shipped build.
namespace pd {
const char* nsf_build_flags() {
  return ""
#if NSF_PF_DEPTH != 4
         " NSF_PF_DEPTH"
#endif
#if NSF_RING_PIN != 0
         " NSF_RING_PIN"
#endif
#if NSF_PAIR_FMO32 != 15
         " NSF_PAIR_FMO32"
#endif
#if NSF_PAIR_FMO128 != 4
         " NSF_PAIR_FMO128"
#endif
#if NSF_PAIR_PF != NSF_PF_DEPTH
         " NSF_PAIR_PF"
#endif
#if NSF_PAIR_FMO64 != 8
         " NSF_PAIR_FMO64"
#endif
      ;
}
}  // namespace pd
