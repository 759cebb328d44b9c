// FastDiff eps-network + 4-step DDPM sampler on gfx950.
//
// Reference: modules/FastDiff/module/FastDiff_model.py:74-102 (network),
// modules/FastDiff/module/modules.py:116-343 (DBlock, TimeAware_LVCBlock,
// location_variable_convolution, KernelPredictor), util.py:158-232 (sampler).
//
// Activations are time-major [B][time][32]; the kernel predictor writes the
// location-variable kernels FRAME-major ([B][T'][64 out][3 tap][32 in]), so the
// LVC consumer reads one contiguous 24 KB block per frame.
#include <cmath>
#include <vector>

#include "../../include/prodiff_hip.h"
#include "gemm.h"
#include "kernels.h"

using namespace pd;

namespace {
constexpr int CI = 32;   // inner channels (base.yaml:21)
constexpr int CC = 80;   // cond channels
constexpr int HK = 64;   // kpnet hidden
constexpr int NLY = 4;   // lvc layers per block
constexpr int KPERLAYER = 2 * CI * CI * 3;   // 6144 kernel values per frame per layer
constexpr int EMB_IN = 128, EMB_MID = 512, EMB_OUT = 512;
constexpr int FD_STEP_CHUNK = 16;   // sampler steps whose embeddings / KP stacks are batched

// Frame-major LVC kernel layout is MFMA-fragment order.  Within each tap the 32 input
// channels are stored in the permuted order pos = lvc_pos(ci): position 16h + reg holds
// channel (reg&3) + 8(reg>>2) + 4h, which is exactly the channel set a lane of a 32x32
// MFMA result holds (rows (reg&3) + 8(reg>>2) + 4h).  So an LVC/pre-conv result computed
// with channels as rows is the next GEMM's k-operand in place (lvc_block_bf16_kernel).
// Value (o, q = tap*32 + ci) of a frame's 64x96 kernel (o = output channel) lives at
//   ((o/32 * 6 + k/16) * 64 + ((k%16)/8) * 32 + o%32) * 8 + k%8,  k = tap*32 + lvc_pos(ci),
// i.e. [gate|filter tile][k-step][lane][8]: each MFMA fragment load is 1 KB per wave.
__host__ __device__ inline int lvc_pos(int ci) { return (((ci >> 2) & 1) << 4) | ((ci >> 3) << 2) | (ci & 3); }
__host__ __device__ inline int lvc_chan(int p) { return (p & 3) | (((p & 15) >> 2) << 3) | ((p >> 4) << 2); }
__host__ __device__ inline int kf_packed(int o, int q) {
  const int k = (q & ~31) | lvc_pos(q & 31);
  return (((o >> 5) * 6 + (k >> 4)) * 64 + ((k & 15) >> 3) * 32 + (o & 31)) * 8 + (k & 7);
}
__host__ __device__ inline void kf_unpack(int p, int& o, int& q) {
  const int j = p & 7, l = (p >> 3) & 63, kkn = p >> 9;
  o = (kkn / 6) * 32 + (l & 31);
  const int k = (kkn % 6) * 16 + (l >> 5) * 8 + j;
  q = (k & ~31) | lvc_chan(k & 31);
}
}  // namespace

struct fd_model {
  int nblocks;
  int ratios[4];
  int hops[4];
  int dtype;
  // Whole-block LVC tile per block kind (measured, r01_ab4): 384 output samples with the
  // next-layer kernel prefetch (8 waves, 1 block/CU, 256 VGPRs) for hop >= 32; 128 for the
  // hop-8 block, whose tiles span several frames (no prefetch).  lvc_ts = 0 selects one
  // fused launch per layer.  Every field below is an fd_set_option (FD_OPT_*) with these
  // measured defaults; the tests use the options to cover each variant.
  int lvc_ts = 384;
  int lvc_ts_sub = 256;        // hop < 32 (hop-8) block tile: r03 A/B with plain K stores 105 vs 112 us (128), 121 (384)
  bool lvc_fuse = true;        // upsample / first conv / final update fused into the LVC block (FD_OPT_LVC_FUSE)
  bool lvc_pf = true;          // next-layer kernel fragments prefetched into registers (FD_OPT_LVC_PF)
  bool lvc_sub = true;         // hop < 32 blocks (hop 8) on the whole-block kernel too (FD_OPT_LVC_SUB)
  // fd_sample (bf16): the kernel-predictor GEMMs run on a second, low-priority stream into a
  // ring of one K buffer per block, so step j+1's kernels for block n are written while
  // step j's later blocks run (FD_OPT_KP_SIDE).  Created on first use.  Off by default:
  // the two streams share the CUs, so each kernel slows down by about the time the overlap
  // saves (r01 ab_v16b: 7.41 vs 7.33 ms/step).
  bool kp_side = false;
  int kp_chunk = 0;   // FD_OPT_KP_CHUNK: utterances per kernel-predictor -> LVC chunk (0 = whole batch)
  int lvc_tpw = 2;    // FD_OPT_LVC_TPW: 32-row tiles per wave of the 384-sample hop >= 32 blocks (2 or 1)
  int lvc_prio = 0;   // FD_OPT_LVC_PRIO: 1 = s_setprio(1) for the second half of an LVC block's waves
  int lvc_ps = 1;     // FD_OPT_LVC_PS (r06): the final block as a persistent kernel with LDS-DMA prefetch

  mutable hipStream_t side = nullptr;
  mutable hipEvent_t ev_hidden = nullptr, ev_kp[4] = {}, ev_lvc[4] = {};
  float* pool = nullptr;
  __bf16* pool_bf = nullptr;   // bf16 mirror of `pool` (PD_DTYPE_BF16), registered with launch_gemm
  void* kps = nullptr;         // the blocks' pre-scaled kernel-predictor weights (kks_w, kks_b)
  // step MLP
  float *fc1_w, *fc1_b, *fc2_w, *fc2_b;
  float *first_w, *first_b;          // [32][7]
  float *final_w, *final_b;          // [7][32], [1]
  struct Block {
    float *up_w, *up_b;              // [2r][32 ci][32 co]
    float *upf_w;                    // [r][32 co][64]: phase k's [W_k^T | W_{k+r}^T] (fused upsample, bf16 mirror)
    float *fct_w, *fct_b;            // [80][512]
    float *kin_w, *kin_b;            // [64][5*96]
    float *kres_w[6], *kres_b[6];    // [64][3*64]
    float *kk_w, *kk_b;              // [4*6144][3*64] frame-major rows
    __bf16* kks_w = nullptr;         // bf16: kk_w rows pre-scaled for the whole-block LVC gate (gate rows
    float* kks_b = nullptr;          //   by -log2 e, filter rows by 2 log2 e), and kk_b likewise
    float *kb_w, *kb_b;              // [256][3*64]
    float *cv_w[NLY], *cv_b[NLY];    // [32][96]
  } blk[4];
  struct Down {
    float *c0_w, *c0_b, *c1_w, *c1_b;   // [32][96]
    float *c2_w, *c2_b;                 // [32][96 + 32] : conv.2 taps ++ residual_dense
  } dn[4];
};

namespace {

// ------------------------------------------------------------------ kernels
// a0[b][t][c] = bias[c] + sum_k w[c][k] x[b][t+k-3]        (FastDiff_model.py:34-36,90)
__global__ __launch_bounds__(256) void first_conv_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out, int L,
                                                         const int* __restrict__ lens, int hop) {
  __shared__ float xs[32 + 6];
  const int b = blockIdx.y, t0 = blockIdx.x * 32, tid = threadIdx.x;
  const int Lv = lens ? min(lens[b] * hop, L) : L;   // ragged batch: the utterance's own end
  if (tid < 38) {
    int t = t0 - 3 + tid;
    xs[tid] = (t >= 0 && t < Lv) ? x[(long long)b * L + t] : 0.f;
  }
  __syncthreads();
  const int s = tid >> 3, q = (tid & 7) * 4, t = t0 + s;
  if (t >= L) return;
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float acc = bias[q + j];
#pragma unroll
    for (int k = 0; k < 7; ++k) acc = fmaf(w[(q + j) * 7 + k], xs[s + k], acc);
    o[j] = acc;
  }
  *reinterpret_cast<float4*>(out + ((long long)b * L + t) * CI + q) = make_float4(o[0], o[1], o[2], o[3]);
}

// ConvTranspose1d(32,32,k=2r,s=r,p=r/2+r%2,op=r%2) of lrelu_0.2(x)   (modules.py:163-166,205-206)
// Output phase phi = blockIdx.y: t = r*m + phi uses taps k0 = (phi+p)%r (input m+d) and
// k0+r (input m+d-1), d = (phi+p)/r.
__global__ __launch_bounds__(256) void upsample_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ Wt,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ out, int Tin, int r,
                                                       int p, const int* __restrict__ lens, int rate_in) {
  __shared__ __attribute__((aligned(16))) float w0[CI * CI], w1[CI * CI];
  __shared__ float xw[34][CI];
  const int b = blockIdx.z, phi = blockIdx.y, m0 = blockIdx.x * 32, tid = threadIdx.x;
  const int k0 = (phi + p) % r, d = (phi + p) / r;
  const int Tv = lens ? min(lens[b] * rate_in, Tin) : Tin;   // input rows past the utterance read zero
  for (int i = tid; i < CI * CI; i += 256) {
    w0[i] = Wt[k0 * CI * CI + i];
    w1[i] = Wt[(k0 + r) * CI * CI + i];
  }
  // rows j = m0 + d - 1 + jj, jj < 34
  for (int i = tid; i < 34 * CI; i += 256) {
    int jj = i / CI, c = i - jj * CI;
    int j = m0 + d - 1 + jj;
    float v = (j >= 0 && j < Tv) ? x[((long long)b * Tin + j) * CI + c] : 0.f;
    xw[jj][c] = v >= 0.f ? v : 0.2f * v;
  }
  __syncthreads();
  const int ml = tid >> 3, q = (tid & 7) * 4, m = m0 + ml;
  if (m >= Tin) return;
  float4 o = *reinterpret_cast<const float4*>(bias + q);
#pragma unroll 8
  for (int ci = 0; ci < CI; ++ci) {
    float xa = xw[ml + 1][ci];   // input m+d
    float xb = xw[ml][ci];       // input m+d-1
    float4 wa = *reinterpret_cast<const float4*>(&w0[ci * CI + q]);
    float4 wb = *reinterpret_cast<const float4*>(&w1[ci * CI + q]);
    o.x = fmaf(wa.x, xa, fmaf(wb.x, xb, o.x));
    o.y = fmaf(wa.y, xa, fmaf(wb.y, xb, o.y));
    o.z = fmaf(wa.z, xa, fmaf(wb.z, xb, o.z));
    o.w = fmaf(wa.w, xa, fmaf(wb.w, xb, o.w));
  }
  const long long t = (long long)r * m + phi;
  *reinterpret_cast<float4*>(out + ((long long)b * Tin * r + t) * CI + q) = o;
}

// x += a + sigmoid(o[:32]) * tanh(o[32:]),  o[t] = Bias_l + K_l . [y[t-1]; y[t]; y[t+1]]
// one block per frame l (modules.py:208-217, 220-253).  Kf rows: o*96 + tap*32 + ci.
template <typename KT>
__global__ __launch_bounds__(256) void lvc_kernel(float* __restrict__ x, const float* __restrict__ a,
                                                  const float* __restrict__ y,
                                                  const KT* __restrict__ Kf, int kf_ld,
                                                  const float* __restrict__ Bf, int bf_ld, int Tc,
                                                  int hop, const int* __restrict__ lens) {
  __shared__ float ks[64 * 97];
  __shared__ float bs[64];
  __shared__ float ys[34 * 33];
  const int g = blockIdx.x, b = g / Tc, l = g - b * Tc, tid = threadIdx.x;
  const long long L = (long long)Tc * hop;
  const long long Lv = lens ? (long long)min(lens[b], Tc) * hop : L;   // ragged batch: the utterance's end
  const KT* kf = Kf + (long long)g * kf_ld;
  for (int i = tid; i < 64 * 96; i += 256) {
    int oo, q2;
    kf_unpack(i, oo, q2);   // fragment-major -> [o][q] rows for the VALU loop
    ks[oo * 97 + q2] = (float)kf[i];
  }
  if (tid < 64) bs[tid] = Bf[(long long)g * bf_ld + tid];
  const int c = tid & 31, sg = tid >> 5;
  for (int s0 = 0; s0 < hop; s0 += 32) {
    const int chunk = hop - s0 < 32 ? hop - s0 : 32;
    __syncthreads();
    for (int i = tid; i < (chunk + 2) * 32; i += 256) {
      int rr = i >> 5, ci = i & 31;
      long long t = (long long)l * hop + s0 - 1 + rr;
      ys[rr * 33 + ci] = (t >= 0 && t < Lv) ? y[((long long)b * L + t) * CI + ci] : 0.f;
    }
    __syncthreads();
    for (int s = sg; s < chunk; s += 8) {
      float og = bs[c], of = bs[c + 32];
      const float* kg = ks + c * 97;
      const float* kfp = ks + (c + 32) * 97;
#pragma unroll
      for (int tap = 0; tap < 3; ++tap) {
        const float* yr = ys + (s + tap) * 33;
#pragma unroll 8
        for (int ci = 0; ci < 32; ++ci) {
          float yv = yr[ci];
          og = fmaf(kg[tap * 32 + ci], yv, og);
          of = fmaf(kfp[tap * 32 + ci], yv, of);
        }
      }
      long long idx = ((long long)b * L + (long long)l * hop + s0 + s) * CI + c;
      x[idx] = x[idx] + a[idx] + sigmoidf_(og) * tanhf_(of);
    }
  }
}

// Fused LVC layer on bf16 MFMA (hop >= 64), one launch per layer (modules.py:208-217, 220-253):
//   u = lrelu_.2(x + a); y = lrelu_.2(conv3_dil(u) + bc); o = Bf_l + K_l . [y(t-1); y(t); y(t+1)]
//   x <- x + a + sigmoid(o[:32]) * tanh(o[32:])
// Block = TS consecutive samples of ONE frame (so one 64x96 kernel K_l), TS/32 waves.
// u (TS + 2 + 2 dil rows) and y (TS + 2 rows) live only in LDS; K_l fragments are
// read straight from the frame-major kernel tensor (16 B per lane per k-step).
template <int TS>
__global__ __launch_bounds__(TS * 2) void lvc_fused_bf16_kernel(
    float* __restrict__ x, const float* __restrict__ a, const __bf16* __restrict__ Kf, int kf_ld,
    const float* __restrict__ Bf, int bf_ld, const __bf16* __restrict__ Wc, const float* __restrict__ bc,
    int Tc, int hop, int dil) {
  constexpr int NT = TS * 2;
  constexpr int LD = 40;                     // bf16 per staged row: 32 + 8 pad (80 B, conflict-free b128 reads)
  constexpr int NMT = (TS + 2 + 31) / 32;    // pre-conv row tiles (TS + 2 rows of y)
  constexpr int YROWS = NMT * 32;
  constexpr int UROWS = YROWS + 2 * 27;      // + 2*dil, dil <= 27 (3^3)
  __shared__ __attribute__((aligned(16))) __bf16 U[UROWS * LD];
  __shared__ __attribute__((aligned(16))) __bf16 Y[YROWS * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int per_frame = hop / TS;
  const int frame = blockIdx.x / per_frame, sub = blockIdx.x - frame * per_frame;
  const int b = frame / Tc, l = frame - b * Tc;
  const long long Lh = (long long)Tc * hop;
  const long long t0 = (long long)l * hop + (long long)sub * TS;
  const long long base = (long long)b * Lh;

  // 1. U[r] = lrelu(x + a) at t = t0 - 1 - dil + r, zero outside the utterance (conv padding)
  const int nU = YROWS + 2 * dil;
  for (int i = tid; i < nU * 8; i += NT) {
    const int r = i >> 3, q = (i & 7) * 4;
    const long long t = t0 - 1 - dil + r;
    bf16x4 v = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
    if (t >= 0 && t < Lh) {
      const float4 xv = *reinterpret_cast<const float4*>(x + (base + t) * CI + q);
      const float4 av = *reinterpret_cast<const float4*>(a + (base + t) * CI + q);
      float u0 = xv.x + av.x, u1 = xv.y + av.y, u2 = xv.z + av.z, u3 = xv.w + av.w;
      u0 = u0 >= 0.f ? u0 : 0.2f * u0; u1 = u1 >= 0.f ? u1 : 0.2f * u1;
      u2 = u2 >= 0.f ? u2 : 0.2f * u2; u3 = u3 >= 0.f ? u3 : 0.2f * u3;
      v = bf16x4{(__bf16)u0, (__bf16)u1, (__bf16)u2, (__bf16)u3};
    }
    *reinterpret_cast<bf16x4*>(U + r * LD + q) = v;
  }
  __syncthreads();

  // 2. pre-conv (32 -> 32, k3, dilation dil): Y[r] = lrelu(W_c . [U(r); U(r+dil); U(r+2dil)] + b)
  {
    bf16x8 wf[6];
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) wf[kk] = *reinterpret_cast<const bf16x8*>(Wc + r32 * 96 + kk * 16 + h * 8);
    const float bias = bc[r32];
    for (int mt = wave; mt < NMT; mt += NT / 64) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
        const int tap = kk >> 1, ci0 = (kk & 1) * 16;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(U + (mt * 32 + r32 + tap * dil) * LD + ci0 + h * 8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wf[kk], acc, 0, 0, 0);
      }
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int r = mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const long long t = t0 - 1 + r;
        float y = acc[reg] + bias;
        y = y >= 0.f ? y : 0.2f * y;
        if (t < 0 || t >= Lh) y = 0.f;        // the LVC zero-pads y at utterance edges
        Y[r * LD + lvc_pos(r32)] = (__bf16)y; // kernel k-order (kf_packed)
      }
    }
  }
  __syncthreads();

  // 3. location-variable conv with this frame's kernel: rows = TS samples, cols = 64
  //    outputs as a gate tile (o = c) and a filter tile (o = 32 + c) in the same lanes.
  {
    const __bf16* kf = Kf + (long long)frame * kf_ld;
    const float* bfp = Bf + (long long)frame * bf_ld;
    const int mt = wave;
    f32x16 ag, afl;
#pragma unroll
    for (int r = 0; r < 16; ++r) { ag[r] = 0.f; afl[r] = 0.f; }
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) {
      const int tap = kk >> 1, ci0 = (kk & 1) * 16;
      const bf16x8 yf = *reinterpret_cast<const bf16x8*>(Y + (mt * 32 + r32 + tap) * LD + ci0 + h * 8);
      const bf16x8 kg = *reinterpret_cast<const bf16x8*>(kf + (kk * 64 + lane) * 8);
      const bf16x8 kl = *reinterpret_cast<const bf16x8*>(kf + ((6 + kk) * 64 + lane) * 8);
      ag = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yf, kg, ag, 0, 0, 0);
      afl = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yf, kl, afl, 0, 0, 0);
    }
    const float bg = bfp[r32], bl = bfp[32 + r32];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int s = mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      const long long idx = (base + t0 + s) * CI + r32;
      x[idx] = x[idx] + a[idx] + gate_fast(ag[reg] + bg, afl[reg] + bl);
    }
  }
}

// ------------------------------------------------------------------ whole LVC block (bf16)
// All 4 LVC layers of one TimeAware_LVCBlock (modules.py:208-217) in ONE launch:
//   for l < 4:  x = x + a + gate(LVC_l(lrelu(conv_{3^l}(lrelu(x + a)) + b_l)))
// Block = TS output samples of one utterance on a grid of NG 32-row tiles covering
// [t0 - 64, t0 + TS + 64).  Tiles are 32-aligned in time; with hop % 32 == 0 every
// tile lies in ONE frame and multiplies one 64x96 kernel (SUB: hop | 32, several frames
// per tile, one masked MFMA chain each).  The state x and audio_down a
// stay in registers in the MFMA C layout (wave w owns tiles w and w + NW); LDS only
// holds the bf16 operands u = lrelu(x + a) and y.  Layer l is valid on rows
// [64 - e_l, 64 + TS + e_l), e = 42, 38, 28, 0 (the remaining dilation reach; +3 each
// when the final conv is fused), and only the tiles overlapping that range are
// computed; rows outside it are never read by a valid row, so they may hold anything.
//
// Optional fusions (template flags), each removing a full-rate HBM round trip:
//  UPS  the block's ConvTranspose upsample (modules.py:205-206) runs in the prologue
//       from x_prev (r x fewer rows), as r phase GEMMs on MFMA: output t = r j + k - p
//       uses taps k and k + r on inputs j and j - 1 (K = 64), staged through LDS.
//  AUD  audio_down = first_conv(audio) (FastDiff_model.py:90) is recomputed per row
//       from the 1-channel audio instead of read as a [L][32] tensor.
//  FIN  the final conv7 32 -> 1 and the sampler update (FastDiff_model.py:100,
//       util.py:222-226) run in the epilogue: only the new audio sample leaves.
struct LvcBlockArgs {
  float* xout;              // [B][Lh][32]                  (!FIN)
  const float* xin;         // [B][Lh][32] upsampled x (!UPS), or x_prev [B][Lh/r][32] (UPS)
  const float* a;           // [B][Lh][32] audio_down       (!AUD)
  const __bf16* Kf[NLY];    // [B*Tc][6144] per layer (frame-major, fragment order)
  const float* Bf;          // [B*Tc][256]: layer l at +64 l
  const __bf16* Wc[NLY];    // [32][96] pre-conv weights (bf16 mirror)
  const float* bc[NLY];
  const __bf16* Wup;        // UPS: [r][32 co][64] = [W_k^T | W_{k+r}^T] per phase k
  const float* bup;         // UPS: [32]
  int r, p;                 // UPS: ratio, ConvTranspose padding
  const float* audio;       // AUD / FIN: [B][Lh] current sample x_t
  const float* fw;          // AUD: first conv [32][7]
  const float* fb;          // AUD: [32]
  const float* wfin;        // FIN: final conv [7][32]
  const float* bfin;        // FIN: [1]
  float* audio_out;         // FIN: [B][Lh]  (x_t - ce eps) / den + sig z
  const float* noise;       // FIN: explicit z [B][Lh] or null (Philox)
  float ce, den, sig;
  unsigned long long seed;
  unsigned stream;
  const int* uid;           // FIN: utterance id per batch row (null -> row index)
  int Tc, hop;
  const int* lens;          // frames of each row's utterance (null: Tc), already offset by b_off
  int b_off;                // utterance index of blockIdx.y = 0 in the whole batch (Philox draws)
  int prio;                 // FD_OPT_LVC_PRIO: s_setprio(1) for the second half of the waves
#ifdef LB_TRACE
  unsigned long long* trace;   // tools/lvc_probe.hip: per-phase s_memtime stamps
#endif
};
#ifdef LB_TRACE
#define LB_STAMP(i)                                                                       \
  do {                                                                                    \
    if (lane == 0 && blockIdx.x % 61 == 0)                                                \
      P.trace[((blockIdx.y * gridDim.x + blockIdx.x) / 61 * NW + wave) * 24 + (i)] =      \
          __builtin_readcyclecounter();                                                   \
  } while (0)
#else
#define LB_STAMP(i) \
  do {              \
  } while (0)
#endif
constexpr int LB_LD = 40;
constexpr int LB_XLD = 36;                          // fp32 staging rows (144 B)
template <int TS, int TPW = 2> struct LbGeo {
  static constexpr int NG = TS / 32 + 4;            // tiles in the grid
  static constexpr int NW = NG / TPW;               // waves; TPW tiles each
  static constexpr int NT = NW * 64;
  static constexpr int UOFF = 28;                   // U index = row + 28 (pre-conv reach 1 + 27)
  static constexpr int UROWS = NG * 32 + 2 * UOFF;
  static constexpr int YROWS = (NG + 1) * 32;       // Y index = row + 1
  static constexpr int UY_BYTES = (UROWS + YROWS) * LB_LD * 2;
  static constexpr int XS_BYTES = NG * 32 * LB_XLD * 4;          // fp32 x rows (prologue / epilogue)
  static constexpr int NTJ_MAX = (NG * 32 / 4 + 2 + 31) / 32;    // phase-GEMM column tiles at r >= 4
  static constexpr int XP_BYTES = (NTJ_MAX * 32 + 1) * LB_LD * 2;
  static constexpr int SMEM = UY_BYTES > XS_BYTES + XP_BYTES ? UY_BYTES : XS_BYTES + XP_BYTES;
};

// fp32 pairs for the LVC epilogues.  Default: a packed vector (v_pk_fma/mul/add_f32 work on two
// values per instruction).  LVC_SCALAR_F32: a plain struct, one v_*_f32 per value (gfx950 issues a
// packed f32 op beside MFMAs at more than twice the cost of a scalar one, MI355X_MICROARCH.md).
#ifdef LVC_SCALAR_F32
struct f32x2 { float x, y; };
__device__ __forceinline__ f32x2 operator+(f32x2 a, f32x2 b) { return f32x2{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ f32x2 operator-(f32x2 a, f32x2 b) { return f32x2{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ f32x2 operator*(f32x2 a, f32x2 b) { return f32x2{a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ f32x2 operator+(f32x2 a, float b) { return f32x2{a.x + b, a.y + b}; }
__device__ __forceinline__ f32x2 operator*(f32x2 a, float b) { return f32x2{a.x * b, a.y * b}; }
__device__ __forceinline__ f32x2& operator+=(f32x2& a, f32x2 b) { a = a + b; return a; }
__device__ __forceinline__ f32x2 efma(f32x2 a, f32x2 b, f32x2 c) { return f32x2{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }
__device__ __forceinline__ f32x2 emax(f32x2 a, f32x2 b) {
  return f32x2{__builtin_elementwise_maximum(a.x, b.x), __builtin_elementwise_maximum(a.y, b.y)};
}
#else
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 efma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 emax(f32x2 a, f32x2 b) { return __builtin_elementwise_maximum(a, b); }
#endif
constexpr float LOG2E = 1.4426950408889634f;
__device__ __forceinline__ f32x2 lrelu2(f32x2 v) {
  // max(v, 0.2 v) as med3(v, 0.2 v, +inf): v_max_f32 would first canonicalize operands
  // the compiler cannot prove canonical (a register state fed from memory)
  const f32x2 s = v * 0.2f;
  return emax(v, s);
}
// sigmoid(g) tanh(f) = (ef - 1) r, ef = exp2(clamped fs), r = 1 / ((ef + 1)(eg + 1)), from the
// exp2 arguments gs = -log2e (g + b_g), fs = 2 log2e (f + b_f) (tanh saturates by |f| = 15)
__device__ __forceinline__ f32x2 gate2ef(f32x2 fs) {
  constexpr float C = 15.f * 2.f * LOG2E;
  return f32x2{__builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(fs.x, -C, C)),
               __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(fs.y, -C, C))};
}
__device__ __forceinline__ f32x2 gate2r(f32x2 gs, f32x2 fs) {
  const f32x2 ef = gate2ef(fs);
  const f32x2 eg1 = f32x2{__builtin_amdgcn_exp2f(gs.x), __builtin_amdgcn_exp2f(gs.y)} + 1.f;
  const f32x2 den = efma(ef, eg1, eg1);
  return f32x2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
}
__device__ __forceinline__ int floordiv(int a, int b) { return (a >= 0 ? a : a - b + 1) / b; }

// TPW = tiles per wave: 2 (NG/2 waves, 2 per SIMD at TS = 384) or 1 (NG waves: 16 at TS = 384,
// 4 per SIMD, so one wave's MFMAs run beside another's gate VALU; <= 128 VGPRs).
template <int TS, bool UPS, bool AUD, bool FIN, bool PF = false, bool SUB = false, int TPW = 2>
__global__ __launch_bounds__((LbGeo<TS, TPW>::NT), (TPW == 1 ? LbGeo<TS, TPW>::NT / 256 : (PF || SUB) ? 2 : 3))
void lvc_block_bf16_kernel(const LvcBlockArgs P) {
  static_assert(!(PF && SUB), "prefetch assumes one frame per tile");
  static_assert(TPW == 1 || TPW == 2, "one or two tiles per wave");
  using G = LbGeo<TS, TPW>;
  constexpr int NW = G::NW, NG = G::NG, UOFF = G::UOFF, GR = NG * 32;
  constexpr int EX = FIN ? 3 : 0;                    // extra valid rows for the fused final conv
  // Rows = time, 40 bf16 per row; position p of a row holds channel lvc_chan(p).
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  __shared__ float AS[AUD ? GR + 6 : 1];             // audio at times [tg - 3, tg + GR + 3)
  __shared__ __attribute__((aligned(16))) float FW[AUD ? 7 * 32 : 4];   // first conv [tap][c]
  __shared__ __attribute__((aligned(16))) float FWF[FIN ? 7 * 32 : 4];  // final conv [tap][c]
  __shared__ __attribute__((aligned(16))) float FBL[AUD ? 32 : 4];       // first conv bias
  __shared__ __attribute__((aligned(16))) float BUL[UPS ? 32 : 4];       // upsample bias
  // PF: the pre-conv weights (fragment order), their biases and the LVC biases of the
  // block's frames (pre-scaled for the gate) live in LDS, so no global load but the
  // next layer's kernel prefetch is in flight across a layer (vmcnt retires in order:
  // a global weight load behind the prefetch would wait for the whole prefetch).
  // SUB (hop 8) stages the pre-conv weights too (WW): a global load per layer made every layer
  // start with an L2 round trip; its LVC biases stay per-frame global reads.
  // (r05: without the staged weights SUB's 69 KB of LDS would fit two blocks per CU, but its
  // registers do not: ~260 VGPRs -- the two-frame K pipeline alone is 96 -- and at the 168-VGPR cap of
  // 3 waves per SIMD it spills 382)
  constexpr bool WL = PF, WW = PF || SUB;
  // frames a block touches: its GR rows span at most GR / hop + 2 frames, and PF (= WL) launches
  // have hop % 64 == 0 (r05: sized for hop >= 32 before, 18 frames -- 8 more than any PF launch reads,
  // 8 KB of LDS and two float4 loads per thread in every block's prologue)
  constexpr int BFR = WL ? GR / 64 + 2 : 1;
  __shared__ __attribute__((aligned(16))) bf16x8 WCL[WW ? NLY * 6 * 64 : 1];
  __shared__ __attribute__((aligned(16))) float BCL[WW ? NLY * CI : 4];
  __shared__ __attribute__((aligned(16))) float BFL[WL ? BFR * 2 * CI * NLY : 4];
  __bf16* U = reinterpret_cast<__bf16*>(smem);
  __bf16* Y = U + G::UROWS * LB_LD;
  float* XS = reinterpret_cast<float*>(smem);                       // aliases U/Y outside the layers
  __bf16* XP = reinterpret_cast<__bf16*>(smem + G::XS_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, n = lane & 31, h = lane >> 5;
  // XCD-aware block order: the hardware deals consecutive block ids round-robin over
  // the 8 XCDs; remap so each XCD walks a contiguous run of (utterance, time) tiles and
  // neighbouring tiles -- which share frames' kernels and halo rows -- share its L2.
  int bx, b;
  {
    const int total = gridDim.x * gridDim.y, id = blockIdx.y * gridDim.x + blockIdx.x;
    const int xcd = id & 7, slot = id >> 3, per = total >> 3, rem = total & 7;
    const int logical = xcd < rem ? xcd * (per + 1) + slot : rem * (per + 1) + (xcd - rem) * per + slot;
    b = logical / gridDim.x;
    bx = logical - b * gridDim.x;
  }
  // Tiles of wave w: PF -- the adjacent pair 2w, 2w + 1 (one frame, one shared kernel);
  // otherwise w and w + NW (better balanced over the shrinking per-layer tile ranges), the
  // upper half first in odd time tiles: a block's last 4 grid tiles are the next block's
  // first 4 (the 2 x 64-row halo), so both read those frames' kernels in the same pass and
  // the second read can hit L2 (hop 8: the halo re-reads were a third of the launch's bytes).
  const int jsw = !PF && (bx & 1);
#define TILE(j) (TPW == 1 ? wave : PF ? 2 * wave + (j) : wave + ((j) ^ jsw) * NW)
  const int Tc = P.Tc, hop = P.hop;
  const int Lh = Tc * hop;                           // utterance-local times fit in 32 bits
  // ragged batch: the utterance ends at Le <= Lh (a multiple of hop, so of 32 when hop % 32 == 0):
  // everything that reads past it -- audio, x_prev, x rows, u, y, the final conv -- reads zero
  const int Le = P.lens ? min(P.lens[b], Tc) * hop : Lh;
  const int t0 = bx * TS, tg = t0 - 64;              // time of grid row 0
  const long long base = (long long)b * Lh;
  constexpr int RLO = 64 - 44 - EX, RHI = 64 + TS + 44 + EX;   // x rows the valid region reads
  LB_STAMP(0);
  // Prologue: every global load of the block -- the LDS-staged operands, x_prev, the
  // phase-GEMM weights and (last, PF) layer 0's kernel fragments -- is issued before the
  // first use, so the block pays about one memory round trip before its first layer
  // (vmcnt retires in order: the prefetch stays in flight while the staging drains).
  const int fbase = (tg > 0 ? tg : 0) / hop;         // first frame of the block (WL)
  constexpr int IT = AUD ? (GR + 6 + G::NT - 1) / G::NT : 1;
  float av[IT], fwv = 0.f, fbv = 0.f, bupv = 0.f, wfv = 0.f;
  if constexpr (AUD) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      // unconditional loads at clamped addresses, masked at the LDS store: a load under a
      // branch makes the compiler wait for it at the branch join
      const int t = tg - 3 + tid + it * G::NT;
      av[it] = P.audio[base + min(max(t, 0), Lh - 1)];
    }
    if (tid < 224) fwv = P.fw[(tid & 31) * 7 + (tid >> 5)];   // fw is [c][tap]
    if (tid < 32) fbv = P.fb[tid];
  }
  if constexpr (UPS) {
    if (tid < 32) bupv = P.bup[tid];
  }
  if constexpr (FIN) {
    if (tid < 224) wfv = P.wfin[tid];                        // already [tap][c]
  }
  constexpr int IW = WW ? (6 * 64 + G::NT - 1) / G::NT : 1;
  constexpr int N4 = BFR * 2 * CI * NLY / 4, IB = WL ? (N4 + G::NT - 1) / G::NT : 1;
  bf16x4 wv[IW][NLY][2];
  float bcv = 0.f;
  float4 bfv[IB];
  if constexpr (WW) {
#pragma unroll
    for (int it = 0; it < IW; ++it) {
      const int i = min(tid + it * G::NT, 6 * 64 - 1), kk = i >> 6, ln = i & 63;
#pragma unroll
      for (int l = 0; l < NLY; ++l) {
        const __bf16* w = P.Wc[l] + (ln & 31) * 96 + (kk >> 1) * 32 + 16 * (ln >> 5) + 4 * (kk & 1);
        wv[it][l][0] = *reinterpret_cast<const bf16x4*>(w);
        wv[it][l][1] = *reinterpret_cast<const bf16x4*>(w + 8);
      }
    }
    if (tid < NLY * CI) {
#pragma unroll
      for (int l = 0; l < NLY; ++l)
        if (tid / CI == l) bcv = P.bc[l][tid % CI];
    }
  }
  if constexpr (WL) {
#pragma unroll
    for (int it = 0; it < IB; ++it) {
      const int i = min(tid + it * G::NT, N4 - 1), fr = min(fbase + i / (2 * CI * NLY / 4), Tc - 1);
      const int c = (i % (2 * CI * NLY / 4)) * 4;
      bfv[it] = *reinterpret_cast<const float4*>(P.Bf + ((long long)b * Tc + fr) * (2 * CI * NLY) + c);
    }
  }
  // UPS: x_prev rows and this wave's first chunk of phase-GEMM weight fragments
  const int r = UPS ? P.r : 1, pp = UPS ? P.p : 0, Tin = Lh / r, Tin_e = Le / r;
  const int ntj = (GR / r + 2 + 31) / 32;
  const int jb = floordiv(tg + pp, r) - 2;           // column j0 = jb + 1 + c, c < 32 ntj
  constexpr int IX = UPS ? ((G::NTJ_MAX * 32 + 1) * 8 + G::NT - 1) / G::NT : 1;
  float4 xv4[IX];
  // NW % r == 0: wave w computes phase w % r on columns w / r, w / r + NW / r, ... and
  // loads that phase's weights once; otherwise jobs run in chunks of 4 (wfj[q]).
  const bool by_phase = NW % r == 0 && ntj <= 4 * (NW / r);
  bf16x8 wfj[4][4];
  // (r05: loading these unconditionally -- no wait at the branch join, the whole prologue's loads in
  // flight together, layer 0's kernel prefetch issued earlier -- measured slower, as r04's fully
  // batched prologue: final block 471-483 -> 505-514 us, lvc_prologue_batch_ab.txt)
  auto wup_load = [&](int job0) {
    if (by_phase) {
      const __bf16* wa = P.Wup + ((long long)(wave % r) * 32 + n) * 64 + 8 * h;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wfj[0][kk] = *reinterpret_cast<const bf16x8*>(wa + kk * 16);
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int job = job0 + q * NW, k = job / ntj;
      if (job < r * ntj) {
        const __bf16* wa = P.Wup + ((long long)k * 32 + n) * 64 + 8 * h;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) wfj[q][kk] = *reinterpret_cast<const bf16x8*>(wa + kk * 16);
      }
    }
  };
  if constexpr (UPS) {
    const float* xp = P.xin + (long long)b * Tin * CI;
#pragma unroll
    for (int it = 0; it < IX; ++it) {
      const int i = tid + it * G::NT, q = (i & 7) * 4, j = min(max(jb + (i >> 3), 0), Tin - 1);
      xv4[it] = *reinterpret_cast<const float4*>(xp + (long long)j * CI + q);
    }
    wup_load(wave);
  }
  // PF (hop % 64 == 0): a wave's two tiles are a 64-aligned pair, so they lie in one frame
  // and share one 64x96 kernel.  Layer l's fragments are loaded into registers while layer
  // l - 1 finishes (issued right after the pair's MFMAs), so their latency hides behind the
  // gates, the staging and the pre-conv.  Loads are unconditional (frame clamped).
  const int fpair = min(max(tg + 32 * TPW * wave + 16 * TPW, 0) / hop, Tc - 1);
  bf16x8 kn[12];
  auto kload = [&](int l) {
    const __bf16* kq = P.Kf[l] + ((long long)b * Tc + fpair) * KPERLAYER;
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) kn[kk] = *reinterpret_cast<const bf16x8*>(kq + (kk * 64 + lane) * 8);
  };
  if constexpr (PF) kload(0);
  // FIN: the sampler noise of this thread's output samples, drawn while the loads fly
  constexpr int IF = FIN ? (TS + G::NT - 1) / G::NT : 1;
  float zr[IF];
  const float bfin = FIN ? P.bfin[0] : 0.f;
  if constexpr (FIN) {
#pragma unroll
    for (int it = 0; it < IF; ++it) {
      const int s = tid + it * G::NT, t = t0 + s;
      zr[it] = 0.f;
      if (s < TS && t < Lh && P.sig != 0.f)
        zr[it] = P.noise ? P.noise[base + t]
                         : philox_normal_u(P.seed, utt_id(P.uid, b + P.b_off), (unsigned)t, P.stream);
    }
  }
  // ---- LDS stores of the staged operands
  if constexpr (AUD) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = tid + it * G::NT;
      const int t = tg - 3 + i;
      if (i < GR + 6) AS[i] = (t >= 0 && t < Le) ? av[it] : 0.f;
    }
    if (tid < 224) FW[tid] = fwv;
    if (tid < 32) FBL[tid] = fbv;
  }
  if constexpr (UPS) {
    if (tid < 32) BUL[tid] = bupv;
  }
  if constexpr (FIN) {
    if (tid < 224) FWF[tid] = wfv;
  }
  if constexpr (WW) {
#pragma unroll
    for (int it = 0; it < IW; ++it) {
      const int i = tid + it * G::NT;
#pragma unroll
      for (int l = 0; l < NLY; ++l) {
        const bf16x4 w0 = wv[it][l][0], w1 = wv[it][l][1];
        if (i < 6 * 64) WCL[l * 384 + i] = bf16x8{w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
      }
    }
    if (tid < NLY * CI) BCL[tid] = bcv;
  }
  if constexpr (WL) {
#pragma unroll
    for (int it = 0; it < IB; ++it) {
      const int i = tid + it * G::NT, c = (i % (2 * CI * NLY / 4)) * 4;
      // gate pre-scale; frames past the utterance end are never read (zero them anyway)
      const float sc = fbase + i / (2 * CI * NLY / 4) >= Tc ? 0.f : (c & 63) < 32 ? -LOG2E : 2.f * LOG2E;
      if (i < N4)
        *reinterpret_cast<float4*>(&BFL[4 * i]) = make_float4(bfv[it].x * sc, bfv[it].y * sc, bfv[it].z * sc, bfv[it].w * sc);
    }
  }
  LB_STAMP(16);
  // ---- x rows (upsampled in-kernel, or loaded) -> registers
  f32x2 xr[TPW][8], ar[TPW][8];
  if constexpr (UPS) {
    // (a) XP[j - jb] = bf16 lrelu(x_prev[j]), j in [jb, jb + 32 ntj]: j0 - 1 .. j0 of every column
#pragma unroll
    for (int it = 0; it < IX; ++it) {
      const int i = tid + it * G::NT, rr = i >> 3, q = (i & 7) * 4, j = jb + rr;
      if (i < (ntj * 32 + 1) * 8) {
        // rows outside x_prev are zero (lrelu(0) = 0)
        const float m = (j >= 0 && j < Tin_e) ? 1.f : 0.f;
        const f32x2 u0 = lrelu2(f32x2{xv4[it].x, xv4[it].y} * m), u1 = lrelu2(f32x2{xv4[it].z, xv4[it].w} * m);
        *reinterpret_cast<bf16x4*>(&XP[rr * LB_LD + q]) = bf16x4{(__bf16)u0.x, (__bf16)u0.y, (__bf16)u1.x, (__bf16)u1.y};
      }
    }
    __syncthreads();
    LB_STAMP(17);
    // (b) phase GEMMs: C^T[co][col] = [W_k^T | W_{k+r}^T] . [xp(j0); xp(j0 - 1)], t = r j0 + k - p
    for (int job0 = wave; job0 < r * ntj; job0 += 4 * NW) {
    if (job0 != wave && !by_phase) wup_load(job0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int k, jt;
      if (by_phase) {
        k = wave % r; jt = wave / r + q * (NW / r);
        if (jt >= ntj) break;
      } else {
        const int job = job0 + q * NW;
        if (job >= r * ntj) break;
        k = job / ntj; jt = job - k * ntj;
      }
      f32x16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        // k-step kk < 2: input j0 (XP row c + 1), kk >= 2: input j0 - 1 (XP row c)
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(
            &XP[(jt * 32 + n + (kk < 2 ? 1 : 0)) * LB_LD + 16 * (kk & 1) + 8 * h]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(by_phase ? wfj[0][kk] : wfj[q][kk], xb, acc, 0, 0, 0);
      }
      const int j0 = jb + 1 + jt * 32 + n, row = r * j0 + k - pp - tg;
      if (row >= RLO && row < RHI) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bv = *reinterpret_cast<const float4*>(&BUL[8 * g + 4 * h]);
          *reinterpret_cast<float4*>(&XS[row * LB_XLD + 8 * g + 4 * h]) =
              make_float4(acc[4 * g] + bv.x, acc[4 * g + 1] + bv.y, acc[4 * g + 2] + bv.z, acc[4 * g + 3] + bv.w);
        }
      }
    }
    if (by_phase) break;
    }
    __syncthreads();
  } else if constexpr (AUD) {
    __syncthreads();                                  // AS / FW visible
  }
  LB_STAMP(18);
  // Transposed C layout: lane (n, h) of tile k holds time tg + 32k + n, channels
  // (reg&3) + 8(reg>>2) + 4h; pair p = regs (2p, 2p+1).  Four float4 loads per tensor
  // (channels 8i + 4h .. +3).
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int k = TILE(j), row = k * 32 + n, t = tg + row;
    const bool ok = row >= RLO && row < RHI && t >= 0 && t < Le;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), av = xv;
      if (ok) {
        if constexpr (UPS) xv = *reinterpret_cast<const float4*>(&XS[row * LB_XLD + 8 * i + 4 * h]);
        else xv = *reinterpret_cast<const float4*>(P.xin + (base + t) * CI + 8 * i + 4 * h);
        if constexpr (AUD) {
          // a0[t][c] = b[c] + sum_tap w[c][tap] audio[t + tap - 3], first_conv_kernel's order
          float a4[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) a4[e] = FBL[8 * i + 4 * h + e];
#pragma unroll
          for (int tap = 0; tap < 7; ++tap) {
            const float s = AS[row + tap];
            const float4 w = *reinterpret_cast<const float4*>(&FW[tap * 32 + 8 * i + 4 * h]);
            a4[0] = fmaf(w.x, s, a4[0]); a4[1] = fmaf(w.y, s, a4[1]);
            a4[2] = fmaf(w.z, s, a4[2]); a4[3] = fmaf(w.w, s, a4[3]);
          }
          av = make_float4(a4[0], a4[1], a4[2], a4[3]);
        } else {
          av = *reinterpret_cast<const float4*>(P.a + (base + t) * CI + 8 * i + 4 * h);
        }
      }
      // registers hold z = x + a (the reference's `x += audio_down`, modules.py:209)
      xr[j][2 * i] = f32x2{xv.x + av.x, xv.y + av.y}; xr[j][2 * i + 1] = f32x2{xv.z + av.z, xv.w + av.w};
      ar[j][2 * i] = f32x2{av.x, av.y}; ar[j][2 * i + 1] = f32x2{av.z, av.w};
    }
  }
  LB_STAMP(19);
  if constexpr (UPS) __syncthreads();                // XS reads done before U/Y (aliased) are written
  // PF: U/Y are not cleared.  A valid row only reads rows staged or computed for it (the
  // e_l bookkeeping), utterance-edge padding is selected, not multiplied, so stale LDS
  // (possibly NaN) reaches only rows that are never stored.
  if constexpr (!PF) {
    const bf16x8 z = {};
    for (int i = tid; i < G::UY_BYTES / 16; i += G::NT) reinterpret_cast<bf16x8*>(smem)[i] = z;
  }
  LB_STAMP(20);
  __syncthreads();
  LB_STAMP(1);
  // static priority for the later-dispatched half of the waves (their SIMD partners are the
  // first half): MI355X_MICROARCH.md "Two waves per SIMD", item 4
  if (P.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int l = 0; l < NLY; ++l) {
    const int d = l == 0 ? 1 : l == 1 ? 3 : l == 2 ? 9 : 27;
    const int e = (l == 0 ? 42 : l == 1 ? 38 : l == 2 ? 28 : 0) + EX;
    const int kf = (64 - e) / 32, kl = (64 + TS + e - 1) / 32;   // LVC tiles of this layer
    const int kpl = kl + 1 < NG - 1 ? kl + 1 : NG - 1;           // last pre-conv tile
    // (1) u = lrelu(z) (z = x + a) of the owned tiles the pre-conv reads: 2 x 16 B per lane
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int k = TILE(j);
      if (k >= kf - 1 && k <= kl + 2) {
        bf16x8 u0, u1;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const f32x2 v0 = lrelu2(xr[j][p]), v1 = lrelu2(xr[j][4 + p]);
          u0[2 * p] = (__bf16)v0.x; u0[2 * p + 1] = (__bf16)v0.y;
          u1[2 * p] = (__bf16)v1.x; u1[2 * p + 1] = (__bf16)v1.y;
        }
        if constexpr (PF) {   // a tile outside the utterance is the convs' zero padding (the PF gate
          const int ts = tg + k * 32;   // updates every tile, so its x is not zero there)
          if (ts < 0 || ts >= Le) { u0 = bf16x8{}; u1 = bf16x8{}; }
        }
        __bf16* dst = &U[(k * 32 + n + UOFF) * LB_LD + 16 * h];
        *reinterpret_cast<bf16x8*>(dst) = u0;
        *reinterpret_cast<bf16x8*>(dst + 8) = u1;
      }
    }
    __syncthreads();
    LB_STAMP(2 + 3 * l);
    // (2) y^T = lrelu(W_c . [u(t-d); u(t); u(t+d)]^T + b): A = weights (rows = out channel,
    //     k in kernel order), B = u rows.  Pre-conv tile kp -> Y index [32kp, 32kp+32) = rows - 1.
    {
      bf16x8 wf[6];
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
        if constexpr (WW) {
          wf[kk] = WCL[(l * 6 + kk) * 64 + lane];
        } else {
          const __bf16* w = P.Wc[l] + n * 96 + (kk >> 1) * 32 + 16 * h + 4 * (kk & 1);
          const bf16x4 w0 = *reinterpret_cast<const bf16x4*>(w), w1 = *reinterpret_cast<const bf16x4*>(w + 8);
          wf[kk] = bf16x8{w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
        }
      }
      f32x2 bias[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 bv = *reinterpret_cast<const float4*>((WW ? &BCL[l * CI] : P.bc[l]) + 8 * i + 4 * h);
        bias[2 * i] = f32x2{bv.x, bv.y}; bias[2 * i + 1] = f32x2{bv.z, bv.w};
      }
      // a wave's pre-conv tiles kp0 = kf + wave and kp1 = kp0 + NW (NG <= 2 NW: no third), their MFMA
      // chains interleaved when it has both -- the same per-tile MFMA order, so the same values
      auto pre_epi = [&](int kp, const f32x16& acc) {
        f32x2 v[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) v[p] = lrelu2(f32x2{acc[2 * p], acc[2 * p + 1]} + bias[p]);
        const int tt = tg + kp * 32 - 1;                  // the tile's first time (wave-uniform)
        if (tt < 0 || tt + 31 >= Le) {                    // utterance-edge tile: zero-pad
          const int t = tt + n;
          const bool in = t >= 0 && t < Le;           // select, not multiply: stale LDS may be NaN
#pragma unroll
          for (int p = 0; p < 8; ++p) v[p] = in ? v[p] : f32x2{0.f, 0.f};
        }
        bf16x8 y0, y1;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          y0[2 * p] = (__bf16)v[p].x; y0[2 * p + 1] = (__bf16)v[p].y;
          y1[2 * p] = (__bf16)v[4 + p].x; y1[2 * p + 1] = (__bf16)v[4 + p].y;
        }
        __bf16* dst = &Y[(kp * 32 + n) * LB_LD + 16 * h];
        *reinterpret_cast<bf16x8*>(dst) = y0;
        *reinterpret_cast<bf16x8*>(dst + 8) = y1;
      };
      static_assert(NG <= 2 * NW, "at most two pre-conv tiles per wave");
      const int kp0 = kf + wave, kp1 = kp0 + NW;
      auto urow = [&](int kp, int kk) {
        return *reinterpret_cast<const bf16x8*>(
            &U[(kp * 32 + n + UOFF - 1 + ((kk >> 1) - 1) * d) * LB_LD + 16 * (kk & 1) + 8 * h]);
      };
      if (kp1 <= kpl) {
        f32x16 a0, a1;
#pragma unroll
        for (int q = 0; q < 16; ++q) { a0[q] = 0.f; a1[q] = 0.f; }
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) {
          const bf16x8 b0 = urow(kp0, kk), b1 = urow(kp1, kk);
          a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[kk], b0, a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[kk], b1, a1, 0, 0, 0);
        }
        pre_epi(kp0, a0);
        pre_epi(kp1, a1);
      } else if (kp0 <= kpl) {
        f32x16 a0;
#pragma unroll
        for (int q = 0; q < 16; ++q) a0[q] = 0.f;
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[kk], urow(kp0, kk), a0, 0, 0, 0);
        pre_epi(kp0, a0);
      }
    }
    __syncthreads();
    LB_STAMP(3 + 3 * l);
    // (3) o^T = K_frame . [y(t-1); y(t); y(t+1)]^T + Bf;  x += a + sigmoid(o_g) tanh(o_f)
    // K is pre-scaled (gate rows by -log2 e, filter rows by 2 log2 e): the accumulators are
    // the exp2 arguments.  z = x + a lives in registers: x_{l+1} = z_l + o, and
    // z_{l+1} = x_{l+1} + a except after the last layer.
    const f32x2 cg = {-LOG2E, -LOG2E}, cf = {2.f * LOG2E, 2.f * LOG2E};
    // bb: the frame's gate / filter biases (bb[i], bb[4 + i]: channels 8i + 4h ..), loaded by the
    // caller all at once -- null when they are folded into the accumulators (PF).  r05: read here, one
    // pair per channel group, they were four L2 round trips in a row per tile and layer (SUB asm)
    auto gate_update = [&](int j, const f32x16& g, const f32x16& f, const float4* bb, bool live) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x2 gs0 = {g[4 * i], g[4 * i + 1]}, gs1 = {g[4 * i + 2], g[4 * i + 3]};
        f32x2 fs0 = {f[4 * i], f[4 * i + 1]}, fs1 = {f[4 * i + 2], f[4 * i + 3]};
        if (bb) {   // bias not folded into the accumulators yet
          const float4 bg = bb[i];
          const float4 bl = bb[4 + i];
          gs0 = efma(f32x2{bg.x, bg.y}, cg, gs0);
          gs1 = efma(f32x2{bg.z, bg.w}, cg, gs1);
          fs0 = efma(f32x2{bl.x, bl.y}, cf, fs0);
          fs1 = efma(f32x2{bl.z, bl.w}, cf, fs1);
        }
        // o = (ef - 1) r with r = 1 / ((ef + 1)(eg + 1)), folded into x as fma(ef, r, x + a - r)
        // (5 packed ops per pair instead of 7: the layer loop is VALU-issue-bound)
        const f32x2 r0 = gate2r(gs0, fs0), r1 = gate2r(gs1, fs1);
        const f32x2 ef0 = gate2ef(fs0), ef1 = gate2ef(fs1);
        if (live) {
          const f32x2 t0 = (l + 1 < NLY ? xr[j][2 * i] + ar[j][2 * i] : xr[j][2 * i]) - r0;
          const f32x2 t1 = (l + 1 < NLY ? xr[j][2 * i + 1] + ar[j][2 * i + 1] : xr[j][2 * i + 1]) - r1;
          xr[j][2 * i] = efma(ef0, r0, t0);
          xr[j][2 * i + 1] = efma(ef1, r1, t1);
        } else if (l + 1 < NLY) {
          xr[j][2 * i] += ar[j][2 * i];
          xr[j][2 * i + 1] += ar[j][2 * i + 1];
        }
      }
    };
    if constexpr (PF) {
      // the pair's 24 MFMAs as 4 interleaved chains on the shared kernel, then the next layer's
      // prefetch, then the two gates.  Accumulators start from the frame's staged bias.
      f32x16 g[TPW], f[TPW];
      const float* bq = &BFL[((fpair - fbase) * NLY + l) * 2 * CI];
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 bg = *reinterpret_cast<const float4*>(bq + 8 * i + 4 * h);
          const float4 bl = *reinterpret_cast<const float4*>(bq + 32 + 8 * i + 4 * h);
          g[j][4 * i] = bg.x; g[j][4 * i + 1] = bg.y; g[j][4 * i + 2] = bg.z; g[j][4 * i + 3] = bg.w;
          f[j][4 * i] = bl.x; f[j][4 * i + 1] = bl.y; f[j][4 * i + 2] = bl.z; f[j][4 * i + 3] = bl.w;
        }
      }
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const bf16x8 yb = *reinterpret_cast<const bf16x8*>(
              &Y[(TILE(j) * 32 + n + (kk >> 1)) * LB_LD + 16 * (kk & 1) + 8 * h]);
          g[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kn[kk], yb, g[j], 0, 0, 0);
          f[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kn[6 + kk], yb, f[j], 0, 0, 0);
        }
      }
      if (l + 1 < NLY) kload(l + 1);
      // every tile is updated, with no branch between the tiles' gates (the compiler interleaves
      // them): a tile outside this layer's valid range is never read by a valid row, one outside
      // the utterance is zeroed where it is read (the u stage above, the final conv's partial sums)
#pragma unroll
      for (int j = 0; j < TPW; ++j) gate_update(j, g[j], f[j], nullptr, true);
    } else {
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int k = TILE(j), ts = tg + k * 32;
      if (k >= kf && k <= kl && ts >= 0 && ts < Le) {
        f32x16 g, f;
#pragma unroll
        for (int r = 0; r < 16; ++r) { g[r] = 0.f; f[r] = 0.f; }
        const float* bq;
        if constexpr (SUB) {
          // hop < 32: the tile spans 32/hop frames.  Column n belongs to frame (ts + n)/hop;
          // one MFMA chain per frame with the other frames' columns zeroed in B, so every
          // column accumulates exactly its own frame's kernel.
          const int f0 = ts / hop, fn = (ts + n) / hop;
          const int nf = min(32 / hop, Tc - f0);
          // the frames' kernel fragments in a 2-deep register pipeline: frame i + 1's loads are
          // in flight under frame i's MFMAs (a load-then-use chain per frame made this block a
          // series of L2 round trips: 79 us for one utterance vs 121 us for eight, r02)
          const __bf16* kq0 = P.Kf[l] + ((long long)b * Tc + f0) * KPERLAYER;
          bf16x8 ka[12], kb[12];
          auto kld = [&](bf16x8 (&d)[12], int i) {   // unconditional: rows past the last frame clamp
            const __bf16* kq = kq0 + (long long)min(i, nf - 1) * KPERLAYER;
#pragma unroll
            for (int kk = 0; kk < 12; ++kk) d[kk] = *reinterpret_cast<const bf16x8*>(kq + (kk * 64 + lane) * 8);
            __builtin_amdgcn_sched_barrier(0);    // keep the loads here (the scheduler sinks them to their use)
          };
          auto kmm = [&](const bf16x8 (&kf)[12], int i) {
            const bool mine = fn == f0 + i;
#pragma unroll
            for (int kk = 0; kk < 6; ++kk) {
              // B operand re-read from LDS per frame (registers go to the kernel pipeline)
              const bf16x8 yv = *reinterpret_cast<const bf16x8*>(&Y[(k * 32 + n + (kk >> 1)) * LB_LD + 16 * (kk & 1) + 8 * h]);
              const bf16x8 z = {};
              const bf16x8 ym = mine ? yv : z;
              g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kk], ym, g, 0, 0, 0);
              f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[6 + kk], ym, f, 0, 0, 0);
            }
          };
          kld(ka, 0);
          for (int i = 0; i < nf; i += 2) {
            kld(kb, i + 1);
            kmm(ka, i);
            if (i + 1 < nf) {
              kld(ka, i + 2);
              kmm(kb, i + 1);
            }
          }
          bq = P.Bf + ((long long)b * Tc + (fn < Tc ? fn : Tc - 1)) * (2 * CI * NLY) + l * 2 * CI;
        } else {
          const int frame = ts / hop;
          const __bf16* kq = P.Kf[l] + ((long long)b * Tc + frame) * KPERLAYER;
          bq = P.Bf + ((long long)b * Tc + frame) * (2 * CI * NLY) + l * 2 * CI;
#pragma unroll
          for (int kk = 0; kk < 6; ++kk) {
            const int tap = kk >> 1;
            const bf16x8 yb = *reinterpret_cast<const bf16x8*>(&Y[(k * 32 + n + tap) * LB_LD + 16 * (kk & 1) + 8 * h]);
            const bf16x8 kg = *reinterpret_cast<const bf16x8*>(kq + (kk * 64 + lane) * 8);
            const bf16x8 kt = *reinterpret_cast<const bf16x8*>(kq + ((6 + kk) * 64 + lane) * 8);
            g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kg, yb, g, 0, 0, 0);
            f = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kt, yb, f, 0, 0, 0);
          }
        }
        // hop < 32: a tile can straddle the utterance end; rows past it stay zero
        // (they are the next layer's conv padding)
        float4 bb[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bb[i] = *reinterpret_cast<const float4*>(bq + 8 * i + 4 * h);
          bb[4 + i] = *reinterpret_cast<const float4*>(bq + 32 + 8 * i + 4 * h);
        }
        __builtin_amdgcn_sched_barrier(0);   // all eight in flight together
        gate_update(j, g, f, bb, !SUB || ts + n < Le);
      }
    }
    }
    if (l < NLY - 1) LB_STAMP(4 + 3 * l);
  }
  LB_STAMP(14);
  if constexpr (FIN) {
    // eps(t) = b + sum_tap E[t + tap - 3][tap],  E[r][tap] = sum_c w[tap][c] x(r)[c]: each lane
    // forms the 7 per-tap partial sums of its row from the x it holds (16 channels; the two
    // channel halves meet by one lane swap), so only 7 floats per row go through LDS
    // (aliasing U/Y: every wave is past its Y reads).  r03: the final conv read 28 x 16 B of
    // fp32 x rows plus 28 x 16 B of weights per output sample from LDS -- 12% of the block.
    float* E = XS;                                   // [GR rows][8]
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int k = TILE(j), row = k * 32 + n;
      if (k >= 1 && k <= NG - 2) {
        float st[7];
#pragma unroll
        for (int tap = 0; tap < 7; ++tap) {
          f32x2 acc = {0.f, 0.f};
#pragma unroll
          for (int i = 0; i < 4; ++i) {             // channels 8i + 4h .. +3 = regs 4i .. 4i+3
            const float4 w = *reinterpret_cast<const float4*>(&FWF[tap * 32 + 8 * i + 4 * h]);
            acc = efma(xr[j][2 * i], f32x2{w.x, w.y}, acc);
            acc = efma(xr[j][2 * i + 1], f32x2{w.z, w.w}, acc);
          }
          st[tap] = acc.x + acc.y;
        }
#pragma unroll
        for (int tap = 0; tap < 7; ++tap) st[tap] += __shfl_xor(st[tap], 32);
        if constexpr (PF) {   // x is zero outside the utterance (the final conv's padding)
          const int ts = tg + k * 32;
          if (ts < 0 || ts >= Le) {
#pragma unroll
            for (int tap = 0; tap < 7; ++tap) st[tap] = 0.f;
          }
        }
        if (h == 0) {
          *reinterpret_cast<float4*>(&E[row * 8]) = make_float4(st[0], st[1], st[2], st[3]);
          *reinterpret_cast<float4*>(&E[row * 8 + 4]) = make_float4(st[4], st[5], st[6], 0.f);
        }
      }
    }
    __syncthreads();
    // one thread per output sample: x_t from the staged audio (AS[i] is time tg - 3 + i,
    // t = tg + 64 + s), the sampler update (util.py:222-226)
    constexpr int IS = (TS + G::NT - 1) / G::NT;
#pragma unroll
    for (int it = 0; it < IS; ++it) {
      const int s = tid + it * G::NT, t = t0 + s;
      if (s < TS && t < Lh) {
        float e = bfin;
#pragma unroll
        for (int tap = 0; tap < 7; ++tap) e += E[(64 + s + tap - 3) * 8 + tap];
        float v = (AS[67 + s] - P.ce * e) / P.den;
        if (P.sig != 0.f) v += P.sig * zr[it];
        P.audio_out[base + t] = v;
      }
    }
  } else {
    // centre tiles [2, 2 + TS/32) -> x out
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int k = TILE(j), t = tg + k * 32 + n;
      if (k >= 2 && k < 2 + TS / 32 && t < Lh) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<float4*>(P.xout + (base + t) * CI + 8 * i + 4 * h) =
              make_float4(xr[j][2 * i].x, xr[j][2 * i].y, xr[j][2 * i + 1].x, xr[j][2 * i + 1].y);
      }
    }
  }
  LB_STAMP(15);
#undef TILE
}

// ------------------------------------------------------------------ persistent final block (r06)
// LDS-DMA by inline asm: one global_load_lds per wave (M0 = the wave's LDS destination, lane i's `bytes`
// land at M0 + i * bytes).  Not the builtin: hipcc cannot tell the DMA's LDS destination from the U / Y
// windows, so after a builtin DMA it waited vmcnt(0) -- for the DMA itself -- before every later LDS access.
// Hidden from the waitcnt pass, the DMA must be OLDER than every load the pass waits on while it is in
// flight (vmcnt retires in order): it is issued right after a tile's layer-0 MFMAs, before the layer-1
// kernel fragments, and waited for explicitly (vmcnt at the next tile's top).  The asm sets M0, which hipcc
// treats as reserved: this kernel has no other M0 use (no LDS-DMA builtin, no indirect register indexing).
__device__ __forceinline__ void lds_dma16(const void* g, void* lds) {
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lds);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(l), "v"(g) : "memory");
}
__device__ __forceinline__ void lds_dma4(const void* g, void* lds) {
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lds);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(l), "v"(g) : "memory");
}
// lvc_block_bf16_kernel<384, UPS, AUD, FIN, PF> as a persistent kernel (FD_OPT_LVC_PS): one 8-wave block
// per CU walks the launch's tiles in the same XCD-aware order.  Each tile's prologue loads -- the audio
// window, the x_prev rows, the frames' LVC biases -- arrive by LDS-DMA (global_load_lds) issued during the
// PREVIOUS tile's layers, and layer 0's kernel fragments by register loads issued after the previous
// tile's last LVC MFMAs: the phase probe (tools/lvc_probe, profiles/r06_ab/lvc_xprev_bf16_ab.txt) put 15%
// of a one-tile block's life in waiting for those loads, with one block per CU and nothing to overlap them.
// The tile-invariant operands (pre-conv weights and biases, first / final conv, upsample bias) are staged
// once per block.  DMA'd values land raw: the masks (zero outside the utterance) and the gate pre-scale of
// the biases are applied in place in the tile's prologue or where they are read -- the same values the
// one-tile kernel stores, so the same arithmetic, roundings and MFMA order: bit-identical
// (tests/test_gpu_bf16.py).
#ifdef LB_TRACE
// tools/lvc_probe ps mode: per-phase s_memtime stamps of iteration 5 of every 4th block, lane 0 of each wave
#define PS_STAMP(i)                                                                                        \
  do {                                                                                                     \
    if (it == 5 && (tq & 63) == 0 && blockIdx.x % 4 == 0)                                                  \
      P.trace[((blockIdx.x / 4) * NW + (tq >> 6)) * 24 + (i)] = __builtin_readcyclecounter();              \
  } while (0)
#else
#define PS_STAMP(i) \
  do {              \
  } while (0)
#endif
// FINAL = the sampler's last block (upsample r = 4, first conv, final conv + sampler update; hop 256); !FINAL
// (r06) = the hop-64 block (upsample r = 8, audio_down from HBM, x out), the one-tile kernel's <384, UPS, PF>.
template <bool FINAL>
__global__ __launch_bounds__(512, 1) void lvc_ps_kernel(const LvcBlockArgs P, int ntx, int ntiles) {
  constexpr int TS = 384, TPW = 2;
  using G = LbGeo<TS, TPW>;
  constexpr int NW = G::NW, NG = G::NG, UOFF = G::UOFF, GR = NG * 32, EX = FINAL ? 3 : 0, NT = G::NT;
  constexpr int BFR = GR / (FINAL ? 256 : 64) + 2;      // frames a tile touches at hop 256 / 64 (host-checked)
  constexpr int XROWS = G::NTJ_MAX * 32 + 1, XROWS8 = (XROWS + 7) / 8 * 8;   // x_prev rows (r >= 4: <= 161)
  constexpr int NAS = GR + 6, NAS64 = (NAS + 63) / 64 * 64;                  // audio samples of a tile
  constexpr int FA = FINAL ? 1 : 0;                     // (the audio / first / final conv arrays: FINAL only)
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  __shared__ __attribute__((aligned(16))) float AS[2][FINAL ? NAS64 : 4];   // audio, times tg - 3 + i (raw)
  __shared__ __attribute__((aligned(16))) float XPN[XROWS8 * CI];           // x_prev rows jb + rr (raw)
  __shared__ __attribute__((aligned(16))) float BFL[2][BFR * 2 * CI * NLY]; // frames' LVC biases (pre-scaled)
  __shared__ __attribute__((aligned(16))) float FW[FA ? 7 * 32 : 4];
  __shared__ __attribute__((aligned(16))) float FWF[FA ? 7 * 32 : 4];
  __shared__ __attribute__((aligned(16))) float FBL[FA ? 32 : 4];
  __shared__ __attribute__((aligned(16))) float BUL[32];
  __shared__ __attribute__((aligned(16))) bf16x8 WCL[NLY * 6 * 64];
  __shared__ __attribute__((aligned(16))) float BCL[NLY * CI];
  __shared__ float EB[FA ? 8 : 1][2][3][8];                                  // FIN: pairs' outer E rows
  __bf16* U = reinterpret_cast<__bf16*>(smem);
  __bf16* Y = U + G::UROWS * LB_LD;
  float* XS = reinterpret_cast<float*>(smem);
  __bf16* XP = reinterpret_cast<__bf16*>(smem + G::XS_BYTES);
  const int tid = threadIdx.x;
  const int Tc = P.Tc, hop = P.hop, Lh = Tc * hop;
  const int r = P.r, pp = P.p, Tin = Lh / r;
  const int ntj = (GR / r + 2 + 31) / 32;
  constexpr int RLO = 64 - 44 - EX, RHI = 64 + TS + 44 + EX;
  // ---- tile-invariant operands, once per block
  if constexpr (FINAL) {
    if (tid < 224) FW[tid] = P.fw[(tid & 31) * 7 + (tid >> 5)];
    if (tid < 32) FBL[tid] = P.fb[tid];
    if (tid < 224) FWF[tid] = P.wfin[tid];
  }
  if (tid < 32) BUL[tid] = P.bup[tid];
  if (tid < 6 * 64) {
    const int kk = tid >> 6, ln = tid & 63;
#pragma unroll
    for (int l = 0; l < NLY; ++l) {
      const __bf16* w = P.Wc[l] + (ln & 31) * 96 + (kk >> 1) * 32 + 16 * (ln >> 5) + 4 * (kk & 1);
      const bf16x4 w0 = *reinterpret_cast<const bf16x4*>(w), w1 = *reinterpret_cast<const bf16x4*>(w + 8);
      WCL[l * 384 + tid] = bf16x8{w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
    }
  }
  if (tid < NLY * CI) BCL[tid] = P.bc[tid / CI][tid % CI];
  const float bfin = FINAL ? P.bfin[0] : 0.f;
  // tile v -> (utterance, time tile): the one-tile kernel's XCD-aware order (gridDim.x % 8 == 0, so tile v
  // runs on the XCD of block v % gridDim.x, as block v did there)
  auto coords = [&](int v, int& b, int& bx) {
    const int xcd = v & 7, slot = v >> 3, per = ntiles >> 3, rem = ntiles & 7;
    const int logical = xcd < rem ? xcd * (per + 1) + slot : rem * (per + 1) + (xcd - rem) * per + slot;
    b = __builtin_amdgcn_readfirstlane(logical / ntx);   // (uniform: scalar loads of lens / uid)
    bx = __builtin_amdgcn_readfirstlane(logical - b * ntx);
  };
  // a tile's loads straight into LDS (buffer s of AS / BFL, and XPN)
  auto dma = [&](int v, int s, int wave, int lane) {
    int b, bx;
    coords(v, b, bx);
    const int tg = bx * TS - 64, jb = floordiv(tg + pp, r) - 2, fbase = (tg > 0 ? tg : 0) / hop;
    const long long base = (long long)b * Lh;
    if constexpr (FINAL) {
#pragma unroll
      for (int q0 = 0; q0 < NAS64 / 64; q0 += NW) {        // 4-B pieces, one sample per lane
        const int q = q0 + wave;
        if (q * 64 < NAS) {
          const int t = tg - 3 + q * 64 + lane;
          lds_dma4(P.audio + base + min(max(t, 0), Lh - 1), &AS[s][q * 64]);
        }
      }
    }
#pragma unroll
    for (int q0 = 0; q0 < XROWS8 / 8; q0 += NW) {          // 16-B pieces, 8 rows of 32 channels per wave
      const int q = q0 + wave;
      if (q * 8 < XROWS) {
        const int j = min(max(jb + q * 8 + (lane >> 3), 0), Tin - 1);
        lds_dma16(P.xin + ((long long)b * Tin + j) * CI + (lane & 7) * 4, &XPN[q * 8 * CI]);
      }
    }
#pragma unroll
    for (int f0 = 0; f0 < BFR; f0 += NW) {                  // one frame (256 floats) per wave and piece
      const int fq = f0 + wave;
      if (fq < BFR) {
        const int fr = min(fbase + fq, Tc - 1);
        lds_dma16(P.Bf + ((long long)b * Tc + fr) * (2 * CI * NLY) + lane * 4, &BFL[s][fq * 2 * CI * NLY]);
      }
    }
  };
  bf16x8 kn[12];
  auto kload = [&](int b, int fpair, int l, int lane) {
    const __bf16* kq = P.Kf[l] + ((long long)b * Tc + fpair) * KPERLAYER;
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) kn[kk] = *reinterpret_cast<const bf16x8*>(kq + (kk * 64 + lane) * 8);
  };
  auto fpair_of = [&](int tg, int wave) { return min(max(tg + 32 * TPW * wave + 16 * TPW, 0) / hop, Tc - 1); };
  // a tile's utterance end and utterance id, loaded a tile ahead (at the DMA) by unconditional loads from a
  // selected pointer: under `P.lens ?` / `P.uid ?` branches the waitcnt pass waited vmcnt(0) at the join --
  // for the DMA and the kernel-fragment loads in flight
  // (raw values only: used -- and so waited for -- at the next tile's top, both loads in flight together;
  // r06 probe: computed at the load, they cost two serial round trips inside layer 0)
  int lv_n = 0, uv_n = 0;
  float zn_n = 0.f;     // the explicit sampler draw of thread tq's sample tq - 64 (P.noise; unconditional load)
  auto tile_scalars = [&](int v, int tq) {
    int b, bx;
    coords(v, b, bx);
    lv_n = *(P.lens ? P.lens + b : reinterpret_cast<const int*>(P.Bf));
    if constexpr (FINAL) {
      uv_n = *(P.uid ? P.uid + b + P.b_off : reinterpret_cast<const int*>(P.Bf));
      zn_n = (P.noise ? P.noise : P.audio)[(long long)b * Lh + min(max(bx * TS + tq - 64, 0), Lh - 1)];
    }
  };
  const int v0 = blockIdx.x;
  __syncthreads();                                         // the invariant operands are staged
  if (v0 < ntiles) {
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    int b, bx;
    coords(v0, b, bx);
    tile_scalars(v0, tid);
    dma(v0, 0, wave, lane);
    kload(b, fpair_of(bx * TS - 64, wave), 0, lane);
  }
  int it = 0;
  for (int v = v0; v < ntiles; v += gridDim.x, ++it) {
    const int cur = it & 1;
    // thread ids through an opaque copy: addresses derived from them are recomputed per tile instead of
    // hoisted out of the loop and spilled
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int lane = tq & 63, n = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tq >> 6);
    // the next tile, pinned in an SGPR here: rematerialised where it is used, its kernarg load waited
    // lgkmcnt(0) -- for the LDS reads in flight -- inside the layer-0 MFMAs
    int vnext = v + (int)gridDim.x;
    asm volatile("" : "+s"(vnext));
    PS_STAMP(0);
    int b, bx;
    coords(v, b, bx);
    const int Le = P.lens ? min(__builtin_amdgcn_readfirstlane(lv_n), Tc) * hop : Lh;
    const unsigned uidv = !FINAL ? 0u : P.uid ? (unsigned)__builtin_amdgcn_readfirstlane(uv_n) : (unsigned)(b + P.b_off);
    const int t0 = bx * TS, tg = t0 - 64;
    const long long base = (long long)b * Lh;
    const int Tin_e = Le / r;
    const int fbase = (tg > 0 ? tg : 0) / hop;
    const int jb = floordiv(tg + pp, r) - 2;
    const int fpair = fpair_of(tg, wave);
    // this tile's DMA (issued a tile ago) has landed for every wave: each waits for its own pieces -- the
    // 12 younger kernel-fragment loads (and at most one audio_out store; !FINAL: 8 x stores) may stay in
    // flight -- then a barrier
    constexpr int VMY = FINAL ? 12 : 20;
    __builtin_amdgcn_s_waitcnt((VMY & 15) | ((VMY >> 4) << 14) | 0x0F70);   // vmcnt(VMY)
    __syncthreads();
    PS_STAMP(1);
    // phase-GEMM weights (NW % r == 0: wave w computes phase w % r), FIN noise
    bf16x8 wfj[4];
    {
      const __bf16* wa = P.Wup + ((long long)(wave % r) * 32 + n) * 64 + 8 * h;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wfj[kk] = *reinterpret_cast<const bf16x8*>(wa + kk * 16);
    }
    // !FINAL: the tile's audio_down rows (x += a, modules.py:209) straight into registers, loaded here so
    // their HBM round trip runs under the XP fill and the phase GEMMs (unconditional at clamped rows,
    // masked where they are used)
    float4 araw[TPW][4];
    if constexpr (!FINAL) {
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int t = min(max(tg + (2 * wave + j) * 32 + n, 0), Lh - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) araw[j][i] = *reinterpret_cast<const float4*>(P.a + (base + t) * CI + 8 * i + 4 * h);
      }
    }
    // (the explicit draw loaded a tile ahead, unconditionally: under `P.noise ?` the waitcnt pass waited for
    // every outstanding load -- the next tile's kernel fragments included -- at the join)
    const float znz = zn_n;
    // (thread tq writes sample s = tq - 64: lane (n, h) of wave w holds row 64 w + 32 h + n of the window)
    const int so = tq - 64;
    float zr = 0.f;
    if constexpr (FINAL) {
      const float zph = philox_normal_u(P.seed, uidv, (unsigned)(t0 + so), P.stream);
      zr = (so >= 0 && so < TS && t0 + so < Lh && P.sig != 0.f) ? (P.noise ? znz : zph) : 0.f;
      // audio samples outside the utterance -> 0 in place (the one-tile kernel's masked staging: the DMA
      // lands raw values; only the out-of-range ones are rewritten, so no LDS read)
#pragma unroll
      for (int ia = 0; ia < NAS64 / NT + 1; ++ia) {
        const int i = tq + ia * NT, t = tg - 3 + i;
        if (i < NAS && (t < 0 || t >= Le)) AS[cur][i] = 0.f;
      }
    }
    // the frames' LVC biases: the gate pre-scale the one-tile kernel applies at staging, once per tile in
    // place (read from the LVC phases on, past the barriers below)
    {
      float* bfs = BFL[cur];
#pragma unroll
      for (int ib = 0; ib < (BFR * 2 * CI * NLY + NT - 1) / NT; ++ib) {
        const int i = tq + ib * NT;
        if (i < BFR * 2 * CI * NLY) bfs[i] *= (i & 63) < 32 ? -LOG2E : 2.f * LOG2E;
      }
    }
    // (a) XP[j - jb] = bf16 lrelu(x_prev[j]), zero outside the utterance
    constexpr int IX = ((G::NTJ_MAX * 32 + 1) * 8 + NT - 1) / NT;
#pragma unroll
    for (int itx = 0; itx < IX; ++itx) {
      const int i = tq + itx * NT, rr = i >> 3, q = (i & 7) * 4, j = jb + rr;
      if (i < (ntj * 32 + 1) * 8) {
        const float m = (j >= 0 && j < Tin_e) ? 1.f : 0.f;
        const float4 xv = *reinterpret_cast<const float4*>(&XPN[rr * CI + q]);
        const f32x2 u0 = lrelu2(f32x2{xv.x, xv.y} * m), u1 = lrelu2(f32x2{xv.z, xv.w} * m);
        *reinterpret_cast<bf16x4*>(&XP[rr * LB_LD + q]) = bf16x4{(__bf16)u0.x, (__bf16)u0.y, (__bf16)u1.x, (__bf16)u1.y};
      }
    }
    __syncthreads();
    PS_STAMP(2);
    // (b) phase GEMMs: C^T[co][col] = [W_k^T | W_{k+r}^T] . [xp(j0); xp(j0 - 1)], t = r j0 + k - p
    {
      const int k = wave % r;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int jt = wave / r + qq * (NW / r);
        if (jt < ntj) {
          f32x16 acc;
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const bf16x8 xb = *reinterpret_cast<const bf16x8*>(
                &XP[(jt * 32 + n + (kk < 2 ? 1 : 0)) * LB_LD + 16 * (kk & 1) + 8 * h]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wfj[kk], xb, acc, 0, 0, 0);
          }
          const int j0 = jb + 1 + jt * 32 + n, row = r * j0 + k - pp - tg;
          if (row >= RLO && row < RHI) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const float4 bv = *reinterpret_cast<const float4*>(&BUL[8 * g + 4 * h]);
              *reinterpret_cast<float4*>(&XS[row * LB_XLD + 8 * g + 4 * h]) =
                  make_float4(acc[4 * g] + bv.x, acc[4 * g + 1] + bv.y, acc[4 * g + 2] + bv.z, acc[4 * g + 3] + bv.w);
            }
          }
        }
      }
    }
    __syncthreads();
    PS_STAMP(3);
    // x rows -> registers: z = x + a, a = first_conv(audio) in first_conv_kernel's order -- from the bias,
    // taps ascending: taps 0..5 as three v_mfma_f32_32x32x2_f32 (exact f32, bitwise the fmaf chain; A = two
    // taps' weights, B = the tile's audio rows shifted by those taps; D lands in the x registers' layout),
    // tap 6 by fmaf.  (The VALU chain: 112 fmaf and 28 16-B LDS reads per lane and tile.)
    f32x2 xr[TPW][8], ar[TPW][8];
    const float* as = AS[cur];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int k = 2 * wave + j, row = k * 32 + n, t = tg + row;
      const bool ok = row >= RLO && row < RHI && t >= 0 && t < Le;
      if constexpr (!FINAL) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), av = xv;
          if (ok) {
            xv = *reinterpret_cast<const float4*>(&XS[row * LB_XLD + 8 * i + 4 * h]);
            av = araw[j][i];
          }
          xr[j][2 * i] = f32x2{xv.x + av.x, xv.y + av.y}; xr[j][2 * i + 1] = f32x2{xv.z + av.z, xv.w + av.w};
          ar[j][2 * i] = f32x2{av.x, av.y}; ar[j][2 * i + 1] = f32x2{av.z, av.w};
        }
      } else {
      f32x16 fa;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 bv = *reinterpret_cast<const float4*>(&FBL[8 * i + 4 * h]);
        fa[4 * i] = bv.x; fa[4 * i + 1] = bv.y; fa[4 * i + 2] = bv.z; fa[4 * i + 3] = bv.w;
      }
#pragma unroll
      for (int q = 0; q < 3; ++q)   // (every lane, masked rows too: row + 6 < NAS, staged finite samples)
        fa = __builtin_amdgcn_mfma_f32_32x32x2f32(FW[(2 * q + h) * 32 + n], as[row + 2 * q + h], fa, 0, 0, 0);
      const float s6 = as[row + 6];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 w = *reinterpret_cast<const float4*>(&FW[6 * 32 + 8 * i + 4 * h]);
        float4 av = make_float4(fmaf(w.x, s6, fa[4 * i]), fmaf(w.y, s6, fa[4 * i + 1]),
                                fmaf(w.z, s6, fa[4 * i + 2]), fmaf(w.w, s6, fa[4 * i + 3]));
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) xv = *reinterpret_cast<const float4*>(&XS[row * LB_XLD + 8 * i + 4 * h]);
        else av = xv;
        xr[j][2 * i] = f32x2{xv.x + av.x, xv.y + av.y}; xr[j][2 * i + 1] = f32x2{xv.z + av.z, xv.w + av.w};
        ar[j][2 * i] = f32x2{av.x, av.y}; ar[j][2 * i + 1] = f32x2{av.z, av.w};
      }
      }
    }
    __syncthreads();                                       // XS reads done before U / Y (aliased) are written
    PS_STAMP(4);
    if (P.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    const float* bfl = BFL[cur];
#pragma unroll
    for (int l = 0; l < NLY; ++l) {
      const int d = l == 0 ? 1 : l == 1 ? 3 : l == 2 ? 9 : 27;
      const int e = (l == 0 ? 42 : l == 1 ? 38 : l == 2 ? 28 : 0) + EX;
      const int kf = (64 - e) / 32, kl = (64 + TS + e - 1) / 32;
      const int kpl = kl + 1 < NG - 1 ? kl + 1 : NG - 1;
      // (1) u = lrelu(z) of the owned tiles the pre-conv reads
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int k = 2 * wave + j;
        if (k >= kf - 1 && k <= kl + 2) {
          bf16x8 u0, u1;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const f32x2 v0 = lrelu2(xr[j][p]), v1 = lrelu2(xr[j][4 + p]);
            u0[2 * p] = (__bf16)v0.x; u0[2 * p + 1] = (__bf16)v0.y;
            u1[2 * p] = (__bf16)v1.x; u1[2 * p + 1] = (__bf16)v1.y;
          }
          const int ts = tg + k * 32;
          if (ts < 0 || ts >= Le) { u0 = bf16x8{}; u1 = bf16x8{}; }
          __bf16* dst = &U[(k * 32 + n + UOFF) * LB_LD + 16 * h];
          *reinterpret_cast<bf16x8*>(dst) = u0;
          *reinterpret_cast<bf16x8*>(dst + 8) = u1;
        }
      }
      __syncthreads();
      PS_STAMP(5 + 3 * l);
      // (2) y^T = lrelu(W_c . [u(t-d); u(t); u(t+d)]^T + b)
      {
        bf16x8 wf[6];
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) wf[kk] = WCL[(l * 6 + kk) * 64 + lane];
        f32x2 bias[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 bv = *reinterpret_cast<const float4*>(&BCL[l * CI + 8 * i + 4 * h]);
          bias[2 * i] = f32x2{bv.x, bv.y}; bias[2 * i + 1] = f32x2{bv.z, bv.w};
        }
        // a wave's pre-conv tiles kp0 = kf + wave and kp1 = kp0 + NW (NG <= 2 NW: no third), their
        // MFMA chains interleaved -- the same per-tile MFMA order, so the same values
        auto pre_epi = [&](int kp, const f32x16& acc) {
          f32x2 vv[8];
#pragma unroll
          for (int p = 0; p < 8; ++p) vv[p] = lrelu2(f32x2{acc[2 * p], acc[2 * p + 1]} + bias[p]);
          const int tt = tg + kp * 32 - 1;
          if (tt < 0 || tt + 31 >= Le) {
            const int t = tt + n;
            const bool in = t >= 0 && t < Le;
#pragma unroll
            for (int p = 0; p < 8; ++p) vv[p] = in ? vv[p] : f32x2{0.f, 0.f};
          }
          bf16x8 y0, y1;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            y0[2 * p] = (__bf16)vv[p].x; y0[2 * p + 1] = (__bf16)vv[p].y;
            y1[2 * p] = (__bf16)vv[4 + p].x; y1[2 * p + 1] = (__bf16)vv[4 + p].y;
          }
          __bf16* dst = &Y[(kp * 32 + n) * LB_LD + 16 * h];
          *reinterpret_cast<bf16x8*>(dst) = y0;
          *reinterpret_cast<bf16x8*>(dst + 8) = y1;
        };
        static_assert(NG <= 2 * NW, "at most two pre-conv tiles per wave");
        const int kp0 = kf + wave, kp1 = kp0 + NW;
        auto urow = [&](int kp, int kk) {
          return *reinterpret_cast<const bf16x8*>(
              &U[(kp * 32 + n + UOFF - 1 + ((kk >> 1) - 1) * d) * LB_LD + 16 * (kk & 1) + 8 * h]);
        };
        if (kp1 <= kpl) {
          f32x16 a0, a1;
#pragma unroll
          for (int q = 0; q < 16; ++q) { a0[q] = 0.f; a1[q] = 0.f; }
#pragma unroll
          for (int kk = 0; kk < 6; ++kk) {
            const bf16x8 b0 = urow(kp0, kk), b1 = urow(kp1, kk);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[kk], b0, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[kk], b1, a1, 0, 0, 0);
          }
          pre_epi(kp0, a0);
          pre_epi(kp1, a1);
        } else if (kp0 <= kpl) {
          f32x16 a0;
#pragma unroll
          for (int q = 0; q < 16; ++q) a0[q] = 0.f;
#pragma unroll
          for (int kk = 0; kk < 6; ++kk) a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[kk], urow(kp0, kk), a0, 0, 0, 0);
          pre_epi(kp0, a0);
        }
      }
      __syncthreads();
      PS_STAMP(6 + 3 * l);
      // (3) o^T = K_frame . [y(t-1); y(t); y(t+1)]^T + Bf;  x += a + sigmoid(o_g) tanh(o_f)
      f32x16 g[TPW], f[TPW];
      const float* bq = &bfl[((fpair - fbase) * NLY + l) * 2 * CI];
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // (pre-scaled in the prologue)
          const float4 bg = *reinterpret_cast<const float4*>(bq + 8 * i + 4 * h);
          const float4 bl = *reinterpret_cast<const float4*>(bq + 32 + 8 * i + 4 * h);
          g[j][4 * i] = bg.x; g[j][4 * i + 1] = bg.y; g[j][4 * i + 2] = bg.z; g[j][4 * i + 3] = bg.w;
          f[j][4 * i] = bl.x; f[j][4 * i + 1] = bl.y; f[j][4 * i + 2] = bl.z; f[j][4 * i + 3] = bl.w;
        }
      }
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const bf16x8 yb = *reinterpret_cast<const bf16x8*>(
              &Y[((2 * wave + j) * 32 + n + (kk >> 1)) * LB_LD + 16 * (kk & 1) + 8 * h]);
          g[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kn[kk], yb, g[j], 0, 0, 0);
          f[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kn[6 + kk], yb, f[j], 0, 0, 0);
        }
      }
      // the next tile's DMA after layer 0's MFMAs (its XPN was read in this tile's prologue, its AS / BFL
      // buffer cur ^ 1 by the previous tile), ahead of the kernel-fragment loads
      if (l == 0) PS_STAMP(18);
      if (l == 0 && vnext < ntiles) {                 // (the scalars' loads first: waiting for them is not
        tile_scalars(vnext, tq);                       // waiting for the DMA)
        dma(vnext, cur ^ 1, wave, lane);
      }
      if (l + 1 < NLY) {
        kload(b, fpair, l + 1, lane);
      } else if (vnext < ntiles) {                         // the next tile's layer-0 fragments
        int b2, bx2;
        coords(vnext, b2, bx2);
        kload(b2, fpair_of(bx2 * TS - 64, wave), 0, lane);
      }
      if (l == 0) PS_STAMP(19);
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x2 gs0 = {g[j][4 * i], g[j][4 * i + 1]}, gs1 = {g[j][4 * i + 2], g[j][4 * i + 3]};
          const f32x2 fs0 = {f[j][4 * i], f[j][4 * i + 1]}, fs1 = {f[j][4 * i + 2], f[j][4 * i + 3]};
          const f32x2 r0 = gate2r(gs0, fs0), r1 = gate2r(gs1, fs1);
          const f32x2 ef0 = gate2ef(fs0), ef1 = gate2ef(fs1);
          const f32x2 q0 = (l + 1 < NLY ? xr[j][2 * i] + ar[j][2 * i] : xr[j][2 * i]) - r0;
          const f32x2 q1 = (l + 1 < NLY ? xr[j][2 * i + 1] + ar[j][2 * i + 1] : xr[j][2 * i + 1]) - r1;
          xr[j][2 * i] = efma(ef0, r0, q0);
          xr[j][2 * i + 1] = efma(ef1, r1, q1);
        }
      }
      PS_STAMP(7 + 3 * l);
    }
    if (P.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(0);
    if constexpr (!FINAL) {
      // centre tiles [2, 2 + TS/32) -> x out (plain stores: they stay in flight into the next tile, whose
      // top waits for at most 20 younger operations -- these 8 and the 12 kernel-fragment loads)
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int k = 2 * wave + j, t = tg + k * 32 + n;
        if (k >= 2 && k < 2 + TS / 32 && t < Lh) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            *reinterpret_cast<float4*>(P.xout + (base + t) * CI + 8 * i + 4 * h) =
                make_float4(xr[j][2 * i].x, xr[j][2 * i].y, xr[j][2 * i + 1].x, xr[j][2 * i + 1].y);
        }
      }
      PS_STAMP(17);
    } else {
    // FIN: eps(t) = b + sum_tap E[t + tap - 3][tap], then the sampler update (util.py:222-226).  E stays in
    // registers: lane (n, h) of wave w holds E of its pair's rows n (tile 2w) and 32 + n (tile 2w + 1) after the
    // halves' partial sums meet, so the row shifts t + tap - 3 are lane permutes (ds_bpermute) within the
    // 64-row pair; only the pair's outer three rows on each side go through LDS to the neighbouring waves.  One
    // barrier instead of two, and no 16 KB E image (the one-tile kernel: 7.1k of 56k cycles per tile)
    float ev[TPW][7];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
#pragma unroll
      for (int tap = 0; tap < 7; ++tap) {
        f32x2 acc = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {             // channels 8i + 4h .. +3 = regs 4i .. 4i+3
          const float4 w = *reinterpret_cast<const float4*>(&FWF[tap * 32 + 8 * i + 4 * h]);
          acc = efma(xr[j][2 * i], f32x2{w.x, w.y}, acc);
          acc = efma(xr[j][2 * i + 1], f32x2{w.z, w.w}, acc);
        }
        ev[j][tap] = acc.x + acc.y;
      }
#pragma unroll
      for (int tap = 0; tap < 7; ++tap) ev[j][tap] += __shfl_xor(ev[j][tap], 32);
      const int ts = tg + (2 * wave + j) * 32;
      if (ts < 0 || ts >= Le) {                    // x is zero outside the utterance (the final conv's padding)
#pragma unroll
        for (int tap = 0; tap < 7; ++tap) ev[j][tap] = 0.f;
      }
    }
    // the pair's rows 0..2 (tile 2w) and 61..63 (tile 2w + 1) for the neighbouring waves
    if (h == 0 && n < 3) {
#pragma unroll
      for (int tap = 0; tap < 7; ++tap) EB[wave][0][n][tap] = ev[0][tap];
    }
    if (h == 0 && n >= 29) {
#pragma unroll
      for (int tap = 0; tap < 7; ++tap) EB[wave][1][n - 29][tap] = ev[1][tap];
    }
    __syncthreads();
    {
      const int rho = lane;                        // = 32 h + n: this lane's row within the pair
      float e = bfin;
#pragma unroll
      for (int tap = 0; tap < 7; ++tap) {
        const int src = rho + tap - 3;             // source row within the pair, [-3, 67)
        const int sl = src & 31;
        const float v0 = __shfl(ev[0][tap], sl), v1 = __shfl(ev[1][tap], sl);
        const float vl = EB[wave > 0 ? wave - 1 : 0][1][min(max(src + 3, 0), 2)][tap];        // wave w - 1, rows 61..63
        const float vr = EB[wave < NW - 1 ? wave + 1 : NW - 1][0][min(max(src - 64, 0), 2)][tap];   // wave w + 1, rows 0..2
        e += src < 0 ? vl : src < 32 ? v0 : src < 64 ? v1 : vr;
      }
      const int t = t0 + so;
      if (so >= 0 && so < TS && t < Lh) {
        float vv = (as[67 + so] - P.ce * e) / P.den;
        if (P.sig != 0.f) vv += P.sig * zr;
        P.audio_out[base + t] = vv;
      }
    }
    PS_STAMP(17);
    }
  }
}
#undef PS_STAMP

// ------------------------------------------------------------------ DiffusionDBlock (bf16)
// modules.py:131-138 in one launch:
//   xs = x[f i];  h1 = lrelu(conv_d1(lrelu(xs)));  h2 = lrelu(conv_d2(h1));
//   out = conv_d4(h2) + W_r xs + (b3 + b_r)        (conv.2 and residual_dense share one K=128 GEMM)
// Block = 128 output rows of one utterance; local row p <-> i = i0 - 7 + p (halo 1+2+4).
// Every intermediate is zeroed outside [0, Lout): each reference conv's zero padding.
// AF: bound on the factor f of an audio-input block (the audio window is (DB_TS + 14) f
// samples); the first DBlock has f = 4 in every shipped config.
// r03 (SQ counters, C3): the audio block was issue-bound -- 1.1k VALU + 0.6k SALU instructions
// per wave at 3 waves per SIMD -- so the first conv keeps its weights in registers and the
// conv epilogues apply the utterance-edge mask only on edge tiles.
// r04: 5 waves -- the two dilated stages are 5 row tiles each, so with 4 waves one wave ran
// two tiles while three idled at the barrier; the 5th wave sits out only the 4-tile final conv.
#ifndef DB_NW
#define DB_NW 5
#endif
#ifndef DB_WPE
#define DB_WPE 5   // waves per SIMD: 4 blocks of 5 waves per CU (<= 96 VGPRs; the LDS allows 4);
                   // the AF = 16 window (8 loads per thread) keeps 4 (it spilled at 96)
#endif
constexpr int DB_TS = 128, DB_ROWS = 168, DB_LD = 40, DB_NT = 64 * DB_NW;
template <int AF>
__global__ __launch_bounds__(DB_NT) __attribute__((amdgpu_waves_per_eu(AF > 4 ? 4 : DB_WPE))) void dblock_bf16_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                          const __bf16* __restrict__ W0, const float* __restrict__ b0,
                                                          const __bf16* __restrict__ W1, const float* __restrict__ b1,
                                                          const __bf16* __restrict__ W2, const float* __restrict__ b2,
                                                          int Lout, int f, const float* __restrict__ audio,
                                                          const float* __restrict__ fw, const float* __restrict__ fb,
                                                          const int* __restrict__ lens, int rate) {
  // U0 = lrelu(x[f i]) is dead after the first conv, so h2 reuses its rows: 3 x 13 KB of
  // bf16 images
  __shared__ __attribute__((aligned(16))) __bf16 U0[DB_ROWS * DB_LD];   // lrelu(x[f i]), then h2
  __shared__ __attribute__((aligned(16))) __bf16 R0[DB_ROWS * DB_LD];   // x[f i] (residual input)
  __shared__ __attribute__((aligned(16))) __bf16 H1[DB_ROWS * DB_LD];
  __bf16* H2 = U0;
  // audio input (the first DBlock): the block's samples t = f i + k - 3 of its rows, staged once
  constexpr bool AUD = AF > 0;   // AF = 0: x input (no audio) -- a compile-time choice: the runtime
                                 // `if constexpr (AUD)` left the x path's loads in the audio kernel, with
                                 // waits at every branch join of the staging
  constexpr int DB_AUM = (DB_TS + 14) * (AUD ? AF : 0) + 8;
  constexpr int DB_AUI = (DB_AUM + DB_NT - 1) / DB_NT;
  // the audio window is dead once the staging has read it (before the barrier that precedes the
  // first write of H1), so it lives in H1's rows: 3 images (40.3 KB) let 4 blocks share a CU
  // where a separate window (43 KB) left room for 3
  static_assert(DB_AUM * 4 <= DB_ROWS * DB_LD * 2, "audio window must fit in H1");
  float* AU = reinterpret_cast<float*>(H1);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int b = blockIdx.y, i0 = blockIdx.x * DB_TS, ib = i0 - 7;
  const long long Lin = (long long)Lout * f;
  const float* src = in + (long long)b * Lin * CI;
  // ragged batch: the utterance's output rows end at Lv (rate output rows per mel frame), its input
  // samples at Lv f; both convs' zero padding starts there
  const int Lv = lens ? min(lens[b] * rate, Lout) : Lout;
  const long long Linv = (long long)Lv * f;
  // the first stage's weight fragments first: their L2 round trip overlaps the staging's;
  // the later stages' are issued after the staging stores (r04: all 20 fragments live across
  // the staging kept the kernel at 148 VGPRs, 3 waves per SIMD)
  bf16x8 wf0[6], wf1[6], wf2[8];
#pragma unroll
  for (int kk = 0; kk < 6; ++kk) wf0[kk] = *reinterpret_cast<const bf16x8*>(W0 + r32 * 96 + kk * 16 + h * 8);
  const float bv0 = b0[r32], bv1 = b1[r32], bv2 = b2[r32];
  if constexpr (AUD) {
    // input = first_conv(audio) at t = f ii (FastDiff_model.py:90), recomputed: no a0 tensor.
    // The window [f ib - 3, f (ib + DB_TS + 14) + 4) arrives in ONE round trip: every thread's
    // loads are unconditional (clamped address) and issued before any LDS store (r03: a
    // branch-guarded load per loop trip made the first DBlock a chain of 3 round trips,
    // ~10x the time of its sibling blocks per row).
    const long long t0 = (long long)ib * f - 3;
    const float* au = audio + (long long)b * Lin;
    const int na = (DB_TS + 14) * f + 8;
    float av[DB_AUI];
#pragma unroll
    for (int it = 0; it < DB_AUI; ++it) {
      const long long t = t0 + tid + DB_NT * it;
      av[it] = au[t < 0 ? 0 : t >= Lin ? Lin - 1 : t];
    }
    // unconditional stores (indices past the window land on AU's last slot, which no row reads):
    // a store under `i < na` let hipcc sink the load into that branch and wait for it there
#pragma unroll
    for (int it = 0; it < DB_AUI; ++it) {
      const int i = tid + DB_NT * it;
      const long long t = t0 + i;
      AU[min(i, DB_AUM - 1)] = (i < na && t >= 0 && t < Linv) ? av[it] : 0.f;
    }
    __syncthreads();
  }
  // staging: every thread's (<= DB_NI) items are loaded before any is converted, so their
  // strided HBM reads are in flight together (one round trip per block, not one per item)
  constexpr int DB_NI = (DB_ROWS * 8 + DB_NT - 1) / DB_NT;
  float4 sv[DB_NI];
  // a thread's channel quad q is the same for all its items: its first-conv weights (7 taps x
  // 4 channels, fw is [c][tap]) and biases live in registers
  float fq[7][4], fbq[4];
  if constexpr (AUD) {
    const int q = (tid & 7) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      fbq[e] = fb[q + e];
#pragma unroll
      for (int k = 0; k < 7; ++k) fq[k][e] = fw[(q + e) * 7 + k];
    }
  }
#pragma unroll
  for (int u = 0; u < DB_NI; ++u) {
    const int i = tid + DB_NT * u;
    const int p = i >> 3, q = (i & 7) * 4, ii = ib + p;
    const bool ok = i < DB_ROWS * 8 && p < DB_TS + 14 && ii >= 0 && ii < Lv;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (AUD) {
      if (ok) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = fbq[e];
#pragma unroll
        for (int k = 0; k < 7; ++k) {                // first_conv_kernel's order
          const float a = AU[p * f + k];             // t = f ii + k - 3
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = fmaf(fq[k][e], a, o[e]);
        }
        v = make_float4(o[0], o[1], o[2], o[3]);
      }
    } else {
      // unconditional load at a clamped row, masked per component: a load under the range
      // branch made the staging one round trip per item (late r03 asm: 5 in a row)
      const int iic = ii < 0 ? 0 : ii >= Lout ? Lout - 1 : ii;
      const float4 x = *reinterpret_cast<const float4*>(src + (long long)iic * f * CI + q);
      v.x = ok ? x.x : 0.f; v.y = ok ? x.y : 0.f; v.z = ok ? x.z : 0.f; v.w = ok ? x.w : 0.f;
    }
    sv[u] = v;
  }
  // (unconditional, as the AU stores: items past the window write the last row, which no stage reads)
#pragma unroll
  for (int u = 0; u < DB_NI; ++u) {
    const int i = tid + DB_NT * u;
    const int p = min(i >> 3, DB_ROWS - 1), q = (i & 7) * 4;
    float4 v = sv[u];
    *reinterpret_cast<bf16x4*>(&R0[p * DB_LD + q]) = bf16x4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    v.x = v.x >= 0.f ? v.x : 0.2f * v.x; v.y = v.y >= 0.f ? v.y : 0.2f * v.y;
    v.z = v.z >= 0.f ? v.z : 0.2f * v.z; v.w = v.w >= 0.f ? v.w : 0.2f * v.w;
    *reinterpret_cast<bf16x4*>(&U0[p * DB_LD + q]) = bf16x4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
  }
#pragma unroll
  for (int kk = 0; kk < 6; ++kk) wf1[kk] = *reinterpret_cast<const bf16x8*>(W1 + r32 * 96 + kk * 16 + h * 8);
  __syncthreads();
  // one dilated 32->32 conv stage over 5 row tiles starting at local row `first`
  auto stage = [&](const __bf16* In, __bf16* Out, const bf16x8 (&wf)[6], float bv, int first, int dil) {
    for (int mt = wave; mt < 5; mt += DB_NW) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) {
        const int tap = kk >> 1, ci0 = (kk & 1) * 16;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(&In[(first + mt * 32 + r32 + (tap - 1) * dil) * DB_LD + ci0 + h * 8]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wf[kk], acc, 0, 0, 0);
      }
      // rows outside [0, Lout) (and past DB_ROWS) are zeroed: tile-uniform test first
      const int pt = first + mt * 32, it0 = ib + pt;
      const bool edge = it0 < 0 || it0 + 31 >= Lv || pt + 31 >= DB_ROWS;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int p = pt + (reg & 3) + 8 * (reg >> 2) + 4 * h, ii = ib + p;
        float v = acc[reg] + bv;
        v = v >= 0.f ? v : 0.2f * v;                        // the next conv's input activation
        if (edge) {
          if (ii < 0 || ii >= Lv || p >= DB_ROWS) v = 0.f;
          if (p < DB_ROWS) Out[p * DB_LD + r32] = (__bf16)v;
        } else {
          Out[p * DB_LD + r32] = (__bf16)v;
        }
      }
    }
  };
  stage(U0, H1, wf0, bv0, 1, 1);    // h1 on p in [1, 161)
  // the last stage's fragments only now (wf0 is dead): all three sets live at once needed
  // 109 VGPRs, over the 96 that 5 waves per SIMD (4 blocks per CU) allow
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) wf2[kk] = *reinterpret_cast<const bf16x8*>(W2 + r32 * 128 + kk * 16 + h * 8);
  __syncthreads();
  stage(H1, H2, wf1, bv1, 3, 2);    // h2 on p in [3, 163)
  __syncthreads();
  // out on p in [7, 135): conv_d4(h2) ++ residual_dense(x), K = 96 + 32
  if (wave < 4) {
    const bf16x8 (&wf)[8] = wf2;
    const float bv = bv2;
    const int mt = wave;   // 4 tiles, one per wave
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      bf16x8 af;
      if (kk < 6) {
        const int tap = kk >> 1, ci0 = (kk & 1) * 16;
        af = *reinterpret_cast<const bf16x8*>(&H2[(7 + mt * 32 + r32 + (tap - 1) * 4) * DB_LD + ci0 + h * 8]);
      } else {
        af = *reinterpret_cast<const bf16x8*>(&R0[(7 + mt * 32 + r32) * DB_LD + (kk - 6) * 16 + h * 8]);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wf[kk], acc, 0, 0, 0);
    }
    float* dst = out + (long long)b * Lout * CI;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int ii = i0 + mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (ii < Lout) dst[(long long)ii * CI + r32] = acc[reg] + bv;
    }
  }
}

// ------------------------------------------------------------------ kernel predictor (bf16)
// Batched over grid.z = step * nb + block: the hidden stack depends only on the mel
// and the step embedding, so a sampler runs it for every step and block in ONE launch.
struct KPArgs {
  const float* condT;       // [B][Tc][80] mel, time-major
  const float* nz;          // fc_t(emb): row of (step s, utterance b, block n) at
  int nz_step, nz_ld;       //   nz + s*nz_step + b*nz_ld + n*80
  int nb, B;
  const __bf16* Win[4];     // per block: [64][5*96]   (tap*96 + ci)
  const float* bin[4];
  const __bf16* Wr[4][6];   // [64][3*64]
  const float* br[4][6];
  const __bf16* Wb[4];      // [256][3*64]  bias_conv
  const float* bb[4];
  __bf16* hout;             // [z][B][Tc][64]  h = h0 + R(h0), bf16 (the kernel GEMM's operand)
  float* Bf;                // [z][B][Tc][256] LVC biases
  int Tc;
  const int* lens;          // frames of each utterance (null: Tc): every conv's zero padding starts there
};

// Fused KernelPredictor hidden stack (modules.py:320-333 + bias_conv :338-342):
//   h0 = lrelu_.1(conv5(c + fc_t(e))), r = 6 x lrelu_.1(conv3(.)), h = h0 + r, Bf = conv3(h)
// Block: 64 output frames of one utterance.  Every stage runs on 96 local rows
// (local row p <-> frame f0 - 16 + p) held in LDS as bf16, and rows outside the
// utterance are zeroed after every stage -- exactly each reference conv's zero
// padding.  The halo shrinks by 1 row per conv (9 rows needed, 16 kept).
__global__ __launch_bounds__(256) void kp_hidden_bf16_kernel(const KPArgs A) {
  constexpr int LDC = 104, LDH = 72;               // 208 B / 144 B rows: conflict-free b128 reads
  __shared__ __attribute__((aligned(16))) __bf16 Cs[101 * LDC];   // + a spare row for the staging's overflow items
  __shared__ __attribute__((aligned(16))) __bf16 Hb[3][98 * LDH];   // H0, R0, R1 (+1 zero row each side)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int b = blockIdx.y, f0 = blockIdx.x * 64, Tc = A.Tc;
  const int Tv = A.lens ? min(A.lens[b], Tc) : Tc;   // ragged batch: the utterance's own end
  const int z = blockIdx.z, step = z / A.nb, nblk = z - step * A.nb;
  const long long rb = (long long)b * Tc;
  const float* nzrow = A.nz + (long long)step * A.nz_step + (long long)b * A.nz_ld + nblk * CC;
  __bf16* hout = A.hout + (long long)z * A.B * Tc * HK;
  float* Bfo = A.Bf + (long long)z * A.B * Tc * (2 * CI * NLY);

  // c' = c + fc_t(e) on frames f0-18 .. f0+81 (channels 80..95 zero).  All loads are issued
  // before any is used (clamped addresses, masked at the store): one round trip, not ten.  r05:
  // issued FIRST, ahead of the weight fragments below -- vmcnt retires in order, so staging them
  // last made the LDS stores wait for every weight load too (the asm: vmcnt(0) after 51 loads)
  constexpr int NCI = (100 * 24 + 255) / 256;
  float4 cv[NCI], nv[NCI];
#pragma unroll
  for (int u = 0; u < NCI; ++u) {
    const int i = min(tid + 256 * u, 100 * 24 - 1), p = i / 24, g = min((i - p * 24) * 4, CC - 4);
    const int f = min(max(f0 - 18 + p, 0), Tc - 1);
    cv[u] = *reinterpret_cast<const float4*>(A.condT + (rb + f) * CC + g);
    nv[u] = *reinterpret_cast<const float4*>(nzrow + g);
  }
  // Stage 0's weight fragments (30 k-steps; both of a wave's jobs use column tile wave & 1)
  // run through a KH0-deep register ring, primed here so the first ones land with the
  // staging loads: a load right before each MFMA made stage 0 thirty L2 round trips per job.
  constexpr int KH0 = 10;
  // every stage's bias for this lane's column, loaded up front (r04: each stage's bias load right
  // before its epilogue was a round trip of its own): stages 0..6 use column (wave & 1) 32 + r32,
  // the bias_conv tiles 2w and 2w + 1
  const int nw = (wave & 1) * 32 + r32;
  const float bias_in = A.bin[nblk][nw];
  float bias_r[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) bias_r[j] = A.br[nblk][j][nw];
  const float bias_b[2] = {A.bb[nblk][2 * wave * 32 + r32], A.bb[nblk][(2 * wave + 1) * 32 + r32]};
  const __bf16* wrow0 = A.Win[nblk] + ((wave & 1) * 32 + r32) * 480 + h * 8;
  bf16x8 w0r[KH0];
#pragma unroll
  for (int s = 0; s < KH0; ++s) w0r[s] = *reinterpret_cast<const bf16x8*>(wrow0 + s * 16);
  bf16x8 bwn[12];   // stage 1's fragments (stages 1..6 below), in flight from here on
  {
    const __bf16* wrow = A.Wr[nblk][0] + ((wave & 1) * 32 + r32) * 192 + h * 8;
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) bwn[kk] = *reinterpret_cast<const bf16x8*>(wrow + kk * 16);
  }
  __builtin_amdgcn_sched_barrier(0);   // every load above in flight before the staging stores
  // (branch-free: items past the 100 rows go to a spare row, padding is masked -- with the stores
  // and conversions under `if`, hipcc sank the last item's loads into the branch and waited there
  // for every load in flight, r05 asm)
#pragma unroll
  for (int u = 0; u < NCI; ++u) {
    const int i = tid + 256 * u;
    const bool in = i < 100 * 24;
    const int p = in ? i / 24 : 100, g = in ? (i - p * 24) * 4 : 0, f = f0 - 18 + p;
    const unsigned mk = (in && g < CC && f >= 0 && f < Tv) ? 0xffffffffu : 0u;
    const float4 c = cv[u], n = nv[u];
    const bf16x4 v = bf16x4{(__bf16)(c.x + n.x), (__bf16)(c.y + n.y), (__bf16)(c.z + n.z), (__bf16)(c.w + n.w)};
    uint2 vb = __builtin_bit_cast(uint2, v);
    vb.x &= mk; vb.y &= mk;
    *reinterpret_cast<uint2*>(Cs + p * LDC + g) = vb;
  }
  for (int i = tid; i < 3 * 2 * LDH; i += 256) {   // zero guard rows 0 and 97
    const int buf = i / (2 * LDH), j = i - buf * 2 * LDH;
    Hb[buf][(j < LDH ? 0 : 97 * LDH) + (j % LDH)] = (__bf16)0.f;
  }
  __syncthreads();

  float keep[2][16];   // h0 in fp32 for the residual add (same job->wave map in every stage)
  // stage 0: h0 = lrelu(conv5(c')) ; jobs = 3 row tiles x 2 column tiles.  Waves 2 and 3 have
  // one job: their second pass runs on a clamped tile and is dropped (they would wait at the
  // barrier anyway), so the ring's step index stays static.
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int job = wave + 4 * q;
    const int mt = min(job >> 1, 2), nt = job & 1;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 30; ++kk) {
      const int st = q * 30 + kk;
      const bf16x8 bw = w0r[st % KH0];
      if (st + KH0 < 60) w0r[st % KH0] = *reinterpret_cast<const bf16x8*>(wrow0 + ((st + KH0) % 30) * 16);
      __builtin_amdgcn_sched_barrier(0);   // keep the load KH0 steps ahead (hipcc sinks loads to their use)
      const int tap = kk / 6, kc = kk - tap * 6;
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(Cs + (mt * 32 + r32 + tap) * LDC + kc * 16 + h * 8);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bw, acc, 0, 0, 0);
    }
    if (job >= 6) continue;
    const int n = nt * 32 + r32;
    const float bias = bias_in;   // (n == nw)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int p = mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, f = f0 - 16 + p;
      float v = acc[reg] + bias;
      v = v >= 0.f ? v : 0.1f * v;
      if (f < 0 || f >= Tv) v = 0.f;
      keep[q][reg] = v;
      Hb[0][(p + 1) * LDH + n] = (__bf16)v;
    }
  }
  __syncthreads();
  // stages 1..6: residual convs H0 -> R0 -> R1 -> R0 -> R1 -> R0 -> R1.
  // A wave's jobs (wave, wave + 4) share the column tile nt = wave & 1: its 12 weight fragments
  // are loaded once per stage and reused by both jobs; stage j + 1's fragments are loaded while
  // stage j computes (no L2 round trip at a stage start).
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const __bf16* In = Hb[j == 0 ? 0 : (j & 1 ? 1 : 2)];
    __bf16* Out = Hb[j & 1 ? 2 : 1];
    bf16x8 bwf[12];
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) bwf[kk] = bwn[kk];
    {
      // next stage's fragments, or the bias_conv's first column tile after the last stage
      const __bf16* wrow = j < 5 ? A.Wr[nblk][j + 1] + ((wave & 1) * 32 + r32) * 192 + h * 8
                                 : A.Wb[nblk] + (2 * wave * 32 + r32) * 192 + h * 8;
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) bwn[kk] = *reinterpret_cast<const bf16x8*>(wrow + kk * 16);
    }
    for (int job = wave, q = 0; job < 6; job += 4, ++q) {
      const int mt = job >> 1, nt = job & 1;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) {
        const int tap = kk >> 2, kc = kk & 3;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(In + (mt * 32 + r32 + tap) * LDH + kc * 16 + h * 8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bwf[kk], acc, 0, 0, 0);
      }
      const int n = nt * 32 + r32;
      const float bias = bias_r[j];   // (n == nw)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int p = mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h, f = f0 - 16 + p;
        float v = acc[reg] + bias;
        v = v >= 0.f ? v : 0.1f * v;
        if (j == 5) v += keep[q][reg];           // h = h0 + R(h0)
        if (f < 0 || f >= Tv) v = 0.f;
        Out[(p + 1) * LDH + n] = (__bf16)v;
        if (j == 5 && p >= 16 && p < 80 && f < Tc) hout[(rb + f) * HK + n] = (__bf16)v;
      }
    }
    __syncthreads();
  }
  bf16x8 bwb[12];
#pragma unroll
  for (int kk = 0; kk < 12; ++kk) bwb[kk] = bwn[kk];   // column tile 2w, loaded during stage 6
  // bias_conv on the 64 output frames: 2 row tiles x 8 column tiles; wave w owns column tiles
  // 2w and 2w+1 (weights loaded once per tile, reused by both row tiles)
#pragma unroll
  for (int job = 0; job < 4; ++job) {
    const int nt = 2 * wave + (job >> 1), mt = job & 1;
    if (job == 1) {   // tile 2w + 1's fragments, in flight under tile 2w's second row tile
      const __bf16* wrow = A.Wb[nblk] + ((nt + 1) * 32 + r32) * 192 + h * 8;
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) bwn[kk] = *reinterpret_cast<const bf16x8*>(wrow + kk * 16);
    }
    if (job == 2) {
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) bwb[kk] = bwn[kk];
    }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) {
      const int tap = kk >> 2, kc = kk & 3;
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(Hb[2] + (16 + mt * 32 + r32 + tap) * LDH + kc * 16 + h * 8);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bwb[kk], acc, 0, 0, 0);
    }
    const int n = nt * 32 + r32;
    const float bias = bias_b[job >> 1];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int f = f0 + mt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (f < Tc) Bfo[(rb + f) * (2 * CI * NLY) + n] = acc[reg] + bias;
    }
  }
}

// Location-variable kernels of ALL 4 layers of an LVC block, frame-major bf16
// (modules.py:335-340):  Kf[l][f][n] = b[l][n] + W[l][n] . [h(f-1); h(f); h(f+1)],
// n < 6144, K = 192: one GEMM with N = 4 x 6144 rows (the MFMA A operand), a column per
// frame, bound by its 340 MB of K stores at C3.  Work item = 512 rows n x 128 frames;
// a persistent block (8 waves, one per CU) walks a contiguous run of items, n-group-major:
//  * wave w holds its 64 rows of W (24 fragments, 96 VGPRs) and their biases in registers
//    for as long as the n-group lasts, so the main loop reads only the frames' h from LDS,
//    one 16-B fragment per TWO MFMAs;
//  * the frames' [h(f-1); h(f); h(f+1)] rows (zero across utterance edges) are double-
//    buffered in LDS: the next item's are loaded at the start of an item and written after
//    its stores, one barrier per item, no barrier inside it;
//  * K stores are unconditional buffer stores (rows past the end are dropped by the range
//    check), so hipcc never drains them before the next LDS write.
// r02's structure (W tile in LDS, one fragment read per MFMA, two barriers per 64-row tile)
// ran ~77 us for its GEMM alone and ~86 us for its stores alone (profiles/r03_ab/kp_kernel_ab.txt).
// A lane of C holds 4 consecutive kernel values of one frame; a per-wave LDS transpose turns
// them into 128-B row segments (8 frames per 1-KiB store: 6.0 TB/s in tools/store_probe.hip).
// r05, measured and not kept (profiles/r05_ab/kp_units_w4_ab.txt): each h row staged once (130 rows
// per item, the tap-0 / tap-2 fragments masked at utterance edges: 76 KB of LDS instead of 141) with
// the work dealt as equal runs of 32-frame tiles (C3's 128-frame items fall 10 or 11 per block): 85-87
// vs 84-85 us; the same as two 4-wave blocks per CU, each with its own barrier phase: 86-87 us.
constexpr int KP_F = 128, KP_NG = 512, KP_LDH = 200;   // 400-B LDS rows: conflict-free b128 reads
// Output transpose tile.  KP_SWZ 0 (default): 32 frames x (64 + 8 pad) bf16 rows (144 B: 16-B aligned
// for the b128 reads; 68 measured 15% slower).  KP_SWZ 1 (r05 A/B): unpadded 128-B rows with an XOR
// swizzle -- at 256 VGPRs the per-slot addresses spill (51 registers) unless KP_STAGGER is off: 8-B slot s
// of frame row r lives at slot s ^ kp_swz(r), kp_swz(r) = 2 (r & 7) + ((r >> 3) & 1).  The epilogue's
// ds_write_b64 (16 lanes = 16 frame rows at one slot) then hits 16 distinct slots -- the 144-B padded
// rows of r02-r04 put rows r and r + 8 on one bank pair (2-way, the SQ pass's 1.62 conflict cycles per
// LDS instruction) -- and the store side's ds_read_b128 (16-B chunk c of row r at chunk c ^ (r & 7),
// halves swapped when (r >> 3) & 1) covers all 64 banks in every lane group.
#ifndef KP_SWZ
#define KP_SWZ 0
#endif
constexpr int KP_LDO = KP_SWZ ? 64 : 72;
__device__ __forceinline__ int kp_swz(int r) { return KP_SWZ ? 2 * (r & 7) + ((r >> 3) & 1) : 0; }
constexpr int KP_NGROUPS = NLY * KPERLAYER / KP_NG;    // 48
constexpr int KP_THREADS = 512;
#ifndef KP_STAGGER
#define KP_STAGGER 0   // r05 same-box ABAB: off 5.68 vs on 5.72-5.76 ms/step, kp 103 vs 107 us (profiles/r05_ab/kp_stagger_swz_ab.txt)
#endif
#ifndef KP_AUX
#define KP_AUX 0   // plain K stores: the lines stay on-die for the LVC block that reads them next (r03 A/B: non-temporal (2) made kp ~4% and the next LVC launch ~4% slower)
#endif
__global__ __launch_bounds__(KP_THREADS, 1) void kp_kernel_bf16_kernel(const __bf16* __restrict__ hin,
                                                                       const __bf16* __restrict__ W,
                                                                       const float* __restrict__ bias,
                                                                       __bf16* __restrict__ Kf, int Tc, int rows,
                                                                       int nfg) {
  __shared__ __attribute__((aligned(16))) __bf16 Hs[2][KP_F * KP_LDH];
  __shared__ __attribute__((aligned(16))) __bf16 Ot[8][32 * KP_LDO];   // swizzled (kp_swz)
  __shared__ __attribute__((aligned(16))) float Bq[8][64];   // wave-private: its rows' biases
  const int tid = threadIdx.x, lane = tid & 63, r32 = lane & 31, h = lane >> 5;
  // wave-uniform, and provably so: the K-store descriptor is built from it (a descriptor hipcc
  // sees as divergent becomes a waterfall loop around every store)
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int items = KP_NGROUPS * nfg;
  const int ib = (int)((long long)blockIdx.x * items / gridDim.x);
  const int ie = (int)((long long)(blockIdx.x + 1) * items / gridDim.x);
  typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
  // H staging: item frames [fg*128, +128) x 192 = 3072 16-B pieces, 6 per thread.  Piece c:
  // frame c / 24, 8 values v = (c % 24) * 8 of [tap][ch] (tap = v / 64).
  uint4 hv[6];
  unsigned hz = 0;        // bit i: piece i is zero padding (applied at the LDS store, so the
                          // load's wait is not pulled up to the load)
  auto h_load = [&](int item) {
    const int fg = item % nfg;
    hz = 0;
    // the item's first frame split once (wave-uniform); piece frames step forward from it
    const int R0 = fg * KP_F, b0 = R0 / Tc, f00 = R0 - b0 * Tc;
    // (ragged batch: kp_hidden_bf16_kernel writes zero h rows past each utterance's end, so the
    // kernel conv's zero padding there needs no lengths here.  r05: reading lens in this loop put
    // loads under branches whose joins waited for every outstanding load and K store: kp 85 -> 103 us)
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int c = tid + KP_THREADS * i, fl = c / 24, v = (c - fl * 24) * 8, tap = v >> 6, ch = v & 63;
      const int R = R0 + fl, Rc = R < rows ? R : rows - 1;
      int b = b0, f = f00 + (Rc - R0);
      if (Tc >= KP_F) {                   // (uniform) the item crosses at most one utterance end
        const bool nx = f >= Tc;
        f -= nx ? Tc : 0;
        b += nx ? 1 : 0;
      } else {
        b = Rc / Tc;
        f = Rc - b * Tc;
      }
      const int ff = f + tap - 1;
      const int ffc = ff < 0 ? 0 : ff >= Tc ? Tc - 1 : ff;     // clamped: unconditional load
      hv[i] = *reinterpret_cast<const uint4*>(hin + ((long long)b * Tc + ffc) * HK + ch);
      hz |= (R >= rows || ff < 0 || ff >= Tc) ? 1u << i : 0u;
    }
  };
  auto h_store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int c = tid + KP_THREADS * i, fl = c / 24, v = (c - fl * 24) * 8;
      // masked with AND: a uint4 ternary here made hipcc select through a scratch array
      const unsigned m = (hz >> i) & 1 ? 0u : ~0u;
      *reinterpret_cast<uint4*>(&Hs[buf][fl * KP_LDH + v]) = make_uint4(hv[i].x & m, hv[i].y & m, hv[i].z & m, hv[i].w & m);
    }
  };
  bf16x8 wa[24];          // A fragments: (j, kk) = rows nb + 32 j + r32, k = 16 kk + 8 h
  float* bw = Bq[wave];
  int ng_cur = -1;
  auto w_load = [&](int ng) {
    const int nb = ng * KP_NG + wave * 64;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 12; ++kk)
        wa[j * 12 + kk] = *reinterpret_cast<const bf16x8*>(W + (long long)(nb + 32 * j + r32) * 192 + kk * 16 + h * 8);
    bw[lane] = bias[nb + lane];   // wave-private: no block barrier (read after this wave's lgkmcnt wait)
  };
  h_load(ib);
  h_store(0);
  __syncthreads();
  __bf16* ot = Ot[wave];
  for (int item = ib; item < ie; ++item) {
    const int buf = (item - ib) & 1, ng = item / nfg, fg = item - ng * nfg;
    if (ng != ng_cur) {   // wave-uniform; once or twice per block
      w_load(ng);
      ng_cur = ng;
      // wait for the weight fragments HERE: otherwise the waitcnt pass cannot tell at the loop's
      // merge point whether wa is still in flight, and waits before its first MFMAs in EVERY item --
      // with vmcnt retiring in order, for all of the previous item's K stores too (r05: a store
      // drain per item; the asm had vmcnt(7) / vmcnt(6) inside the first frame tile's MFMAs)
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    }
    h_load(min(item + 1, ie - 1));   // the next item's frames, under this item's work
    const int nb = ng * KP_NG + wave * 64, layer = nb / KPERLAYER, n0 = nb - layer * KPERLAYER;
    const __amdgpu_buffer_rsrc_t kout =
        __builtin_amdgcn_make_buffer_rsrc(Kf + (long long)layer * rows * KPERLAYER, 0, rows * KPERLAYER * 2, 0x00020000);
    const __bf16* hs = Hs[buf];
    // C[n][frame]: lane owns frame r32, rows n = 32j + 8g + 4h + (0..3); the accumulators start
    // from the rows' biases, so the epilogue is a conversion only
    auto mma = [&](int ft, f32x16 (&acc)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 bn = *reinterpret_cast<const float4*>(&bw[j * 32 + 8 * g + 4 * h]);
          acc[j][4 * g] = bn.x; acc[j][4 * g + 1] = bn.y; acc[j][4 * g + 2] = bn.z; acc[j][4 * g + 3] = bn.w;
        }
#pragma unroll
      for (int kk = 0; kk < 12; ++kk) {
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(&hs[(ft * 32 + r32) * KP_LDH + kk * 16 + h * 8]);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[kk], hb, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[12 + kk], hb, acc[1], 0, 0, 0);
      }
    };
    const int swz = kp_swz(r32);
    auto epi = [&](int ft, const f32x16 (&acc)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)   // 8-B slot 8j + 2g + h of frame row r32 (swizzled: KP_SWZ)
          *reinterpret_cast<bf16x4*>(&ot[r32 * KP_LDO + 4 * (KP_SWZ ? (8 * j + 2 * g + h) ^ swz : 8 * j + 2 * g + h)]) =
              bf16x4{(__bf16)acc[j][4 * g], (__bf16)acc[j][4 * g + 1], (__bf16)acc[j][4 * g + 2], (__bf16)acc[j][4 * g + 3]};
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS writes landed (wave-private tile)
      __builtin_amdgcn_wave_barrier();
      const int f0 = fg * KP_F + ft * 32;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int fl = i * 8 + (lane >> 3), ch = (lane & 7) * 8;
        // chunk (lane & 7) of row fl sits at chunk (lane & 7) ^ (fl & 7), its halves swapped when
        // (fl >> 3) & 1 = i & 1 (compile-time here)
        uint4 v = *reinterpret_cast<const uint4*>(&ot[fl * KP_LDO + 8 * (KP_SWZ ? (lane & 7) ^ (lane >> 3) : lane & 7)]);
        if (KP_SWZ && (i & 1)) v = make_uint4(v.z, v.w, v.x, v.y);
        // 340 MB per launch, read back by the next launch
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_{v.x, v.y, v.z, v.w}, kout,
                                               ((f0 + fl) * KPERLAYER + n0 + ch) * 2, 0, KP_AUX);
      }
      __builtin_amdgcn_wave_barrier();      // the next frame tile rewrites ot
    };
    // (unrolled: hipcc counts the stores in vmcnt.)  Waves 4..7 -- each one's SIMD partner is
    // wave - 4 -- run one frame tile behind on their epilogues (KP_STAGGER): a tile's
    // conversion, LDS transpose and stores then issue beside the partner's MFMAs instead of in
    // the same phase (MI355X_MICROARCH.md "Two waves per SIMD", item 9).
    f32x16 acc0[2], acc1[2];
    if (!KP_STAGGER || wave < 4) {
#pragma unroll
      for (int ft = 0; ft < KP_F / 32; ++ft) {
        mma(ft, acc0);
        epi(ft, acc0);
      }
    } else {
      mma(0, acc0);
#pragma unroll
      for (int ft = 1; ft < KP_F / 32; ++ft) {
        if (ft & 1) { mma(ft, acc1); epi(ft - 1, acc0); }
        else { mma(ft, acc0); epi(ft - 1, acc1); }
      }
      if ((KP_F / 32 - 1) & 1) epi(KP_F / 32 - 1, acc1);
      else epi(KP_F / 32 - 1, acc0);
    }
    // the next item's frames into the other buffer, whose readers (the previous item) are
    // past the last barrier; the barrier makes them visible
    __builtin_amdgcn_sched_barrier(0);
    h_store(buf ^ 1);
    __syncthreads();
  }
}

// prescale: the gate half scaled by -log2(e), the filter half by 2 log2(e) (the whole-block
// LVC kernel's gate takes exp2 arguments straight from its accumulators): the pre-scaled weight
// copy, so the kernel's epilogue is a bf16 conversion only.
// kks_w = bf16(kk_w * s(n)), kks_b = kk_b * s(n): s = -log2 e on a layer's gate rows (n % 6144 <
// 3072: output channels 0..31), 2 log2 e on its filter rows.
__global__ void kp_prescale_kernel(const float* __restrict__ w, const float* __restrict__ b, __bf16* __restrict__ ws,
                                   float* __restrict__ bs) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr long long NW = (long long)NLY * KPERLAYER * 3 * HK;
  if (i >= NW) return;
  const int n = (int)(i / (3 * HK));
  const float s = n % KPERLAYER < KPERLAYER / 2 ? -LOG2E : 2.f * LOG2E;
  ws[i] = (__bf16)(w[i] * s);
  if (i % (3 * HK) == 0) bs[n] = b[n] * s;
}

// (ragged batches need no lengths here: hk rows past an utterance's end are zero, kp_hidden_bf16_kernel)
int kp_kernels_all(const fd_model::Block& K, const __bf16* hk, __bf16* Kb, int B, int Tc, hipStream_t st,
                   bool prescale = false) {
  const int rows = B * Tc;
  const int nfg = cdiv(rows, KP_F);
  // buffer-store offsets are 32-bit bytes, up to the last (partial) item's rows
  PD_CHECK_ARG((long long)nfg * KP_F * KPERLAYER * 2 < (1ll << 31), "kernel predictor: B*T' too large");
  const int items = KP_NGROUPS * nfg;
  const int grid = items < 256 ? items : 256;   // persistent: one block per CU
  ProfScope ps("fd_kp_kernel", st);
  hipLaunchKernelGGL(kp_kernel_bf16_kernel, dim3(grid), dim3(KP_THREADS), 0, st, hk,
                     prescale ? K.kks_w : lookup_bf16(K.kk_w), prescale ? K.kks_b : K.kk_b, Kb, Tc, rows, nfg);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// eps[b][t] = bias + sum_{k<7,c<32} w[k][c] x[b][t+k-3][c]      (FastDiff_model.py:67-68,100)
// mode 0: eps_out = eps.  mode 1 (sampler, util.py:222-226):
//   xa = (xa - ce*eps) / den + sig * z
__global__ __launch_bounds__(256) void final_conv_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w, const float* bias,
                                                         float* eps_out, float* xa, float ce, float den,
                                                         float sig, const float* noise,
                                                         unsigned long long seed, unsigned stream,
                                                         const int* uid, long long L, const int* lens, int hop) {
  // rows of 36 floats (144 B): 16-B reads, slot 9*row mod 16 -> conflict-free across lanes
  __shared__ __attribute__((aligned(16))) float xs[262 * 36];
  __shared__ __attribute__((aligned(16))) float wsh[7 * 32];
  const int b = blockIdx.y, tid = threadIdx.x;
  const long long t0 = (long long)blockIdx.x * 256;
  const long long Lv = lens ? (long long)lens[b] * hop : L;   // ragged batch: x reads zero past the utterance
  if (tid < 224) wsh[tid] = w[tid];
  for (int i = tid; i < 262 * 8; i += 256) {
    const int rr = i >> 3, q = (i & 7) * 4;
    const long long t = t0 - 3 + rr;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t >= 0 && t < L && t < Lv) v = *reinterpret_cast<const float4*>(x + ((long long)b * L + t) * CI + q);
    *reinterpret_cast<float4*>(&xs[rr * 36 + q]) = v;
  }
  __syncthreads();
  const long long t = t0 + tid;
  if (t >= L) return;
  float e = bias[0];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const float* xr = xs + (tid + k) * 36;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(xr + 4 * q);
      const float4 ww = *reinterpret_cast<const float4*>(&wsh[k * 32 + 4 * q]);
      e = fmaf(ww.x, v.x, fmaf(ww.y, v.y, fmaf(ww.z, v.z, fmaf(ww.w, v.w, e))));
    }
  }
  const long long idx = (long long)b * L + t;
  if (eps_out) eps_out[idx] = e;
  if (xa) {
    float v = (xa[idx] - ce * e) / den;
    if (sig != 0.f) v += sig * (noise ? noise[idx] : philox_normal_u(seed, utt_id(uid, b), (unsigned)t, stream));
    xa[idx] = v;
  }
}

// kernel_conv pack: dst row (i*6144 + o*96 + tap*32 + ci), col (kt*64 + h)
//   <- src [(((i*32+ci)*64+o)*3+tap)][h][kt]            (modules.py:335-340 view)
__global__ void pack_kernel_conv_kernel(float* dst, float* dst_b, const float* src, const float* src_b) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)NLY * KPERLAYER * HK * 3;
  if (i >= total) return;
  int kt = (int)(i % 3);
  long long r = i / 3;
  int h = (int)(r % HK);
  int ch = (int)(r / HK);
  int tap = ch % 3, o = (ch / 3) % 64, ci = (ch / 192) % 32, layer = ch / (192 * 32);
  long long row = (long long)layer * KPERLAYER + kf_packed(o, tap * 32 + ci);
  dst[row * (3 * HK) + kt * HK + h] = src[i];
  if (kt == 0 && h == 0) dst_b[row] = src_b[ch];
}

// upsample weight [ci][co][k] -> [k][ci][co]
__global__ void pack_upsample_kernel(float* dst, const float* src, int K) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= CI * CI * K) return;
  int k = i % K, co = (i / K) % CI, ci = i / (K * CI);
  dst[(k * CI + ci) * CI + co] = src[i];
}

// fused-upsample phase weights: dst[(k*32 + co)*64 + q] = q < 32 ? W[k][q][co] : W[k+r][q-32][co]
// from the [2r][ci][co] packing above
__global__ void pack_upsample_phase_kernel(float* dst, const float* wp, int r) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= CI * CI * 2 * r) return;
  const int q = i & 63, co = (i >> 6) & 31, k = i >> 11;
  const int kk = q < 32 ? k : k + r, ci = q & 31;
  dst[i] = wp[(kk * CI + ci) * CI + co];
}

// final conv weight [1][32][7] -> [7][32]
__global__ void pack_final_kernel(float* dst, const float* src) {
  int i = threadIdx.x;
  if (i < 224) dst[(i % 7) * 32 + i / 7] = src[i];
}

// ------------------------------------------------------------------ workspace
// Does block n run as the whole-block LVC kernel (bf16; hop % 32 == 0: one frame per
// 32-row tile; hop | 32: several, masked per frame)?
bool fd_block_fused(const fd_model* m, int n) {
  return m->pool_bf && m->lvc_ts > 0 && (m->hops[n] % 32 == 0 || (32 % m->hops[n] == 0 && m->lvc_sub));
}
// Kernel predictor on the side stream (fd_sample): every block on the whole-block kernel.
bool fd_kp_side(const fd_model* m) {
  if (!m->kp_side || !m->pool_bf) return false;
  for (int n = 0; n < m->nblocks; ++n)
    if (!fd_block_fused(m, n)) return false;
  return true;
}

struct FdWs {
  size_t steps, e128, e512a, e512, nz;  // step MLP (nvec = S*B)
  size_t a0, d[3], dtmp0, dtmp1, xs, wav2;
  size_t X0, X1, y, h0, ra, rb, Bf, Kf, condT, hall, bfall, total;
};

FdWs fd_layout(const fd_model* m, int B, int Tc, int S) {
  FdWs w{};
  size_t off = 0;
  auto take = [&](size_t n) { size_t o = off; off += (n + 63) / 64 * 64; return o; };
  const size_t L = (size_t)Tc * m->hops[m->nblocks - 1];
  const size_t nv = (size_t)S * B;
  w.steps = take(nv);
  w.e128 = take(nv * EMB_IN);
  w.e512a = take(nv * EMB_MID);
  w.e512 = take(nv * EMB_OUT);
  w.nz = take(nv * m->nblocks * CC);
  w.a0 = take((size_t)B * L * CI);
  w.wav2 = take((size_t)B * L);   // sampler ping-pong buffer (fused final update)
  size_t Ld = L;
  for (int n = 0; n < m->nblocks; ++n) {
    Ld /= m->ratios[m->nblocks - 1 - n];
    w.d[n] = take((size_t)B * Ld * CI);
  }
  w.dtmp0 = take((size_t)B * (L / m->ratios[m->nblocks - 1]) * CI);
  w.dtmp1 = take((size_t)B * (L / m->ratios[m->nblocks - 1]) * CI);
  w.X0 = take((size_t)B * L * CI);
  w.X1 = take((size_t)B * L * CI);
  w.y = take((size_t)B * L * CI);
  w.h0 = take((size_t)B * Tc * HK);
  w.ra = take((size_t)B * Tc * HK);
  w.rb = take((size_t)B * Tc * HK);
  w.Bf = take((size_t)B * Tc * 2 * CI * NLY);
  // bf16 path: kernel-predictor hidden outputs of every (step, block), one batched launch
  w.hall = take((size_t)S * m->nblocks * B * Tc * HK);
  w.bfall = take((size_t)S * m->nblocks * B * Tc * 2 * CI * NLY);
  // fp32: one layer; bf16: all 4 layers (one block's worth per block with the side stream)
  w.Kf = take((size_t)B * Tc * KPERLAYER * 2 * (fd_kp_side(m) ? m->nblocks : 1));
  w.condT = take((size_t)B * Tc * CC);
  w.total = off * sizeof(float);
  return w;
}

// step embedding -> fc_t1/swish -> fc_t2/swish -> per-block fc_t   (util.py:404-429,
// FastDiff_model.py:85-87, modules.py:202)
int fd_step_mlp(const fd_model* m, float* ws, const FdWs& W, int nv, hipStream_t st) {
  PD_TRY(sinusoidal_embed(ws + W.steps, ws + W.e128, nv, EMB_IN, st));
  PD_TRY(matvec(m->fc1_w, m->fc1_b, ws + W.e128, EMB_IN, ws + W.e512a, EMB_MID, EMB_MID, EMB_IN, nv, ACT_SWISH, st));
  PD_TRY(matvec(m->fc2_w, m->fc2_b, ws + W.e512a, EMB_MID, ws + W.e512, EMB_OUT, EMB_OUT, EMB_MID, nv, ACT_SWISH, st));
  for (int n = 0; n < m->nblocks; ++n)
    PD_TRY(matvec(m->blk[n].fct_w, m->blk[n].fct_b, ws + W.e512, EMB_OUT, ws + W.nz + n * CC,
                  m->nblocks * CC, CC, EMB_OUT, nv, ACT_NONE, st));
  return PD_OK;
}

// DiffusionDBlock (modules.py:131-138): out = conv_d4(lr(conv_d2(lr(conv_d1(lr(x[f i])))))) + Wr x[f i]
// lens / rate: ragged batch (utterance b's output rows end at lens[b] * rate), or null
int dblock(const fd_model::Down& D, const float* in, float* out, float* t0, float* t1, int B, int Tout,
           int f, hipStream_t st, const fd_model* m = nullptr, const float* audio = nullptr,
           const int* lens = nullptr, int rate = 1) {
  const long long bsi = (long long)Tout * f * CI, bso = (long long)Tout * CI;
  if (const __bf16* w0 = lookup_bf16(D.c0_w)) {   // bf16: one fused launch, intermediates in LDS
    ProfScope ps("fd_dblock_fused", st);
    if (audio && f <= 4)
      hipLaunchKernelGGL(dblock_bf16_kernel<4>, dim3(cdiv(Tout, DB_TS), B), dim3(DB_NT), 0, st, in, out, w0, D.c0_b,
                         lookup_bf16(D.c1_w), D.c1_b, lookup_bf16(D.c2_w), D.c2_b, Tout, f, audio, m->first_w,
                         m->first_b, lens, rate);
    else if (audio)
      hipLaunchKernelGGL(dblock_bf16_kernel<16>, dim3(cdiv(Tout, DB_TS), B), dim3(DB_NT), 0, st, in, out, w0, D.c0_b,
                         lookup_bf16(D.c1_w), D.c1_b, lookup_bf16(D.c2_w), D.c2_b, Tout, f, audio, m->first_w,
                         m->first_b, lens, rate);
    else
      hipLaunchKernelGGL(dblock_bf16_kernel<0>, dim3(cdiv(Tout, DB_TS), B), dim3(DB_NT), 0, st, in, out, w0, D.c0_b,
                         lookup_bf16(D.c1_w), D.c1_b, lookup_bf16(D.c2_w), D.c2_b, Tout, f, nullptr, nullptr, nullptr,
                         lens, rate);
    PD_LAUNCH_CHECK();
    return PD_OK;
  }
  {
    GemmArgs a = make_gemm(B, Tout, CI, D.c0_w, 96, D.c0_b, t0, bso, CI);
    for (int tap = 0; tap < 3; ++tap) {
      Seg s = make_seg(in, bsi, CI, CI, tap - 1, f);
      s.act = ACT_LRELU; s.alpha = 0.2f;
      add_seg(a, s);
    }
    a.lens = lens; a.lens_mul = rate;
    PD_TRY((launch_gemm<1, 1, 4, 1, EPI_STORE, U_FD_DBLOCK>(a, st, "fd_dblock")));
  }
  {
    GemmArgs a = make_gemm(B, Tout, CI, D.c1_w, 96, D.c1_b, t1, bso, CI);
    for (int tap = 0; tap < 3; ++tap) {
      Seg s = make_seg(t0, bso, CI, CI, (tap - 1) * 2);
      s.act = ACT_LRELU; s.alpha = 0.2f;
      add_seg(a, s);
    }
    a.lens = lens; a.lens_mul = rate;
    PD_TRY((launch_gemm<1, 1, 4, 1, EPI_STORE, U_FD_DBLOCK>(a, st, "fd_dblock")));
  }
  {
    GemmArgs a = make_gemm(B, Tout, CI, D.c2_w, 128, D.c2_b, out, bso, CI);
    for (int tap = 0; tap < 3; ++tap) {
      Seg s = make_seg(t1, bso, CI, CI, (tap - 1) * 4);
      s.act = ACT_LRELU; s.alpha = 0.2f;
      add_seg(a, s);
    }
    add_seg(a, make_seg(in, bsi, CI, CI, 0, f));   // residual_dense on x[f i]
    a.lens = lens; a.lens_mul = rate;
    PD_TRY((launch_gemm<1, 1, 4, 1, EPI_STORE, U_FD_DBLOCK>(a, st, "fd_dblock")));
  }
  return PD_OK;
}

// Kernel-predictor hidden stacks (bf16) for `nsteps` steps x every block in one launch.
// nz: [nsteps*B][nb*80] (the step-MLP output); results in ws.hall / ws.bfall, z = s*nb + n.
int fd_kp_hidden_all(const fd_model* m, float* ws, const FdWs& W, const float* condT, const float* nz,
                     int nsteps, int B, int Tc, hipStream_t st, const int* lens = nullptr) {
  const int nb = m->nblocks;
  KPArgs ka{};
  ka.condT = condT; ka.nz = nz; ka.nz_step = B * nb * CC; ka.nz_ld = nb * CC; ka.nb = nb; ka.B = B;
  for (int n = 0; n < nb; ++n) {
    const fd_model::Block& K = m->blk[n];
    ka.Win[n] = lookup_bf16(K.kin_w); ka.bin[n] = K.kin_b;
    for (int j = 0; j < 6; ++j) { ka.Wr[n][j] = lookup_bf16(K.kres_w[j]); ka.br[n][j] = K.kres_b[j]; }
    ka.Wb[n] = lookup_bf16(K.kb_w); ka.bb[n] = K.kb_b;
  }
  ka.hout = reinterpret_cast<__bf16*>(ws + W.hall); ka.Bf = ws + W.bfall; ka.Tc = Tc; ka.lens = lens;
  ProfScope ps("fd_kp_hidden", st);
  hipLaunchKernelGGL(kp_hidden_bf16_kernel, dim3(cdiv(Tc, 64), B, nsteps * nb), dim3(256), 0, st, ka);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// Does the last LVC block run as the fused kernel (upsample + first conv + final update)?
bool fd_final_fused(const fd_model* m) {
  const int n = m->nblocks - 1;
  return m->pool_bf && m->lvc_ts > 0 && m->hops[n] % 32 == 0 && m->lvc_fuse && m->ratios[n] >= 4;
}

// The sampler update fused into the last LVC block (FIN): audio_out = (xa - ce eps)/den + sig z.
struct FdFinal {
  float* audio_out;
  const float* noise;
  float ce, den, sig;
  unsigned long long seed;
  unsigned stream;
  const int* uid;
};

template <int TS, bool UPS, bool AUD, bool FIN, bool PF, bool SUB = false, int TPW = 2>
void launch_lvc_block_t(const LvcBlockArgs& la, long long Tout, int B, hipStream_t st) {
  hipLaunchKernelGGL((lvc_block_bf16_kernel<TS, UPS, AUD, FIN, PF, SUB, TPW>), dim3(cdiv(Tout, TS), B),
                     dim3(LbGeo<TS, TPW>::NT), 0, st, la);
}
template <int TS, int TPW = 2>
int launch_lvc_block_ts(const LvcBlockArgs& la, bool ups, bool aud, bool fin, bool pf, long long Tout, int B,
                        hipStream_t st) {
  if constexpr (TPW == 1) {   // one tile per wave (hop >= 32 only)
    if (la.hop < 32 || !ups || (aud != fin)) { set_error("lvc_block: one tile per wave needs hop >= 32 and the fused upsample"); return PD_ERR_ARG; }
    if (fin) {
      if (pf) launch_lvc_block_t<TS, true, true, true, true, false, 1>(la, Tout, B, st);
      else launch_lvc_block_t<TS, true, true, true, false, false, 1>(la, Tout, B, st);
    } else {
      if (pf) launch_lvc_block_t<TS, true, false, false, true, false, 1>(la, Tout, B, st);
      else launch_lvc_block_t<TS, true, false, false, false, false, 1>(la, Tout, B, st);
    }
    PD_LAUNCH_CHECK();
    return PD_OK;
  }
  if (la.hop < 32) {   // several frames per 32-row tile (the hop-8 block)
    if (aud || fin) { set_error("lvc_block: audio/final fusion needs hop >= 32"); return PD_ERR_ARG; }
    if (ups) launch_lvc_block_t<TS, true, false, false, false, true>(la, Tout, B, st);
    else launch_lvc_block_t<TS, false, false, false, false, true>(la, Tout, B, st);
  } else if (!ups) {
    if (aud || fin) { set_error("lvc_block: audio/final fusion needs the fused upsample"); return PD_ERR_ARG; }
    launch_lvc_block_t<TS, false, false, false, false>(la, Tout, B, st);
  } else if (!aud && !fin) {
    if (pf) launch_lvc_block_t<TS, true, false, false, true>(la, Tout, B, st);
    else launch_lvc_block_t<TS, true, false, false, false>(la, Tout, B, st);
  } else if (aud && !fin) {
    launch_lvc_block_t<TS, true, true, false, false>(la, Tout, B, st);
  } else if (aud && fin) {
    if (pf) launch_lvc_block_t<TS, true, true, true, true>(la, Tout, B, st);
    else launch_lvc_block_t<TS, true, true, true, false>(la, Tout, B, st);
  } else {
    set_error("lvc_block: final fusion needs the audio fusion"); return PD_ERR_ARG;
  }
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// One eps-network evaluation.  xa: audio [B][L]; condT: [B][Tc][80];
// nz: this step's per-block fc_t(emb) rows ([B][nblocks*80]).  Leaves the LVC output in
// *xout, or -- when `fin` is given and the last block is the fused LVC kernel -- applies
// the sampler update itself and sets *xout = nullptr.
// lens (device, B ints, or null): ragged batch -- utterance b is lens[b] mel frames of the padded Tc;
// every conv of the network reads zero past it ("Ragged batches").
int fd_net(const fd_model* m, float* ws, const FdWs& W, const float* xa, const float* condT,
           const float* nz, int step, int B, int Tc, float** xout, hipStream_t st,
           const FdFinal* fin = nullptr, bool side = false, const int* lens = nullptr) {
  const int nb = m->nblocks;
  if (lens && m->pool_bf && m->lvc_ts == 0) {
    set_error("FD_OPT_LVC_TS 0 (per-layer LVC launches) does not take ragged batches (lens)");
    return PD_ERR_UNSUPPORTED;
  }
  const long long L = (long long)Tc * m->hops[nb - 1];
  const bool bf = m->pool_bf != nullptr;
  // whole-block LVC kernel with its prologue/epilogue fusions (bf16)
  // (hop % 32 == 0: one frame per 32-row tile; hop | 32: several, masked per frame)
  auto fused_block = [&](int n) { return fd_block_fused(m, n); };
  auto fused_ups = [&](int n) { return fused_block(n) && m->lvc_fuse && m->ratios[n] >= 4; };
  const bool aud = fd_final_fused(m);              // a0 = first_conv(audio) recomputed by its consumers
  float* a0 = ws + W.a0;
  if (!aud) {
    ProfScope ps("fd_first_conv", st);
    hipLaunchKernelGGL(first_conv_kernel, dim3(cdiv(L, 32), B), dim3(256), 0, st, xa, m->first_w,
                       m->first_b, a0, (int)L, lens, m->hops[nb - 1]);
    PD_LAUNCH_CHECK();
  }
  // downsample chain: a0 -> d[0] -> ... -> d[nb-1]   (FastDiff_model.py:89-93)
  const float* cur = a0;
  long long Lc = L;
  const float* downs[4];
  for (int n = 0; n < nb; ++n) {
    downs[n] = cur;
    const int f = m->ratios[nb - 1 - n];
    Lc /= f;
    PD_TRY(dblock(m->dn[n], cur, ws + W.d[n], ws + W.dtmp0, ws + W.dtmp1, B, (int)Lc, f, st, m,
                  n == 0 && aud ? xa : nullptr, lens, (int)(Lc / Tc)));
    cur = ws + W.d[n];
  }
  // LVC blocks (FastDiff_model.py:95-97)
  const float* x = cur;   // [B][Tc][32]
  float* bufs[2] = {ws + W.X0, ws + W.X1};
  long long Tin = Tc;
  for (int n = 0; n < nb; ++n) {
    const fd_model::Block& K = m->blk[n];
    const int r = m->ratios[n], hop = m->hops[n];
    const float* ad = downs[nb - 1 - n];
    float* xn = bufs[n & 1];
    const long long Tout = Tin * r;
    const long long bsC = (long long)Tc * CC, bsH = (long long)Tc * HK;
    // --- kernel predictor on c + fc_t(emb)   (modules.py:202-204, 320-343)
    const float* hk = nullptr;   // final h  [B][Tc][64] (fp32 path)
    const __bf16* hkb = nullptr; // final h, bf16 path
    float* Bfp = ws + W.Bf;      // LVC biases of this block [B][Tc][256]
    if (bf) {
      // computed for every step and block up front (fd_kp_hidden_all)
      const size_t z = (size_t)step * nb + n;
      hkb = reinterpret_cast<const __bf16*>(ws + W.hall) + z * B * Tc * HK;
      Bfp = ws + W.bfall + z * B * Tc * 2 * CI * NLY;
    } else {
    {
      GemmArgs a = make_gemm(B, Tc, HK, K.kin_w, 5 * 96, K.kin_b, ws + W.h0, bsH, HK);
      for (int tap = 0; tap < 5; ++tap) {
        Seg s = make_seg(condT, bsC, CC, CC, tap - 2);
        s.add_vec = nz + n * CC;
        s.add_ld = nb * CC;
        add_seg(a, s);
      }
      a.act = ACT_LRELU; a.alpha = 0.1f;
      a.lens = lens; a.lens_mul = 1;
      PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_FD_KP_IN>(a, st, "fd_kp_in")));
    }
    const float* src = ws + W.h0;
    float* rbuf[2] = {ws + W.ra, ws + W.rb};
    for (int j = 0; j < 6; ++j) {
      float* dst = rbuf[j & 1];
      GemmArgs a = make_gemm(B, Tc, HK, K.kres_w[j], 3 * HK, K.kres_b[j], dst, bsH, HK);
      for (int tap = 0; tap < 3; ++tap) add_seg(a, make_seg(src, bsH, HK, HK, tap - 1));
      a.act = ACT_LRELU; a.alpha = 0.1f;
      if (j == 5) { a.res = ws + W.h0; a.res_bs = bsH; a.res_ld = HK; }   // h + R(h)
      a.lens = lens; a.lens_mul = 1;
      PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_FD_KP_RES>(a, st, "fd_kp_res")));
      src = dst;
    }
    hk = src;
    {
      GemmArgs a = make_gemm(B, Tc, 2 * CI * NLY, K.kb_w, 3 * HK, K.kb_b, ws + W.Bf,
                             (long long)Tc * 2 * CI * NLY, 2 * CI * NLY);
      for (int tap = 0; tap < 3; ++tap) add_seg(a, make_seg(hk, bsH, HK, HK, tap - 1));
      a.lens = lens; a.lens_mul = 1;
      PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_FD_KP_BIAS>(a, st, "fd_kp_bias")));
    }
    }
    if (fused_block(n)) {
      // every layer's kernels first (frame-major bf16), then the whole block in one launch
      const bool ups = fused_ups(n), last = n == nb - 1;
      const bool fuse_fin = ups && last && fin != nullptr;
      if (!ups) {   // separate upsample (modules.py:205-206)
        ProfScope ps("fd_upsample", st);
        hipLaunchKernelGGL(upsample_kernel, dim3(cdiv(Tin, 32), r, B), dim3(256), 0, st, x, K.up_w, K.up_b,
                           xn, (int)Tin, r, r / 2 + r % 2, lens, (int)(Tin / Tc));
        PD_LAUNCH_CHECK();
      }
      __bf16* Kb = reinterpret_cast<__bf16*>(ws + W.Kf);
      // FD_OPT_KP_CHUNK: kernel predictor + LVC block per chunk of utterances, so a chunk's
      // kernel tensor can still be on-die (Infinity Cache) when the LVC block reads it
      const int cb = (!side && m->kp_chunk > 0 && m->kp_chunk < B) ? m->kp_chunk : B;
      for (int b0 = 0; b0 < B; b0 += cb) {
      const int nbk = B - b0 < cb ? B - b0 : cb;
      const int rows = nbk * Tc;
      __bf16* Kc = Kb;
      if (side) {   // written on the side stream (fd_sample)
        Kc += (size_t)n * rows * NLY * KPERLAYER;
        PD_HIP(hipStreamWaitEvent(st, m->ev_kp[n], 0));
      } else {
        PD_TRY(kp_kernels_all(K, hkb + (size_t)b0 * Tc * HK, Kc, nbk, Tc, st, true));
      }
      LvcBlockArgs la{};
      for (int i = 0; i < NLY; ++i) {
        la.Kf[i] = Kc + (size_t)i * rows * KPERLAYER;
        la.Wc[i] = lookup_bf16(K.cv_w[i]);
        la.bc[i] = K.cv_b[i];
      }
      // never write the buffer this launch reads: with the upsample fused, x_prev is the
      // previous block's output (the other ping-pong buffer, or the DBlock output)
      la.xin = (ups ? x : xn) + (size_t)b0 * (ups ? Tin : Tout) * CI;
      la.xout = (ups ? xn : ws + W.y) + (size_t)b0 * Tout * CI;
      la.a = (last && aud) ? nullptr : ad + (size_t)b0 * Tout * CI;
      la.Bf = Bfp + (size_t)b0 * Tc * 2 * CI * NLY; la.Tc = Tc; la.hop = hop; la.b_off = b0;
      la.lens = lens ? lens + b0 : nullptr;
      la.prio = m->lvc_prio;
      la.Wup = lookup_bf16(K.upf_w); la.bup = K.up_b; la.r = r; la.p = r / 2 + r % 2;
      la.audio = xa + (size_t)b0 * L; la.fw = m->first_w; la.fb = m->first_b;
      la.wfin = m->final_w; la.bfin = m->final_b;
      if (fuse_fin) {
        la.audio_out = fin->audio_out + (size_t)b0 * L; la.noise = fin->noise ? fin->noise + (size_t)b0 * L : nullptr;
        la.ce = fin->ce; la.den = fin->den;
        la.sig = fin->sig; la.seed = fin->seed; la.stream = fin->stream; la.uid = fin->uid;
      }
      {
        ProfScope ps(fuse_fin ? "fd_lvc_block_final" : hop < 32 ? "fd_lvc_block_sub" : ups ? "fd_lvc_block_ups"
                                                                                   : "fd_lvc_block", st);
        const int ts = hop < 32 ? m->lvc_ts_sub : m->lvc_ts;
        const bool pf = m->lvc_pf && hop % 64 == 0;   // a 64-row tile pair shares one frame
        // r06: the persistent kernel -- the final block (upsample r = 4, hop 256) and the hop-64 block
        // (upsample r = 8, audio_down from HBM): the phase GEMMs one phase per wave (NW % r == 0), the
        // frames' biases staged for hop >= 256 / 64
        const bool ps_fin = fuse_fin && r == 4 && hop % 256 == 0;
        const bool ps_ups = ups && !fuse_fin && !(last && aud) && la.a && r == 8 && hop % 64 == 0;
        if (pf && ts == 384 && m->lvc_tpw == 2 && m->lvc_ps && (ps_fin || ps_ups)) {
          // one block per CU (a multiple of 8 blocks keeps the XCD-aware tile order; any grid size walks
          // every tile once)
          int dev = 0, ncu = 0;
          PD_HIP(hipGetDevice(&dev));
          PD_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
          const int ntx = (int)cdiv(Tout, 384), ntiles = ntx * nbk;
          const int grid = ntiles <= ncu ? ntiles : ncu >= 8 ? ncu / 8 * 8 : ncu;
          if (ps_fin) hipLaunchKernelGGL(lvc_ps_kernel<true>, dim3(grid), dim3(512), 0, st, la, ntx, ntiles);
          else hipLaunchKernelGGL(lvc_ps_kernel<false>, dim3(grid), dim3(512), 0, st, la, ntx, ntiles);
          PD_LAUNCH_CHECK();
        } else if (ts == 256) PD_TRY(launch_lvc_block_ts<256>(la, ups, last && aud, fuse_fin, pf, Tout, nbk, st));
        else if (ts == 384 && m->lvc_tpw == 1 && hop >= 32 && ups && (last && aud) == fuse_fin)
          PD_TRY((launch_lvc_block_ts<384, 1>(la, ups, last && aud, fuse_fin, pf, Tout, nbk, st)));
        else if (ts == 384) PD_TRY(launch_lvc_block_ts<384>(la, ups, last && aud, fuse_fin, pf, Tout, nbk, st));
        else PD_TRY(launch_lvc_block_ts<128>(la, ups, last && aud, fuse_fin, pf, Tout, nbk, st));
      }
      }
      float* xo = ups ? xn : ws + W.y;
      if (side) PD_HIP(hipEventRecord(m->ev_lvc[n], st));   // ring slot n free again
      if (fuse_fin) { *xout = nullptr; return PD_OK; }
      x = xo;
      Tin = Tout;
      continue;
    }
    // --- upsample (modules.py:205-206)
    {
      const int p = r / 2 + r % 2;
      ProfScope ps("fd_upsample", st);
      hipLaunchKernelGGL(upsample_kernel, dim3(cdiv(Tin, 32), r, B), dim3(256), 0, st, x, K.up_w, K.up_b,
                         xn, (int)Tin, r, p, lens, (int)(Tin / Tc));
      PD_LAUNCH_CHECK();
    }
    // --- 4 LVC layers (modules.py:208-217)
    if (bf) PD_TRY(kp_kernels_all(K, hkb, reinterpret_cast<__bf16*>(ws + W.Kf), B, Tc, st, false));   // all 4 layers
    for (int i = 0; i < NLY; ++i) {
      const __bf16* Kbl = reinterpret_cast<const __bf16*>(ws + W.Kf) + (size_t)i * B * Tc * KPERLAYER;
      if (!bf) {
        GemmArgs a = make_gemm(B, Tc, KPERLAYER, K.kk_w + (size_t)i * KPERLAYER * 3 * HK, 3 * HK,
                               K.kk_b + (size_t)i * KPERLAYER, ws + W.Kf, (long long)Tc * KPERLAYER,
                               KPERLAYER);
        for (int tap = 0; tap < 3; ++tap) add_seg(a, make_seg(hk, bsH, HK, HK, tap - 1));
        a.lens = lens; a.lens_mul = 1;
        PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_FD_KP_KERNEL>(a, st, "fd_kp_kernel")));
      }
      const int dil = (int)std::pow(3, i);
      if (bf && hop % 64 == 0) {
        // one fused launch per layer: pre-conv + LVC + gate (bf16 MFMA)
        ProfScope ps("fd_lvc_fused", st);
        const __bf16* Kb = Kbl;
        const __bf16* Wc = lookup_bf16(K.cv_w[i]);
        if (hop % 128 == 0)
          hipLaunchKernelGGL(lvc_fused_bf16_kernel<128>, dim3(B * Tc * (hop / 128)), dim3(256), 0, st, xn, ad, Kb,
                             KPERLAYER, Bfp + i * 2 * CI, 2 * CI * NLY, Wc, K.cv_b[i], Tc, hop, dil);
        else
          hipLaunchKernelGGL(lvc_fused_bf16_kernel<64>, dim3(B * Tc * (hop / 64)), dim3(128), 0, st, xn, ad, Kb,
                             KPERLAYER, Bfp + i * 2 * CI, 2 * CI * NLY, Wc, K.cv_b[i], Tc, hop, dil);
      } else {
        {  // y = lrelu(conv_dil3^i(lrelu(x + a)) + b)
          GemmArgs a = make_gemm(B, (int)Tout, CI, K.cv_w[i], 96, K.cv_b[i], ws + W.y, Tout * CI, CI);
          for (int tap = 0; tap < 3; ++tap) {
            Seg sg = make_seg(xn, Tout * CI, CI, CI, (tap - 1) * dil);
            sg.add_ten = ad;
            sg.act = ACT_LRELU; sg.alpha = 0.2f;
            add_seg(a, sg);
          }
          a.act = ACT_LRELU; a.alpha = 0.2f;
          a.lens = lens; a.lens_mul = hop;
          PD_TRY((launch_gemm<1, 1, 4, 1, EPI_STORE, U_FD_LVC_PRECONV>(a, st, "fd_lvc_preconv")));
        }
        ProfScope ps("fd_lvc", st);
        if (bf)
          hipLaunchKernelGGL(lvc_kernel<__bf16>, dim3(B * Tc), dim3(256), 0, st, xn, ad, ws + W.y,
                             Kbl, KPERLAYER, Bfp + i * 2 * CI,
                             2 * CI * NLY, Tc, hop, lens);
        else
          hipLaunchKernelGGL(lvc_kernel<float>, dim3(B * Tc), dim3(256), 0, st, xn, ad, ws + W.y, ws + W.Kf,
                             KPERLAYER, Bfp + i * 2 * CI, 2 * CI * NLY, Tc, hop, lens);
      }
      PD_LAUNCH_CHECK();
    }
    x = xn;
    Tin = Tout;
  }
  *xout = const_cast<float*>(x);
  return PD_OK;
}

}  // namespace

extern "C" {

int fd_create(const fd_dims* dims, const float* const* params, int dtype, void* stream, fd_model** out) {
  PD_CHECK_ARG(dims && params && out, "null pointer");
  PD_CHECK_ARG(dtype == PD_DTYPE_F32 || dtype == PD_DTYPE_BF16, "dtype must be PD_DTYPE_F32 or PD_DTYPE_BF16");
  PD_CHECK_ARG(dims->audio_channels == 1 && dims->inner_channels == CI && dims->cond_channels == CC &&
                   dims->lvc_layers_each_block == NLY && dims->lvc_kernel_size == 3 &&
                   dims->kpnet_hidden_channels == HK && dims->kpnet_conv_size == 3 &&
                   dims->step_embed_in == EMB_IN && dims->step_embed_mid == EMB_MID &&
                   dims->step_embed_out == EMB_OUT,
               "only the FastDiff base.yaml architecture (32/80/64, 4 LVC layers) is supported");
  PD_CHECK_ARG(dims->num_blocks >= 1 && dims->num_blocks <= 4, "num_blocks in [1,4]");
  hipStream_t st = (hipStream_t)stream;
  fd_model* m = new fd_model();
  m->nblocks = dims->num_blocks;
  m->dtype = dtype;
  int hop = 1;
  for (int n = 0; n < m->nblocks; ++n) {
    m->ratios[n] = dims->upsample_ratios[n];
    if (m->ratios[n] < 2 || m->ratios[n] > 16) { delete m; set_error("upsample ratio in [2,16]"); return PD_ERR_ARG; }
    hop *= m->ratios[n];
    m->hops[n] = hop;
  }
  // allocation plan
  std::vector<std::pair<float**, size_t>> plan;
  plan.push_back({&m->fc1_w, (size_t)EMB_MID * EMB_IN}); plan.push_back({&m->fc1_b, EMB_MID});
  plan.push_back({&m->fc2_w, (size_t)EMB_OUT * EMB_MID}); plan.push_back({&m->fc2_b, EMB_OUT});
  plan.push_back({&m->first_w, 224}); plan.push_back({&m->first_b, CI});
  plan.push_back({&m->final_w, 224}); plan.push_back({&m->final_b, 1});
  for (int n = 0; n < m->nblocks; ++n) {
    auto& K = m->blk[n];
    plan.push_back({&K.up_w, (size_t)2 * m->ratios[n] * CI * CI}); plan.push_back({&K.up_b, CI});
    plan.push_back({&K.upf_w, (size_t)2 * m->ratios[n] * CI * CI});
    plan.push_back({&K.fct_w, (size_t)CC * EMB_OUT}); plan.push_back({&K.fct_b, CC});
    plan.push_back({&K.kin_w, (size_t)HK * 5 * 96}); plan.push_back({&K.kin_b, HK});
    for (int j = 0; j < 6; ++j) { plan.push_back({&K.kres_w[j], (size_t)HK * 3 * HK}); plan.push_back({&K.kres_b[j], HK}); }
    plan.push_back({&K.kk_w, (size_t)NLY * KPERLAYER * 3 * HK}); plan.push_back({&K.kk_b, (size_t)NLY * KPERLAYER});
    plan.push_back({&K.kb_w, (size_t)2 * CI * NLY * 3 * HK}); plan.push_back({&K.kb_b, (size_t)2 * CI * NLY});
    for (int i = 0; i < NLY; ++i) { plan.push_back({&K.cv_w[i], (size_t)CI * 96}); plan.push_back({&K.cv_b[i], CI}); }
  }
  for (int n = 0; n < m->nblocks; ++n) {
    auto& D = m->dn[n];
    plan.push_back({&D.c0_w, (size_t)CI * 96}); plan.push_back({&D.c0_b, CI});
    plan.push_back({&D.c1_w, (size_t)CI * 96}); plan.push_back({&D.c1_b, CI});
    plan.push_back({&D.c2_w, (size_t)CI * 128}); plan.push_back({&D.c2_b, CI});
  }
  size_t off = 0;
  std::vector<size_t> offs;
  for (auto& p : plan) { offs.push_back(off); off += (p.second + 63) / 64 * 64; }
  if (hipMalloc((void**)&m->pool, off * sizeof(float)) != hipSuccess) {
    delete m; set_error("hipMalloc failed for FastDiff weights"); return PD_ERR_HIP;
  }
  for (size_t i = 0; i < plan.size(); ++i) *plan[i].first = m->pool + offs[i];

  auto run = [&]() -> int {
    PD_HIP(hipMemsetAsync(m->pool, 0, off * sizeof(float), st));
    auto cp = [&](float* dst, const float* src, size_t n) -> int {
      PD_HIP(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, st));
      return PD_OK;
    };
    int p = 0;
    auto nxt = [&]() { const float* q = params[p++]; return q; };
    // order: see include/prodiff_hip.h (FD_PARAM_ORDER)
    {
      const float* w = nxt(); const float* b = nxt();
      PD_TRY(cp(m->first_w, w, 224)); PD_TRY(cp(m->first_b, b, CI));
    }
    PD_TRY(cp(m->fc1_w, nxt(), (size_t)EMB_MID * EMB_IN)); PD_TRY(cp(m->fc1_b, nxt(), EMB_MID));
    PD_TRY(cp(m->fc2_w, nxt(), (size_t)EMB_OUT * EMB_MID)); PD_TRY(cp(m->fc2_b, nxt(), EMB_OUT));
    for (int n = 0; n < m->nblocks; ++n) {
      auto& K = m->blk[n];
      const int r = m->ratios[n];
      {
        const float* w = nxt();
        hipLaunchKernelGGL(pack_upsample_kernel, dim3(cdiv(CI * CI * 2 * r, 256)), dim3(256), 0, st, K.up_w, w, 2 * r);
        PD_LAUNCH_CHECK();
        hipLaunchKernelGGL(pack_upsample_phase_kernel, dim3(cdiv(CI * CI * 2 * r, 256)), dim3(256), 0, st, K.upf_w,
                           K.up_w, r);
        PD_LAUNCH_CHECK();
        PD_TRY(cp(K.up_b, nxt(), CI));
      }
      PD_TRY(pack_conv(K.kin_w, 5 * 96, 0, 0, 96, nxt(), HK, CC, 5, st));
      PD_TRY(cp(K.kin_b, nxt(), HK));
      for (int j = 0; j < 6; ++j) {
        PD_TRY(pack_conv(K.kres_w[j], 3 * HK, 0, 0, HK, nxt(), HK, HK, 3, st));
        PD_TRY(cp(K.kres_b[j], nxt(), HK));
      }
      {
        const float* w = nxt(); const float* b = nxt();
        const long long total = (long long)NLY * KPERLAYER * HK * 3;
        hipLaunchKernelGGL(pack_kernel_conv_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, K.kk_w, K.kk_b, w, b);
        PD_LAUNCH_CHECK();
      }
      PD_TRY(pack_conv(K.kb_w, 3 * HK, 0, 0, HK, nxt(), 2 * CI * NLY, HK, 3, st));
      PD_TRY(cp(K.kb_b, nxt(), 2 * CI * NLY));
      PD_TRY(cp(K.fct_w, nxt(), (size_t)CC * EMB_OUT));
      PD_TRY(cp(K.fct_b, nxt(), CC));
      for (int i = 0; i < NLY; ++i) {
        PD_TRY(pack_conv(K.cv_w[i], 96, 0, 0, CI, nxt(), CI, CI, 3, st));
        PD_TRY(cp(K.cv_b[i], nxt(), CI));
      }
    }
    for (int n = 0; n < m->nblocks; ++n) {
      auto& D = m->dn[n];
      const float* rw = nxt(); const float* rb = nxt();
      const float* w0 = nxt(); const float* b0 = nxt();
      const float* w1 = nxt(); const float* b1 = nxt();
      const float* w2 = nxt(); const float* b2 = nxt();
      PD_TRY(pack_conv(D.c0_w, 96, 0, 0, CI, w0, CI, CI, 3, st)); PD_TRY(cp(D.c0_b, b0, CI));
      PD_TRY(pack_conv(D.c1_w, 96, 0, 0, CI, w1, CI, CI, 3, st)); PD_TRY(cp(D.c1_b, b1, CI));
      PD_TRY(pack_conv(D.c2_w, 128, 0, 0, CI, w2, CI, CI, 3, st));
      PD_TRY(pack_conv(D.c2_w, 128, 0, 96, CI, rw, CI, CI, 1, st));
      PD_TRY(add_vectors(D.c2_b, b2, rb, CI, st));
    }
    {
      const float* w = nxt(); const float* b = nxt();
      hipLaunchKernelGGL(pack_final_kernel, dim3(1), dim3(256), 0, st, m->final_w, w);
      PD_LAUNCH_CHECK();
      PD_TRY(cp(m->final_b, b, 1));
    }
    if (p != FD_NUM_PARAMS(m->nblocks)) { set_error("fd_create: parameter count mismatch"); return PD_ERR_ARG; }
    if (dtype == PD_DTYPE_BF16) {
      PD_HIP(hipMalloc((void**)&m->pool_bf, off * sizeof(__bf16)));
      PD_TRY(convert_f32_bf16(m->pool, m->pool_bf, (long long)off, st));
      register_bf16_pool(m->pool, off, m->pool_bf);
      // pre-scaled kernel-predictor weights of every block (bf16 rows, fp32 biases)
      const size_t nw = (size_t)NLY * KPERLAYER * 3 * HK, nbias = (size_t)NLY * KPERLAYER;
      PD_HIP(hipMalloc(&m->kps, m->nblocks * (nw * sizeof(__bf16) + nbias * sizeof(float))));
      for (int n = 0; n < m->nblocks; ++n) {
        auto& K = m->blk[n];
        K.kks_b = reinterpret_cast<float*>(m->kps) + n * nbias;
        K.kks_w = reinterpret_cast<__bf16*>(reinterpret_cast<float*>(m->kps) + m->nblocks * nbias) + n * nw;
        hipLaunchKernelGGL(kp_prescale_kernel, dim3(cdiv((long long)nw, 256)), dim3(256), 0, st, K.kk_w, K.kk_b, K.kks_w,
                           K.kks_b);
        PD_LAUNCH_CHECK();
      }
    }
    return PD_OK;
  };
  for (int i = 0; i < FD_NUM_PARAMS(m->nblocks); ++i)
    if (!params[i]) { (void)hipFree(m->pool); delete m; set_error("null parameter " + std::to_string(i)); return PD_ERR_ARG; }
  int rc = run();
  if (rc != PD_OK) {
    (void)hipFree(m->pool);
    if (m->pool_bf) (void)hipFree(m->pool_bf);
    if (m->kps) (void)hipFree(m->kps);
    delete m;
    return rc;
  }
  *out = m;
  return PD_OK;
}

void fd_destroy(fd_model* m) {
  if (!m) return;
  if (m->side) {
    (void)hipStreamSynchronize(m->side);
    (void)hipStreamDestroy(m->side);
    (void)hipEventDestroy(m->ev_hidden);
    for (int n = 0; n < 4; ++n) {
      if (m->ev_kp[n]) (void)hipEventDestroy(m->ev_kp[n]);
      if (m->ev_lvc[n]) (void)hipEventDestroy(m->ev_lvc[n]);
    }
  }
  if (m->pool_bf) {
    unregister_bf16_pool(m->pool);
    (void)hipFree(m->pool_bf);
  }
  if (m->kps) (void)hipFree(m->kps);
  (void)hipFree(m->pool);
  delete m;
}

int fd_hop(const fd_model* m) { return m ? m->hops[m->nblocks - 1] : 0; }

size_t fd_workspace_size(const fd_model* m, int B, int Tc, int S) {
  if (!m || B < 0 || Tc < 0 || S < 1) return 0;
  return fd_layout(m, B, Tc, S < FD_STEP_CHUNK ? S : FD_STEP_CHUNK).total;
}

int fd_draw_x_T(const fd_model* m, float* x_T, int B, int Tc, unsigned long long seed, const int* utt_ids,
                void* stream) {
  PD_CHECK_ARG(m && x_T, "null pointer");
  PD_CHECK_ARG(B >= 0 && Tc >= 0, "bad shape");
  const long long L = (long long)Tc * m->hops[m->nblocks - 1];
  return fill_normal_utt(x_T, B, L, seed, 0xFFFF0001u, utt_ids, (hipStream_t)stream);   // fd_sample_coefs' x_T stream
}

int fd_set_option(fd_model* m, int option, int value) {
  PD_CHECK_ARG(m, "null pointer");
  switch (option) {
    case FD_OPT_LVC_TS:
      PD_CHECK_ARG(value == 0 || value == 128 || value == 256 || value == 384, "FD_OPT_LVC_TS in {0,128,256,384}");
      m->lvc_ts = value;
      m->lvc_pf = value >= 384;   // the register prefetch is tuned for the 384 tile
      return PD_OK;
    case FD_OPT_LVC_TS_SUB:
      PD_CHECK_ARG(value == 128 || value == 256 || value == 384, "FD_OPT_LVC_TS_SUB in {128,256,384}");
      m->lvc_ts_sub = value;
      return PD_OK;
    case FD_OPT_LVC_FUSE: m->lvc_fuse = value != 0; return PD_OK;
    case FD_OPT_LVC_PF: m->lvc_pf = value != 0; return PD_OK;
    case FD_OPT_LVC_SUB: m->lvc_sub = value != 0; return PD_OK;
    case FD_OPT_KP_SIDE: m->kp_side = value != 0; return PD_OK;
    case FD_OPT_KP_CHUNK:
      PD_CHECK_ARG(value >= 0, "FD_OPT_KP_CHUNK >= 0");
      m->kp_chunk = value;
      return PD_OK;
    case FD_OPT_LVC_PRIO:
      PD_CHECK_ARG(value == 0 || value == 1, "FD_OPT_LVC_PRIO in {0,1}");
      m->lvc_prio = value;
      return PD_OK;
    case FD_OPT_LVC_PS:
      PD_CHECK_ARG(value == 0 || value == 1, "FD_OPT_LVC_PS in {0,1}");
      m->lvc_ps = value;
      return PD_OK;
    case FD_OPT_LVC_TPW:
      PD_CHECK_ARG(value == 1 || value == 2, "FD_OPT_LVC_TPW in {1,2}");
      m->lvc_tpw = value;
      return PD_OK;
    default: break;
  }
  set_error("fd_set_option: unknown option " + std::to_string(option));
  return PD_ERR_ARG;
}

int fd_forward(const fd_model* m, const float* audio, const float* cond, const float* steps, float* eps,
               int B, int Tc, void* workspace, size_t ws_bytes, void* stream) {
  PD_CHECK_ARG(m && audio && cond && steps && eps && workspace, "null pointer");
  PD_CHECK_ARG(B > 0 && Tc > 0, "B and T' must be positive");
  FdWs W = fd_layout(m, B, Tc, 1);
  if (ws_bytes < W.total) { set_error("workspace too small"); return PD_ERR_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  const long long L = (long long)Tc * m->hops[m->nblocks - 1];
  PD_HIP(hipMemcpyAsync(ws + W.steps, steps, sizeof(float) * B, hipMemcpyDeviceToDevice, st));
  PD_TRY(fd_step_mlp(m, ws, W, B, st));
  PD_TRY(transpose_ct_to_tc(cond, ws + W.condT, B, CC, Tc, st));
  float* x = nullptr;
  if (m->pool_bf) PD_TRY(fd_kp_hidden_all(m, ws, W, ws + W.condT, ws + W.nz, 1, B, Tc, st));
  PD_TRY(fd_net(m, ws, W, audio, ws + W.condT, ws + W.nz, 0, B, Tc, &x, st));
  hipLaunchKernelGGL(final_conv_kernel, dim3(cdiv(L, 256), B), dim3(256), 0, st, x, m->final_w, m->final_b,
                     eps, (float*)nullptr, 0.f, 0.f, 0.f, (const float*)nullptr, 0ull, 0u, (const int*)nullptr, L,
                     (const int*)nullptr, 1);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

int fd_sample_coefs(const fd_model* m, const float* mel, const float* ce_, const float* den_, const float* sg_,
                    const float* steps_, int N, const float* x_T, const float* noise, unsigned long long seed,
                    const int* utt_ids, const int* lens, int draw0, float* wav, int B, int Tc, void* workspace,
                    size_t ws_bytes, void* stream) {
  PD_CHECK_ARG(m && mel && ce_ && den_ && sg_ && steps_ && wav && workspace, "null pointer");
  PD_CHECK_ARG(B > 0 && Tc > 0 && N >= 1 && draw0 >= 0, "bad B/T'/N/draw0");
  // Long schedules (the 200- and 1000-step ones, fastdiff.py:58-61) run in chunks of
  // FD_STEP_CHUNK steps: each chunk's step embeddings and kernel-predictor hidden stacks
  // are computed in one batched launch, so the workspace is bounded by the chunk.
  const int CH = N < FD_STEP_CHUNK ? N : FD_STEP_CHUNK;
  FdWs W = fd_layout(m, B, Tc, CH);
  if (ws_bytes < W.total) { set_error("workspace too small"); return PD_ERR_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  const long long L = (long long)Tc * m->hops[m->nblocks - 1];
  // With the update fused into the last LVC block, step j reads one audio buffer and
  // writes the other (its neighbours' halos still read the old samples): start in the
  // buffer that makes the last step land in `wav`.
  const bool fused = fd_final_fused(m);
  float* cur = (!fused || N % 2 == 0) ? wav : ws + W.wav2;
  float* other = cur == wav ? ws + W.wav2 : wav;
  // x_T ~ N(0,1)  (util.py:208)
  if (x_T) {
    PD_HIP(hipMemcpyAsync(cur, x_T, sizeof(float) * B * L, hipMemcpyDeviceToDevice, st));
  } else {
    PD_TRY(fill_normal_utt(cur, B, L, seed, 0xFFFF0001u, utt_ids, st));
  }
  const bool side = fd_kp_side(m);
  if (side && !m->side) {
    int lo = 0, hi = 0;
    PD_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));   // lo = least urgent
    PD_HIP(hipStreamCreateWithPriority(&m->side, hipStreamNonBlocking, lo));
    PD_HIP(hipEventCreateWithFlags(&m->ev_hidden, hipEventDisableTiming));
    for (int b = 0; b < m->nblocks; ++b) {
      PD_HIP(hipEventCreateWithFlags(&m->ev_kp[b], hipEventDisableTiming));
      PD_HIP(hipEventCreateWithFlags(&m->ev_lvc[b], hipEventDisableTiming));
    }
  }
  const int nb = m->nblocks, rows = B * Tc;
  for (int j0 = 0; j0 < N; j0 += CH) {
    const int nc = N - j0 < CH ? N - j0 : CH;
    // the chunk's step embeddings at once
    std::vector<float> sv(nc);
    for (int j = 0; j < nc; ++j) sv[j] = steps_[j0 + j];
    PD_TRY(fill_steps(ws + W.steps, sv.data(), nc, B, st));
    PD_TRY(fd_step_mlp(m, ws, W, nc * B, st));
    if (m->pool_bf) PD_TRY(fd_kp_hidden_all(m, ws, W, mel, ws + W.nz, nc, B, Tc, st, lens));
    if (side) {
      PD_HIP(hipEventRecord(m->ev_hidden, st));
      PD_HIP(hipStreamWaitEvent(m->side, m->ev_hidden, 0));
    }
    for (int jl = 0; jl < nc; ++jl) {
      const int j = j0 + jl;
      if (side) {
        // step j's kernels for every block; slot b is rewritten once step j-1's block b has run
        for (int b = 0; b < nb; ++b) {
          if (j > 0) PD_HIP(hipStreamWaitEvent(m->side, m->ev_lvc[b], 0));
          const __bf16* hkb = reinterpret_cast<const __bf16*>(ws + W.hall) + ((size_t)jl * nb + b) * rows * HK;
          __bf16* Kb = reinterpret_cast<__bf16*>(ws + W.Kf) + (size_t)b * rows * NLY * KPERLAYER;
          PD_TRY(kp_kernels_all(m->blk[b], hkb, Kb, B, Tc, m->side, true));
          PD_HIP(hipEventRecord(m->ev_kp[b], m->side));
        }
      }
      float* x = nullptr;
      // x = (x - ce eps) / den + sg z  (pass j's coefficients, fd_sample / util.py:222-231)
      const float ce = ce_[j], den = den_[j], sg = sg_[j];
      const FdFinal fin{other, noise ? noise + (size_t)j * B * L : (const float*)nullptr, ce, den, sg, seed,
                        0x10000u + draw0 + j, utt_ids};
      PD_TRY(fd_net(m, ws, W, cur, mel, ws + W.nz + (size_t)jl * B * nb * CC, jl, B, Tc, &x, st,
                    fused ? &fin : nullptr, side, lens));
      if (x == nullptr) {   // updated inside the last LVC block
        std::swap(cur, other);
        continue;
      }
      {
        ProfScope ps("fd_final_update", st);
        hipLaunchKernelGGL(final_conv_kernel, dim3(cdiv(L, 256), B), dim3(256), 0, st, x, m->final_w,
                           m->final_b, (float*)nullptr, cur, ce, den, sg, fin.noise, seed, 0x10000u + draw0 + j, utt_ids, L,
                           lens, m->hops[nb - 1]);
      }
      PD_LAUNCH_CHECK();
    }
  }
  if (cur != wav) PD_HIP(hipMemcpyAsync(wav, cur, sizeof(float) * B * L, hipMemcpyDeviceToDevice, st));
  return PD_OK;
}

int fd_sample(const fd_model* m, const float* mel, const float* beta, const float* alpha, const float* sigma,
              const float* steps, int N, const float* x_T, const float* noise, unsigned long long seed,
              const int* utt_ids, const int* lens, float* wav, int B, int Tc, void* workspace, size_t ws_bytes,
              void* stream) {
  PD_CHECK_ARG(m && mel && beta && alpha && sigma && steps && wav && workspace, "null pointer");
  PD_CHECK_ARG(N >= 1, "bad N");
  // pass j runs schedule index n = N-1-j:
  //   x = (x - beta/sqrt(1-alpha^2) eps) / sqrt(1-beta) + [n>0] sigma z   (util.py:222-226)
  std::vector<float> ce(N), den(N), sg(N), st(N);
  for (int j = 0; j < N; ++j) {
    const int n = N - 1 - j;
    ce[j] = beta[n] / sqrtf(1.f - alpha[n] * alpha[n]);
    den[j] = sqrtf(1.f - beta[n]);
    sg[j] = n > 0 ? sigma[n] : 0.f;
    st[j] = steps[n];
  }
  return fd_sample_coefs(m, mel, ce.data(), den.data(), sg.data(), st.data(), N, x_T, noise, seed, utt_ids, lens, 0,
                         wav, B, Tc, workspace, ws_bytes, stream);
}

}  // extern "C"

// Non-default compile-time knobs of this file (pd_build_config): "" for the shipped build.
namespace pd {
const char* fastdiff_build_flags() {
  return ""
#ifdef LB_TRACE
         " LB_TRACE"
#endif
#ifdef LVC_SCALAR_F32
         " LVC_SCALAR_F32"
#endif
#if DB_NW != 5
         " DB_NW"
#endif
#if DB_WPE != 5
         " DB_WPE"
#endif
#if KP_STAGGER != 0
         " KP_STAGGER"
#endif
#if KP_AUX != 0
         " KP_AUX"
#endif
#if KP_SWZ != 0
         " KP_SWZ"
#endif
      ;
}
}  // namespace pd

extern "C" int fd_fold_weight_norm(float* w, const float* g, const float* v, int cout, int per_row,
                                   void* stream) {
  PD_CHECK_ARG(w && g && v && cout > 0 && per_row > 0, "bad weight-norm arguments");
  return pd::weight_norm_fold(w, g, v, cout, per_row, (hipStream_t)stream);
}
