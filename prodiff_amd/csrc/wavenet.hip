// ProDiff WaveNet denoiser + x0-predict reverse sampler on gfx950.
//
// Reference: modules/decoder/wavenet.py:22-123 (WaveNet), modules/diffusion/
// prodiff.py:106-153 (GaussianDiffusion sampler).  See include/prodiff_hip.h
// for the C-ABI and DESIGN.md for the data layout and kernel plan.
//
// Per reverse step:   1 input-projection GEMM (+ReLU)
//                     L x [ GEMM1: dil-conv(3 taps of x+dproj) ++ cond-proj, K=3C+H,
//                                  fused sigmoid*tanh gate        -> g
//                           GEMM2: out-proj K=C, fused residual/sqrt2 + skip sum ]
//                     skip-proj GEMM (prologue 1/sqrt(L), ReLU)
//                     out-proj GEMM with the posterior update fused in its epilogue.
#include <cmath>
#include <vector>

#include "../../include/prodiff_hip.h"
#include "gemm.h"
#include "kernels.h"

using namespace pd;

struct pd_wavenet {
  int M, H, L, C, cyc, dtype;
  int ldw_in, ldw1;
  float* pool = nullptr;
  __bf16* pool_bf = nullptr;   // bf16 mirror of `pool` (PD_DTYPE_BF16), registered with launch_gemm
  size_t pool_n = 0;
  float *Win, *b_in, *W1, *b1, *W2, *b2, *Wd, *bd, *Wl1, *bl1, *Wl2, *bl2, *Ws, *bs, *Wo, *bo;
  // bf16 path, C == 256: residual-layer weights in MFMA-fragment order (wn_layer_bf16_kernel)
  __bf16* frag = nullptr;
  __bf16* W1f = nullptr;   // [L][2C/32 tiles][K/16 steps][64 lanes][8]
  __bf16* W2f = nullptr;
};

namespace {

constexpr int WNF_C = 256;   // channels the fused layer kernel is built for (base_config.yaml:211)

// dst[((nt*KS + ks)*64 + lane)*8 + j] = bf16(src[(nt*32 + lane%32) * ld + ks*16 + (lane/32)*8 + j])
__global__ void pack_frag_kernel(__bf16* dst, const float* src, int N, int K, int ld) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)N * K) return;
  const int j = (int)(i & 7), lane = (int)((i >> 3) & 63);
  const long long rest = i >> 9;
  const int KS = K / 16, ks = (int)(rest % KS), nt = (int)(rest / KS);
  const int n = nt * 32 + (lane & 31), k = ks * 16 + (lane >> 5) * 8 + j;
  dst[i] = (__bf16)src[(long long)n * ld + k];
}

// One WaveNet residual layer, bf16 MFMA, fully fused (wavenet.py:60-72):
//   z = W1 . [x(t-d)+dp; x(t)+dp; x(t+d)+dp; cond(t)] + b1      (K = 3C + H)
//   g = sigmoid(z[:C]) * tanh(z[C:])
//   o = W2 . g + b2 ;  x = (x + o[:C]) / sqrt2 ;  skip (+)= o[C:]
// Block = 32 rows (frames, may straddle utterances), 8 waves; wave w owns gate/filter
// columns [32w, 32w+32) / [C+32w, ...) of GEMM1 and residual/skip columns of GEMM2,
// so both epilogues pair their halves in registers.  The K=1024 input row lives in
// LDS (bf16); weights stream from L2 in fragment order (1 KB per wave-load).
struct WnLayerArgs {
  const float* xin;       // [B][T][C] layer input (other blocks read its halo rows,
  float* xout;            //            so the update goes to a second buffer)
  float* skip;            // [B][T][C]
  const float* cond;      // [B][T][H]
  const float* dp;        // this layer's diffusion projection, dp[b*dp_ld + c]
  int dp_ld;
  const __bf16* W1f;      // [2C/32][K1/16][64][8]
  const float* b1;        // [2C]
  const __bf16* W2f;      // [2C/32][C/16][64][8]
  const float* b2;        // [2C]
  int B, T, H, dil, first;
};

template <int KMAX>
__global__ __launch_bounds__(512) void wn_layer_bf16_kernel(const WnLayerArgs P) {
  constexpr int C = WNF_C;
  constexpr int LDA = KMAX + 8, LDG = C + 8;     // 16-B-offset rows: conflict-free b128 fragment reads
  __shared__ __attribute__((aligned(16))) __bf16 As[32 * LDA];
  __shared__ __attribute__((aligned(16))) __bf16 Gs[32 * LDG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r32 = lane & 31, h = lane >> 5;
  const int H = P.H, K1 = 3 * C + H, rows = P.B * P.T, R0 = blockIdx.x * 32;
  // stage [x(t-d)+dp; x(t)+dp; x(t+d)+dp; cond] as bf16 (zero outside each row's utterance)
  const int ng = K1 / 4;
  for (int i = tid; i < 32 * ng; i += 512) {
    const int r = i / ng, g = (i - r * ng) * 4, R = R0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (R < rows) {
      const int b = R / P.T, t = R - b * P.T;
      if (g < 3 * C) {
        const int tap = g / C, c = g - tap * C, tt = t + (tap - 1) * P.dil;
        if (tt >= 0 && tt < P.T) {
          v = *reinterpret_cast<const float4*>(P.xin + ((long long)b * P.T + tt) * C + c);
          const float4 d = *reinterpret_cast<const float4*>(P.dp + (long long)b * P.dp_ld + c);
          v.x += d.x; v.y += d.y; v.z += d.z; v.w += d.w;
        }
      } else {
        v = *reinterpret_cast<const float4*>(P.cond + ((long long)b * P.T + t) * H + (g - 3 * C));
      }
    }
    *reinterpret_cast<bf16x4*>(&As[r * LDA + g]) = bf16x4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
  }
  __syncthreads();

  // GEMM1: gate tile nt = wave, filter tile nt = 8 + wave
  const int KS1 = K1 / 16;
  const bf16x8* wg = reinterpret_cast<const bf16x8*>(P.W1f) + (long long)wave * KS1 * 64 + lane;
  const bf16x8* wf = reinterpret_cast<const bf16x8*>(P.W1f) + (long long)(8 + wave) * KS1 * 64 + lane;
  f32x16 ag, af;
#pragma unroll
  for (int r = 0; r < 16; ++r) { ag[r] = 0.f; af[r] = 0.f; }
#pragma unroll 8
  for (int ks = 0; ks < KS1; ++ks) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(&As[r32 * LDA + ks * 16 + h * 8]);
    const bf16x8 bgt = wg[ks * 64], bft = wf[ks * 64];
    ag = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bgt, ag, 0, 0, 0);
    af = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bft, af, 0, 0, 0);
  }
  {
    const int n = wave * 32 + r32;
    const float bgv = P.b1[n], bfv = P.b1[C + n];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int r = (reg & 3) + 8 * (reg >> 2) + 4 * h;
      Gs[r * LDG + n] = (__bf16)(sigmoidf_(ag[reg] + bgv) * tanhf_(af[reg] + bfv));
    }
  }
  __syncthreads();

  // GEMM2: residual tile nt = wave, skip tile nt = 8 + wave
  constexpr int KS2 = C / 16;
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(P.W2f) + (long long)wave * KS2 * 64 + lane;
  const bf16x8* wsk = reinterpret_cast<const bf16x8*>(P.W2f) + (long long)(8 + wave) * KS2 * 64 + lane;
  f32x16 ar, as_;
#pragma unroll
  for (int r = 0; r < 16; ++r) { ar[r] = 0.f; as_[r] = 0.f; }
#pragma unroll
  for (int ks = 0; ks < KS2; ++ks) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Gs[r32 * LDG + ks * 16 + h * 8]);
    ar = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, wr[ks * 64], ar, 0, 0, 0);
    as_ = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, wsk[ks * 64], as_, 0, 0, 0);
  }
  const int n = wave * 32 + r32;
  const float brv = P.b2[n], bsv = P.b2[C + n];
  const float rs2 = 0.70710678118654752440f;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int R = R0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
    if (R < rows) {
      const long long o = (long long)R * C + n;      // rows are b*T + t: contiguous [B][T][C]
      P.xout[o] = (P.xin[o] + ar[reg] + brv) * rs2;
      P.skip[o] = (P.first ? 0.f : P.skip[o]) + as_[reg] + bsv;
    }
  }
}

struct WsLayout {
  size_t x, x2, g, skip, hs, xin, condT, outT, steps, emb, h1, d, dproj, total;
};

WsLayout ws_layout(const pd_wavenet* h, int B, int T, int S) {
  WsLayout w{};
  size_t off = 0;
  auto take = [&](size_t nfloats) {
    size_t o = off;
    off += (nfloats + 63) / 64 * 64;  // 256-byte aligned
    return o;
  };
  const size_t BT = (size_t)B * T;
  w.x = take(BT * h->C);
  w.x2 = take(BT * h->C);
  w.g = take(BT * h->C);
  w.skip = take(BT * h->C);
  w.hs = take(BT * h->C);
  w.xin = take(BT * h->M);
  w.condT = take(BT * h->H);
  w.outT = take(BT * h->M);
  w.steps = take((size_t)S * B);
  w.emb = take((size_t)S * B * h->C);
  w.h1 = take((size_t)S * B * 4 * h->C);
  w.d = take((size_t)S * B * h->C);
  w.dproj = take((size_t)S * B * h->L * h->C);
  w.total = off * sizeof(float);
  return w;
}

// Step embedding + MLP + all layers' diffusion projections for S*B steps.
int step_mlp(const pd_wavenet* h, float* ws, const WsLayout& L, int nvec, hipStream_t st) {
  const int C = h->C;
  PD_TRY(sinusoidal_embed(ws + L.steps, ws + L.emb, nvec, C, st));
  PD_TRY(matvec(h->W1, h->b1, ws + L.emb, C, ws + L.h1, 4 * C, 4 * C, C, nvec, ACT_MISH, st));
  PD_TRY(matvec(h->W2, h->b2, ws + L.h1, 4 * C, ws + L.d, C, C, 4 * C, nvec, ACT_NONE, st));
  PD_TRY(matvec(h->Wd, h->bd, ws + L.d, C, ws + L.dproj, h->L * C, h->L * C, C, nvec, ACT_NONE, st));
  return PD_OK;
}

// Input projection + residual stack + skip head.  xin: time-major [B][T][M];
// cond: time-major [B][T][H]; dproj: [B][L][C].  Leaves relu(skip head) in ws.hs.
int wavenet_core(const pd_wavenet* h, float* ws, const WsLayout& Lw, const float* xin,
                 const float* cond, const float* dproj, int B, int T, hipStream_t st) {
  const int M = h->M, H = h->H, C = h->C, Ly = h->L;
  const long long BTs = (long long)T;
  float* x = ws + Lw.x;
  float* g = ws + Lw.g;
  float* skip = ws + Lw.skip;
  float* hs = ws + Lw.hs;
  {  // x = relu(W_in spec + b)   (wavenet.py:108-111)
    GemmArgs a = make_gemm(B, T, C, h->Win, h->ldw_in, h->b_in, x, BTs * C, C);
    add_seg(a, make_seg(xin, BTs * M, M, M, 0));
    a.act = ACT_RELU;
    PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_WN_INPROJ>(a, st, "wn_inproj")));
  }
  if (h->W1f) {
    // bf16, C == 256: one fused launch per residual layer, x ping-pongs x <-> x2
    float* xb[2] = {x, ws + Lw.x2};
    for (int l = 0; l < Ly; ++l) {
      WnLayerArgs P{};
      P.xin = xb[l & 1]; P.xout = xb[(l + 1) & 1]; P.skip = skip; P.cond = cond;
      P.dp = dproj + (size_t)l * C; P.dp_ld = Ly * C;
      P.W1f = h->W1f + (size_t)l * 2 * C * (3 * C + H); P.b1 = h->bl1 + (size_t)l * 2 * C;
      P.W2f = h->W2f + (size_t)l * 2 * C * C; P.b2 = h->bl2 + (size_t)l * 2 * C;
      P.B = B; P.T = T; P.H = H; P.dil = 1 << (l % h->cyc); P.first = (l == 0);
      ProfScope ps("wn_layer", st);
      hipLaunchKernelGGL(wn_layer_bf16_kernel<1024>, dim3(cdiv((long long)B * T, 32)), dim3(512), 0, st, P);
      PD_LAUNCH_CHECK();
    }
  } else
  for (int l = 0; l < Ly; ++l) {
    const int dil = 1 << (l % h->cyc);
    {  // z = dilconv(x + dproj) + condproj ; g = sigmoid(z[:C]) * tanh(z[C:])   (wavenet.py:60-67)
      GemmArgs a = make_gemm(B, T, 2 * C, h->Wl1 + (size_t)l * 2 * C * h->ldw1, h->ldw1,
                             h->bl1 + (size_t)l * 2 * C, g, BTs * C, C);
      for (int tap = 0; tap < 3; ++tap) {
        Seg s = make_seg(x, BTs * C, C, C, (tap - 1) * dil);
        s.add_vec = dproj + (size_t)l * C;
        s.add_ld = Ly * C;
        add_seg(a, s);
      }
      add_seg(a, make_seg(cond, BTs * H, H, H, 0));
      a.half = C;
      PD_TRY((launch_gemm<1, 2, 4, 1, EPI_GATE, U_WN_GATE>(a, st, "wn_gate")));
    }
    {  // o = W_out g + b ; x = (x + o[:C]) / sqrt2 ; skip += o[C:]   (wavenet.py:69-72)
      GemmArgs a = make_gemm(B, T, 2 * C, h->Wl2 + (size_t)l * 2 * C * C, C, h->bl2 + (size_t)l * 2 * C,
                             x, BTs * C, C);
      add_seg(a, make_seg(g, BTs * C, C, C, 0));
      a.half = C;
      a.out2 = skip; a.out2_bs = BTs * C; a.out2_ld = C;
      a.flag = (l == 0);
      PD_TRY((launch_gemm<1, 2, 4, 1, EPI_RESSKIP, U_WN_RESSKIP>(a, st, "wn_resskip")));
    }
  }
  {  // hs = relu(W_skip (sum skip / sqrt(L)) + b)   (wavenet.py:119-121)
    GemmArgs a = make_gemm(B, T, C, h->Ws, C, h->bs, hs, BTs * C, C);
    Seg s = make_seg(skip, BTs * C, C, C, 0);
    s.scale = 1.0f / sqrtf((float)Ly);
    add_seg(a, s);
    a.act = ACT_RELU;
    PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_WN_SKIP>(a, st, "wn_skiphead")));
  }
  return PD_OK;
}

}  // namespace

extern "C" {

int pd_wavenet_create(const pd_wavenet_dims* dims, const float* const* params, int dtype,
                      void* stream, pd_wavenet** out) {
  PD_CHECK_ARG(dims && params && out, "null pointer");
  PD_CHECK_ARG(dtype == PD_DTYPE_F32 || dtype == PD_DTYPE_BF16, "dtype must be PD_DTYPE_F32 or PD_DTYPE_BF16");
  const int M = dims->in_dims, H = dims->hidden_size, L = dims->residual_layers,
            C = dims->residual_channels, cyc = dims->dilation_cycle_length;
  PD_CHECK_ARG(M > 0 && M % 4 == 0, "in_dims must be a positive multiple of 4");
  PD_CHECK_ARG(H > 0 && H % 4 == 0, "hidden_size must be a positive multiple of 4");
  PD_CHECK_ARG(C > 0 && C % 32 == 0, "residual_channels must be a positive multiple of 32");
  PD_CHECK_ARG(L > 0 && cyc > 0, "residual_layers/dilation_cycle_length must be positive");
  for (int i = 0; i < PD_WAVENET_NUM_PARAMS(L); ++i)
    PD_CHECK_ARG(params[i] != nullptr, "null parameter pointer " + std::to_string(i));
  hipStream_t st = (hipStream_t)stream;

  pd_wavenet* h = new pd_wavenet();
  h->M = M; h->H = H; h->L = L; h->C = C; h->cyc = cyc; h->dtype = dtype;
  h->ldw_in = round_up(M, GEMM_BK);
  h->ldw1 = 3 * C + round_up(H, GEMM_BK);
  size_t off = 0;
  std::vector<std::pair<float**, size_t>> plan = {
      {&h->Win, (size_t)C * h->ldw_in}, {&h->b_in, (size_t)C},
      {&h->W1, (size_t)4 * C * C}, {&h->b1, (size_t)4 * C},
      {&h->W2, (size_t)C * 4 * C}, {&h->b2, (size_t)C},
      {&h->Wd, (size_t)L * C * C}, {&h->bd, (size_t)L * C},
      {&h->Wl1, (size_t)L * 2 * C * h->ldw1}, {&h->bl1, (size_t)L * 2 * C},
      {&h->Wl2, (size_t)L * 2 * C * C}, {&h->bl2, (size_t)L * 2 * C},
      {&h->Ws, (size_t)C * C}, {&h->bs, (size_t)C},
      {&h->Wo, (size_t)M * C}, {&h->bo, (size_t)M}};
  std::vector<size_t> offs;
  for (auto& p : plan) { offs.push_back(off); off += (p.second + 63) / 64 * 64; }
  if (hipMalloc((void**)&h->pool, off * sizeof(float)) != hipSuccess) {
    delete h;
    set_error("hipMalloc failed for WaveNet weights");
    return PD_ERR_HIP;
  }
  for (size_t i = 0; i < plan.size(); ++i) *plan[i].first = h->pool + offs[i];
  int rc = PD_OK;
  auto run = [&]() -> int {
    PD_HIP(hipMemsetAsync(h->pool, 0, off * sizeof(float), st));
    auto cp = [&](float* dst, const float* src, size_t n) -> int {
      PD_HIP(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, st));
      return PD_OK;
    };
    int p = 0;
    PD_TRY(pack_conv(h->Win, h->ldw_in, 0, 0, h->ldw_in, params[p++], C, M, 1, st));
    PD_TRY(cp(h->b_in, params[p++], C));
    PD_TRY(cp(h->W1, params[p++], (size_t)4 * C * C));
    PD_TRY(cp(h->b1, params[p++], 4 * C));
    PD_TRY(cp(h->W2, params[p++], (size_t)4 * C * C));
    PD_TRY(cp(h->b2, params[p++], C));
    for (int l = 0; l < L; ++l) {
      const float* dil_w = params[p++];
      const float* dil_b = params[p++];
      const float* dif_w = params[p++];
      const float* dif_b = params[p++];
      const float* con_w = params[p++];
      const float* con_b = params[p++];
      const float* out_w = params[p++];
      const float* out_b = params[p++];
      float* W1l = h->Wl1 + (size_t)l * 2 * C * h->ldw1;
      PD_TRY(pack_conv(W1l, h->ldw1, 0, 0, C, dil_w, 2 * C, C, 3, st));
      PD_TRY(pack_conv(W1l, h->ldw1, 0, 3 * C, round_up(H, GEMM_BK), con_w, 2 * C, H, 1, st));
      PD_TRY(add_vectors(h->bl1 + (size_t)l * 2 * C, dil_b, con_b, 2 * C, st));
      PD_TRY(cp(h->Wd + (size_t)l * C * C, dif_w, (size_t)C * C));
      PD_TRY(cp(h->bd + (size_t)l * C, dif_b, C));
      PD_TRY(cp(h->Wl2 + (size_t)l * 2 * C * C, out_w, (size_t)2 * C * C));
      PD_TRY(cp(h->bl2 + (size_t)l * 2 * C, out_b, 2 * C));
    }
    PD_TRY(cp(h->Ws, params[p++], (size_t)C * C));
    PD_TRY(cp(h->bs, params[p++], C));
    PD_TRY(cp(h->Wo, params[p++], (size_t)M * C));
    PD_TRY(cp(h->bo, params[p++], M));
    h->pool_n = off;
    if (dtype == PD_DTYPE_BF16) {
      PD_HIP(hipMalloc(&h->pool_bf, off * sizeof(__bf16)));
      PD_TRY(convert_f32_bf16(h->pool, h->pool_bf, (long long)off, st));
      register_bf16_pool(h->pool, off, h->pool_bf);
      if (C == WNF_C && H % 32 == 0 && 3 * C + H <= 1024) {
        const int K1 = 3 * C + H;
        const size_t per = (size_t)2 * C * K1 + (size_t)2 * C * C;
        PD_HIP(hipMalloc(&h->frag, (size_t)L * per * sizeof(__bf16)));
        h->W1f = h->frag;
        h->W2f = h->frag + (size_t)L * 2 * C * K1;
        for (int l = 0; l < L; ++l) {
          const long long n1 = (long long)2 * C * K1, n2 = (long long)2 * C * C;
          hipLaunchKernelGGL(pack_frag_kernel, dim3(cdiv(n1, 256)), dim3(256), 0, st, h->W1f + l * n1,
                             h->Wl1 + (size_t)l * 2 * C * h->ldw1, 2 * C, K1, h->ldw1);
          PD_LAUNCH_CHECK();
          hipLaunchKernelGGL(pack_frag_kernel, dim3(cdiv(n2, 256)), dim3(256), 0, st, h->W2f + l * n2,
                             h->Wl2 + (size_t)l * 2 * C * C, 2 * C, C, C);
          PD_LAUNCH_CHECK();
        }
      }
    }
    return PD_OK;
  };
  rc = run();
  if (rc != PD_OK) {
    (void)hipFree(h->pool);
    if (h->pool_bf) (void)hipFree(h->pool_bf);
    if (h->frag) (void)hipFree(h->frag);
    delete h;
    return rc;
  }
  *out = h;
  return PD_OK;
}

void pd_wavenet_destroy(pd_wavenet* h) {
  if (!h) return;
  if (h->pool_bf) {
    unregister_bf16_pool(h->pool);
    (void)hipFree(h->pool_bf);
  }
  if (h->frag) (void)hipFree(h->frag);
  (void)hipFree(h->pool);
  delete h;
}

size_t pd_wavenet_workspace_size(const pd_wavenet* h, int B, int T, int S) {
  if (!h || B < 0 || T < 0 || S < 1) return 0;
  return ws_layout(h, B, T, S).total;
}

int pd_wavenet_forward(const pd_wavenet* h, const float* spec, const float* steps, const float* cond,
                       float* out, int B, int T, void* workspace, size_t ws_bytes, void* stream) {
  PD_CHECK_ARG(h && spec && steps && cond && out && workspace, "null pointer");
  PD_CHECK_ARG(B > 0 && T > 0, "B and T must be positive");
  WsLayout Lw = ws_layout(h, B, T, 1);
  if (ws_bytes < Lw.total) { set_error("workspace too small"); return PD_ERR_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  PD_HIP(hipMemcpyAsync(ws + Lw.steps, steps, sizeof(float) * B, hipMemcpyDeviceToDevice, st));
  PD_TRY(step_mlp(h, ws, Lw, B, st));
  PD_TRY(transpose_ct_to_tc(spec, ws + Lw.xin, B, h->M, T, st));
  PD_TRY(transpose_ct_to_tc(cond, ws + Lw.condT, B, h->H, T, st));
  PD_TRY(wavenet_core(h, ws, Lw, ws + Lw.xin, ws + Lw.condT, ws + Lw.dproj, B, T, st));
  const long long BTs = T;
  GemmArgs a = make_gemm(B, T, h->M, h->Wo, h->C, h->bo, ws + Lw.outT, BTs * h->M, h->M);
  add_seg(a, make_seg(ws + Lw.hs, BTs * h->C, h->C, h->C, 0));
  PD_TRY((launch_gemm<1, 2, 4, 1, EPI_STORE, U_WN_OUT>(a, st, "wn_outproj")));
  PD_TRY(transpose_tc_to_ct(ws + Lw.outT, out, B, T, h->M, st));
  return PD_OK;
}

int pd_prodiff_sample(const pd_wavenet* h, const float* cond, const float* coef1, const float* coef2,
                      const float* sigma, int S, const float* x_T, const float* noise,
                      unsigned long long seed, float* mel, int B, int T, void* workspace,
                      size_t ws_bytes, void* stream) {
  PD_CHECK_ARG(h && cond && coef1 && coef2 && sigma && mel && workspace, "null pointer");
  PD_CHECK_ARG(B > 0 && T > 0 && S >= 1 && S <= 64, "bad B/T/S");
  WsLayout Lw = ws_layout(h, B, T, S);
  if (ws_bytes < Lw.total) { set_error("workspace too small"); return PD_ERR_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  const int M = h->M, C = h->C, Ly = h->L;
  const long long BTM = (long long)B * T * M;
  // x_T ~ U[0,1) (prodiff.py:147) -- the state lives in `mel` (time-major [B][T][M])
  if (x_T) {
    PD_HIP(hipMemcpyAsync(mel, x_T, sizeof(float) * BTM, hipMemcpyDeviceToDevice, st));
  } else {
    PD_TRY(fill_uniform(mel, BTM, seed, 0xFFFF0000u, st));
  }
  // all S steps' embeddings at once: step index i = S-1-j for the j-th pass
  PD_TRY(fill_reverse_steps(ws + Lw.steps, S, B, S - 1, st));
  PD_TRY(step_mlp(h, ws, Lw, S * B, st));
  const long long BTs = T;
  for (int j = 0; j < S; ++j) {
    const int i = S - 1 - j;
    PD_TRY(wavenet_core(h, ws, Lw, mel, cond, ws + Lw.dproj + (size_t)j * B * Ly * C, B, T, st));
    // x0 = W_out hs + b ; x = c1[i] x0 + c2[i] x + [i>0] exp(.5 logvar[i]) n   (prodiff.py:106-126)
    GemmArgs a = make_gemm(B, T, M, h->Wo, C, h->bo, mel, BTs * M, M);
    add_seg(a, make_seg(ws + Lw.hs, BTs * C, C, C, 0));
    a.res = mel; a.res_bs = BTs * M; a.res_ld = M;
    a.c1 = coef1[i]; a.c2 = coef2[i];
    a.sigma = (i == 0) ? 0.f : sigma[i];
    a.noise = noise ? noise + (size_t)j * BTM : nullptr;
    a.noise_bs = BTs * M; a.noise_ld = M;
    a.seed = seed; a.stream_id = (unsigned)j;
    PD_TRY((launch_gemm<1, 2, 4, 1, EPI_POSTERIOR, U_WN_POSTERIOR>(a, st, "wn_outproj_posterior")));
  }
  return PD_OK;
}

}  // extern "C"
