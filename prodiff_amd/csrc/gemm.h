// Implicit-GEMM Conv1d engine for gfx950 (fp32 in / fp32 accumulate on MFMA).
//
// Every Conv1d/Linear on the ProDiff/FastDiff hot path is computed here as
//     out[b, t, n] = epilogue( sum_k A(b, t, k) * W[n][k] )
// over TIME-MAJOR activations ([batch][time][channel], channels contiguous).
// The reduction axis k is a concatenation of "segments": each segment is one
// conv tap (or one extra input tensor) read at row  v*row_mul  with
// v = t + row_off, zero outside [0, T) of its utterance (the conv zero
// padding), optionally pre-processed on load (per-(b,c) add, tensor add,
// activation, scale).  Weights are pre-packed once as W[n][sum(kpad)].
//
// Tile: 256 threads = 4 waves; each wave owns WM_T x WN_T 32x32 accumulator
// tiles of v_mfma_f32_32x32x2_f32 (exact f32 fmaf chain).
// K is staged through LDS 32 deep, double-buffered, the next chunk's global
// loads in flight under the current chunk's MFMAs.
#pragma once
#include <type_traits>

#include "common.h"

namespace pd {

constexpr int GEMM_BK = 32;
constexpr int MAX_SEGS = 12;   // NSF-HiFiGAN resblock convs have up to 11 taps

struct Seg {
  const float* src;        // points at channel c_off of batch 0, row 0
  long long bstride;       // elements between utterances
  int ld;                  // elements between rows
  int cs;                  // channels read (multiple of 4)
  int row_mul;             // source row = v * row_mul
  int row_off;             // v = t + row_off  (zero padding outside [0,T))
  const float* add_vec;    // optional [B][add_ld] per-(b,c) add (before act)
  int add_ld;
  const float* add_ten;    // optional tensor add, same layout as src (before act)
  int act;
  float alpha;
  float scale;
  int kpad;                // cs rounded up to GEMM_BK
};

enum Epi { EPI_STORE = 0, EPI_GATE = 1, EPI_RESSKIP = 2, EPI_POSTERIOR = 3 };

// GEMM uses on the hot path (template ID -> distinct kernel symbol per use)
enum GemmUse {
  U_WN_INPROJ = 0, U_WN_GATE = 1, U_WN_RESSKIP = 2, U_WN_SKIP = 3, U_WN_OUT = 4, U_WN_POSTERIOR = 5,
  U_FD_DBLOCK = 10, U_FD_KP_IN = 11, U_FD_KP_RES = 12, U_FD_KP_BIAS = 13, U_FD_KP_KERNEL = 14,
  U_FD_LVC_PRECONV = 15,
  U_NSF_CONV_PRE = 20, U_NSF_UPS = 21, U_NSF_RES = 22, U_NSF_POST = 23
};

struct GemmArgs {
  int B, T, N, nseg;
  Seg seg[MAX_SEGS];
  const float* W;           // packed fp32 [N][ldw]  (fp32 path)
  const __bf16* Wb;         // packed bf16 [N][ldw]  (bf16 path; selects it when non-null)
  int out_bf16;             // STORE: write `out` as bf16
  int ldw;                  // = sum of seg kpad
  const float* bias;        // [N]
  float* out;
  long long out_bs;
  int out_ld;
  int act;
  float alpha, scale;
  const float* res;         // STORE: added after act/scale; POSTERIOR: x_t
  long long res_bs;
  int res_ld;
  int half;                 // paired modes: columns n and n+half combine
  float* out2;              // RESSKIP: skip accumulator
  long long out2_bs;
  int out2_ld;
  int flag;                 // RESSKIP: 1 -> first layer (skip = value)
  float c1, c2, sigma;      // POSTERIOR: x = c1*x0 + c2*x_t + sigma*n
  const float* noise;       // POSTERIOR: explicit draws (time-major) or null -> Philox
  long long noise_bs;
  int noise_ld;
  unsigned long long seed;
  unsigned int stream_id;
  const int* uid;           // POSTERIOR: utterance id per batch row (null -> row index)
  int ksplit;               // STORE, > 1: split-K -- blockIdx.z sums one K range into `part`,
  float* part;              //   [ksplit][B*T][N] fp32, and gemm_splitk_reduce applies the epilogue
  const int* lens;          // ragged batch: utterance b's segments read zero from row lens[b] * lens_mul
  int lens_mul;             //   on (null: from row T), the rows being in units of 1 / lens_mul frame
};

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// TW = float : v_mfma_f32_32x32x2_f32 (exact fp32, the parity path)
// TW = __bf16: v_mfma_f32_32x32x16_bf16 (weights bf16, activations rounded to bf16
//              when staged into LDS, fp32 accumulate/epilogue)
// ID only makes each hot-path use a distinct symbol in rocprof traces (DESIGN.md lists them).
template <typename TW, int WM_T, int WN_T, int WAVES_M, int WAVES_N, int EPI, int ID>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs a) {
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
  constexpr bool BF = !std::is_same<TW, float>::value;
  constexpr int BM = 32 * WM_T * WAVES_M;
  constexpr int BN = 32 * WN_T * WAVES_N;
  constexpr int BK = GEMM_BK;
  // padded LDS rows: 144 B (fp32) / 80 B (bf16) keep the ds_read_b128 fragment reads
  // conflict-free (16-B slot = 9r (fp32) or 5r (bf16) + const mod 16)
  constexpr int LDL = BF ? BK + 8 : BK + 4;
  constexpr bool PAIRED = (EPI == EPI_GATE || EPI == EPI_RESSKIP);
  static_assert(!PAIRED || (WN_T == 2 && WAVES_N == 1), "paired epilogue layout");
  constexpr int A_IT = BM / 32, B_IT = BN / 32;

  __shared__ __attribute__((aligned(16))) TW smem[2][(BM + BN) * LDL];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int rows = a.B * a.T;
  const int row0 = blockIdx.x * BM;
  const int nb = PAIRED ? blockIdx.y * (BN / 2) : blockIdx.y * BN;
  const int q4 = (tid & 7) * 4;

  int a_b[A_IT], a_t[A_IT], a_len[A_IT];
  bool a_ok[A_IT];
#pragma unroll
  for (int i = 0; i < A_IT; ++i) {
    int R = row0 + (tid >> 3) + 32 * i;
    a_ok[i] = R < rows;
    int b = a_ok[i] ? R / a.T : 0;
    a_b[i] = b;
    a_t[i] = R - b * a.T;
    a_len[i] = a.lens ? min(a.lens[b] * a.lens_mul, a.T) : a.T;   // the conv's zero padding starts here
  }
  const TW* w_ptr[B_IT];
  bool w_ok[B_IT];
#pragma unroll
  for (int i = 0; i < B_IT; ++i) {
    int local = (tid >> 3) + 32 * i;
    int n = PAIRED ? (local < BN / 2 ? nb + local : a.half + nb + local - BN / 2) : nb + local;
    w_ok[i] = n < a.N;
    const TW* W;
    if constexpr (BF) W = a.Wb; else W = a.W;
    w_ptr[i] = W + (long long)(w_ok[i] ? n : 0) * a.ldw + q4;
  }

  float4 ra[A_IT];
  typename std::conditional<BF, uint2, float4>::type rb[B_IT];
  auto load_chunk = [&](int s, int c0, int kg) {
    const Seg& sg = a.seg[s];
    const int c = c0 + q4;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      int vv = a_t[i] + sg.row_off;
      if (a_ok[i] && c < sg.cs && vv >= 0 && vv < a_len[i]) {
        long long off = (long long)a_b[i] * sg.bstride + (long long)vv * sg.row_mul * sg.ld + c;
        v = *reinterpret_cast<const float4*>(sg.src + off);
        if (sg.add_ten) {
          float4 w = *reinterpret_cast<const float4*>(sg.add_ten + off);
          v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
        }
        if (sg.add_vec) {
          float4 w = *reinterpret_cast<const float4*>(sg.add_vec + (long long)a_b[i] * sg.add_ld + c);
          v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
        }
        if (sg.act != ACT_NONE) {
          v.x = act_apply(v.x, sg.act, sg.alpha); v.y = act_apply(v.y, sg.act, sg.alpha);
          v.z = act_apply(v.z, sg.act, sg.alpha); v.w = act_apply(v.w, sg.act, sg.alpha);
        }
        if (sg.scale != 1.f) { v.x *= sg.scale; v.y *= sg.scale; v.z *= sg.scale; v.w *= sg.scale; }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      if constexpr (BF)
        rb[i] = w_ok[i] ? *reinterpret_cast<const uint2*>(w_ptr[i] + kg) : make_uint2(0u, 0u);
      else
        rb[i] = w_ok[i] ? *reinterpret_cast<const float4*>(w_ptr[i] + kg) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_chunk = [&](int buf) {
    TW* As = smem[buf];
    TW* Bs = smem[buf] + BM * LDL;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      TW* dst = As + ((tid >> 3) + 32 * i) * LDL + q4;
      if constexpr (BF) {
        bf16x4 v = {(__bf16)ra[i].x, (__bf16)ra[i].y, (__bf16)ra[i].z, (__bf16)ra[i].w};
        *reinterpret_cast<bf16x4*>(dst) = v;
      } else {
        *reinterpret_cast<float4*>(dst) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      TW* dst = Bs + ((tid >> 3) + 32 * i) * LDL + q4;
      if constexpr (BF) *reinterpret_cast<uint2*>(dst) = rb[i];
      else *reinterpret_cast<float4*>(dst) = rb[i];
    }
  };

  f32x16 acc[WM_T][WN_T];
#pragma unroll
  for (int i = 0; i < WM_T; ++i)
#pragma unroll
    for (int j = 0; j < WN_T; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  int ch_begin = 0, nchunks = a.ldw / BK;
  constexpr bool SPLITTABLE = (EPI == EPI_STORE || PAIRED);
  if (SPLITTABLE && a.ksplit > 1) {   // this block's K range (host makes every range non-empty)
    const int cps = (nchunks + a.ksplit - 1) / a.ksplit;
    ch_begin = blockIdx.z * cps;
    nchunks = min(nchunks, ch_begin + cps);
  }
  int s = 0, c0 = ch_begin * BK;
  while (c0 >= a.seg[s].kpad) { c0 -= a.seg[s].kpad; ++s; }
  load_chunk(s, c0, ch_begin * BK);
  store_chunk(ch_begin & 1);
  __syncthreads();
  const int r32 = lane & 31, h = lane >> 5;
  for (int ch = ch_begin; ch < nchunks; ++ch) {
    const bool more = ch + 1 < nchunks;
    if (more) {
      c0 += BK;
      if (c0 >= a.seg[s].kpad) { ++s; c0 = 0; }
      load_chunk(s, c0, (ch + 1) * BK);
    }
    const TW* As = smem[ch & 1];
    const TW* Bs = smem[ch & 1] + BM * LDL;
    if constexpr (BF) {
      // 32x32x16: lane (r, h) holds A[r][8h + j], B[8h + j][r]; two k-steps per 32-deep chunk
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[WM_T], bfr[WN_T];
#pragma unroll
        for (int i = 0; i < WM_T; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 32 * WM_T + i * 32 + r32) * LDL + kk * 16 + h * 8);
#pragma unroll
        for (int j = 0; j < WN_T; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 32 * WN_T + j * 32 + r32) * LDL + kk * 16 + h * 8);
#pragma unroll
        for (int i = 0; i < WM_T; ++i)
#pragma unroll
          for (int j = 0; j < WN_T; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // 32x32x2 f32: MFMA kk pairs k = kk (lanes h=0) with k = 16 + kk (h=1), so each
      // lane reads 16 contiguous floats per operand
      float af[WM_T][16], bf[WN_T][16];
#pragma unroll
      for (int i = 0; i < WM_T; ++i) {
        const float* p = As + (wm * 32 * WM_T + i * 32 + r32) * LDL + h * 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 v = *reinterpret_cast<const float4*>(p + 4 * q);
          af[i][4 * q] = v.x; af[i][4 * q + 1] = v.y; af[i][4 * q + 2] = v.z; af[i][4 * q + 3] = v.w;
        }
      }
#pragma unroll
      for (int j = 0; j < WN_T; ++j) {
        const float* p = Bs + (wn * 32 * WN_T + j * 32 + r32) * LDL + h * 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 v = *reinterpret_cast<const float4*>(p + 4 * q);
          bf[j][4 * q] = v.x; bf[j][4 * q + 1] = v.y; bf[j][4 * q + 2] = v.z; bf[j][4 * q + 3] = v.w;
        }
      }
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
#pragma unroll
        for (int i = 0; i < WM_T; ++i)
#pragma unroll
          for (int j = 0; j < WN_T; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][kk], bf[j][kk], acc[i][j], 0, 0, 0);
    }
    if (more) store_chunk((ch + 1) & 1);
    __syncthreads();
  }

  // ------------------------------------------------------------ epilogue
  // C/D map of 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  const float rs2 = 0.70710678118654752440f;
#pragma unroll
  for (int i = 0; i < WM_T; ++i) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int rl = wm * 32 * WM_T + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      const int R = row0 + rl;
      if (R >= rows) continue;
      if constexpr (PAIRED) {
        if (a.ksplit > 1) {   // raw partial sums of both halves; gemm_splitk_reduce applies the epilogue
          float* pz = a.part + ((long long)blockIdx.z * rows + R) * a.N + nb + r32;
          pz[0] = acc[i][0][reg];
          pz[a.half] = acc[i][1][reg];
          continue;
        }
      }
      const int b = R / a.T, t = R - b * a.T;
      if constexpr (EPI == EPI_GATE) {
        const int n = nb + r32;
        float v0 = acc[i][0][reg] + a.bias[n];
        float v1 = acc[i][1][reg] + a.bias[a.half + n];
        a.out[(long long)b * a.out_bs + (long long)t * a.out_ld + n] = sigmoidf_(v0) * tanhf_(v1);
      } else if constexpr (EPI == EPI_RESSKIP) {
        const int n = nb + r32;
        float v0 = acc[i][0][reg] + a.bias[n];
        float v1 = acc[i][1][reg] + a.bias[a.half + n];
        float* xp = a.out + (long long)b * a.out_bs + (long long)t * a.out_ld + n;
        *xp = (*xp + v0) * rs2;
        float* sp = a.out2 + (long long)b * a.out2_bs + (long long)t * a.out2_ld + n;
        *sp = a.flag ? v1 : (*sp + v1);
      } else {
#pragma unroll
        for (int j = 0; j < WN_T; ++j) {
          const int n = nb + wn * 32 * WN_T + j * 32 + r32;
          if (n >= a.N) continue;
          if (EPI == EPI_STORE && a.ksplit > 1) {
            a.part[((long long)blockIdx.z * rows + R) * a.N + n] = acc[i][j][reg];
            continue;
          }
          float v = acc[i][j][reg] + (a.bias ? a.bias[n] : 0.f);
          const long long oi = (long long)b * a.out_bs + (long long)t * a.out_ld + n;
          if constexpr (EPI == EPI_POSTERIOR) {
            float xt = a.res[(long long)b * a.res_bs + (long long)t * a.res_ld + n];
            float x = a.c1 * v + a.c2 * xt;
            if (a.sigma != 0.f) {
              float z = a.noise ? a.noise[(long long)b * a.noise_bs + (long long)t * a.noise_ld + n]
                                : philox_normal_u(a.seed, utt_id(a.uid, b), (unsigned)(t * a.N + n), a.stream_id);
              x += a.sigma * z;
            }
            a.out[oi] = x;
          } else {
            v = act_apply(v, a.act, a.alpha) * a.scale;
            if (a.res) v += a.res[(long long)b * a.res_bs + (long long)t * a.res_ld + n];
            if (a.out_bf16) reinterpret_cast<__bf16*>(a.out)[oi] = (__bf16)v;
            else a.out[oi] = v;
          }
        }
      }
    }
  }
}

// Host-side validation + launch.  Returns PD_OK or an error code.
int validate_gemm(const GemmArgs& a);

// Split-K epilogue: out = act(sum_z part[z] + bias) * scale (+ res), as EPI_STORE's; or the
// paired GATE / RESSKIP epilogues on the summed halves.
int gemm_splitk_reduce(const GemmArgs& a, int epi, hipStream_t st);

const __bf16* lookup_bf16(const float* p);

template <int WM_T, int WN_T, int WAVES_M, int WAVES_N, int EPI, int ID>
int launch_gemm(const GemmArgs& a0, hipStream_t st, const char* tag) {
  GemmArgs a = a0;
  if (!a.Wb) a.Wb = lookup_bf16(a.W);   // bf16 handle -> bf16 MFMA path
  PD_TRY(validate_gemm(a));
  constexpr int BM = 32 * WM_T * WAVES_M;
  constexpr int BN = 32 * WN_T * WAVES_N;
  constexpr bool PAIRED = (EPI == EPI_GATE || EPI == EPI_RESSKIP);
  const long long rows = (long long)a.B * a.T;
  if (rows == 0) return PD_OK;
  dim3 grid(cdiv(rows, BM), PAIRED ? a.half / 32 : cdiv(a.N, BN));
  if (PAIRED && (a.half % 32 != 0 || a.N != 2 * a.half)) {
    set_error("paired gemm needs N == 2*half, half % 32 == 0");
    return PD_ERR_ARG;
  }
  if (a.ksplit > 1) {
    const int nch = a.ldw / GEMM_BK;
    if (!(EPI == EPI_STORE || PAIRED) || !a.part || a.ksplit > nch) {
      set_error("split-K needs EPI_STORE / GATE / RESSKIP, a partial-sum buffer and ksplit <= K / 32");
      return PD_ERR_ARG;
    }
    const int cps = cdiv(nch, a.ksplit);
    a.ksplit = cdiv(nch, cps);          // every K range non-empty
    grid.z = a.ksplit;
  }
  {
    ProfScope ps(tag, st);
    if (a.Wb)
      hipLaunchKernelGGL((gemm_kernel<__bf16, WM_T, WN_T, WAVES_M, WAVES_N, EPI, ID>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((gemm_kernel<float, WM_T, WN_T, WAVES_M, WAVES_N, EPI, ID>), grid, dim3(256), 0, st, a);
    PD_LAUNCH_CHECK();
    if (a.ksplit > 1) PD_TRY(gemm_splitk_reduce(a, EPI, st));
  }
  return PD_OK;
}

// Convenience constructors ---------------------------------------------------
inline Seg make_seg(const float* src, long long bstride, int ld, int cs, int row_off,
                    int row_mul = 1) {
  Seg s{};
  s.src = src; s.bstride = bstride; s.ld = ld; s.cs = cs;
  s.row_mul = row_mul; s.row_off = row_off;
  s.add_vec = nullptr; s.add_ld = 0; s.add_ten = nullptr;
  s.act = ACT_NONE; s.alpha = 0.f; s.scale = 1.f;
  s.kpad = round_up(cs, GEMM_BK);
  return s;
}

inline GemmArgs make_gemm(int B, int T, int N, const float* W, int ldw, const float* bias,
                          float* out, long long out_bs, int out_ld) {
  GemmArgs a{};
  a.B = B; a.T = T; a.N = N; a.nseg = 0;
  a.W = W; a.ldw = ldw; a.bias = bias;
  a.out = out; a.out_bs = out_bs; a.out_ld = out_ld;
  a.act = ACT_NONE; a.alpha = 0.f; a.scale = 1.f;
  return a;
}

inline void add_seg(GemmArgs& a, const Seg& s) { a.seg[a.nseg++] = s; }

}  // namespace pd
