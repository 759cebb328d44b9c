// Condition encoder of the SVS teacher: ProDiffTeacher.forward_condition
// (modules/svs/prodiff_teacher.py:103-146) -- the stage that produces the
// denoiser's `cond` [B, T_mel, H].
//
//   extra  = dur_embed(mel2ph_to_dur(mel2ph)) + lang_embed(lang_seq)      :110-119
//   x      = sqrt(H) * embed_tokens(txt) + extra + sinusoid(positions)    tts_modules.py:319-330
//   x      = FFT encoder (enc_layers x EncSALayer, final LayerNorm)       tts_modules.py:264-289
//   cond   = gather(pad(x), mel2ph) + pitch + spk (+ gender) + voicing + breath, * (mel2ph > 0)
//
// Activations are TIME-MAJOR [batch][token][channel] throughout (the teacher's own
// [B, T, C] layout; the reference's T x B x C transposes are pure views of it).
// Launch sequence per call (all on `stream`, allocation-free):
//   enc_embed    one pass over the tokens: token/lang/dur/position sums, padding mask
//   per layer:   enc_ln (mask x in place, LN1)  -> QKV GEMM  -> enc_attn (online-softmax
//                attention, key-padding mask)  -> out-proj GEMM (+ residual)
//                -> enc_ln (mask, LN2) -> FFN conv GEMM (9 taps, * k^-0.5, GELU)
//                -> FFN linear GEMM (+ residual)
//   enc_ln (final LayerNorm * mask) -> enc_cond (length-regulator gather + variance sums)
// The GEMMs are the implicit-GEMM Conv1d engine (gemm.h) -- MFMA fp32 or bf16.
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/prodiff_hip.h"
#include "common.h"
#include "gemm.h"
#include "kernels.h"

using namespace pd;

namespace {

enum EncUse { U_ENC_QKV = 30, U_ENC_OUT = 31, U_ENC_FFN1 = 32, U_ENC_FFN2 = 33 };

// ---------------------------------------------------------------- embeddings
// FastspeechEncoder.forward_embedding (tts_modules.py:319-330) with the teacher's
// extra_embed (prodiff_teacher.py:110-119).  One block per (8 tokens, utterance):
//  * dur[t] = #{ frames f : mel2ph[f] == t+1 }        (mel2ph_to_dur, tts_modules.py:223-229)
//  * pos[t] = #{ t' <= t : tok[t'] != 0 } for tokens, 0 for padding (make_positions,
//             utils/tts_utils.py:6-18, on ~padding_mask)
//  * x[t,c] = ((sqrt(H) emb[tok][c] + ((dur dw[c] + db[c]) + lang[l][c])) + pe(pos, c)) * [tok != 0]
//    with pe(p, c) = sin(p f_c) | cos(p f_{c-H/2}), f_i = exp(-i ln(1e4)/(H/2-1))
//    (SinusoidalPositionalEmbedding.get_embedding, common_layers.py:111-128, fp32 as there).
//  * rel_pos: x[t,c] = ((sqrt(H) emb[tok][c] + extra) sqrt(H) + pr(t, c)) * [tok != 0], with
//    the RelPositionalEncoding table pr(t, 2i) = sin(q g_i), pr(t, 2i+1) = cos(q g_i),
//    q = max(P, T) - 1 - t (reversed positions; P = the rows of the reference's table, 5000 at
//    first and the longest input seen since: pd_cond_dims.rel_pos), g_i = exp(2i (-ln(1e4)/H))
//    (espnet_positional_embedding.py:24-45,108-115; FFTBlocks masks the padding, tts_modules.py:274).
constexpr int EMB_TOK = 8;

__global__ __launch_bounds__(256) void enc_embed_kernel(
    const long long* __restrict__ tok, const long long* __restrict__ lang, const long long* __restrict__ mel2ph,
    int Tt, int Tm, int H, const float* __restrict__ emb, int V, float scale, const float* __restrict__ dur_w,
    const float* __restrict__ dur_b, const float* __restrict__ lang_emb, int NL, float neg_freq, int rel_pos,
    float neg_rel, float* __restrict__ x) {
  const int b = blockIdx.y, t0 = blockIdx.x * EMB_TOK, tid = threadIdx.x;
  __shared__ int cnt[EMB_TOK];
  __shared__ int npre;
  __shared__ int pos[EMB_TOK];
  if (tid < EMB_TOK) cnt[tid] = 0;
  if (tid == 0) npre = 0;
  __syncthreads();
  const long long* tk = tok + (long long)b * Tt;
  if (dur_w) {
    const long long* mp = mel2ph + (long long)b * Tm;
    for (int f = tid; f < Tm; f += 256) {
      const long long v = mp[f];
      const long long j = v - 1 - t0;
      if (v >= 1 && v <= Tt && j >= 0 && j < EMB_TOK) atomicAdd(&cnt[j], 1);
    }
  }
  int pre = 0;
  for (int i = tid; i < t0 && i < Tt; i += 256) pre += tk[i] != 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) pre += __shfl_xor(pre, o);
  if ((tid & 63) == 0 && pre) atomicAdd(&npre, pre);
  __syncthreads();
  if (tid == 0) {
    int run = npre;
    for (int j = 0; j < EMB_TOK; ++j) {
      const int t = t0 + j;
      const bool np = t < Tt && tk[t] != 0;
      run += np;
      pos[j] = np ? run : 0;
    }
  }
  __syncthreads();
  const int half = H / 2;
  for (int j = 0; j < EMB_TOK; ++j) {
    const int t = t0 + j;
    if (t >= Tt) break;
    const long long id = tk[t];
    const bool np = id != 0;
    // ids index tables of V / NL rows; out-of-range ids (an IndexError in the reference) are
    // clamped so a bad input cannot fault the device
    const float* er = emb + min(max(id, 0ll), (long long)V - 1) * H;
    const float* lr = lang ? lang_emb + min(max(lang[(long long)b * Tt + t], 0ll), (long long)NL - 1) * H : nullptr;
    const float d = (float)cnt[j];
    const float p = (float)pos[j];
    float* xr = x + ((long long)b * Tt + t) * H;
    for (int c = tid; c < H; c += 256) {
      float extra = 0.f;
      if (dur_w) extra = d * dur_w[c] + dur_b[c];
      if (lr) extra = extra + lr[c];
      float v;
      if (rel_pos) {
        const int P = rel_pos > 5000 ? rel_pos : 5000;   // the reference table never has fewer than 5000 rows
        const float q = (float)((Tt > P ? Tt : P) - 1 - t);
        const float arg = q * expf((float)(c & ~1) * neg_rel);
        v = (scale * er[c] + extra) * scale + ((c & 1) ? cosf(arg) : sinf(arg));
      } else {
        const int i = c < half ? c : c - half;
        const float arg = p * expf((float)i * neg_freq);
        const float pe = pos[j] == 0 ? 0.f : (c < half ? sinf(arg) : cosf(arg));
        v = (scale * er[c] + extra) + pe;
      }
      xr[c] = np ? v : 0.f;
    }
  }
}

// ---------------------------------------------------------------- LayerNorm
// One wave per token row.  mode 0 (EncSALayer's LN1/LN2, common_layers.py:656-669): the
// row is first multiplied by the padding mask in place -- the `x * (1 - mask)` that ends the
// previous sub-layer (:666,673, tts_modules.py:285) -- then y = LN(x).  mode 1 (FFTBlocks'
// final norm, :286-287): y = LN(x) * mask.  Two-pass fp32 moments, eps as the module's.
__global__ __launch_bounds__(256) void enc_ln_kernel(float* __restrict__ x, const float* __restrict__ g,
                                                     const float* __restrict__ bta, const long long* __restrict__ tok,
                                                     float* __restrict__ y, int rows, int H, float eps, int mode) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const bool pad = tok[r] == 0;
  float* xr = x + (long long)r * H;
  float* yr = y + (long long)r * H;
  if (mode == 1 && pad) {
    for (int c = lane; c < H; c += 64) yr[c] = 0.f;
    return;
  }
  if (mode == 0 && pad)
    for (int c = lane; c < H; c += 64) xr[c] = 0.f;
  float s = 0.f;
  if (!pad)
    for (int c = lane; c < H; c += 64) s += xr[c];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)H;
  float v = 0.f;
  if (!pad)
    for (int c = lane; c < H; c += 64) {
      const float d = xr[c] - mean;
      v += d * d;
    }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const float rstd = 1.f / sqrtf(v / (float)H + eps);
  for (int c = lane; c < H; c += 64) {
    const float xv = pad ? 0.f : xr[c];
    yr[c] = (xv - mean) * rstd * g[c] + bta[c];
  }
}

// ---------------------------------------------------------------- attention
// Self-attention core of MultiheadAttention (common_layers.py:172-300 -> torch's
// multi_head_attention_forward, bias=False, need_weights path): per head
//   softmax(q k^T / sqrt(D) + mask) v,  mask = -inf on padding keys (key_padding_mask).
// One block = 32 queries of one (utterance, head); keys stream through LDS 32 at a time
// with the online-softmax recurrence (running max m, sum l).  Thread (q = tid/8, sub =
// tid%8) scores keys sub + 8j and owns output columns 4 sub + 32 i.  fp32 VALU: the
// whole encoder attention is O(T_txt^2 H) on T_txt <= a few hundred tokens.
// A query whose keys are all padding (an all-padding utterance) yields 0, not NaN.
constexpr int AQ = 32, AK = 32;

template <int D>
__global__ __launch_bounds__(256) void enc_attn_kernel(const float* __restrict__ qkv, const long long* __restrict__ tok,
                                                       float* __restrict__ out, int Tt, int H, float qscale) {
  constexpr int LD = D + 4;
  constexpr int ND4 = D / 4;
  constexpr int OI = D / 32;   // float4 column groups per thread
  __shared__ __attribute__((aligned(16))) float Qs[AQ * LD];
  __shared__ __attribute__((aligned(16))) float Ks[AK * LD];
  __shared__ __attribute__((aligned(16))) float Vs[AK * LD];
  __shared__ float Ps[AQ][AK + 1];
  __shared__ int kval[AK];
  const int b = blockIdx.z, head = blockIdx.y, q0 = blockIdx.x * AQ;
  const int tid = threadIdx.x, q = tid >> 3, sub = tid & 7;
  const long long row0 = (long long)b * Tt;
  const int ld3 = 3 * H;
  for (int e = tid; e < AQ * ND4; e += 256) {
    const int r = e / ND4, c4 = e - r * ND4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q0 + r < Tt) {
      v = *reinterpret_cast<const float4*>(qkv + (row0 + q0 + r) * ld3 + head * D + 4 * c4);
      v.x *= qscale; v.y *= qscale; v.z *= qscale; v.w *= qscale;
    }
    *reinterpret_cast<float4*>(Qs + r * LD + 4 * c4) = v;
  }
  float m = -1e30f, l = 0.f;
  float4 o[OI];
#pragma unroll
  for (int i = 0; i < OI; ++i) o[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k0 = 0; k0 < Tt; k0 += AK) {
    __syncthreads();   // previous chunk's K/V/P reads are done
    for (int e = tid; e < AK * ND4; e += 256) {
      const int r = e / ND4, c4 = e - r * ND4;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
      if (k0 + r < Tt) {
        const float* src = qkv + (row0 + k0 + r) * ld3 + head * D + 4 * c4;
        kv = *reinterpret_cast<const float4*>(src + H);
        vv = *reinterpret_cast<const float4*>(src + 2 * H);
      }
      *reinterpret_cast<float4*>(Ks + r * LD + 4 * c4) = kv;
      *reinterpret_cast<float4*>(Vs + r * LD + 4 * c4) = vv;
    }
    if (tid < AK) kval[tid] = (k0 + tid < Tt) && tok[row0 + k0 + tid] != 0;
    __syncthreads();
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    const float* qr = Qs + q * LD;
#pragma unroll 4
    for (int d4 = 0; d4 < ND4; ++d4) {
      const float4 qv = *reinterpret_cast<const float4*>(qr + 4 * d4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 kv = *reinterpret_cast<const float4*>(Ks + (sub + 8 * j) * LD + 4 * d4);
        s[j] += qv.x * kv.x + qv.y * kv.y + qv.z * kv.z + qv.w * kv.w;
      }
    }
    float cm = -1e30f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (kval[sub + 8 * j]) cm = fmaxf(cm, s[j]);
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) cm = fmaxf(cm, __shfl_xor(cm, off));
    const float mn = fmaxf(m, cm);
    const float corr = expf(m - mn);
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float p = kval[sub + 8 * j] ? expf(s[j] - mn) : 0.f;
      Ps[q][sub + 8 * j] = p;
      ps += p;
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) ps += __shfl_xor(ps, off);
    l = l * corr + ps;
    m = mn;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < OI; ++i) {
      o[i].x *= corr; o[i].y *= corr; o[i].z *= corr; o[i].w *= corr;
    }
#pragma unroll 8
    for (int k = 0; k < AK; ++k) {
      const float p = Ps[q][k];
#pragma unroll
      for (int i = 0; i < OI; ++i) {
        const float4 vv = *reinterpret_cast<const float4*>(Vs + k * LD + 4 * sub + 32 * i);
        o[i].x += p * vv.x; o[i].y += p * vv.y; o[i].z += p * vv.z; o[i].w += p * vv.w;
      }
    }
  }
  const int t = q0 + q;
  if (t >= Tt) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  float* orow = out + (row0 + t) * H + head * D;
#pragma unroll
  for (int i = 0; i < OI; ++i) {
    float4 v = o[i];
    v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
    *reinterpret_cast<float4*>(orow + 4 * sub + 32 * i) = v;
  }
}

// ---------------------------------------------------------------- condition assembly
// prodiff_teacher.py:121-145 for one mel frame per wave:
//   m = mel2ph[f];  cond = m ? ((((enc[m-1] + (log(1 + f0/700) pw + pb)) + spk) + gender)
//                              + (voicing vw + vb + breath bw + bb)) : 0
// (the gather from the zero-padded encoder output, LengthRegulator's mel2ph convention,
// then the nonpadding multiply; the reference's F.pad row 0 makes m = 0 frames exactly 0).
struct CondArgs {
  const float* enc;            // [B, Tt, H]
  const long long* mel2ph;       // [B, Tm]
  const float* f0;             // [B, Tm]
  const float* pw;             // pitch_embed.weight [H] / bias [H]
  const float* pb;
  const float* spk_tab;        // spk_embed.weight rows (n_spk), indexed by spk_id ...
  const long long* spk_id;
  int n_spk;
  const float* spk_mix;        // ... or a mix [B, spk_ts ? Tm : 1, H]
  int spk_ts;
  const float* gen_tab;        // add_gender_embed (prodiff_teacher.py:91-95): lang_embed rows (n_gen)
  const long long* gen_id;
  int n_gen;
  const float* gen_mix;
  int gen_ts;
  const float* voicing;        // [B, Tm] or null
  const float* vw;
  const float* vb;
  const float* breath;         // [B, Tm] or null
  const float* bw;
  const float* bb;
  float* out;                  // [B, Tm, H]
  int B, Tt, Tm, H;
};

__global__ __launch_bounds__(256) void enc_cond_kernel(const CondArgs a) {
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= (long long)a.B * a.Tm) return;
  const int b = (int)(r / a.Tm), f = (int)(r - (long long)b * a.Tm);
  float* orow = a.out + r * a.H;
  const long long m = a.mel2ph[r];
  if (m <= 0 || m > a.Tt) {
    for (int c = lane; c < a.H; c += 64) orow[c] = 0.f;
    return;
  }
  const float* er = a.enc + ((long long)b * a.Tt + (m - 1)) * a.H;
  const float f0m = logf(1.f + a.f0[r] / 700.f);
  const float* sr = nullptr;
  if (a.spk_mix) sr = a.spk_mix + ((long long)b * (a.spk_ts ? a.Tm : 1) + (a.spk_ts ? f : 0)) * a.H;
  else if (a.spk_tab) sr = a.spk_tab + min(max(a.spk_id[b], 0ll), (long long)a.n_spk - 1) * a.H;
  const float* gr = nullptr;
  if (a.gen_mix) gr = a.gen_mix + ((long long)b * (a.gen_ts ? a.Tm : 1) + (a.gen_ts ? f : 0)) * a.H;
  else if (a.gen_tab) gr = a.gen_tab + min(max(a.gen_id[b], 0ll), (long long)a.n_gen - 1) * a.H;
  const float vo = a.voicing ? a.voicing[r] : 0.f;
  const float br = a.breath ? a.breath[r] : 0.f;
  for (int c = lane; c < a.H; c += 64) {
    float v = er[c] + (f0m * a.pw[c] + a.pb[c]);
    if (sr) v += sr[c];
    if (gr) v += gr[c];
    if (a.voicing && a.breath) v += (vo * a.vw[c] + a.vb[c]) + (br * a.bw[c] + a.bb[c]);
    else if (a.voicing) v += vo * a.vw[c] + a.vb[c];
    else if (a.breath) v += br * a.bw[c] + a.bb[c];
    orow[c] = v;
  }
}

// GEMM tile by grid size: 128 x 64 tiles once they give every CU a block, else 32 x 128 tiles
// with the K axis split over up to 8 blocks (the B = 1 encoder has a few hundred rows: its
// 32-deep K steps run back to back on ~30 blocks otherwise, latency-bound).
bool enc_big_tile(long long rows, int N) { return (long long)cdiv(rows, 128) * cdiv(N, 64) >= 256; }
int enc_ksplit(long long rows, int N, int K) {
  if (enc_big_tile(rows, N)) return 1;
  const long long gxy = (long long)cdiv(rows, 32) * cdiv(N, 128);
  int ks = (int)std::min<long long>(8, (256 + gxy - 1) / gxy);
  ks = std::min(ks, std::max(1, K / GEMM_BK / 4));   // >= 4 K steps per block
  return std::max(ks, 1);
}

template <int EPI, int ID>
int enc_gemm(GemmArgs a, float* part, hipStream_t st, const char* tag) {
  const long long rows = (long long)a.B * a.T;
  if (enc_big_tile(rows, a.N)) return launch_gemm<1, 2, 4, 1, EPI, ID>(a, st, tag);
  a.ksplit = enc_ksplit(rows, a.N, a.ldw);
  a.part = part;
  return launch_gemm<1, 1, 1, 4, EPI, ID>(a, st, tag);
}

}  // namespace

struct pd_cond {
  pd_cond_dims d;
  int H, L, K, heads, D, F;
  float* pool = nullptr;
  __bf16* pool_bf = nullptr;
  // per layer
  std::vector<float*> ln1g, ln1b, Wqkv, Wo, ln2g, ln2b, W1, b1, W2, b2;
  float *lnfg = nullptr, *lnfb = nullptr, *emb = nullptr, *dur_w = nullptr, *dur_b = nullptr;
  float *spk = nullptr, *gender = nullptr, *lang = nullptr, *pw = nullptr, *pb = nullptr;
  float *vw = nullptr, *vb = nullptr, *bw = nullptr, *bb = nullptr;
};

namespace {
struct CondWs {
  size_t x, h, qkv, att, f, enc, part, total;
};
CondWs cond_ws(const pd_cond* h, int B, int Tt) {
  const size_t R = (size_t)B * Tt;
  auto al = [](size_t n) { return (n + 63) / 64 * 64; };
  CondWs w{};
  size_t o = 0;
  w.x = o; o += al(R * h->H);
  w.h = o; o += al(R * h->H);
  w.qkv = o; o += al(R * 3 * h->H);
  w.att = o; o += al(R * h->H);
  w.f = o; o += al(R * h->F);
  w.enc = o; o += al(R * h->H);
  // split-K partial sums: the largest ksplit * rows * N over the four GEMMs
  const int H = h->H, F = h->F;
  size_t part = 0;
  const int NK[4][2] = {{3 * H, H}, {H, H}, {F, h->K * H}, {H, F}};
  for (auto& nk : NK) {
    const int ks = enc_ksplit((long long)R, nk[0], nk[1]);
    if (ks > 1) part = std::max(part, (size_t)ks * R * nk[0]);
  }
  w.part = o; o += al(part);
  w.total = o * sizeof(float);
  return w;
}
}  // namespace

extern "C" {

int pd_cond_num_params(const pd_cond_dims* d) {
  if (!d) return -1;
  return 10 * d->enc_layers + 3 + 2 * !!d->use_dur_embed + !!d->use_spk_id + !!d->use_gender_id +
         !!d->use_lang_id + 2 + 2 * !!d->use_voicing_embed + 2 * !!d->use_breath_embed;
}

int pd_cond_create(const pd_cond_dims* dims, const float* const* params, int dtype, void* stream, pd_cond** out) {
  PD_CHECK_ARG(dims && params && out, "null pointer");
  const pd_cond_dims& d = *dims;
  PD_CHECK_ARG(dtype == PD_DTYPE_F32 || dtype == PD_DTYPE_BF16, "dtype must be PD_DTYPE_F32 or PD_DTYPE_BF16");
  PD_CHECK_ARG(d.hidden_size > 0 && d.hidden_size % 64 == 0, "hidden_size must be a positive multiple of 64");
  PD_CHECK_ARG(d.num_heads > 0 && d.hidden_size % d.num_heads == 0, "hidden_size % num_heads != 0");
  PD_CHECK_ARG(d.rel_pos >= 0, "rel_pos must be >= 0 (0: sinusoid; > 0: table of max(rel_pos, 5000) rows)");
  const int D = d.hidden_size / d.num_heads;
  if (D != 64 && D != 128 && D != 256) {
    set_error("pd_cond: head dim (hidden_size / num_heads) must be 64, 128 or 256");
    return PD_ERR_UNSUPPORTED;
  }
  PD_CHECK_ARG(d.enc_ffn_kernel_size % 2 == 1 && d.enc_ffn_kernel_size <= MAX_SEGS,
               "enc_ffn_kernel_size must be odd and <= 11 (SAME padding)");
  PD_CHECK_ARG(d.enc_layers >= 0 && d.vocab_size > 0, "bad enc_layers / vocab_size");
  PD_CHECK_ARG(!d.use_spk_id || d.num_spk > 0, "num_spk must be positive with use_spk_id");
  PD_CHECK_ARG(!d.use_lang_id || d.num_langs > 0, "num_langs must be positive with use_lang_id");
  // add_gender_embed looks the ids up in lang_embed (prodiff_teacher.py:91-95), so gender ids need it
  PD_CHECK_ARG(!d.use_gender_id || d.use_lang_id, "use_gender_id needs use_lang_id (gender ids index lang_embed)");
  hipStream_t st = (hipStream_t)stream;
  pd_cond* h = new pd_cond();
  h->d = d;
  h->H = d.hidden_size; h->L = d.enc_layers; h->K = d.enc_ffn_kernel_size;
  h->heads = d.num_heads; h->D = D; h->F = 4 * d.hidden_size;
  const int H = h->H, F = h->F, K = h->K, L = h->L;
  // pool layout (floats, 64-aligned); GEMM weights packed as W[n][k]
  std::vector<std::pair<float**, size_t>> plan;
  h->ln1g.resize(L); h->ln1b.resize(L); h->Wqkv.resize(L); h->Wo.resize(L); h->ln2g.resize(L);
  h->ln2b.resize(L); h->W1.resize(L); h->b1.resize(L); h->W2.resize(L); h->b2.resize(L);
  for (int l = 0; l < L; ++l) {
    plan.push_back({&h->ln1g[l], H}); plan.push_back({&h->ln1b[l], H});
    plan.push_back({&h->Wqkv[l], (size_t)3 * H * H}); plan.push_back({&h->Wo[l], (size_t)H * H});
    plan.push_back({&h->ln2g[l], H}); plan.push_back({&h->ln2b[l], H});
    plan.push_back({&h->W1[l], (size_t)F * K * H}); plan.push_back({&h->b1[l], F});
    plan.push_back({&h->W2[l], (size_t)H * F}); plan.push_back({&h->b2[l], H});
  }
  plan.push_back({&h->lnfg, H}); plan.push_back({&h->lnfb, H});
  plan.push_back({&h->emb, (size_t)d.vocab_size * H});
  if (d.use_dur_embed) { plan.push_back({&h->dur_w, H}); plan.push_back({&h->dur_b, H}); }
  if (d.use_spk_id) plan.push_back({&h->spk, (size_t)d.num_spk * H});
  if (d.use_gender_id) plan.push_back({&h->gender, (size_t)2 * H});
  if (d.use_lang_id) plan.push_back({&h->lang, (size_t)d.num_langs * H});
  plan.push_back({&h->pw, H}); plan.push_back({&h->pb, H});
  if (d.use_voicing_embed) { plan.push_back({&h->vw, H}); plan.push_back({&h->vb, H}); }
  if (d.use_breath_embed) { plan.push_back({&h->bw, H}); plan.push_back({&h->bb, H}); }
  size_t off = 0;
  std::vector<size_t> offs;
  for (auto& p : plan) { offs.push_back(off); off += (p.second + 63) / 64 * 64; }
  if (hipMalloc(&h->pool, off * sizeof(float)) != hipSuccess) {
    delete h;
    set_error("hipMalloc failed for condition-encoder weights");
    return PD_ERR_HIP;
  }
  for (size_t i = 0; i < plan.size(); ++i) *plan[i].first = h->pool + offs[i];
  auto run = [&]() -> int {
    auto cp = [&](float* dst, const float* src, size_t n) -> int {
      PD_CHECK_ARG(src, "null parameter pointer");
      PD_HIP(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, st));
      return PD_OK;
    };
    int p = 0;
    for (int l = 0; l < L; ++l) {
      PD_TRY(cp(h->ln1g[l], params[p++], H));
      PD_TRY(cp(h->ln1b[l], params[p++], H));
      PD_TRY(cp(h->Wqkv[l], params[p++], (size_t)3 * H * H));   // in_proj_weight [3H, H] = W[n][k]
      PD_TRY(cp(h->Wo[l], params[p++], (size_t)H * H));
      PD_TRY(cp(h->ln2g[l], params[p++], H));
      PD_TRY(cp(h->ln2b[l], params[p++], H));
      PD_CHECK_ARG(params[p], "null parameter pointer");
      PD_TRY(pack_conv(h->W1[l], K * H, 0, 0, H, params[p++], F, H, K, st));   // ffn_1 [F, H, K]
      PD_TRY(cp(h->b1[l], params[p++], F));
      PD_TRY(cp(h->W2[l], params[p++], (size_t)H * F));
      PD_TRY(cp(h->b2[l], params[p++], H));
    }
    PD_TRY(cp(h->lnfg, params[p++], H));
    PD_TRY(cp(h->lnfb, params[p++], H));
    PD_TRY(cp(h->emb, params[p++], (size_t)d.vocab_size * H));
    if (d.use_dur_embed) { PD_TRY(cp(h->dur_w, params[p++], H)); PD_TRY(cp(h->dur_b, params[p++], H)); }
    if (d.use_spk_id) PD_TRY(cp(h->spk, params[p++], (size_t)d.num_spk * H));
    if (d.use_gender_id) PD_TRY(cp(h->gender, params[p++], (size_t)2 * H));
    if (d.use_lang_id) PD_TRY(cp(h->lang, params[p++], (size_t)d.num_langs * H));
    PD_TRY(cp(h->pw, params[p++], H));
    PD_TRY(cp(h->pb, params[p++], H));
    if (d.use_voicing_embed) { PD_TRY(cp(h->vw, params[p++], H)); PD_TRY(cp(h->vb, params[p++], H)); }
    if (d.use_breath_embed) { PD_TRY(cp(h->bw, params[p++], H)); PD_TRY(cp(h->bb, params[p++], H)); }
    if (dtype == PD_DTYPE_BF16) {
      PD_HIP(hipMalloc(&h->pool_bf, off * sizeof(__bf16)));
      PD_TRY(convert_f32_bf16(h->pool, h->pool_bf, (long long)off, st));
      register_bf16_pool(h->pool, off, h->pool_bf);
    }
    return PD_OK;
  };
  const int rc = run();
  if (rc != PD_OK) {
    (void)hipFree(h->pool);
    if (h->pool_bf) (void)hipFree(h->pool_bf);
    delete h;
    return rc;
  }
  *out = h;
  return PD_OK;
}

void pd_cond_destroy(pd_cond* h) {
  if (!h) return;
  if (h->pool_bf) {
    unregister_bf16_pool(h->pool);
    (void)hipFree(h->pool_bf);
  }
  (void)hipFree(h->pool);
  delete h;
}

size_t pd_cond_workspace_size(const pd_cond* h, int B, int T_txt, int T_mel) {
  if (!h || B < 1 || T_txt < 1 || T_mel < 0) return 0;
  return cond_ws(h, B, T_txt).total;
}

int pd_cond_forward(const pd_cond* h, const pd_cond_inputs* in, float* cond, float* enc_out, int B, int T_txt,
                    int T_mel, void* workspace, size_t ws_bytes, void* stream) {
  PD_CHECK_ARG(h && in && workspace, "null pointer");
  PD_CHECK_ARG(B > 0 && T_txt > 0 && T_mel >= 0, "bad B / T_txt / T_mel");
  PD_CHECK_ARG(in->txt_tokens && in->mel2ph, "txt_tokens and mel2ph are required");
  PD_CHECK_ARG(cond || enc_out, "nothing to write: cond and enc_out are both null");
  const pd_cond_dims& d = h->d;
  if (cond) {
    PD_CHECK_ARG(in->f0, "f0 is required");   // add_pitch (prodiff_teacher.py:97-100)
    if (d.use_spk_id)   // add_spk_embed's assert (prodiff_teacher.py:84)
      PD_CHECK_ARG(in->spk_embed_id || in->spk_mix_embed, "use_spk_id: spk_embed_id or spk_mix_embed is required");
    if (d.use_gender_id)
      PD_CHECK_ARG(in->gender_embed_id || in->gender_mix_embed,
                   "use_gender_id: gender_embed_id or gender_mix_embed is required");
    if (d.use_voicing_embed) PD_CHECK_ARG(in->voicing, "use_voicing_embed: voicing is required");
    if (d.use_breath_embed) PD_CHECK_ARG(in->breath, "use_breath_embed: breath is required");
  }
  if (d.use_lang_id) PD_CHECK_ARG(in->lang_seq, "use_lang_embed is True, lang_seq is required");   // :116
  const CondWs w = cond_ws(h, B, T_txt);
  if (ws_bytes < w.total) { set_error("workspace too small"); return PD_ERR_WORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  const int H = h->H, F = h->F, K = h->K;
  const int rows = B * T_txt;
  const long long bs = (long long)T_txt;
  float* x = ws + w.x;
  float* hn = ws + w.h;
  float* qkv = ws + w.qkv;
  float* att = ws + w.att;
  float* ff = ws + w.f;
  float* enc = enc_out ? enc_out : ws + w.enc;
  float* part = ws + w.part;
  const float neg_freq = (float)(-(std::log(10000.0) / (H / 2 - 1)));
  const float neg_rel = (float)(-(std::log(10000.0) / H));
  {
    ProfScope ps("enc_embed", st);
    hipLaunchKernelGGL(enc_embed_kernel, dim3(cdiv(T_txt, EMB_TOK), B), dim3(256), 0, st, in->txt_tokens,
                       d.use_lang_id ? in->lang_seq : nullptr, in->mel2ph, T_txt, T_mel, H, h->emb, d.vocab_size,
                       (float)std::sqrt((double)H), h->dur_w, h->dur_b, h->lang, d.num_langs, neg_freq, d.rel_pos,
                       neg_rel, x);
  }
  PD_LAUNCH_CHECK();
  const float eps = 1e-5f;
  const float qscale = (float)std::sqrt(1.0 / (double)h->D);
  for (int l = 0; l < h->L; ++l) {
    {
      ProfScope ps("enc_ln", st);
      hipLaunchKernelGGL(enc_ln_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, h->ln1g[l], h->ln1b[l],
                         in->txt_tokens, hn, rows, H, eps, 0);
    }
    PD_LAUNCH_CHECK();
    {
      GemmArgs a = make_gemm(B, T_txt, 3 * H, h->Wqkv[l], H, nullptr, qkv, bs * 3 * H, 3 * H);
      add_seg(a, make_seg(hn, bs * H, H, H, 0));
      PD_TRY((enc_gemm<EPI_STORE, U_ENC_QKV>(a, part, st, "enc_qkv")));
    }
    {
      ProfScope ps("enc_attn", st);
      dim3 grid(cdiv(T_txt, AQ), h->heads, B);
      if (h->D == 64)
        hipLaunchKernelGGL(enc_attn_kernel<64>, grid, dim3(256), 0, st, qkv, in->txt_tokens, att, T_txt, H, qscale);
      else if (h->D == 128)
        hipLaunchKernelGGL(enc_attn_kernel<128>, grid, dim3(256), 0, st, qkv, in->txt_tokens, att, T_txt, H, qscale);
      else
        hipLaunchKernelGGL(enc_attn_kernel<256>, grid, dim3(256), 0, st, qkv, in->txt_tokens, att, T_txt, H, qscale);
    }
    PD_LAUNCH_CHECK();
    {   // x = x + attn Wo^T   (out_proj, bias=False; residual, common_layers.py:658-665)
      GemmArgs a = make_gemm(B, T_txt, H, h->Wo[l], H, nullptr, x, bs * H, H);
      add_seg(a, make_seg(att, bs * H, H, H, 0));
      a.res = x; a.res_bs = bs * H; a.res_ld = H;
      PD_TRY((enc_gemm<EPI_STORE, U_ENC_OUT>(a, part, st, "enc_outproj")));
    }
    {
      ProfScope ps("enc_ln", st);
      hipLaunchKernelGGL(enc_ln_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, h->ln2g[l], h->ln2b[l],
                         in->txt_tokens, hn, rows, H, eps, 0);
    }
    PD_LAUNCH_CHECK();
    {   // f = gelu(k^-0.5 (conv_k(hn) + b1))   (TransformerFFNLayer, common_layers.py:570-576)
      GemmArgs a = make_gemm(B, T_txt, F, h->W1[l], K * H, h->b1[l], ff, bs * F, F);
      for (int tap = 0; tap < K; ++tap) add_seg(a, make_seg(hn, bs * H, H, H, tap - K / 2));
      a.lens = in->txt_lens; a.lens_mul = 1;   // ragged token batch: zero past each row's own tokens
      a.act = ACT_GELU;
      a.alpha = (float)std::pow((double)K, -0.5);
      PD_TRY((enc_gemm<EPI_STORE, U_ENC_FFN1>(a, part, st, "enc_ffn1")));
    }
    {   // x = x + (f W2^T + b2)   (ffn_2, residual, :667-672)
      GemmArgs a = make_gemm(B, T_txt, H, h->W2[l], F, h->b2[l], x, bs * H, H);
      add_seg(a, make_seg(ff, bs * F, F, F, 0));
      a.res = x; a.res_bs = bs * H; a.res_ld = H;
      PD_TRY((enc_gemm<EPI_STORE, U_ENC_FFN2>(a, part, st, "enc_ffn2")));
    }
  }
  {
    ProfScope ps("enc_ln", st);
    hipLaunchKernelGGL(enc_ln_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, h->lnfg, h->lnfb, in->txt_tokens,
                       enc, rows, H, eps, 1);
  }
  PD_LAUNCH_CHECK();
  if (!cond || T_mel == 0) return PD_OK;
  CondArgs a{};
  a.enc = enc; a.mel2ph = in->mel2ph; a.f0 = in->f0; a.pw = h->pw; a.pb = h->pb;
  if (d.use_spk_id) {
    if (in->spk_mix_embed) { a.spk_mix = in->spk_mix_embed; a.spk_ts = in->spk_mix_frames > 1; }
    else { a.spk_tab = h->spk; a.spk_id = in->spk_embed_id; a.n_spk = d.num_spk; }
  }
  if (d.use_gender_id) {
    if (in->gender_mix_embed) { a.gen_mix = in->gender_mix_embed; a.gen_ts = in->gender_mix_frames > 1; }
    else { a.gen_tab = h->lang; a.gen_id = in->gender_embed_id; a.n_gen = d.num_langs; }
  }
  if (d.use_voicing_embed) { a.voicing = in->voicing; a.vw = h->vw; a.vb = h->vb; }
  if (d.use_breath_embed) { a.breath = in->breath; a.bw = h->bw; a.bb = h->bb; }
  a.out = cond; a.B = B; a.Tt = T_txt; a.Tm = T_mel; a.H = H;
  if (a.spk_ts) PD_CHECK_ARG(in->spk_mix_frames == T_mel, "spk_mix_embed frames must be 1 or T_mel");
  if (a.gen_ts) PD_CHECK_ARG(in->gender_mix_frames == T_mel, "gender_mix_embed frames must be 1 or T_mel");
  {
    ProfScope ps("enc_cond", st);
    hipLaunchKernelGGL(enc_cond_kernel, dim3(cdiv((long long)B * T_mel, 4)), dim3(256), 0, st, a);
  }
  PD_LAUNCH_CHECK();
  return PD_OK;
}

}  // extern "C"
