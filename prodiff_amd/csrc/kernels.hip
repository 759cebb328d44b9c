// Small utility kernels + error plumbing.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <mutex>
#include <vector>

#include "gemm.h"
#include "kernels.h"

namespace pd {

static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
const char* get_error() { return g_err.c_str(); }

int validate_gemm(const GemmArgs& a) {
  if (a.B < 0 || a.T < 0 || a.N <= 0) { set_error("gemm: bad B/T/N"); return PD_ERR_ARG; }
  if (a.nseg <= 0 || a.nseg > MAX_SEGS) { set_error("gemm: bad segment count"); return PD_ERR_ARG; }
  int k = 0;
  for (int i = 0; i < a.nseg; ++i) {
    const Seg& s = a.seg[i];
    if (!s.src || s.cs <= 0 || (s.cs & 3) || (s.ld & 3) || (s.bstride & 3) ||
        (reinterpret_cast<uintptr_t>(s.src) & 15) || s.kpad % GEMM_BK || s.kpad < s.cs ||
        s.row_mul < 1) {
      set_error("gemm: segment " + std::to_string(i) + " not 16-byte aligned / padded");
      return PD_ERR_ARG;
    }
    if (s.add_vec && ((s.add_ld & 3) || (reinterpret_cast<uintptr_t>(s.add_vec) & 15))) {
      set_error("gemm: add_vec alignment"); return PD_ERR_ARG;
    }
    if (s.add_ten && (reinterpret_cast<uintptr_t>(s.add_ten) & 15)) {
      set_error("gemm: add_ten alignment"); return PD_ERR_ARG;
    }
    k += s.kpad;
  }
  if (k != a.ldw) { set_error("gemm: sum(kpad) != ldw"); return PD_ERR_ARG; }
  if (reinterpret_cast<uintptr_t>(a.W) & 15) { set_error("gemm: W alignment"); return PD_ERR_ARG; }
  return PD_OK;
}

// ---------------------------------------------------------------- split-K reduce
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmArgs a) {
  const long long rows = (long long)a.B * a.T;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * a.N) return;
  const long long R = i / a.N;
  const int n = (int)(i - R * a.N);
  float v = 0.f;
  for (int z = 0; z < a.ksplit; ++z) v += a.part[(z * rows + R) * a.N + n];
  v += a.bias ? a.bias[n] : 0.f;
  v = act_apply(v, a.act, a.alpha) * a.scale;
  const long long b = R / a.T, t = R - b * a.T;
  if (a.res) v += a.res[b * a.res_bs + t * a.res_ld + n];
  const long long oi = b * a.out_bs + t * a.out_ld + n;
  if (a.out_bf16) reinterpret_cast<__bf16*>(a.out)[oi] = (__bf16)v;
  else a.out[oi] = v;
}

// paired epilogues over (row, n < half): columns n and n + half combine (gemm.h EPI_GATE / EPI_RESSKIP)
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_paired_kernel(const GemmArgs a) {
  const long long rows = (long long)a.B * a.T;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * a.half) return;
  const long long R = i / a.half;
  const int n = (int)(i - R * a.half);
  float v0 = a.bias[n], v1 = a.bias[a.half + n];
  for (int z = 0; z < a.ksplit; ++z) {
    const float* pz = a.part + (z * rows + R) * a.N + n;
    v0 += pz[0];
    v1 += pz[a.half];
  }
  const long long b = R / a.T, t = R - b * a.T;
  if constexpr (EPI == EPI_GATE) {
    a.out[b * a.out_bs + t * a.out_ld + n] = sigmoidf_(v0) * tanhf_(v1);
  } else {
    float* xp = a.out + b * a.out_bs + t * a.out_ld + n;
    *xp = (*xp + v0) * 0.70710678118654752440f;
    float* sp = a.out2 + b * a.out2_bs + t * a.out2_ld + n;
    *sp = a.flag ? v1 : (*sp + v1);
  }
}

int gemm_splitk_reduce(const GemmArgs& a, int epi, hipStream_t st) {
  const long long rows = (long long)a.B * a.T;
  if (epi == EPI_GATE || epi == EPI_RESSKIP) {
    const long long n = rows * a.half;
    if (epi == EPI_GATE)
      hipLaunchKernelGGL(splitk_reduce_paired_kernel<EPI_GATE>, dim3(cdiv(n, 256)), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL(splitk_reduce_paired_kernel<EPI_RESSKIP>, dim3(cdiv(n, 256)), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(cdiv(rows * a.N, 256)), dim3(256), 0, st, a);
  }
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- matvec
// out[v][n] = act(W[n] . in[v] + bias[n]).  One wave per output n and MV_NV vectors at
// once (grid.y covers the vector groups), so each W row is read once per group and
// the MV_NV dot products run side by side instead of one after another.
constexpr int MV_NV = 8;
__global__ __launch_bounds__(256) void matvec_kernel(const float* __restrict__ W,
                                                     const float* __restrict__ bias,
                                                     const float* __restrict__ in, int in_ld,
                                                     float* __restrict__ out, int out_ld, int N,
                                                     int K, int nvec, int act) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int v0 = blockIdx.y * MV_NV;
  if (n >= N) return;
  const int nv = nvec - v0 < MV_NV ? nvec - v0 : MV_NV;
  const float* w = W + (long long)n * K;
  float s[MV_NV];
#pragma unroll
  for (int j = 0; j < MV_NV; ++j) s[j] = 0.f;
  // 4 k-steps per trip with every load issued before the FMAs (K is a multiple of 64 for
  // every caller; the tail loop covers the rest)
  const float* iv = in + (long long)v0 * in_ld;
  int k = lane;
  for (; k + 192 < K; k += 256) {
    float wk[4], x[4][MV_NV];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      wk[u] = w[k + 64 * u];
#pragma unroll
      for (int j = 0; j < MV_NV; ++j) x[u][j] = j < nv ? iv[(long long)j * in_ld + k + 64 * u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < MV_NV; ++j) s[j] = fmaf(wk[u], x[u][j], s[j]);
  }
  for (; k < K; k += 64) {
    const float wk = w[k];
#pragma unroll
    for (int j = 0; j < MV_NV; ++j)
      if (j < nv) s[j] = fmaf(wk, iv[(long long)j * in_ld + k], s[j]);
  }
#pragma unroll
  for (int j = 0; j < MV_NV; ++j) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s[j] += __shfl_xor(s[j], o);
  }
  if (lane < nv) {
    float r = s[0];
#pragma unroll
    for (int j = 1; j < MV_NV; ++j) r = lane == j ? s[j] : r;
    out[(long long)(v0 + lane) * out_ld + n] = act_apply(r + (bias ? bias[n] : 0.f), act, 0.f);
  }
}

int matvec(const float* W, const float* bias, const float* in, int in_ld, float* out, int out_ld,
           int N, int K, int nvec, int act, hipStream_t st) {
  if (nvec <= 0) return PD_OK;
  ProfScope ps("step_mlp", st);
  hipLaunchKernelGGL(matvec_kernel, dim3(cdiv(N, 4), cdiv(nvec, MV_NV)), dim3(256), 0, st, W, bias, in, in_ld,
                     out, out_ld, N, K, nvec, act);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- embeddings
__global__ void sinusoidal_kernel(const float* __restrict__ steps, float* __restrict__ out, int nvec,
                                  int dim, float neg_e) {
  const int half = dim / 2;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec * half) return;
  int v = i / half, k = i - v * half;
  float f = expf((float)k * neg_e);          // torch: exp(arange(half) * -e) in fp32
  float arg = steps[v] * f;                  // long/float step * fp32 freq -> fp32
  out[(long long)v * dim + k] = sinf(arg);
  out[(long long)v * dim + half + k] = cosf(arg);
}

int sinusoidal_embed(const float* steps, float* out, int nvec, int dim, hipStream_t st) {
  const int half = dim / 2;
  float neg_e = -(float)(std::log(10000.0) / (half - 1));
  int n = nvec * half;
  if (n == 0) return PD_OK;
  hipLaunchKernelGGL(sinusoidal_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, steps, out, nvec, dim,
                     neg_e);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

__global__ void rev_steps_kernel(float* steps, int S, int B, int first) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < S * B) steps[i] = (float)(first - i / B);
}

int fill_reverse_steps(float* steps, int S, int B, int first, hipStream_t st) {
  hipLaunchKernelGGL(rev_steps_kernel, dim3(cdiv(S * B, 256)), dim3(256), 0, st, steps, S, B, first);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

struct StepVals { float v[PD_MAX_STEP_VALS]; };
__global__ void steps_kernel(float* steps, StepVals vals, int S, int B) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < S * B) steps[i] = vals.v[i / B];
}

int fill_steps(float* steps, const float* host_vals, int S, int B, hipStream_t st) {
  if (S > PD_MAX_STEP_VALS) { set_error("fill_steps: too many step values"); return PD_ERR_ARG; }
  StepVals sv{};
  for (int j = 0; j < S; ++j) sv.v[j] = host_vals[j];
  hipLaunchKernelGGL(steps_kernel, dim3(cdiv(S * B, 256)), dim3(256), 0, st, steps, sv, S, B);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- rectified flow helpers
// out[i] = x[i] + sum_j c[j] k[j][i]  (RK stage inputs / final update, reflow.py:48-84)
__global__ void axpy_multi_kernel(float* out, const float* x, AxpyTerms t, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = x[i];
  for (int j = 0; j < t.n; ++j) v = fmaf(t.c[j], t.k[j][i], v);
  out[i] = v;
}

int axpy_multi(float* out, const float* x, const AxpyTerms& t, long long n, hipStream_t st) {
  if (t.n < 0 || t.n > 6) { set_error("axpy_multi: 0..6 terms"); return PD_ERR_ARG; }
  if (n <= 0) return PD_OK;
  hipLaunchKernelGGL(axpy_multi_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, out, x, t, n);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// denorm_spec: (x + 1) / 2 * (max - min) + min  (reflow.py:106-107); mean_clamp: the
// PitchRectifiedFlow form, mean over the bins then clamp (reflow.py:138-144)
__global__ void reflow_denorm_kernel(const float* __restrict__ x, const float* __restrict__ smin,
                                     const float* __restrict__ smax, int nspec, int M, long long rows,
                                     int mean_clamp, float cmin, float cmax, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (mean_clamp) {
    if (i >= rows) return;
    float s = 0.f;
    for (int m = 0; m < M; ++m) {
      const int k = nspec == 1 ? 0 : m;
      s += (x[i * M + m] + 1.f) / 2.f * (smax[k] - smin[k]) + smin[k];
    }
    out[i] = fminf(fmaxf(s / (float)M, cmin), cmax);
  } else {
    if (i >= rows * M) return;
    const int k = nspec == 1 ? 0 : (int)(i % M);
    out[i] = (x[i] + 1.f) / 2.f * (smax[k] - smin[k]) + smin[k];
  }
}

int reflow_denorm(const float* x, const float* smin, const float* smax, int nspec, int M, long long rows,
                  int mean_clamp, float cmin, float cmax, float* out, hipStream_t st) {
  const long long n = mean_clamp ? rows : rows * M;
  if (n <= 0) return PD_OK;
  hipLaunchKernelGGL(reflow_denorm_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, x, smin, smax, nspec, M, rows,
                     mean_clamp, cmin, cmax, out);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- transposes
// in [B][R][Cc] -> out [B][Cc][R] via 32x32 LDS tiles
__global__ void transpose_kernel(const float* __restrict__ in, float* __restrict__ out, int R, int Cc) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const float* src = in + (long long)b * R * Cc;
  float* dst = out + (long long)b * R * Cc;
  for (int i = threadIdx.y; i < 32; i += 8) {
    int r = r0 + i, c = c0 + threadIdx.x;
    tile[i][threadIdx.x] = (r < R && c < Cc) ? src[(long long)r * Cc + c] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    int c = c0 + i, r = r0 + threadIdx.x;
    if (r < R && c < Cc) dst[(long long)c * R + r] = tile[threadIdx.x][i];
  }
}

int transpose_ct_to_tc(const float* in, float* out, int B, int C, int T, hipStream_t st) {
  if (B * C * T == 0) return PD_OK;
  hipLaunchKernelGGL(transpose_kernel, dim3(cdiv(T, 32), cdiv(C, 32), B), dim3(32, 8), 0, st, in, out,
                     C, T);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

int transpose_tc_to_ct(const float* in, float* out, int B, int T, int C, hipStream_t st) {
  if (B * C * T == 0) return PD_OK;
  hipLaunchKernelGGL(transpose_kernel, dim3(cdiv(C, 32), cdiv(T, 32), B), dim3(32, 8), 0, st, in, out,
                     T, C);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- packing
__global__ void pack_conv_kernel(float* dst, int ldw, int n_off, int k_off, int cpad,
                                 const float* src, int Cout, int Cin, int taps) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)Cout * Cin * taps;
  if (i >= total) return;
  int tap = (int)(i % taps);
  long long r = i / taps;
  int ci = (int)(r % Cin);
  int co = (int)(r / Cin);
  dst[(long long)(n_off + co) * ldw + k_off + tap * cpad + ci] = src[i];
}

int pack_conv(float* dst, int ldw, int n_off, int k_off, int cpad, const float* src, int Cout, int Cin,
              int taps, hipStream_t st) {
  long long total = (long long)Cout * Cin * taps;
  hipLaunchKernelGGL(pack_conv_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, dst, ldw, n_off, k_off,
                     cpad, src, Cout, Cin, taps);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

__global__ void add_vec_kernel(float* d, const float* a, const float* b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = a[i] + b[i];
}

int add_vectors(float* dst, const float* a, const float* b, int n, hipStream_t st) {
  hipLaunchKernelGGL(add_vec_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, dst, a, b, n);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

__global__ void wn_fold_kernel(float* w, const float* g, const float* v, int per_row) {
  const int co = blockIdx.x;
  const float* vr = v + (long long)co * per_row;
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < per_row; i += blockDim.x) s += (double)vr[i] * vr[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float scale = (float)((double)g[co] / sqrt(red[0]));
  for (int i = threadIdx.x; i < per_row; i += blockDim.x) w[(long long)co * per_row + i] = vr[i] * scale;
}

int weight_norm_fold(float* w, const float* g, const float* v, int Cout, int per_row, hipStream_t st) {
  hipLaunchKernelGGL(wn_fold_kernel, dim3(Cout), dim3(256), 0, st, w, g, v, per_row);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

// ---------------------------------------------------------------- bf16 pools
__global__ void f2bf_kernel(const float* s, __bf16* d, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = (__bf16)s[i];
}

int convert_f32_bf16(const float* src, __bf16* dst, long long n, hipStream_t st) {
  if (n == 0) return PD_OK;
  hipLaunchKernelGGL(f2bf_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, src, dst, n);
  PD_LAUNCH_CHECK();
  return PD_OK;
}

namespace {
struct PoolRec { const float* base; size_t n; const __bf16* bf; };
std::vector<PoolRec> g_pools;
std::mutex g_pool_mu;
}  // namespace

void register_bf16_pool(const float* base, size_t n, const __bf16* bf) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pools.push_back({base, n, bf});
}

void unregister_bf16_pool(const float* base) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (size_t i = 0; i < g_pools.size(); ++i)
    if (g_pools[i].base == base) { g_pools.erase(g_pools.begin() + i); return; }
}

const __bf16* lookup_bf16(const float* p) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (auto& r : g_pools)
    if (p >= r.base && p < r.base + r.n) return r.bf + (p - r.base);
  return nullptr;
}

// ---------------------------------------------------------------- RNG fills
__global__ void fill_utt_kernel(float* out, long long per, unsigned long long seed, unsigned stream, const int* ids,
                                bool normal) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (e >= per) return;
  const unsigned u = utt_id(ids, b);
  out[(long long)b * per + e] =
      normal ? philox_normal_u(seed, u, (unsigned)e, stream) : philox_uniform_u(seed, u, (unsigned)e, stream);
}
static int fill_utt(float* out, int B, long long per, unsigned long long seed, unsigned stream, const int* ids,
                    bool normal, hipStream_t st) {
  if (B == 0 || per == 0) return PD_OK;
  PD_CHECK_ARG(per < (1ll << 32), "per-utterance draw index exceeds 32 bits");
  hipLaunchKernelGGL(fill_utt_kernel, dim3(cdiv(per, 256), B), dim3(256), 0, st, out, per, seed, stream, ids, normal);
  PD_LAUNCH_CHECK();
  return PD_OK;
}
int fill_uniform_utt(float* out, int B, long long per, unsigned long long seed, unsigned stream, const int* ids,
                     hipStream_t st) {
  return fill_utt(out, B, per, seed, stream, ids, false, st);
}
int fill_normal_utt(float* out, int B, long long per, unsigned long long seed, unsigned stream, const int* ids,
                    hipStream_t st) {
  return fill_utt(out, B, per, seed, stream, ids, true, st);
}

// ---------------------------------------------------------------- profiling
namespace {
struct ProfRec { const char* tag; int slot; };
bool g_prof_on = false;
std::string g_prof_filter;   // ",tag1,tag2," or empty (every tag)
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_pool;
std::vector<ProfRec> g_recs;
}  // namespace

ProfScope::ProfScope(const char* tag, hipStream_t st) : tag_(tag), st_(st), slot_(-1) {
  if (!g_prof_on || !tag) return;
  if (!g_prof_filter.empty() && g_prof_filter.find("," + std::string(tag) + ",") == std::string::npos) return;
  slot_ = (int)g_recs.size();
  if ((size_t)slot_ >= g_pool.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { slot_ = -1; return; }
    g_pool.push_back({a, b});
  }
  g_recs.push_back({tag, slot_});
  (void)hipEventRecord(g_pool[slot_].first, st_);
}

ProfScope::~ProfScope() {
  if (slot_ >= 0) (void)hipEventRecord(g_pool[slot_].second, st_);
}

}  // namespace pd

extern "C" int pd_profile_filter(const char* tags) {
  pd::g_prof_filter = (tags && *tags) ? "," + std::string(tags) + "," : std::string();
  return PD_OK;
}

extern "C" int pd_profile_enable(int on) {
  pd::g_prof_on = on != 0;
  pd::g_recs.clear();
  return PD_OK;
}

// Waits for every recorded launch, then writes "tag count total_ms\n" lines
// (sorted by tag) into buf.  Returns the number of bytes needed (incl. NUL).
extern "C" int pd_profile_summary(char* buf, int buflen) {
  std::map<std::string, std::pair<int, double>> agg;
  for (auto& r : pd::g_recs) {
    auto& ev = pd::g_pool[r.slot];
    if (hipEventSynchronize(ev.second) != hipSuccess) { pd::set_error("hipEventSynchronize failed"); return -1; }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev.first, ev.second) != hipSuccess) { pd::set_error("hipEventElapsedTime failed"); return -1; }
    auto& a = agg[r.tag];
    a.first += 1;
    a.second += ms;
  }
  std::string out;
  char line[256];
  for (auto& kv : agg) {
    snprintf(line, sizeof line, "%s %d %.6f\n", kv.first.c_str(), kv.second.first, kv.second.second);
    out += line;
  }
  if (buf && buflen > 0) {
    size_t n = std::min((size_t)buflen - 1, out.size());
    memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return (int)out.size() + 1;
}

extern "C" const char* pd_last_error(void) { return pd::get_error(); }
extern "C" int pd_version(void) { return 2; }

namespace pd {
const char* fastdiff_build_flags();
const char* nsf_build_flags();
const char* wavenet_build_flags();
}  // namespace pd

// "default" for the shipped build, else the non-default compile-time knobs (A/B variant libraries
// built by tools/build_variant_lib.sh): bench.py records it, the GPU tests refuse a variant build
// unless PRODIFF_ALLOW_VARIANT=1.
extern "C" const char* pd_build_config(void) {
  static const std::string s = [] {
    std::string f = std::string(pd::fastdiff_build_flags()) + pd::nsf_build_flags() + pd::wavenet_build_flags();
    return f.empty() ? std::string("default") : f.substr(1);
  }();
  return s.c_str();
}
