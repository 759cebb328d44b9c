// Small utility kernels shared by the WaveNet and FastDiff paths.
#pragma once
#include "common.h"

namespace pd {

// out[v][n] = act(sum_k W[n][k] * in[v][k] + bias[n]) for v < nvec.
// One wave per output row, lanes stride K (coalesced rows of W).
int matvec(const float* W, const float* bias, const float* in, int in_ld, float* out,
           int out_ld, int N, int K, int nvec, int act, hipStream_t st);

// Sinusoidal step embedding (wavenet.py:26-38, FastDiff util.py:404-429, same
// formula): e[v] = [sin(s_v f_k), cos(s_v f_k)], f_k = exp(-k ln(1e4)/(half-1)),
// with f_k and s_v*f_k rounded to float32 as torch computes them.
int sinusoidal_embed(const float* steps, float* out, int nvec, int dim, hipStream_t st);

// steps[j*B + b] = first - j  (ProDiff reverse indices), j < S.
int fill_reverse_steps(float* steps, int S, int B, int first, hipStream_t st);
// steps[j*B + b] = vals[j] for host-provided values (FastDiff fractional steps, the
// rectified-flow stage times), S <= PD_MAX_STEP_VALS (passed as a kernel argument).
constexpr int PD_MAX_STEP_VALS = 128;
int fill_steps(float* steps, const float* host_vals, int S, int B, hipStream_t st);

// out[i] = x[i] + sum_j c[j] * k[j][i], j < n <= 6  (explicit Runge-Kutta stage inputs and
// the final update of the rectified-flow sampler, reflow.py:48-84).  out may alias x.
struct AxpyTerms {
  const float* k[6];
  float c[6];
  int n;
};
int axpy_multi(float* out, const float* x, const AxpyTerms& t, long long n, hipStream_t st);

// denorm_spec of the rectified flow (reflow.py:106-107, 138-144):
//   y[r][m] = (x[r][m] + 1) / 2 * (smax[m'] - smin[m']) + smin[m'],  m' = nspec == 1 ? 0 : m
//   mean_clamp: out[r] = clamp(mean_m y[r][m], cmin, cmax); else out[r][m] = y[r][m].
int reflow_denorm(const float* x, const float* smin, const float* smax, int nspec, int M, long long rows,
                  int mean_clamp, float cmin, float cmax, float* out, hipStream_t st);

// [B][C][T] (channel-major, PyTorch Conv1d layout) <-> [B][T][C] (time-major)
int transpose_ct_to_tc(const float* in, float* out, int B, int C, int T, hipStream_t st);
int transpose_tc_to_ct(const float* in, float* out, int B, int T, int C, hipStream_t st);

// Weight packing: dst[(n_off+co)*ldw + k_off + tap*cpad + ci] = src[(co*Cin+ci)*taps + tap]
int pack_conv(float* dst, int ldw, int n_off, int k_off, int cpad, const float* src, int Cout,
              int Cin, int taps, hipStream_t st);
// dst[i] = a[i] + b[i]
int add_vectors(float* dst, const float* a, const float* b, int n, hipStream_t st);
// weight-norm fold on device: w[co,:] = g[co] * v[co,:] / ||v[co,:]||
int weight_norm_fold(float* w, const float* g, const float* v, int Cout, int per_row, hipStream_t st);

// fp32 -> bf16 (round to nearest even)
int convert_f32_bf16(const float* src, __bf16* dst, long long n, hipStream_t st);
// bf16 mirrors of packed fp32 weight pools: launch_gemm uses the bf16 copy of any
// weight pointer inside a registered pool (same element offset).
void register_bf16_pool(const float* base, size_t n, const __bf16* bf);
void unregister_bf16_pool(const float* base);
const __bf16* lookup_bf16(const float* p);

// Philox fills, U[0,1) or N(0,1), per utterance (common.h philox_*_u): out[b][e], e < per, keyed by utt_id(ids, b).
int fill_uniform_utt(float* out, int B, long long per, unsigned long long seed, unsigned stream, const int* ids,
                     hipStream_t st);
int fill_normal_utt(float* out, int B, long long per, unsigned long long seed, unsigned stream, const int* ids,
                    hipStream_t st);

}  // namespace pd
