// Common helpers for the ProDiff/FastDiff gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#define PD_OK 0
#define PD_ERR_ARG 1
#define PD_ERR_HIP 2
#define PD_ERR_WORKSPACE 3
#define PD_ERR_UNSUPPORTED 4

namespace pd {

void set_error(const std::string& msg);
const char* get_error();

}  // namespace pd

#define PD_CHECK_ARG(cond, msg)                       \
  do {                                                \
    if (!(cond)) {                                    \
      pd::set_error(std::string("argument: ") + msg); \
      return PD_ERR_ARG;                              \
    }                                                 \
  } while (0)

#define PD_HIP(expr)                                                               \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      pd::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));           \
      return PD_ERR_HIP;                                                           \
    }                                                                              \
  } while (0)

#define PD_LAUNCH_CHECK()                                                          \
  do {                                                                             \
    hipError_t _e = hipGetLastError();                                             \
    if (_e != hipSuccess) {                                                        \
      pd::set_error(std::string("kernel launch: ") + hipGetErrorString(_e) +      \
                    " at " + __FILE__ + ":" + std::to_string(__LINE__));          \
      return PD_ERR_HIP;                                                           \
    }                                                                              \
  } while (0)

#define PD_TRY(expr)                \
  do {                              \
    int _rc = (expr);               \
    if (_rc != PD_OK) return _rc;   \
  } while (0)

namespace pd {

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_MISH = 3, ACT_SWISH = 4, ACT_TANH = 5, ACT_GELU = 6 };

__device__ __forceinline__ float act_apply(float v, int act, float alpha) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_LRELU: return v >= 0.f ? v : alpha * v;
    case ACT_MISH: {
      // x * tanh(softplus(x)), softplus threshold 20 (torch default)
      float sp = v > 20.f ? v : log1pf(expf(v));
      return v * tanhf(sp);
    }
    case ACT_SWISH: return v / (1.f + expf(-v));
    case ACT_TANH: return tanhf(v);
    case ACT_GELU: {
      // exact (erf) GELU of alpha * v: the FFT-encoder FFN scales its conv output by
      // kernel_size^-0.5 BEFORE the activation (common_layers.py:570-576)
      const float x = v * alpha;
      return 0.5f * x * (1.f + erff(x * 0.70710678118654752440f));
    }
    default: return v;
  }
}

// Gate nonlinearities on the hardware transcendentals (v_exp_f32 + v_rcp_f32, ~1 ulp
// each): ~10 VALU ops instead of the IEEE divide + libm tanh (~60), which made the
// gated epilogues VALU-bound.  Saturation is exact: exp -> inf gives rcp -> 0.
__device__ __forceinline__ float exp_fast(float v) {
  return __builtin_amdgcn_exp2f(v * 1.4426950408889634f);
}
__device__ __forceinline__ float sigmoidf_(float v) {
  return __builtin_amdgcn_rcpf(1.f + exp_fast(-v));
}
__device__ __forceinline__ float tanhf_(float v) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(exp_fast(2.f * v) + 1.f);
}

// sigmoid(g) * tanh(f) with 2 exp + 1 rcp:  (E_f - 1) / ((E_f + 1)(1 + E_g)),
// E_f = e^{2f} (f clamped to +-15, where tanh is 1 in fp32), E_g = e^{-g} (inf -> 0).
__device__ __forceinline__ float gate_fast(float g, float f) {
  const float ef = __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(f, -15.f, 15.f) * 2.8853900817779268f);
  const float eg = __builtin_amdgcn_exp2f(g * -1.4426950408889634f);
  return (ef - 1.f) * __builtin_amdgcn_rcpf((ef + 1.f) * (1.f + eg));
}

// ---------------------------------------------------------------------------
// Counter-based normal/uniform draws (Philox4x32-10), used when the caller does
// not hand in explicit noise.  key = seed.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
    uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += W0; k1 += W1;
  }
}

__device__ __forceinline__ float u01_from(uint32_t x) {
  // (0,1]: never 0, so log() is finite
  return (float)((x >> 8) + 1u) * (1.0f / 16777216.0f);
}

// Per-utterance draws (what every sampler uses): counter = (element within the utterance,
// utterance id, stream).  An utterance's noise depends on its id, never on its row in a
// batch or on how a job is sharded over ranks, so batched, length-grouped and multi-GPU
// runs of the same utterance produce the same output.  Ids come from the caller
// (`utt_ids`, one per batch row) or default to the row index.
__device__ __forceinline__ unsigned utt_id(const int* ids, int b) { return ids ? (unsigned)ids[b] : (unsigned)b; }
__device__ __forceinline__ float philox_normal_u(uint64_t seed, unsigned uid, unsigned elem, uint32_t stream) {
  uint32_t c[4] = {elem, uid, stream, 0x5EEDu};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float u1 = u01_from(c[0]), u2 = u01_from(c[1]);
  return sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
}
__device__ __forceinline__ float philox_uniform_u(uint64_t seed, unsigned uid, unsigned elem, uint32_t stream) {
  uint32_t c[4] = {elem, uid, stream, 0x0F00u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return (float)(c[0] >> 8) * (1.0f / 16777216.0f);
}

// Optional per-launch timing (pd_profile_enable): HIP events recorded on the
// launch stream around every tagged kernel; read back after the timed region.
struct ProfScope {
  ProfScope(const char* tag, hipStream_t st);
  ~ProfScope();
  const char* tag_;
  hipStream_t st_;
  int slot_;
};

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace pd
