/*
 * prodiff_hip.h -- C-ABI of libprodiff_hip.so, the MI355X (gfx950) ProDiff/FastDiff
 * inference hot path.
 *
 * Conventions
 *  - Every tensor pointer is a caller-owned DEVICE buffer (e.g. torch.cuda tensors),
 *    float32, contiguous, 16-byte aligned.  Host pointers appear only where a
 *    parameter is documented as "host" (per-step scalars).
 *  - Calls are asynchronous and stream-ordered on `stream` (a hipStream_t; NULL =
 *    the default stream).  Nothing allocates or synchronises inside forward/sample
 *    calls, so they can be captured into a hipGraph.  Scratch memory is passed in
 *    (`workspace`, at least *_workspace_size() bytes).
 *  - Handles are immutable after create; concurrent calls on different streams
 *    need separate workspaces.
 *  - Return 0 (PD_OK) or an error code; pd_last_error() gives a thread-local text.
 *    Argument checks mirror the reference's assert points (e.g. the LVC length
 *    check, modules/FastDiff/module/modules.py:236).
 *  - Layouts: "time-major" = [batch][time][channel] (channels contiguous), the
 *    layout ProDiff's condition/mel already have at the sampler boundary
 *    (prodiff.py:136-138 receives cond [B,T,H]; :151 returns mel [B,T,M]).
 *    "channel-major" = PyTorch Conv1d layout [batch][channel][time].
 */
#ifndef PRODIFF_HIP_H
#define PRODIFF_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PD_OK 0
#define PD_ERR_ARG 1
#define PD_ERR_HIP 2
#define PD_ERR_WORKSPACE 3
#define PD_ERR_UNSUPPORTED 4

#define PD_DTYPE_F32 0
#define PD_DTYPE_BF16 1

const char* pd_last_error(void);
int pd_version(void);
/* "default" for the shipped build; otherwise the non-default compile-time knobs it was built with
 * (A/B variant libraries, tools/build_variant_lib.sh).  bench.py records it; the GPU tests refuse a
 * variant library unless PRODIFF_ALLOW_VARIANT=1. */
const char* pd_build_config(void);

/* Per-launch timing for benchmarks: when enabled, HIP events are recorded on the
 * launch stream around every hot-path kernel (tagged by use, e.g. "fd_kp_kernel").
 * pd_profile_enable(1) also clears previous records.  pd_profile_summary waits
 * for the recorded events and writes "tag count total_ms" lines; it returns the
 * buffer size needed (including the NUL), or -1 on error. */
int pd_profile_enable(int on);
int pd_profile_summary(char* buf, int buflen);
/* Restrict recording to the tags in a comma-separated list (NULL or "" = every tag).
 * An event pair costs GPU time at every launch it brackets; bench.py times its step with
 * only the dominant kernel recorded. */
int pd_profile_filter(const char* tags);

/* ===================================================================== ProDiff
 * WaveNet denoiser -- replaces modules/decoder/wavenet.py:74-123 (WaveNet) as the
 * `denoise_fn` of GaussianDiffusion (modules/diffusion/prodiff.py:49-54,125).
 */
typedef struct pd_wavenet pd_wavenet;

typedef struct {
  int in_dims;               /* M: mel bins (80 LJSpeech, 128 SVS)          wavenet.py:75 */
  int hidden_size;           /* H: condition channels (encoder_hidden)                   */
  int residual_layers;       /* L: 20 (handler/base_config.yaml:210)                     */
  int residual_channels;     /* C: 256 (base_config.yaml:211), multiple of 32            */
  int dilation_cycle_length; /* dilation 2^(l % cycle) (wavenet.py:93-96)                */
} pd_wavenet_dims;

/* Parameter order = the reference state-dict order (wavenet.py:84-99), all float32
 * in their PyTorch shapes:
 *   input_projection.{weight[C,M,1],bias[C]}, mlp.0.{weight[4C,C],bias},
 *   mlp.2.{weight[C,4C],bias},
 *   for l < L: residual_layers.l.{dilated_conv.weight[2C,C,3], dilated_conv.bias,
 *              diffusion_projection.weight[C,C], diffusion_projection.bias,
 *              conditioner_projection.weight[2C,H,1], conditioner_projection.bias,
 *              output_projection.weight[2C,C,1], output_projection.bias},
 *   skip_projection.{weight[C,C,1],bias}, output_projection.{weight[M,C,1],bias}. */
#define PD_WAVENET_NUM_PARAMS(L) (6 + 8 * (L) + 4)

/* Packs the weights into the kernels' layouts (device-to-device, on `stream`). */
int pd_wavenet_create(const pd_wavenet_dims* dims, const float* const* params, int dtype,
                      void* stream, pd_wavenet** out);
void pd_wavenet_destroy(pd_wavenet* h);
/* Kernel-variant option of a handle; set before its first call.  PD_WN_OPT_LAYER selects the
 * bf16 residual-layer implementation: 0 the fused kernel with 32-frame blocks, 3 the fused
 * kernel with 64-frame blocks, 1 two launches per layer (GATE: 128 frames x 64 gated channels
 * per block, activation window staged once; RESSKIP: 64 frames x 128 outputs), 2 (default)
 * 64-frame fused blocks when they still give every CU a block (B*T >= 16384 frames) else 32.
 * DESIGN.md §4 has the measurements. */
#define PD_WN_OPT_LAYER 0
/* PD_WN_OPT_KSPLIT (fp32 path): the residual-layer GEMMs split their K range over several blocks
 * until the grid holds 512 (default) or 256 blocks; 0 = never split. */
#define PD_WN_OPT_KSPLIT 1
/* PD_WN_OPT_L2PF (bf16 fused layer): 1 (default) each layer launch pulls the next layer's weight
 * fragments into every XCD's L2 while it runs; 0 = off. */
#define PD_WN_OPT_L2PF 2
/* PD_WN_OPT_STACK (bf16, C = H = 256, dilation_cycle_length 1, T >= 64, PD_WN_OPT_LAYER 2): n = 1..16
 * residual layers per launch (wn_stack_bf16_kernel: a 64-frame window per 32 output frames stays
 * resident for the n layers; bit-identical to the one-layer kernel), default 10; 0 = one launch
 * per layer. */
#define PD_WN_OPT_STACK 3
/* PD_WN_OPT_STACK_RO: output frames per wn_stack_bf16_kernel block, 16..48, capped at 64 - 2 max(nl, 8)
 * (the 64-frame window less a halo of one frame per layer each side); 0 (default) = that cap (44 at
 * the default 10 layers per launch). */
#define PD_WN_OPT_STACK_RO 4
/* 5: reserved (r04's in-kernel split-K reduction by arrival counters, removed: measured slower) */
/* PD_WN_OPT_STACK_FUSE (bf16 stack path): 1 (default) the input projection runs inside the first
 * stack launch and, in pd_prodiff_sample, the skip head + output projection + posterior update
 * inside the last one (same roundings and k order as the separate launches); 0 = separate launches. */
#define PD_WN_OPT_STACK_FUSE 6
/* PD_WN_OPT_F32_LAYER (fp32 path): 1 (default) residual layers whose GEMMs would split K (small
 * batches, e.g. B = 1) run as two launches of 32-frame x 32-channel-pair blocks with no split-K
 * partials (wn_f32_layer_kernel); 2 = always; 0 = the split-K GEMM engine. */
#define PD_WN_OPT_F32_LAYER 7
int pd_wavenet_set_option(pd_wavenet* h, int option, int value);
/* S = number of reverse steps the workspace must serve (1 for pd_wavenet_forward). */
size_t pd_wavenet_workspace_size(const pd_wavenet* h, int B, int T, int S);

/* One denoiser call, reference signature WaveNet.forward(spec, diffusion_step, cond)
 * (wavenet.py:100-123):
 *   spec  [B,1,M,T] channel-major, steps [B] (float; integer steps as floats),
 *   cond  [B,H,T] channel-major  ->  out [B,1,M,T]. */
int pd_wavenet_forward(const pd_wavenet* h, const float* spec, const float* steps,
                       const float* cond, float* out, int B, int T, void* workspace,
                       size_t ws_bytes, void* stream);

/* Ragged batches (every sampler below, and nsf_forward): `lens` is a device array of B ints, the
 * length of each row's utterance in mel frames (1 <= lens[b] <= T), or NULL (every row is T frames).
 * Rows stay laid out at the padded length T; frames t >= lens[b] are padding, and every convolution
 * of the network reads them as its zero padding -- so row b's first lens[b] frames (and samples)
 * equal a run of that utterance alone (B = 1, T = lens[b]), the reference's one-segment-at-a-time
 * inference (handler/infer/handler.py:373-388).  Outputs in the padding are unspecified.  With the
 * on-device draws below, the draws of an utterance's frames are the same padded or alone.  A few
 * A/B kernel variants do not take lens (PD_WN_OPT_LAYER 1, FD_OPT_LVC_TS 0, FD_OPT_KP_SIDE, FD_OPT_KP_CHUNK)
 * and return PD_ERR_UNSUPPORTED. */
/* Random draws (every sampler below).  When the caller passes no explicit draws they come
 * from an on-device Philox4x32-10 generator keyed by (seed, utterance id, element index
 * within the utterance, stream): `utt_ids` is a device array of B ints (one id per batch
 * row) or NULL (ids 0..B-1).  An utterance's output therefore depends on (seed, its id) only,
 * not on its row in the batch or on how a job is sharded over GPUs. */
/* The whole x0-predict reverse sampler, GaussianDiffusion.forward(cond, infer=True)
 * (prodiff.py:136-153) for S = clip(infer_step, 1, timesteps) steps:
 *   x ~ U[0,1); for i = S-1..0: x0 = WaveNet(x, i, cond);
 *   x = coef1[i]*x0 + coef2[i]*x + [i>0]*sigma[i]*n_i
 * with coef1/coef2 = posterior_mean_coef1/2 and sigma = exp(0.5*posterior_log_variance_clipped)
 * (host arrays of length >= S, taken from the checkpoint buffers).
 *   cond  [B,T,H] time-major (as the teacher hands it, prodiff_teacher.py:167)
 *   x_T   [B,T,M] time-major draw, or NULL -> Philox U[0,1) from `seed`
 *   noise [S][B,T,M] time-major draws (pass j uses noise[j]), or NULL -> Philox N(0,1)
 *   mel   [B,T,M] output (the reference's x[:,0].transpose(1,2), prodiff.py:151). */
int pd_prodiff_sample(const pd_wavenet* h, const float* cond, const float* coef1,
                      const float* coef2, const float* sigma, int S, const float* x_T,
                      const float* noise, unsigned long long seed, const int* utt_ids, const int* lens,
                      float* mel, int B, int T, void* workspace, size_t ws_bytes, void* stream);

/* ============================================================= rectified flow
 * RectifiedFlow / PitchRectifiedFlow inference (modules/diffusion/reflow.py:5-144) with
 * the WaveNet velocity field -- the SVS teacher's diff_type "reflow"
 * (modules/svs/prodiff_teacher.py:67-82) and the pitch predictor's sampler
 * (modules/variance_predictor/pitch_predictor.py:40-55):
 *   x ~ N(0,1); dt = 1/max(1,S); for i < S: x = step(x, t = i*dt)      (reflow.py:86-101)
 *   v(x, t) = WaveNet(x, time_scale*t, cond); step = euler / rk2 / rk4 / rk5 (reflow.py:48-84).
 * Euler's update is fused into the velocity output projection. */
#define PD_REFLOW_EULER 0
#define PD_REFLOW_RK2 1
#define PD_REFLOW_RK4 2
#define PD_REFLOW_RK5 3

/* 0 if the arguments are invalid (S * stages > 128, unknown algorithm). */
size_t pd_reflow_workspace_size(const pd_wavenet* h, int B, int T, int S, int algo);

/*   cond [B,T,H] time-major (the condition before the transpose at reflow.py:33)
 *   x_T  [B,T,M] time-major draw, or NULL -> Philox N(0,1) from `seed`
 *   x    [B,T,M] output: the reference's x.transpose(2,3).squeeze(1) before denorm_spec. */
int pd_reflow_sample(const pd_wavenet* h, const float* cond, int S, int algo, float time_scale,
                     const float* x_T, unsigned long long seed, const int* utt_ids, const int* lens, float* x,
                     int B, int T, void* workspace, size_t ws_bytes, void* stream);

/* denorm_spec (reflow.py:106-107): y = (x+1)/2 * (spec_max - spec_min) + spec_min with
 * spec_min/spec_max device arrays of length nspec (1, broadcast, or M);  x [rows,M].
 * mean_clamp = 0: out [rows,M] = y.  mean_clamp = 1 (PitchRectifiedFlow, :138-144):
 * out [rows] = clamp(mean over the M bins of y, clamp_min, clamp_max). */
int pd_reflow_denorm(const float* x, const float* spec_min, const float* spec_max, int nspec, int M,
                     int rows, int mean_clamp, float clamp_min, float clamp_max, float* out,
                     void* stream);

/* ==================================================================== FastDiff
 * eps-network -- replaces modules/FastDiff/module/FastDiff_model.py:10-102 (FastDiff)
 * and the sampler util.py:158-232 (sampling_given_noise_schedule, ddim=False).
 */
typedef struct fd_model fd_model;

typedef struct {
  int audio_channels;        /* 1    (modules/FastDiff/config/base.yaml:20) */
  int inner_channels;        /* 32   */
  int cond_channels;         /* 80   */
  int num_blocks;            /* len(upsample_ratios) = 3 */
  int upsample_ratios[4];    /* 8, 8, 4 (hop 256) */
  int lvc_layers_each_block; /* 4    */
  int lvc_kernel_size;       /* 3    */
  int kpnet_hidden_channels; /* 64   */
  int kpnet_conv_size;       /* 3    */
  int step_embed_in;         /* 128  */
  int step_embed_mid;        /* 512  */
  int step_embed_out;        /* 512  */
} fd_dims;

/* Parameter order (weight-norm already folded, w = g*v/||v||, FastDiff_model.py:104-113;
 * fd_fold_weight_norm does it on device): for every Conv1d "weight" then "bias":
 *   first_audio_conv, fc_t1.{weight,bias}, fc_t2.{weight,bias},
 *   for n < num_blocks (lvc_blocks.n): upsample.{weight[32,32,2r],bias},
 *       kernel_predictor.input_conv.0, kernel_predictor.residual_conv.{1,3,6,8,11,13},
 *       kernel_predictor.kernel_conv, kernel_predictor.bias_conv, fc_t.{weight,bias},
 *       convs.{0..3},
 *   for n < num_blocks (downsample.n): residual_dense, conv.{0,1,2},
 *   final_conv.0. */
#define FD_NUM_PARAMS(nb) (2 + 4 + 30 * (nb) + 8 * (nb) + 2)

int fd_create(const fd_dims* dims, const float* const* params, int dtype, void* stream,
              fd_model** out);
void fd_destroy(fd_model* m);
int fd_hop(const fd_model* m);   /* prod(upsample_ratios) = samples per mel frame */
/* Workspace of fd_forward (S = 1) or fd_sample (S = N steps; bounded: steps run in chunks of
 * 16, so the 200- and 1000-step schedules of fastdiff.py:58-61 need the 16-step size). */
size_t fd_workspace_size(const fd_model* m, int B, int Tc, int S);

/* Kernel-variant options of a handle (bf16 LVC-block tiling and fusions).  The defaults are
 * the measured production configuration; the tests select each variant.
 * Set them before the handle's first forward/sample call; not thread-safe against calls. */
#define FD_OPT_LVC_TS 0       /* whole-block LVC tile, hop >= 32: 384 (default), 256, 128; 0 = per-layer launches */
#define FD_OPT_LVC_TS_SUB 1   /* whole-block LVC tile of the hop < 32 block: 256 (default), 128, 384 */
#define FD_OPT_LVC_FUSE 2     /* 1: upsample / first conv / sampler update fused into the LVC blocks */
#define FD_OPT_LVC_PF 3       /* 1: next-layer kernel fragments prefetched into registers (tile 384) */
#define FD_OPT_LVC_SUB 4      /* 1: the hop < 32 block on the whole-block kernel too */
#define FD_OPT_KP_SIDE 5      /* 1: kernel-predictor GEMMs of fd_sample on a low-priority side stream */
/* 6: reserved (r02's streaming LVC kernel, removed in r03: measured slower) */
#define FD_OPT_KP_CHUNK 7     /* n > 0: kernel predictor + LVC block per chunk of n utterances (default 0 = whole batch) */
/* 8, 9: reserved (r03's skewed persistent LVC kernel, removed: measured slower) */
#define FD_OPT_LVC_TPW 10     /* 32-row tiles per wave of the 384-sample hop >= 32 LVC blocks: 2 (8 waves) or 1 (16 waves) */
#define FD_OPT_LVC_PRIO 11    /* 1: s_setprio(1) for the second half of an LVC block's waves */
/* 12: reserved (r04's persistent LVC kernel with LDS-DMA prefetch, removed: measured slower) */
#define FD_OPT_LVC_PS 14      /* 1 (r06): the final (fused, prefetching, 384-sample) LVC block as a persistent kernel whose
                               * next tile's audio / x_prev / biases arrive by LDS-DMA under the current tile's layers */
/* 13: reserved (r04's multi-tile fused-DBlock blocks, removed: measured slower) */
int fd_set_option(fd_model* m, int option, int value);

/* w[co,:] = g[co] * v[co,:] / ||v[co,:]||  (torch.nn.utils.weight_norm, dim 0). */
int fd_fold_weight_norm(float* w, const float* g, const float* v, int cout, int per_row,
                        void* stream);

/* One network call, reference net((audio, c, steps)) (FastDiff_model.py:74-102):
 *   audio [B,1,L] (L = Tc*hop), cond [B,80,Tc] channel-major, steps [B] float
 *   -> eps [B,1,L]. */
int fd_forward(const fd_model* m, const float* audio, const float* cond, const float* steps,
               float* eps, int B, int Tc, void* workspace, size_t ws_bytes, void* stream);

/* sampling_given_noise_schedule(net, (B,1,L), dh, schedule, condition) (util.py:158-232):
 *   x ~ N(0,1); for n = N-1..0: x = (x - beta[n]/sqrt(1-alpha[n]^2) eps(x,c,steps[n]))
 *                                     / sqrt(1-beta[n]) + [n>0] sigma[n] z
 *   mel   [B,Tc,80] time-major (the ProDiff sampler's output, no transpose needed)
 *   beta/alpha/sigma/steps: host arrays of length N (util.py:181-206)
 *   x_T   [B,L] draw or NULL -> Philox N(0,1); noise [N-1][B,L] (pass j uses noise[j])
 *   or NULL -> Philox;  wav [B,L] output. */
int fd_sample(const fd_model* m, const float* mel, const float* beta, const float* alpha,
              const float* sigma, const float* steps, int N, const float* x_T,
              const float* noise, unsigned long long seed, const int* utt_ids, const int* lens, float* wav,
              int B, int Tc, void* workspace, size_t ws_bytes, void* stream);

/* The same reverse process with the per-pass update given directly: pass j (j < N, sampling
 * order) evaluates eps at step value steps[j] and sets x = (x - ce[j] eps) / den[j] + sg[j] z.
 * fd_sample is this with DDPM coefficients (util.py:222-226); DDIM (util.py:215-220,
 * ddim=True) is ce = -(c2 + c3) / c1, den = 1 / c1, sg = 0.  `draw0` offsets the passes'
 * Philox stream ids (a sampler run pass by pass, return_sequence=True, keeps the fused
 * run's draws); the x_T draw is taken only when x_T is NULL. */
int fd_sample_coefs(const fd_model* m, const float* mel, const float* ce, const float* den,
                    const float* sg, const float* steps, int N, const float* x_T,
                    const float* noise, unsigned long long seed, const int* utt_ids, const int* lens,
                    int draw0, float* wav, int B, int Tc, void* workspace, size_t ws_bytes, void* stream);

/* The sampler's x_T ~ N(0,1) draw alone (util.py:208): exactly the [B,L] array fd_sample /
 * fd_sample_coefs draw when their x_T is NULL (same seed and utt_ids), written to x_T.  A
 * pass-by-pass run (return_sequence=True) takes its first state from here. */
int fd_draw_x_T(const fd_model* m, float* x_T, int B, int Tc, unsigned long long seed, const int* utt_ids,
                void* stream);

/* ==================================================================== NSF-HiFiGAN
 * SVS vocoder -- replaces modules/nsf_hifigan/models.py:222-283
 * (Generator, with SourceModuleHnNSF/SineGen :100-219 and ResBlock1/2 :36-97) as
 * called by NsfHifiGAN.spec2wav_torch (component/vocoder/nsf_hifigan.py:29-56).
 */
typedef struct nsf_model nsf_model;

typedef struct {
  int num_mels;                    /* 128 (handler/base_config.yaml:7) */
  int upsample_initial_channel;    /* 512 */
  int num_upsamples;               /* len(upsample_rates) <= 6 */
  int upsample_rates[6];           /* 8, 8, 2, 2 (hop 512) */
  int upsample_kernel_sizes[6];    /* 16, 16, 4, 4; k % u == 0, k - u even */
  int resblock;                    /* 1 (ResBlock1) or 2 (ResBlock2) */
  int num_kernels;                 /* len(resblock_kernel_sizes) <= 4 */
  int resblock_kernel_sizes[4];    /* 3, 7, 11 (odd, <= 11) */
  int num_dilations;               /* len(resblock_dilation_sizes[j]) <= 4 */
  int resblock_dilation_sizes[4][4];
  int sampling_rate;               /* 44100 */
  int harmonic_num;                /* 8 (models.py:229) */
} nsf_dims;

/* Parameter order = the reference state dict after remove_weight_norm (models.py:285-293):
 *   m_source.l_linear.{weight,bias}, noise_convs.i.{weight,bias} (i < num_upsamples),
 *   conv_pre.{weight,bias}, ups.i.{weight [Cin,Cout,k], bias},
 *   resblocks.n.convs1.j / convs2.j (ResBlock1) or convs.j (ResBlock2) {weight,bias},
 *   conv_post.{weight,bias}.  All device pointers, fp32. */
int nsf_num_params(const nsf_dims* dims);
/* dtype PD_DTYPE_F32: exact fp32 (parity path); PD_DTYPE_BF16: bf16 weights/activations on the
 * MFMA, fp32 accumulate, fp32 source module and epilogues. */
int nsf_create(const nsf_dims* dims, const float* const* params, int dtype, void* stream, nsf_model** out);
void nsf_destroy(nsf_model* m);
int nsf_hop(const nsf_model* m);   /* prod(upsample_rates) */
size_t nsf_workspace_size(const nsf_model* m, int B, int T);
/* NSF_OPT_SMALL_MAX: ResBlock convs with at most this many channels run on the LDS/VALU small-channel
 * kernel (default 16, measured; 0 = never).  Set before the first forward call. */
#define NSF_OPT_SMALL_MAX 0
/* NSF_OPT_WCONV: 1 (default) runs the bf16 ResBlock convs with 16..256 channels on the windowed
 * MFMA conv kernels (input window staged once in LDS for all taps), ahead of
 * NSF_OPT_SMALL_MAX; 0 = the implicit-GEMM engine / small kernel.  No effect on the fp32 path. */
#define NSF_OPT_WCONV 1
/* NSF_OPT_PAIR: 1 (default) runs each ResBlock1 conv pair c2(lrelu(c1(lrelu(x)))) + x with 32, 64 or 128
 * channels (16: NSF_OPT_PAIR16) as ONE windowed launch (the inner activation stays in LDS, x is read once); 0 = two
 * windowed launches with the inner activation through HBM in bf16.  Same roundings either way. */
#define NSF_OPT_PAIR 2
/* NSF_OPT_PAIR16: 1 (default) runs the 16-channel ResBlock1 pairs of the shipped shapes (taps 3/7/11,
 * dilation 1/3/5) the same way, on 16x16x32 MFMAs; 0 = two launches for them.  Needs NSF_OPT_PAIR. */
#define NSF_OPT_PAIR16 3
/* NSF_OPT_UPS_NC: 1 (default) lets the bf16 windowed upsample compute the noise conv of its stage itself when
 * the source kernel has at most 8 taps (the last three stages) instead of reading nsf_noise_conv's output;
 * 0 = always the separate noise conv.  Same fp32 operations in the same order. */
#define NSF_OPT_UPS_NC 4
/* NSF_OPT_RB16 (r06): 1 (default) runs each 16-channel ResBlock1 of the shipped shapes (taps 3/7/11, c1
 * dilations 1, 3, 5) as ONE launch that keeps the residual in registers across its three conv pairs and reads
 * x / writes the ResBlock sum once (32-tile windows, 4 waves); 2 = 64-tile windows of 8 waves; 0 = one
 * launch per pair (NSF_OPT_PAIR16).  Same roundings and MFMA order: bit-identical either way. */
#define NSF_OPT_RB16 5
/* NSF_OPT_RB32 / NSF_OPT_RB64 (r06): the same whole-ResBlock1 launch at 32 / 64 channels, for the kernel sizes
 * whose bit is set (1: taps 3, 2: taps 7, 4: taps 11); 0 = one launch per pair.  Bit-identical either way.
 * Defaults: RB32 1 (taps 3 only), RB64 0 (measured). */
#define NSF_OPT_RB32 6
#define NSF_OPT_RB64 7
/* NSF_OPT_C256 (r06): the 256-channel ResBlock convs' block shape -- 0: 4 waves and 128 output channels per
 * block (two blocks stage each row tile's window), 1 (default): 8 waves and all 256.  Bit-identical. */
#define NSF_OPT_C256 8
/* NSF_OPT_NC_MFMA (r06): 2 (default) runs the first two stages' source convs (K = 128 / 16, stride K / 2) on the
 * f32 MFMA (fmaf chains from the bias, k ascending: bit-identical), 1 only the K = 128 one, 0 = the fp32 VALU kernel. */
#define NSF_OPT_NC_MFMA 9
int nsf_set_option(nsf_model* m, int option, int value);

/* spec2wav_torch(mel, f0=f0) for a batch of independent utterances:
 *   mel [B,T,num_mels] time-major, scaled by mel_scale on load: 2.30259 turns the log10
 *   mel of spec2wav_torch into the natural-log mel the Generator takes (nsf_hifigan.py:50-53);
 *   1.0 is Generator.forward(c, f0) itself (models.py:265)
 *   f0  [B,T] Hz (0 = unvoiced)
 *   rand_ini [harmonic_num+1] (torch.rand(1,dim), models.py:139; element 0 ignored) and
 *   noise [B, T*hop, harmonic_num+1] (randn_like, models.py:182), or NULL -> Philox from seed
 *   wav [B, T*hop] output in [-1, 1]. */
int nsf_forward(const nsf_model* m, const float* mel, float mel_scale, const float* f0, const float* rand_ini,
                const float* noise, unsigned long long seed, const int* utt_ids, const int* lens, float* wav,
                int B, int T, void* workspace, size_t ws_bytes, void* stream);

/* ============================================================ condition encoder
 * SVS teacher condition -- replaces ProDiffTeacher.forward_condition
 * (modules/svs/prodiff_teacher.py:103-146): FastspeechEncoder (modules/fastspeech/
 * tts_modules.py:232-330: token + position embedding, enc_layers x EncSALayer with 2-head
 * self-attention and the k=9 conv FFN, final LayerNorm), mel2ph_to_dur (:223-229), the
 * mel2ph length-regulator gather and the pitch / speaker / gender / voicing / breath sums.
 */
typedef struct pd_cond pd_cond;

typedef struct {
  int vocab_size;            /* len(ph_encoder)                         prodiff_teacher.py:13 */
  int hidden_size;           /* H: 256 (handler/base_config.yaml:112), multiple of 64       */
  int enc_layers;            /* 4                                                            */
  int enc_ffn_kernel_size;   /* 9 (odd, <= 11)                                               */
  int num_heads;             /* 2; head dim H / num_heads in {64, 128, 256}                  */
  int num_spk;               /* spk_embed rows                                               */
  int num_langs;             /* lang_embed rows = len(hparams["languages"]) + 1              */
  int use_dur_embed, use_spk_id, use_gender_id, use_lang_id, use_voicing_embed, use_breath_embed;
  int rel_pos;               /* > 0: RelPositionalEncoding (tts_modules.py:299-300,324-325,
                                espnet_positional_embedding.py:89-115) instead of the sinusoid,
                                with a table of max(rel_pos, 5000) rows (< 0 rejected): the
                                reference's table starts at 5000 rows and extend_pe (:24-45)
                                keeps the longest input's length, which then sets the
                                reversed positions of every later, shorter batch         */
} pd_cond_dims;

/* Parameter order = the reference state-dict order (buffers and `diffusion.*` skipped), fp32:
 *   for l < enc_layers: encoder.layers.l.op.{layer_norm1.weight, layer_norm1.bias,
 *       self_attn.in_proj_weight [3H,H], self_attn.out_proj.weight [H,H], layer_norm2.weight,
 *       layer_norm2.bias, ffn.ffn_1.weight [4H,H,k], ffn.ffn_1.bias, ffn.ffn_2.weight [H,4H],
 *       ffn.ffn_2.bias},
 *   encoder.layer_norm.{weight,bias}, encoder.embed_tokens.weight [V,H],
 *   [dur_embed.{weight [H,1],bias}], [spk_embed.weight], [gender_embed.weight [2,H]],
 *   [lang_embed.weight], pitch_embed.{weight,bias}, [voicing_embed.{weight,bias}],
 *   [breath_embed.{weight,bias}]   ([...] present iff its use_* flag is set).
 * The reference's add_gender_embed looks gender ids up in lang_embed (prodiff_teacher.py:95);
 * that is reproduced, so use_gender_id requires use_lang_id. */
int pd_cond_num_params(const pd_cond_dims* dims);
int pd_cond_create(const pd_cond_dims* dims, const float* const* params, int dtype, void* stream,
                   pd_cond** out);
void pd_cond_destroy(pd_cond* h);
size_t pd_cond_workspace_size(const pd_cond* h, int B, int T_txt, int T_mel);

/* forward_condition's inputs, all device pointers (int64 = torch.long), NULL when absent:
 *   txt_tokens [B,T_txt] (0 = padding), mel2ph [B,T_mel] (0 = padding frame, else token
 *   index + 1, <= T_txt), f0 [B,T_mel] Hz, lang_seq [B,T_txt], spk_embed_id [B] or
 *   spk_mix_embed [B, spk_mix_frames (1 or T_mel), H], gender_embed_id [B] or
 *   gender_mix_embed [B, gender_mix_frames, H], voicing [B,T_mel], breath [B,T_mel].
 * Embedding ids outside their table (an IndexError in the reference) are clamped on the device
 * and mel2ph values above T_txt give zero frames, so a malformed input cannot fault the GPU. */
typedef struct {
  const long long* txt_tokens;
  const long long* mel2ph;
  const float* f0;
  const long long* lang_seq;
  const long long* spk_embed_id;
  const float* spk_mix_embed;
  int spk_mix_frames;
  const long long* gender_embed_id;
  const float* gender_mix_embed;
  int gender_mix_frames;
  const float* voicing;
  const float* breath;
  /* Ragged token batch (device, B ints, or NULL = every row T_txt tokens): row b's phonemes are its
   * first txt_lens[b] tokens.  The FFN conv (k = 9 over tokens) then reads zero past each row's own
   * end -- the zero padding of the row encoded alone (B = 1, T_txt = txt_lens[b]), the reference's
   * one-segment-at-a-time inference -- where it would otherwise read the padded rows' LayerNorm(0) =
   * beta (common_layers.py:668-669).  Attention and LayerNorm already mask padding tokens. */
  const int* txt_lens;
} pd_cond_inputs;

/* cond [B,T_mel,H] time-major (what pd_prodiff_sample / pd_reflow_sample take), and optionally
 * enc_out [B,T_txt,H] = the FastspeechEncoder output (tts_modules.py:310-317); either may be
 * NULL (not both); with cond NULL, mel2ph / T_mel still feed the duration embedding.  Every
 * utterance needs at least one non-padding token. */
int pd_cond_forward(const pd_cond* h, const pd_cond_inputs* in, float* cond, float* enc_out, int B,
                    int T_txt, int T_mel, void* workspace, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PRODIFF_HIP_H */
