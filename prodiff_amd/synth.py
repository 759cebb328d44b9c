"""Seeded synthetic parameters and inputs shared by the golden-vector script,
the parity tests and ``bench.py``.

No pretrained checkpoint exists offline, so every parity
fixture is produced with weights drawn here.  The draw is keyed by
``(seed, crc32(parameter name))`` with numpy's PCG64 generator, which is
bit-stable across machines, so the GPU box regenerates exactly the weights the
reference saw in this container without any weight file travelling.

Parameter names and shapes follow the reference state dicts:
  * ``WaveNet``  -- modules/decoder/wavenet.py:74-99
  * ``FastDiff`` -- modules/FastDiff/module/FastDiff_model.py:13-72 (weight-norm
    form, ``weight_g``/``weight_v``, as the checkpoints store it:
    component/vocoder/fastdiff.py:41)
"""
from __future__ import annotations

import zlib
from collections import OrderedDict

import numpy as np


# --------------------------------------------------------------------------
# parameter name/shape tables
# --------------------------------------------------------------------------
def wavenet_param_shapes(in_dims=80, hidden_size=256, residual_layers=20,
                         residual_channels=256):
    """Ordered ``{state-dict key: shape}`` of reference ``WaveNet``."""
    C, H, M = residual_channels, hidden_size, in_dims
    s = OrderedDict()
    s["input_projection.weight"] = (C, M, 1)
    s["input_projection.bias"] = (C,)
    s["mlp.0.weight"] = (4 * C, C)
    s["mlp.0.bias"] = (4 * C,)
    s["mlp.2.weight"] = (C, 4 * C)
    s["mlp.2.bias"] = (C,)
    for l in range(residual_layers):
        p = f"residual_layers.{l}."
        s[p + "dilated_conv.weight"] = (2 * C, C, 3)
        s[p + "dilated_conv.bias"] = (2 * C,)
        s[p + "diffusion_projection.weight"] = (C, C)
        s[p + "diffusion_projection.bias"] = (C,)
        s[p + "conditioner_projection.weight"] = (2 * C, H, 1)
        s[p + "conditioner_projection.bias"] = (2 * C,)
        s[p + "output_projection.weight"] = (2 * C, C, 1)
        s[p + "output_projection.bias"] = (2 * C,)
    s["skip_projection.weight"] = (C, C, 1)
    s["skip_projection.bias"] = (C,)
    s["output_projection.weight"] = (M, C, 1)
    s["output_projection.bias"] = (M,)
    return s


KPNET_RES_IDX = (1, 3, 6, 8, 11, 13)   # Conv1d positions inside residual_conv (modules.py:297-313)


def _wn(s, name, shape):
    s[name + ".bias"] = (shape[0],)
    s[name + ".weight_g"] = (shape[0], 1, 1)
    s[name + ".weight_v"] = tuple(shape)


def fastdiff_param_shapes(audio_channels=1, inner_channels=32, cond_channels=80,
                          upsample_ratios=(8, 8, 4), lvc_layers_each_block=4,
                          lvc_kernel_size=3, kpnet_hidden_channels=64,
                          kpnet_conv_size=3, diffusion_step_embed_dim_in=128,
                          diffusion_step_embed_dim_mid=512,
                          diffusion_step_embed_dim_out=512, weight_norm=True):
    """Ordered ``{state-dict key: shape}`` of reference ``FastDiff``.

    With ``weight_norm`` every ``nn.Conv1d`` carries ``weight_g``/``weight_v``
    (FastDiff_model.py:115-122); ``ConvTranspose1d`` and ``Linear`` do not.
    """
    Ci, Cc, Hk = inner_channels, cond_channels, kpnet_hidden_channels
    Lyr, ks, kp = lvc_layers_each_block, lvc_kernel_size, kpnet_conv_size
    s = OrderedDict()

    def conv(name, shape):
        if weight_norm:
            _wn(s, name, shape)
        else:
            s[name + ".weight"] = tuple(shape)
            s[name + ".bias"] = (shape[0],)

    conv("first_audio_conv", (Ci, audio_channels, 7))
    s["fc_t1.weight"] = (diffusion_step_embed_dim_mid, diffusion_step_embed_dim_in)
    s["fc_t1.bias"] = (diffusion_step_embed_dim_mid,)
    s["fc_t2.weight"] = (diffusion_step_embed_dim_out, diffusion_step_embed_dim_mid)
    s["fc_t2.bias"] = (diffusion_step_embed_dim_out,)
    nb = len(upsample_ratios)
    for n in range(nb):
        r = upsample_ratios[n]
        p = f"lvc_blocks.{n}."
        s[p + "upsample.weight"] = (Ci, Ci, 2 * r)
        s[p + "upsample.bias"] = (Ci,)
        conv(p + "kernel_predictor.input_conv.0", (Hk, Cc, 5))
        for j in KPNET_RES_IDX:
            conv(p + f"kernel_predictor.residual_conv.{j}", (Hk, Hk, kp))
        conv(p + "kernel_predictor.kernel_conv", (Ci * 2 * Ci * ks * Lyr, Hk, kp))
        conv(p + "kernel_predictor.bias_conv", (2 * Ci * Lyr, Hk, kp))
        s[p + "fc_t.weight"] = (Cc, diffusion_step_embed_dim_out)
        s[p + "fc_t.bias"] = (Cc,)
        for i in range(Lyr):
            conv(p + f"convs.{i}", (Ci, Ci, ks))
    for n in range(nb):
        p = f"downsample.{n}."
        conv(p + "residual_dense", (Ci, Ci, 1))
        for j in range(3):
            conv(p + f"conv.{j}", (Ci, Ci, 3))
    conv("final_conv.0", (audio_channels, Ci, 7))
    return s


# --------------------------------------------------------------------------
# draws
# --------------------------------------------------------------------------
def _rng(seed, name):
    return np.random.default_rng([int(seed), zlib.crc32(name.encode())])


def _gain(name):
    # the LVC kernels multiply 96 taps each; keep them from saturating the gate
    if "kernel_conv" in name or "bias_conv" in name:
        return 0.3
    # a trained eps-network predicts ~N(0,1); keep the synthetic one there too
    if "final_conv" in name:
        return 0.2
    # NSF-HiFiGAN output conv feeds a tanh: keep it out of saturation
    if name.startswith("conv_post"):
        return 0.3
    # durations reach tens of frames; keep dur * w at the embedding scale
    if name.startswith("dur_embed"):
        return 0.1
    return 1.0


def synth_tensor(name, shape, seed):
    """Deterministic float32 draw for one parameter."""
    rng = _rng(seed, name)
    z = rng.standard_normal(size=shape, dtype=np.float32)
    if name.endswith(".bias"):
        return (0.02 * z).astype(np.float32)
    if name.endswith(".weight_g"):
        return (_gain(name) * (1.0 + 0.1 * z)).astype(np.float32)
    if name.endswith(".weight_v"):
        return z
    if "layer_norm" in name and name.endswith(".weight"):   # LayerNorm gamma ~ 1
        return (1.0 + 0.1 * z).astype(np.float32)
    if "upsample" in name or name.startswith("ups."):   # ConvTranspose1d [Cin, Cout, k]: 2 taps hit each output
        fan_in = shape[0] * 2
    else:
        fan_in = int(np.prod(shape[1:]))
    return (z * (_gain(name) / np.sqrt(fan_in))).astype(np.float32)


def synth_params(shapes, seed):
    return OrderedDict((k, synth_tensor(k, v, seed)) for k, v in shapes.items())


def fold_weight_norm_np(g, v):
    """w = g * v / ||v|| with the norm over every dim but 0 (torch.nn.utils.weight_norm, dim=0)."""
    n = np.sqrt(np.sum(v.astype(np.float64) ** 2, axis=tuple(range(1, v.ndim)), keepdims=True))
    return (g.astype(np.float64) * v / n).astype(np.float32)


def synth_inputs(seed, shape, kind="normal", loc=0.0, scale=1.0):
    rng = np.random.default_rng([int(seed), 0xC0FFEE])
    if kind == "uniform":
        return rng.random(size=shape, dtype=np.float32)
    return (loc + scale * rng.standard_normal(size=shape, dtype=np.float32)).astype(np.float32)


# NSF-HiFiGAN generator (modules/nsf_hifigan/models.py:208-265), plain (weight-norm
# removed) keys in state-dict order.  Default dims are the SVS vocoder's
# (handler/base_config.yaml:7-11: 128 mels, 44.1 kHz, hop 512 = 8*8*2*2*2).
NSF_DEFAULTS = dict(num_mels=128, upsample_initial_channel=512, upsample_rates=(8, 8, 2, 2, 2),
                    upsample_kernel_sizes=(16, 16, 4, 4, 4), resblock="1", resblock_kernel_sizes=(3, 7, 11),
                    resblock_dilation_sizes=((1, 3, 5), (1, 3, 5), (1, 3, 5)), sampling_rate=44100)


def nsf_param_shapes(num_mels=128, upsample_initial_channel=512, upsample_rates=(8, 8, 2, 2, 2),
                     upsample_kernel_sizes=(16, 16, 4, 4, 4), resblock="1", resblock_kernel_sizes=(3, 7, 11),
                     resblock_dilation_sizes=((1, 3, 5), (1, 3, 5), (1, 3, 5)), harmonic_num=8, **_):
    s = OrderedDict()
    s["m_source.l_linear.weight"] = (1, harmonic_num + 1)
    s["m_source.l_linear.bias"] = (1,)
    ch0 = upsample_initial_channel
    for i in range(len(upsample_rates)):
        c = ch0 // 2 ** (i + 1)
        if i + 1 < len(upsample_rates):
            sf = int(np.prod(upsample_rates[i + 1:]))
            s[f"noise_convs.{i}.weight"] = (c, 1, 2 * sf)
        else:
            s[f"noise_convs.{i}.weight"] = (c, 1, 1)
        s[f"noise_convs.{i}.bias"] = (c,)
    s["conv_pre.weight"] = (ch0, num_mels, 7)
    s["conv_pre.bias"] = (ch0,)
    for i, (u, k) in enumerate(zip(upsample_rates, upsample_kernel_sizes)):
        s[f"ups.{i}.weight"] = (ch0 // 2 ** i, ch0 // 2 ** (i + 1), k)
        s[f"ups.{i}.bias"] = (ch0 // 2 ** (i + 1),)
    n = 0
    for i in range(len(upsample_rates)):
        c = ch0 // 2 ** (i + 1)
        for k, d in zip(resblock_kernel_sizes, resblock_dilation_sizes):
            names = ([f"convs1.{j}" for j in range(len(d))] + [f"convs2.{j}" for j in range(len(d))]
                     if str(resblock) == "1" else [f"convs.{j}" for j in range(len(d))])
            for nm in names:
                s[f"resblocks.{n}.{nm}.weight"] = (c, c, k)
                s[f"resblocks.{n}.{nm}.bias"] = (c,)
            n += 1
    s["conv_post.weight"] = (1, ch0 // 2 ** len(upsample_rates), 7)
    s["conv_post.bias"] = (1,)
    return s


# --------------------------------------------------------------------------
# SVS teacher condition stage (modules/svs/prodiff_teacher.py:10-47, encoder
# modules/fastspeech/tts_modules.py:291-308, layers common_layers.py:625-648)
# --------------------------------------------------------------------------
COND_DEFAULTS = dict(hidden_size=256, enc_layers=4, enc_ffn_kernel_size=9, num_heads=2, num_spk=1, num_langs=3,
                     use_dur_embed=True, use_spk_id=True, use_gender_id=False, use_lang_id=True,
                     use_voicing_embed=True, use_breath_embed=True)


def cond_param_shapes(vocab_size, hidden_size=256, enc_layers=4, enc_ffn_kernel_size=9, num_spk=1, num_langs=3,
                      use_dur_embed=True, use_spk_id=True, use_gender_id=False, use_lang_id=True,
                      use_voicing_embed=True, use_breath_embed=True, **_):
    """Ordered ``{state-dict key: shape}`` of the teacher minus ``diffusion.*`` and buffers."""
    H, k = hidden_size, enc_ffn_kernel_size
    s = OrderedDict()
    for l in range(enc_layers):
        p = f"encoder.layers.{l}.op."
        s[p + "layer_norm1.weight"] = (H,)
        s[p + "layer_norm1.bias"] = (H,)
        s[p + "self_attn.in_proj_weight"] = (3 * H, H)
        s[p + "self_attn.out_proj.weight"] = (H, H)
        s[p + "layer_norm2.weight"] = (H,)
        s[p + "layer_norm2.bias"] = (H,)
        s[p + "ffn.ffn_1.weight"] = (4 * H, H, k)
        s[p + "ffn.ffn_1.bias"] = (4 * H,)
        s[p + "ffn.ffn_2.weight"] = (H, 4 * H)
        s[p + "ffn.ffn_2.bias"] = (H,)
    s["encoder.layer_norm.weight"] = (H,)
    s["encoder.layer_norm.bias"] = (H,)
    s["encoder.embed_tokens.weight"] = (vocab_size, H)
    if use_dur_embed:
        s["dur_embed.weight"] = (H, 1)
        s["dur_embed.bias"] = (H,)
    if use_spk_id:
        s["spk_embed.weight"] = (num_spk, H)
    if use_gender_id:
        s["gender_embed.weight"] = (2, H)
    if use_lang_id:
        s["lang_embed.weight"] = (num_langs, H)
    s["pitch_embed.weight"] = (H, 1)
    s["pitch_embed.bias"] = (H,)
    if use_voicing_embed:
        s["voicing_embed.weight"] = (H, 1)
        s["voicing_embed.bias"] = (H,)
    if use_breath_embed:
        s["breath_embed.weight"] = (H, 1)
        s["breath_embed.bias"] = (H,)
    return s


def synth_cond_params(shapes, seed):
    """synth_params + the padding rows Embedding(..., padding_idx=0) keeps at zero
    (common_layers.py:63-68: initialised to 0 and never updated)."""
    P = synth_params(shapes, seed)
    for k in ("encoder.embed_tokens.weight", "lang_embed.weight"):
        if k in P:
            P[k][0] = 0.0
    return P


def synth_cond_inputs(seed, lengths, vocab_size, num_spk=1, num_langs=3, max_dur=12, pad_tokens=0):
    """Ragged batch of phoneme sequences with durations: ``lengths[b]`` tokens (ids >= 1) then
    zero padding to max(lengths) + pad_tokens; mel2ph repeats token i+1 dur[i] times, then
    0-padding to the longest utterance (the binarizer's layout, tts_modules.py:135-171)."""
    rng = np.random.default_rng([int(seed), 0xC0D])
    B = len(lengths)
    Tt = max(lengths) + pad_tokens
    tok = np.zeros((B, Tt), np.int64)
    lang = np.zeros((B, Tt), np.int64)
    durs = []
    for b, n in enumerate(lengths):
        tok[b, :n] = rng.integers(1, vocab_size, n)
        lang[b, :n] = rng.integers(1, max(num_langs, 2), n)
        durs.append(rng.integers(1, max_dur + 1, n))
    Tm = max(int(d.sum()) for d in durs)
    mel2ph = np.zeros((B, Tm), np.int64)
    for b, d in enumerate(durs):
        mel2ph[b, :int(d.sum())] = np.repeat(np.arange(1, len(d) + 1), d)
    f0 = rng.uniform(80.0, 800.0, (B, Tm)).astype(np.float32)
    f0[rng.random((B, Tm)) < 0.15] = 0.0        # unvoiced frames
    voicing = rng.uniform(-1.5, 1.0, (B, Tm)).astype(np.float32)
    breath = rng.uniform(-1.5, 1.0, (B, Tm)).astype(np.float32)
    spk = rng.integers(0, num_spk, B).astype(np.int64)
    return dict(txt_tokens=tok, mel2ph=mel2ph, f0=f0, lang_seq=lang, spk_embed_id=spk,
                voicing=voicing, breath=breath)


def synth_svs_utterance(seed, frames, n_tokens, vocab_size, num_langs=3, hidden=256):
    """One SVS segment as the inference handler builds it (handler/infer/handler.py:220-262):
    n_tokens phonemes whose durations sum to exactly `frames` mel frames, f0 with unvoiced
    gaps, voicing / breath curves and a time-invariant speaker mix [1, H]."""
    rng = np.random.default_rng([int(seed), 0x5F5])
    cuts = np.sort(rng.choice(np.arange(1, frames), n_tokens - 1, replace=False))
    dur = np.diff(np.concatenate([[0], cuts, [frames]]))
    tok = rng.integers(1, vocab_size, n_tokens).astype(np.int64)
    lang = rng.integers(1, max(num_langs, 2), n_tokens).astype(np.int64)
    mel2ph = np.repeat(np.arange(1, n_tokens + 1), dur).astype(np.int64)
    f0 = rng.uniform(120.0, 700.0, frames).astype(np.float32)
    f0[rng.random(frames) < 0.1] = 0.0
    return dict(txt_tokens=tok, mel2ph=mel2ph, f0=f0, lang_seq=lang,
                spk_mix_embed=(0.3 * rng.standard_normal((1, hidden))).astype(np.float32),
                voicing=rng.uniform(-1.5, 1.0, frames).astype(np.float32),
                breath=rng.uniform(-1.5, 1.0, frames).astype(np.float32))
