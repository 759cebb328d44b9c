"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU (numpy, float64) restatement of the reference NSF-HiFiGAN generator
(SURVEY §8(f) row 2).  Only ``tests/`` uses it, as the checker.  Pinned against
``tests/golden/nsf_*.npz`` (made by running the reference, tests/golden/gen_golden_nsf.py).

Follows modules/nsf_hifigan/models.py:
  * ResBlock1 / ResBlock2   -- :36-97 (lrelu slope 0.1, get_padding = d*(k-1)/2, utils.py:12-13)
  * SineGen._f02sine        -- :130-166.  The reference also cumsums a 0/1 "shift" counter
                               derived from tmp_over_one (:143-160); it only ever adds integers
                               to the phase, so sin(2*pi*phase) is unchanged and the restatement
                               omits it (the golden vectors confirm it).
  * SineGen.forward         -- :168-185 (uv, noise_amp, randn draws)
  * SourceModuleHnNSF       -- :188-219 (Linear(harm+1 -> 1) + tanh)
  * Generator.forward       -- :222-283
and component/vocoder/nsf_hifigan.py:42-56 (spec2wav_torch: c = 2.30259 * mel^T).
"""
import numpy as np

from oracle.oracle_prodiff import conv1d

LRELU = 0.1


def lrelu(x, a=LRELU):
    return np.where(x >= 0, x, a * x)


def conv1d_strided(x, w, b, stride, padding):
    """torch.nn.Conv1d with stride (noise_convs, models.py:241-245)."""
    x = np.asarray(x, np.float64)
    w = np.asarray(w, np.float64)
    B, Cin, T = x.shape
    Cout, _, K = w.shape
    xp = np.pad(x, ((0, 0), (0, 0), (padding, padding)))
    Tout = (T + 2 * padding - K) // stride + 1
    out = np.zeros((B, Cout, Tout))
    for k in range(K):
        seg = xp[:, :, k:k + stride * (Tout - 1) + 1:stride]
        out += np.einsum("oi,bit->bot", w[:, :, k], seg)
    return out + np.asarray(b, np.float64)[None, :, None]


def conv_transpose1d(x, w, b, stride, padding):
    """torch.nn.ConvTranspose1d: w [Cin, Cout, K] (models.py:236-238)."""
    x = np.asarray(x, np.float64)
    w = np.asarray(w, np.float64)
    B, Cin, T = x.shape
    _, Cout, K = w.shape
    full = np.zeros((B, Cout, (T - 1) * stride + K))
    for k in range(K):
        full[:, :, k:k + stride * (T - 1) + 1:stride] += np.einsum("io,bit->bot", w[:, :, k], x)
    Tout = (T - 1) * stride - 2 * padding + K
    return full[:, :, padding:padding + Tout] + np.asarray(b, np.float64)[None, :, None]


def sine_source(f0, upp, sr, lin_w, lin_b, rand_ini, noise, sine_amp=0.1, noise_std=0.003):
    """SourceModuleHnNSF(f0, upp) -> har [B, L] (models.py:130-219).
    f0 [B,T] (Hz, 0 = unvoiced); rand_ini [dim] (element 0 is forced to 0, :140);
    noise [B, L, dim] the randn_like draw (:182)."""
    f0 = np.asarray(f0, np.float32)
    dim = lin_w.shape[-1]
    fn = f0[:, :, None] * np.arange(1, dim + 1, dtype=np.float32)[None, None, :]     # fp32 (:177)
    rad = np.fmod(fn / np.float32(sr), np.float32(1.0)).astype(np.float32)             # fp32 (:138)
    ini = np.asarray(rand_ini, np.float32).reshape(-1).copy()
    ini[0] = 0.0
    rad[:, 0, :] = rad[:, 0, :] + ini                                                # fp32 (:141)
    rad_up = np.repeat(rad.astype(np.float64), upp, axis=1)                         # nearest (:153)
    sines = np.sin(np.cumsum(rad_up, axis=1) * 2 * np.pi)                            # (:161)
    uv = np.repeat((f0 > 0).astype(np.float64), upp, axis=1)[:, :, None]
    noise_amp = uv * noise_std + (1 - uv) * sine_amp / 3
    sw = sines * sine_amp * uv + noise_amp * np.asarray(noise, np.float64)
    lw = np.asarray(lin_w, np.float64).reshape(-1)
    return np.tanh(sw @ lw + float(np.asarray(lin_b).reshape(-1)[0]))


def resblock(p, pre, x, k, dils, kind):
    if str(kind) == "1":
        for j, d in enumerate(dils):
            xt = conv1d(lrelu(x), p[f"{pre}.convs1.{j}.weight"], p[f"{pre}.convs1.{j}.bias"], d, d * (k - 1) // 2)
            xt = conv1d(lrelu(xt), p[f"{pre}.convs2.{j}.weight"], p[f"{pre}.convs2.{j}.bias"], 1, (k - 1) // 2)
            x = xt + x
    else:
        for j, d in enumerate(dils):
            x = conv1d(lrelu(x), p[f"{pre}.convs.{j}.weight"], p[f"{pre}.convs.{j}.bias"], d, d * (k - 1) // 2) + x
    return x


def generator_forward(p, h, c, f0, rand_ini, noise):
    """Generator.forward(c [B,M,T], f0 [B,T]) -> [B,1,T*upp] (models.py:265-283)."""
    rates, ks = h["upsample_rates"], h["upsample_kernel_sizes"]
    upp = int(np.prod(rates))
    har = sine_source(f0, upp, h["sampling_rate"], p["m_source.l_linear.weight"], p["m_source.l_linear.bias"],
                      rand_ini, noise)[:, None, :]
    x = conv1d(c, p["conv_pre.weight"], p["conv_pre.bias"], 1, 3)
    nk = len(h["resblock_kernel_sizes"])
    for i, (u, k) in enumerate(zip(rates, ks)):
        x = lrelu(x)
        x = conv_transpose1d(x, p[f"ups.{i}.weight"], p[f"ups.{i}.bias"], u, (k - u) // 2)
        if i + 1 < len(rates):
            sf = int(np.prod(rates[i + 1:]))
            xs_ = conv1d_strided(har, p[f"noise_convs.{i}.weight"], p[f"noise_convs.{i}.bias"], sf, sf // 2)
        else:
            xs_ = conv1d_strided(har, p[f"noise_convs.{i}.weight"], p[f"noise_convs.{i}.bias"], 1, 0)
        x = x + xs_
        xs = None
        for j, (rk, d) in enumerate(zip(h["resblock_kernel_sizes"], h["resblock_dilation_sizes"])):
            r = resblock(p, f"resblocks.{i * nk + j}", x, rk, d, h["resblock"])
            xs = r if xs is None else xs + r
        x = xs / nk
    x = lrelu(x, 0.01)                    # F.leaky_relu default slope (:280)
    x = conv1d(x, p["conv_post.weight"], p["conv_post.bias"], 1, 3)
    return np.tanh(x)


def spec2wav(p, h, mel, f0, rand_ini, noise):
    """component/vocoder/nsf_hifigan.py:50-56: mel [B,T,M] (log10) -> wav [B, T*upp]."""
    c = 2.30259 * np.transpose(np.asarray(mel, np.float64), (0, 2, 1))
    return generator_forward(p, h, c, f0, rand_ini, noise)[:, 0, :]
