"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU (numpy, float64) restatement of the reference FastDiff vocoder hot path.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg use it, as the checker.  Pinned against ``tests/golden/fastdiff_*.npz``
and ``schedules.npz`` (tests/test_oracle.py).

Follows:
  * step embedding   -- modules/FastDiff/module/util.py:404-429, FastDiff_model.py:7-8,85-87
  * DiffusionDBlock  -- modules/FastDiff/module/modules.py:116-138
  * LVC block        -- modules.py:141-218 (TimeAware_LVCBlock.forward)
  * LVC op           -- modules.py:220-253 (location_variable_convolution)
  * KernelPredictor  -- modules.py:257-343
  * network          -- FastDiff_model.py:74-102
  * weight-norm fold -- FastDiff_model.py:104-113 (torch.nn.utils.remove_weight_norm)
  * schedules        -- util.py:158-206 (alpha/sigma/steps), :362-401,
                        component/vocoder/fastdiff.py:44-73
  * sampler          -- util.py:207-232 (ddim=False)
"""
import math

import numpy as np

from oracle.oracle_prodiff import conv1d, linear, sigmoid

UPSAMPLE = (8, 8, 4)     # base.yaml:23 upsample_ratios
LAYERS = 4               # base.yaml:24 lvc_layers_each_block


def fold_weight_norm(sd):
    """Return a plain state dict: w = g * v / ||v||_{dims != 0}."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_g"):
            base = k[:-len(".weight_g")]
            vv = np.asarray(sd[base + ".weight_v"], np.float64)
            n = np.sqrt(np.sum(vv ** 2, axis=tuple(range(1, vv.ndim)), keepdims=True))
            out[base + ".weight"] = np.asarray(v, np.float64) * vv / n
        elif k.endswith(".weight_v"):
            continue
        else:
            out[k] = np.asarray(v, np.float64)
    return out


def lrelu(x, a):
    return np.where(x >= 0, x, a * x)


def swish(x):
    return x * sigmoid(x)


def step_embedding(steps, dim_in=128):
    """util.py:404-429; frequencies and s*f are float32 in the reference."""
    half = dim_in // 2
    e = np.float32(np.log(10000) / (half - 1))
    freqs = np.exp((np.arange(half, dtype=np.float32) * -e).astype(np.float32)).astype(np.float32)
    arg = (np.asarray(steps, np.float32).reshape(-1, 1) * freqs[None, :]).astype(np.float32)
    arg = arg.astype(np.float64)
    return np.concatenate([np.sin(arg), np.cos(arg)], axis=1)


def interp_nearest(x, size):
    """F.interpolate(mode='nearest') along the last axis."""
    L = x.shape[-1]
    scale = np.float32(L) / np.float32(size)
    idx = np.minimum(np.floor(np.arange(size, dtype=np.float32) * scale).astype(np.int64), L - 1)
    return x[..., idx]


def conv_transpose1d(x, w, b, stride, padding, output_padding):
    """x [B,Cin,T], w [Cin,Cout,K] (torch.nn.ConvTranspose1d)."""
    B, Cin, T = x.shape
    _, Cout, K = w.shape
    Lout = (T - 1) * stride - 2 * padding + K + output_padding
    full = np.zeros((B, Cout, (T - 1) * stride + K + output_padding))
    for k in range(K):
        full[:, :, k:k + (T - 1) * stride + 1:stride] += np.einsum("io,bit->bot", w[:, :, k], x)
    out = full[:, :, padding:padding + Lout]
    return out + b[None, :, None]


def dblock(p, q, x, factor):
    """modules.py:131-138."""
    size = x.shape[-1] // factor
    res = interp_nearest(conv1d(x, p[q + "residual_dense.weight"], p[q + "residual_dense.bias"]), size)
    x = interp_nearest(x, size)
    for j, dil in enumerate((1, 2, 4)):
        x = lrelu(x, 0.2)
        x = conv1d(x, p[q + f"conv.{j}.weight"], p[q + f"conv.{j}.bias"], dil, dil)
    return x + res


def kernel_predictor(p, q, c):
    """modules.py:320-343.  c [B,80,T'] -> kernels [B,4,32,64,3,T'], bias [B,4,64,T']."""
    B, _, T = c.shape
    h = lrelu(conv1d(c, p[q + "input_conv.0.weight"], p[q + "input_conv.0.bias"], 1, 2), 0.1)
    r = h
    for j in (1, 3, 6, 8, 11, 13):
        r = lrelu(conv1d(r, p[q + f"residual_conv.{j}.weight"], p[q + f"residual_conv.{j}.bias"], 1, 1), 0.1)
    h = h + r
    k = conv1d(h, p[q + "kernel_conv.weight"], p[q + "kernel_conv.bias"], 1, 1)
    bb = conv1d(h, p[q + "bias_conv.weight"], p[q + "bias_conv.bias"], 1, 1)
    return k.reshape(B, LAYERS, 32, 64, 3, T), bb.reshape(B, LAYERS, 64, T)


def lvc(x, kernel, bias, hop):
    """modules.py:220-253 with dilation 1 (the only value passed, :216).
    out[b,o,l*h+s] = bias[b,o,l] + sum_{i,k} K[b,i,o,k,l] * xpad[b,i,l*h+s+k]."""
    B, Cin, L = x.shape
    _, _, Cout, K, T = kernel.shape
    assert L == T * hop, "length of (x, kernel) is not matched"
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1)))
    out = np.empty((B, Cout, T, hop))
    for l in range(T):
        win = np.stack([xp[:, :, l * hop + k:l * hop + k + hop] for k in range(K)], axis=2)  # [B,Cin,K,hop]
        out[:, :, l, :] = np.einsum("biks,biok->bos", win, kernel[..., l]) + bias[:, :, l, None]
    return out.reshape(B, Cout, L)


def lvc_block(p, n, x, audio_down, c, emb):
    """modules.py:190-218."""
    q = f"lvc_blocks.{n}."
    r = UPSAMPLE[n]
    hop = int(np.prod(UPSAMPLE[:n + 1]))
    noise = linear(emb, p[q + "fc_t.weight"], p[q + "fc_t.bias"])[:, :, None]
    kernels, bias = kernel_predictor(p, q + "kernel_predictor.", c + noise)
    x = lrelu(x, 0.2)
    x = conv_transpose1d(x, p[q + "upsample.weight"], p[q + "upsample.bias"], r, r // 2 + r % 2, r % 2)
    for i in range(LAYERS):
        x = x + audio_down
        y = lrelu(x, 0.2)
        y = conv1d(y, p[q + f"convs.{i}.weight"], p[q + f"convs.{i}.bias"], 3 ** i, 3 ** i)
        y = lrelu(y, 0.2)
        y = lvc(y, kernels[:, i], bias[:, i], hop)
        x = x + sigmoid(y[:, :32]) * np.tanh(y[:, 32:])
    return x


def fastdiff_forward(p, audio, c, steps, capture=None):
    """FastDiff_model.py:74-102.  p: weight-norm-folded state dict.
    audio [B,1,L], c [B,80,T'], steps [B,1] -> eps [B,1,L]."""
    e = step_embedding(steps)
    e = swish(linear(e, p["fc_t1.weight"], p["fc_t1.bias"]))
    e = swish(linear(e, p["fc_t2.weight"], p["fc_t2.bias"]))
    a = conv1d(audio, p["first_audio_conv.weight"], p["first_audio_conv.bias"], 1, 3)
    downs = []
    for n, f in enumerate(UPSAMPLE[::-1]):
        downs.append(a)
        a = dblock(p, f"downsample.{n}.", a, f)
        if capture is not None:
            capture[f"downsample{n}"] = a
    x = a
    for n, ad in enumerate(reversed(downs)):
        x = lvc_block(p, n, x, ad, c, e)
        if capture is not None:
            capture[f"lvc{n}"] = x
    return conv1d(x, p["final_conv.0.weight"], p["final_conv.0.bias"], 1, 3)


# ---------------------------------------------------------------- schedules
def train_alpha(T=1000, beta_0=1e-6, beta_T=0.01):
    """fastdiff.py:44-51 -> util.py:362-387, in float32 like torch."""
    beta = np.linspace(beta_0, beta_T, T).astype(np.float32)
    a = (1 - beta).astype(np.float32)
    for t in range(1, T):
        a[t] = np.float32(a[t] * a[t - 1])
    return np.sqrt(a).astype(np.float32)


def infer_schedule(beta_infer, alpha_train):
    """util.py:181-206 -> beta, alpha, sigma, fractional steps (float32)."""
    b = np.asarray(beta_infer, np.float32)
    a = (1 - b).astype(np.float32)
    s = b.copy()
    for n in range(1, len(b)):
        a[n] = np.float32(a[n] * a[n - 1])
        s[n] = np.float32(s[n] * np.float32((1 - a[n - 1]) / (1 - a[n])))
    a, s = np.sqrt(a).astype(np.float32), np.sqrt(s).astype(np.float32)
    steps = []
    for n in range(len(b)):
        ai = a[n]
        if ai < alpha_train[-1]:
            steps.append(float(len(alpha_train) - 1))
            continue
        if ai > alpha_train[0]:
            steps.append(0.0)
            continue
        for t in range(len(alpha_train) - 1):
            if alpha_train[t + 1] <= ai <= alpha_train[t]:
                d = np.float32(np.float32(alpha_train[t] - ai) / np.float32(alpha_train[t] - alpha_train[t + 1]))
                steps.append(t + float(d))
                break
    return b, a, s, np.asarray(steps, np.float32)


def fastdiff_sample(p, c, x_T, noises, beta, alpha, sigma, steps):
    """util.py:207-232 (ddim=False) with the draws supplied.
    c [B,80,T'], x_T [B,1,L], noises[j] for n = N-1-j (n > 0)."""
    x = np.asarray(x_T, np.float64)
    N = len(steps)
    B = x.shape[0]
    for j, n in enumerate(range(N - 1, -1, -1)):
        eps = fastdiff_forward(p, x, c, np.full((B, 1), steps[n], np.float32))
        x = x - float(beta[n]) / math.sqrt(1 - float(alpha[n]) ** 2) * eps
        x = x / math.sqrt(1 - float(beta[n]))
        if n > 0:
            x = x + float(sigma[n]) * np.asarray(noises[j], np.float64)
    return x
