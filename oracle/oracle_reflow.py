"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU (numpy, float64) restatement of the reference rectified-flow sampler with the
WaveNet velocity field, used by ``tests/`` as the checker.  Nothing in
``prodiff_amd`` imports this module.

Pinned against ``tests/golden/reflow_*.npz``, produced by running the reference
itself (tests/golden/gen_golden.py, tests/test_oracle.py).

Follows:
  * RectifiedFlow.inference       -- modules/diffusion/reflow.py:86-101
  * sample_euler / rk2 / rk4 / rk5 -- reflow.py:48-84
  * denorm_spec                   -- reflow.py:106-107 (RectifiedFlow),
                                     :138-144 (PitchRectifiedFlow: mean over bins, clamp)
  * velocity_fn                   -- the WaveNet denoiser (oracle_prodiff.wavenet_forward)
"""
import numpy as np

from oracle.oracle_prodiff import wavenet_forward

ALGORITHMS = ("euler", "rk2", "rk4", "rk5")


def stage_times(infer_step, algorithm, time_scale):
    """The float32 step values the reference hands the WaveNet, in evaluation order.

    reflow.py:89-98: dt = 1/max(1, S) (Python float), dts = float32 tensor [dt],
    t = i * dts (float32); a stage at t + c*dt is `t + c*dt` with the Python-float
    offset rounded to float32, then `time_scale * (...)` in float32."""
    S = int(infer_step)
    dt = 1.0 / max(1, S)
    f = np.float32
    offs = {"euler": [None], "rk2": [None, 0.5], "rk4": [None, 0.5, 0.5, 1.0],
            "rk5": [None, 0.25, 0.25, 0.5, 0.75, 1.0]}[algorithm]
    out = []
    for i in range(S):
        t = f(f(i) * f(dt))
        for c in offs:
            tt = t if c is None else f(t + f(c * dt))
            out.append(f(f(time_scale) * tt))
    return np.array(out, np.float32), dt


def reflow_sample(p, cond, x_T, infer_step=20, algorithm="euler", time_scale=1000,
                  residual_layers=20, dilation_cycle=1):
    """reflow.py:86-101 with the initial draw supplied.
    cond [B,T,H] (the teacher's condition before the transpose at :33);
    x_T [B,1,M,T] (torch.randn at :88).  Returns x [B,T,M] (before denorm_spec)."""
    condT = np.transpose(cond, (0, 2, 1))
    x = np.asarray(x_T, np.float64)
    B = x.shape[0]
    times, dt = stage_times(infer_step, algorithm, time_scale)
    it = iter(times)

    def v(xx):
        return wavenet_forward(p, xx, np.full((B,), next(it), np.float32), condT, residual_layers, dilation_cycle)

    for _ in range(int(infer_step)):
        if algorithm == "euler":
            x = x + v(x) * dt
        elif algorithm == "rk2":
            k1 = v(x)
            k2 = v(x + 0.5 * k1 * dt)
            x = x + k2 * dt
        elif algorithm == "rk4":
            k1 = v(x)
            k2 = v(x + 0.5 * k1 * dt)
            k3 = v(x + 0.5 * k2 * dt)
            k4 = v(x + k3 * dt)
            x = x + (k1 + 2 * k2 + 2 * k3 + k4) * dt / 6
        elif algorithm == "rk5":
            k1 = v(x)
            k2 = v(x + 0.25 * k1 * dt)
            k3 = v(x + 0.125 * (k2 + k1) * dt)
            k4 = v(x + 0.5 * (-k2 + 2 * k3) * dt)
            k5 = v(x + 0.0625 * (3 * k1 + 9 * k4) * dt)
            k6 = v(x + (-3 * k1 + 2 * k2 + 12 * k3 - 12 * k4 + 8 * k5) * dt / 7)
            x = x + (7 * k1 + 32 * k3 + 12 * k4 + 32 * k5 + 7 * k6) * dt / 90
        else:
            raise ValueError(algorithm)
    return np.transpose(x[:, 0], (0, 2, 1))


def denorm_spec(x, spec_min, spec_max):
    """reflow.py:106-107: (x + 1) / 2 * (max - min) + min, min/max broadcast over bins."""
    smin = np.asarray(spec_min, np.float64).reshape(-1)
    smax = np.asarray(spec_max, np.float64).reshape(-1)
    return (x + 1) / 2 * (smax - smin) + smin


def pitch_denorm(x, spec_min, spec_max, clamp_min, clamp_max):
    """reflow.py:138-144 (PitchRectifiedFlow): mean over the repeat bins, clamp."""
    return np.clip(denorm_spec(x, spec_min, spec_max).mean(axis=-1), clamp_min, clamp_max)
