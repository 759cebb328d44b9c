"""The bf16 parity bar, shared by every bf16 GPU test.

bf16 (C3's compute dtype) is judged against the fp32 reference/oracle with a
stated, looser bound (SURVEY §8(c) suggests rel-L2 <= 1e-2):

  relative L2  ||got - ref|| / ||ref||   <= REL_L2
  max relative max|got - ref| / max|ref| <= REL_MAX

bf16 keeps 8 significant bits (per-GEMM rounding ~4e-3 relative); the 20-layer
denoiser and the 12-layer LVC stacks compound it.  Every call prints its measured
errors ("BF16ERR ...") so the GPU test log records them (DESIGN.md §3 tabulates
them); the bars sit just above the largest measured value (r02, profiles/
r02_bf16_errors.txt):
  * sampler / denoiser / vocoder OUTPUTS (mel, waveform, WaveNet x0, NSF wav):
    measured <= 8.4e-3 rel-L2 and <= 1.41e-2 max-rel -> bars 1e-2 / 2e-2;
  * the FastDiff eps-network alone (fd_forward, an intermediate the sampler
    scales by beta/sqrt(1-alpha^2) before it reaches the waveform): measured
    <= 1.51e-2 rel-L2, <= 3.42e-2 max-rel -> bars EPS_REL_L2 / EPS_REL_MAX.
"""
import numpy as np

REL_L2 = 1e-2
REL_MAX = 2e-2
EPS_REL_L2 = 2e-2
EPS_REL_MAX = 4e-2


def bf16_errors(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    assert np.isfinite(got).all()
    rel = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    mx = float(np.abs(got - ref).max() / np.abs(ref).max())
    return rel, mx


def assert_bf16_close(got, ref, label="", rel_l2=REL_L2, rel_max=REL_MAX):
    rel, mx = bf16_errors(got, ref)
    print(f"BF16ERR {label} rel-L2={rel:.3e} max-rel={mx:.3e}", flush=True)
    assert rel <= rel_l2 and mx <= rel_max, f"{label}: rel-L2 {rel:.3e} (bar {rel_l2}), max-rel {mx:.3e} (bar {rel_max})"
