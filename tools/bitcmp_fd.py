"""Bit-for-bit comparison of the bf16 FastDiff sampler across two library builds (GPU box).

A kernel change meant to keep every value (a reordered schedule, an interleave of independent MFMA
chains) is checked here against the library it replaces: both run the same seeded 4-step samples --
dense, ragged, and the C3 shape -- and the outputs must be equal bit for bit.

usage: python tools/bitcmp_fd.py <out.npz>                 (PRODIFF_HIP_LIB selects the library)
       python tools/bitcmp_fd.py --compare <a.npz> <b.npz>
"""
import sys

import numpy as np

CASES = [("dense_2x67", 2, 67, None), ("ragged_3x90", 3, 90, [90, 41, 7]), ("c3_8x861", 8, 861, None)]


def run(out):
    import torch
    sys.path.insert(0, ".")
    from prodiff_amd import FastDiff, synth
    from prodiff_amd.schedules import fastdiff_infer_params, fastdiff_reverse_schedule, fastdiff_train_alpha
    dev = torch.device("cuda:0")
    p = synth.synth_params(synth.fastdiff_param_shapes(), 31)
    b, a, s, st = fastdiff_infer_params(fastdiff_reverse_schedule(4), fastdiff_train_alpha())
    res = {}
    for name, B, Tc, lens in CASES:
        m = FastDiff()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
        m = m.to(dev).set_compute_dtype("bf16")
        mel = torch.from_numpy(synth.synth_inputs(80 + B, (B, Tc, 80), loc=-5.0, scale=2.0)).to(dev)
        for ps in (0, 1):
            m.set_options(lvc_ps=ps)
            o = m.sample(mel, b, a, s, st, lens=lens, seed=77).cpu().numpy()
            torch.cuda.synchronize()
            res[f"{name}_ps{ps}"] = o
            print(name, ps, o.shape, float(np.abs(o).max()), flush=True)
    np.savez(out, **res)


def compare(fa, fb):
    A, Bz = np.load(fa), np.load(fb)
    bad = 0
    for k in A.files:
        d = np.abs(A[k].astype(np.float64) - Bz[k].astype(np.float64)).max()
        same = np.array_equal(A[k], Bz[k])
        print(f"{k}: {'bit-identical' if same else 'DIFFERENT'} (max |d| {d:.3g})")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
