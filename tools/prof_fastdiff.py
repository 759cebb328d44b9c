"""Profiling driver: C3-size FastDiff sampler calls (bf16) for rocprofv3 runs.

    rocprofv3 --kernel-trace --stats -d gpurun_out/p -- python tools/prof_fastdiff.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from prodiff_amd.pipeline import Synthesizer  # noqa: E402


def main():
    dtype = os.environ.get("DTYPE", "bf16")
    reps = int(os.environ.get("REPS", "2"))
    B, T = 8, 861
    dev = torch.device("cuda:0")
    syn = Synthesizer.synthetic(dev, seed=0, dtype=dtype)
    mel = torch.from_numpy(np.random.default_rng(0).normal(-5, 2, (B, T, 80)).astype(np.float32)).to(dev)
    for i in range(reps):
        wav = syn.vocoder.spec2wav_torch(mel, seed=i)
    torch.cuda.synchronize()
    print("ok", float(wav.abs().mean()))


if __name__ == "__main__":
    main()
