"""Shared loader for the NSF-HiFiGAN golden fixtures (tests/golden/nsf_*.npz)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["nsf_c64_r8822", "nsf_c32_r44_rb2", "nsf_c512_full"]


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    h = dict(num_mels=int(z["num_mels"]), upsample_initial_channel=int(z["upsample_initial_channel"]),
             upsample_rates=tuple(z["upsample_rates"].tolist()),
             upsample_kernel_sizes=tuple(z["upsample_kernel_sizes"].tolist()),
             resblock=str(int(z["resblock"])), resblock_kernel_sizes=tuple(z["resblock_kernel_sizes"].tolist()),
             resblock_dilation_sizes=tuple(tuple(d) for d in z["resblock_dilation_sizes"].tolist()),
             sampling_rate=int(z["sampling_rate"]))
    return h, {k: z[k] for k in ("mel", "f0", "rand_ini", "noise", "wav")}, int(z["seed"])
