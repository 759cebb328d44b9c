"""Golden vectors for the NSF-HiFiGAN generator, made by running
the REFERENCE ``modules/nsf_hifigan/models.py`` Generator in this container:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_nsf.py

Weights come from ``prodiff_amd.synth`` (plain, weight-norm-removed keys), so only
inputs, the two random draws and the output are stored.  The draws are
``torch.rand(1, dim)`` (models.py:139) then ``torch.randn_like`` (:182) from the
default CPU generator: they are replayed from the same seed and recorded.
The input follows ``spec2wav_torch`` (component/vocoder/nsf_hifigan.py:50-56):
c = 2.30259 * mel^T.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")

from prodiff_amd import synth  # noqa: E402
from modules.nsf_hifigan.env import AttrDict  # noqa: E402
from modules.nsf_hifigan.models import Generator  # noqa: E402

CASES = {
    # The reference SineGen is batch-1 only (models.py:162-163 concatenates a [1,1,dim] zero row).
    # small channels, hop 256 (8*8*2*2), the SVS kernels/resblocks
    "nsf_c64_r8822": dict(synth.NSF_DEFAULTS, upsample_initial_channel=64, upsample_rates=(8, 8, 2, 2),
                          upsample_kernel_sizes=(16, 16, 4, 4), B=1, T=8, seed=41),
    # ResBlock2, two upsamples
    "nsf_c32_r44_rb2": dict(synth.NSF_DEFAULTS, upsample_initial_channel=32, upsample_rates=(4, 4),
                            upsample_kernel_sizes=(8, 8), resblock="2", resblock_kernel_sizes=(3, 5),
                            resblock_dilation_sizes=((1, 3), (2, 6)), sampling_rate=22050, B=1, T=7, seed=42),
    # the full SVS vocoder dims (512 channels, hop 512), short input
    "nsf_c512_full": dict(synth.NSF_DEFAULTS, B=1, T=2, seed=43),
}


def run(name, cfg):
    B, T, seed = cfg.pop("B"), cfg.pop("T"), cfg.pop("seed")
    h = AttrDict(num_mels=cfg["num_mels"], upsample_initial_channel=cfg["upsample_initial_channel"],
                 upsample_rates=list(cfg["upsample_rates"]), upsample_kernel_sizes=list(cfg["upsample_kernel_sizes"]),
                 resblock=cfg["resblock"], resblock_kernel_sizes=list(cfg["resblock_kernel_sizes"]),
                 resblock_dilation_sizes=[list(d) for d in cfg["resblock_dilation_sizes"]],
                 sampling_rate=cfg["sampling_rate"])
    g = Generator(h)
    g.remove_weight_norm()
    p = synth.synth_params(synth.nsf_param_shapes(**cfg), seed)
    g.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()}, strict=True)
    g.eval()
    mel = synth.synth_inputs(seed, (B, T, cfg["num_mels"]), loc=-2.0, scale=1.0)
    rng = np.random.default_rng(seed)
    f0 = rng.uniform(80.0, 600.0, size=(B, T)).astype(np.float32)
    f0[:, 1] = 0.0                                     # an unvoiced frame
    upp = int(np.prod(cfg["upsample_rates"]))
    torch.manual_seed(seed)
    with torch.no_grad():
        c = torch.from_numpy(mel).transpose(2, 1) * 2.30259
        wav = g(c, torch.from_numpy(f0)).view(B, -1).numpy()
    torch.manual_seed(seed)
    rand_ini = torch.rand(1, 9).numpy()[0]
    noise = torch.randn(B, T * upp, 9).numpy()
    cfgs = {k: np.asarray(v, dtype=object if k == "resblock_dilation_sizes" else None) for k, v in cfg.items()}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), mel=mel, f0=f0, rand_ini=rand_ini, noise=noise,
                        wav=wav.astype(np.float32), seed=np.int64(seed),
                        num_mels=cfg["num_mels"], upsample_initial_channel=cfg["upsample_initial_channel"],
                        upsample_rates=np.asarray(cfg["upsample_rates"]),
                        upsample_kernel_sizes=np.asarray(cfg["upsample_kernel_sizes"]),
                        resblock=np.int64(int(cfg["resblock"])),
                        resblock_kernel_sizes=np.asarray(cfg["resblock_kernel_sizes"]),
                        resblock_dilation_sizes=np.asarray(cfg["resblock_dilation_sizes"]),
                        sampling_rate=np.int64(cfg["sampling_rate"]))
    del cfgs
    print(name, wav.shape, float(np.abs(wav).max()))


if __name__ == "__main__":
    torch.set_num_threads(8)
    for n, c in CASES.items():
        run(n, dict(c))
