"""prodiff_amd -- MI355X-native ProDiff mel denoiser/sampler and FastDiff vocoder.

Drop-in replacements for the reference hot path (see DESIGN.md / INTEGRATION.md):
  * prodiff_amd.prodiff.WaveNet            <- modules/decoder/wavenet.py:WaveNet
  * prodiff_amd.prodiff.GaussianDiffusion  <- modules/diffusion/prodiff.py:GaussianDiffusion
  * prodiff_amd.fastdiff.FastDiff          <- modules/FastDiff/module/FastDiff_model.py:FastDiff
  * prodiff_amd.fastdiff.sampling_given_noise_schedule <- modules/FastDiff/module/util.py
  * prodiff_amd.vocoder.FastDiff (registered vocoder) <- component/vocoder/fastdiff.py
  * prodiff_amd.reflow.RectifiedFlow / PitchRectifiedFlow <- modules/diffusion/reflow.py
  * prodiff_amd.teacher.ProDiffTeacher (forward_condition on the GPU)
        <- modules/svs/prodiff_teacher.py:ProDiffTeacher
  * prodiff_amd.nsf_hifigan.Generator / NsfHifiGAN (registered vocoder)
        <- modules/nsf_hifigan/models.py, component/vocoder/nsf_hifigan.py
All compute runs in libprodiff_hip.so (hand-written gfx950 HIP kernels).
"""
from .prodiff import GaussianDiffusion, WaveNet  # noqa: F401
from .fastdiff import FastDiff, sampling_given_noise_schedule  # noqa: F401
from .reflow import PitchRectifiedFlow, RectifiedFlow  # noqa: F401
from .nsf_hifigan import Generator as NsfGenerator, NsfHifiGAN  # noqa: F401
from .teacher import ProDiffTeacher  # noqa: F401

__all__ = ["WaveNet", "GaussianDiffusion", "FastDiff", "sampling_given_noise_schedule", "RectifiedFlow",
           "PitchRectifiedFlow", "NsfGenerator", "NsfHifiGAN", "ProDiffTeacher"]
