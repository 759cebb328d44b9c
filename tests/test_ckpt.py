"""Checkpoint layouts: the reference's training checkpoints load into
the GPU modules unchanged.

  * utils/ckpt_utils.py:8-68 -- newest model_ckpt_steps_<N>.ckpt, `model.` prefix stripping,
    nested {model_name: sd}, dotted model names, strict=False shape filtering, force;
  * FastDiff vocoder dir -- config.yaml + {'state_dict': {'model': weight-norm sd}}
    (component/vocoder/fastdiff.py:17-41, :92-115);
  * NSF-HiFiGAN -- config.json beside the file + {'generator': weight-norm sd}
    (modules/nsf_hifigan/models.py:21-36).
CPU tests check the loaded parameters; the `gpu` tests run the loaded modules against
the golden vectors (same weights, so the outputs must match the fixtures)."""
import json
import os

import numpy as np
import pytest
import torch
import yaml

from prodiff_amd import GaussianDiffusion, WaveNet, synth
from prodiff_amd.ckpt import get_all_ckpts, load_ckpt
from tests import golden_io as G
from tests import nsf_cases as NC


def _save(path, obj):
    torch.save(obj, path)
    return path


def _wn_sd(seed, dims=(80, 32, 4, 64)):
    return {k: torch.from_numpy(v) for k, v in synth.synth_params(synth.wavenet_param_shapes(*dims), seed).items()}


def test_get_all_ckpts_newest_first(tmp_path):
    for s in (100, 2000, 350):
        _save(tmp_path / f"model_ckpt_steps_{s}.ckpt", {"state_dict": {}})
    paths = get_all_ckpts(str(tmp_path))
    assert [os.path.basename(p) for p in paths] == [f"model_ckpt_steps_{s}.ckpt" for s in (2000, 350, 100)]
    assert len(get_all_ckpts(str(tmp_path), steps=350)) == 1


def test_load_ckpt_prefix_newest_and_file(tmp_path):
    for step, seed in ((100, 1), (2000, 2)):
        _save(tmp_path / f"model_ckpt_steps_{step}.ckpt",
              {"state_dict": {"model." + k: v for k, v in _wn_sd(seed).items()}, "global_step": step})
    net = WaveNet(80, 32, 4, 64, 2)
    load_ckpt(net, str(tmp_path), "model")
    for k, v in _wn_sd(2).items():
        assert torch.equal(net.state_dict()[k], v), k
    load_ckpt(net, str(tmp_path / "model_ckpt_steps_100.ckpt"), "model")
    for k, v in _wn_sd(1).items():
        assert torch.equal(net.state_dict()[k], v), k


def test_load_ckpt_nested_and_dotted_names(tmp_path):
    sd = _wn_sd(3)
    _save(tmp_path / "model_ckpt_steps_5.ckpt", {"state_dict": {"model": sd}})
    net = WaveNet(80, 32, 4, 64, 2)
    load_ckpt(net, str(tmp_path), "model")
    assert all(torch.equal(net.state_dict()[k], v) for k, v in sd.items())
    # {'model': {'diffusion.denoise_fn.*': ...}} loaded as 'model.diffusion'
    d2 = tmp_path / "d2"
    d2.mkdir()
    _save(d2 / "model_ckpt_steps_7.ckpt",
          {"state_dict": {"model": {"diffusion.denoise_fn." + k: v for k, v in _wn_sd(4).items()}}})
    gd = GaussianDiffusion(80, WaveNet(80, 32, 4, 64, 2), timesteps=4, max_beta=40.0)
    load_ckpt(gd, str(d2), "model.diffusion", strict=False)
    assert all(torch.equal(gd.denoise_fn.state_dict()[k], v) for k, v in _wn_sd(4).items())


def test_load_ckpt_strict_false_drops_mismatched_shapes(tmp_path, capsys):
    sd = _wn_sd(5)
    sd["output_projection.weight"] = torch.zeros(7, 64, 1)
    _save(tmp_path / "model_ckpt_steps_1.ckpt", {"state_dict": {"model." + k: v for k, v in sd.items()}})
    net = WaveNet(80, 32, 4, 64, 2)
    before = net.output_projection.weight.detach().clone()
    load_ckpt(net, str(tmp_path), "model", strict=False)
    assert "Unmatched keys" in capsys.readouterr().out
    assert torch.equal(net.output_projection.weight, before)
    assert torch.equal(net.input_projection.weight, sd["input_projection.weight"])
    with pytest.raises(RuntimeError):
        load_ckpt(net, str(tmp_path), "model", strict=True)


def test_load_ckpt_force_and_safe_loader(tmp_path, capsys):
    with pytest.raises(AssertionError):
        load_ckpt(WaveNet(80, 32, 4, 64, 2), str(tmp_path), "model")
    load_ckpt(WaveNet(80, 32, 4, 64, 2), str(tmp_path), "model", force=False)
    assert "ckpt not found" in capsys.readouterr().out
    # anything beyond tensors/containers is refused (weights_only=True), never unpickled
    _save(tmp_path / "model_ckpt_steps_1.ckpt", {"state_dict": {}, "obj": _Opaque()})
    with pytest.raises(Exception):
        load_ckpt(WaveNet(80, 32, 4, 64, 2), str(tmp_path), "model")


class _Opaque:
    pass


def test_load_ckpt_numpy_scalar_metadata(tmp_path):
    """A resumed reference training checkpoint stores checkpoint_callback_best as a numpy
    scalar (np.load(best_valid.npy)[0], utils/pl_utils.py:321,751; dumped by
    handler/train/handler.py:389-402): the weights-only loader accepts numpy scalars/dtypes."""
    sd = _wn_sd(6)
    _save(tmp_path / "model_ckpt_steps_9.ckpt",
          {"epoch": 3, "global_step": 9, "checkpoint_callback_best": np.float64(0.1234),
           "best_int": np.int64(7), "optimizer_states": [{}], "state_dict": {"model." + k: v for k, v in sd.items()}})
    net = WaveNet(80, 32, 4, 64, 2)
    load_ckpt(net, str(tmp_path), "model")
    assert all(torch.equal(net.state_dict()[k], v) for k, v in sd.items())


# ---------------------------------------------------------------- vocoder layouts
FASTDIFF_CONFIG = dict(audio_channels=1, inner_channels=32, cond_channels=80, upsample_ratios=[8, 8, 4],
                       lvc_layers_each_block=4, lvc_kernel_size=3, kpnet_hidden_channels=64, kpnet_conv_size=3,
                       dropout=0.0, diffusion_step_embed_dim_in=128, diffusion_step_embed_dim_mid=512,
                       diffusion_step_embed_dim_out=512, use_weight_norm=True, T=1000, beta_0=1e-6, beta_T=0.01,
                       noise_schedule="")


def fastdiff_dir(tmp_path, seed=31):
    with open(tmp_path / "config.yaml", "w") as f:
        yaml.safe_dump(FASTDIFF_CONFIG, f)
    sd = {k: torch.from_numpy(v) for k, v in G.fastdiff_params(seed).items()}
    _save(tmp_path / "model_ckpt_steps_500000.ckpt", {"state_dict": {"model": sd}})
    _save(tmp_path / "model_ckpt_steps_20.ckpt", {"state_dict": {"model": {}}})   # older, must not be picked
    return str(tmp_path)


def test_fastdiff_vocoder_dir_layout(tmp_path):
    from prodiff_amd.vocoder import FastDiff as FastDiffVocoder
    voc = FastDiffVocoder({"vocoder_ckpt": fastdiff_dir(tmp_path)}, device=torch.device("cpu"))
    p = G.fastdiff_params(31)
    got = voc.model.state_dict()
    for k in p:
        if k.endswith(".weight_v"):
            base = k[:-len("_v")]
            ref = synth.fold_weight_norm_np(p[base + "_g"], p[k])
            np.testing.assert_allclose(got[base].numpy(), ref, rtol=2e-6, atol=1e-7, err_msg=base)
        elif not k.endswith(".weight_g"):
            assert torch.equal(got[k], torch.from_numpy(p[k])), k
    assert len(voc.sched[3]) == 4   # reverse_step 4 -> the 4-iter schedule (fastdiff.py:62-73)


def nsf_weight_norm_sd(h, seed):
    """The checkpoint form of a synth generator: every conv (not m_source) as weight_g / weight_v."""
    p = synth.synth_params(synth.nsf_param_shapes(**h), seed)
    out = {}
    for k, v in p.items():
        if k.endswith(".weight") and not k.startswith("m_source"):
            g = np.sqrt((v.astype(np.float64) ** 2).sum(axis=tuple(range(1, v.ndim)), keepdims=True)).astype(np.float32)
            out[k[:-len("weight")] + "weight_g"] = torch.from_numpy(g)
            out[k[:-len("weight")] + "weight_v"] = torch.from_numpy(v)
        else:
            out[k] = torch.from_numpy(v)
    return out, p


def nsf_file(tmp_path, name):
    h, _, seed = NC.load(name)
    cfg = dict(h, resblock=h["resblock"], upsample_rates=list(h["upsample_rates"]),
               upsample_kernel_sizes=list(h["upsample_kernel_sizes"]),
               resblock_kernel_sizes=list(h["resblock_kernel_sizes"]),
               resblock_dilation_sizes=[list(d) for d in h["resblock_dilation_sizes"]],
               n_fft=2048, win_size=2048, hop_size=int(np.prod(h["upsample_rates"])))
    with open(tmp_path / "config.json", "w") as f:
        json.dump(cfg, f)
    sd, p = nsf_weight_norm_sd(h, seed)
    return _save(tmp_path / "model", {"generator": sd}), p


def test_nsf_checkpoint_layout(tmp_path):
    from prodiff_amd.nsf_hifigan import load_model
    path, p = nsf_file(tmp_path, "nsf_c64_r8822")
    g, h = load_model(path, device="cpu")
    got = g.state_dict()
    for k, v in p.items():
        np.testing.assert_allclose(got[k].numpy(), v, rtol=2e-6, atol=1e-7, err_msg=k)
    assert h.num_mels == 128 or h.num_mels > 0


# ---------------------------------------------------------------- GPU: loaded modules vs goldens
@pytest.mark.gpu
def test_teacher_from_checkpoint_matches_golden(tmp_path):
    from tests.test_gpu_cond import cuda_inputs
    from prodiff_amd.teacher import ProDiffTeacher
    hp, P, ins, d = G.cond_case("cond_small")
    rhp = dict(hp, audio_num_mel_bins=128, dropout=0.1, languages=["a", "b"], residual_layers=2,
               residual_channels=256, dilation_cycle_length=1, timesteps=4, timescale=1000, schedule_type="vpsde",
               max_beta=40.0, spec_min=[-12], spec_max=[0])
    src = ProDiffTeacher(int(d["vocab"]), rhp)
    src.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()}, strict=False)
    _save(tmp_path / "model_ckpt_steps_160000.ckpt",
          {"state_dict": {"model." + k: v for k, v in src.state_dict().items()}})
    t = ProDiffTeacher(int(d["vocab"]), rhp)
    load_ckpt(t, str(tmp_path), "model", strict=True)
    t = t.cuda()
    x = cuda_inputs(ins)
    cond = t.forward_condition(x.pop("txt_tokens"), x.pop("mel2ph"), x.pop("f0"), **x).cpu().numpy()
    assert np.abs(cond - d["cond"]).max() <= 1e-4


@pytest.mark.gpu
def test_fastdiff_vocoder_from_checkpoint_matches_golden(tmp_path):
    from prodiff_amd.vocoder import FastDiff as FastDiffVocoder
    voc = FastDiffVocoder({"vocoder_ckpt": fastdiff_dir(tmp_path)})
    d = G.load("fastdiff_sample_n4")
    t = lambda a: torch.from_numpy(a).cuda()
    wav = voc.spec2wav_torch(t(np.ascontiguousarray(d["c"].transpose(0, 2, 1))), x_T=t(d["x_T"]),
                             noise=t(d["noise"])).cpu().numpy()
    ref = d["wav"].reshape(wav.shape)
    assert np.abs(wav - ref).max() <= max(1e-4, 1e-5 * np.abs(ref).max())


@pytest.mark.gpu
def test_nsf_from_checkpoint_matches_golden(tmp_path):
    from prodiff_amd.nsf_hifigan import NsfHifiGAN
    path, _ = nsf_file(tmp_path, "nsf_c64_r8822")
    voc = NsfHifiGAN({"vocoder_ckpt": str(path)})
    _, io, _ = NC.load("nsf_c64_r8822")
    t = lambda a: torch.from_numpy(a).cuda()
    wav = voc.spec2wav_torch(t(io["mel"]), f0=t(io["f0"]), rand_ini=t(io["rand_ini"]), noise=t(io["noise"]))
    assert float(np.abs(wav.cpu().numpy() - io["wav"].reshape(-1)).max()) < 1e-4
