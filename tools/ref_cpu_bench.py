"""Time the REFERENCE's own CPU path (SURVEY §8(d) CPU-baseline procedure).

Runs only where /root/reference exists (this container; the GPU box has no reference):

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_cpu_bench.py [--threads N] [--repeats 5]

Imports the reference modules read-only with the SURVEY §8(c) shims (lower-case
``modules.fastdiff`` alias for FastDiff_model.py:4-5; ``Tensor.cuda`` as identity
for the hard-coded ``.cuda()`` in util.py:68,214,424), loads the shared seeded
synthetic weights (prodiff_amd.synth) and times, fp32 under torch.no_grad():

  C3: ProDiff 2-iter (GaussianDiffusion + WaveNet 20x256, M=80, vpsde max_beta 40,
      prodiff.py:136-153) on cond [8,861,256], then FastDiff 4-iter
      (util.py:158-232 with the fastdiff.py:72-73 schedule) on the mel -> wav [8,1,220416]
  C2: ProDiff 2-iter alone, B=1, T=1000
  C5: the SVS path on one GPU's share of C5: ProDiffTeacher.forward(infer=True)
      (modules/svs/prodiff_teacher.py:148-168: FFT-encoder condition + 4-iter ProDiff, M=128)
      then the NSF-HiFiGAN Generator (modules/nsf_hifigan/models.py:222-283, 44.1 kHz, hop 512)
      on 8 segments x 861 frames (10 s each)
  PITCH: the pitch predictor's sampler (r06): PitchRectifiedFlow (reflow.py:86-144) over
      WaveNet(64, 256, 20, 256, dilation cycle 5) (pitch_predictor.py:40-55,
      handler/base_config.yaml:135-149), 20 Euler steps + denorm_spec, segments one at a time

``--configs C5`` re-times only the named configs and merges them into the JSON.

1 warm-up + median of N timed runs.  Writes profiles/r02_ref_cpu.json, which
bench.py reports as ``cpu_baseline`` (kind "reference").
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

from prodiff_amd import synth  # noqa: E402

torch.Tensor.cuda = lambda self, *a, **k: self          # shim (util.py:68,214,424)

from modules.decoder.wavenet import WaveNet            # noqa: E402
from modules.diffusion.prodiff import GaussianDiffusion  # noqa: E402
import modules.FastDiff                                # noqa: E402
import modules.FastDiff.module                         # noqa: E402
import modules.FastDiff.module.modules as fd_modules   # noqa: E402
import modules.FastDiff.module.util as fd_util         # noqa: E402
sys.modules["modules.fastdiff"] = modules.FastDiff
sys.modules["modules.fastdiff.module"] = modules.FastDiff.module
sys.modules["modules.fastdiff.module.modules"] = fd_modules
sys.modules["modules.fastdiff.module.util"] = fd_util
from modules.FastDiff.module.FastDiff_model import FastDiff  # noqa: E402
sys.modules.setdefault("chardet", __import__("types").ModuleType("chardet"))   # utils/__init__.py:6

HOP, SR = 256, 22050
SCHED4 = [3.2176e-04, 2.5743e-03, 2.5376e-02, 7.0414e-01]   # component/vocoder/fastdiff.py:72-73


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def build(seed=0):
    net = WaveNet(80, 256, 20, 256, 1)
    gd = GaussianDiffusion(out_dims=80, denoise_fn=net, timesteps=2, time_scale=1000, schedule_type="vpsde",
                           max_beta=40.0, spec_min=[-12], spec_max=[0]).eval()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in
                         synth.synth_params(synth.wavenet_param_shapes(80, 256, 20, 256), seed).items()})
    fd = FastDiff()
    fd.load_state_dict({k: torch.from_numpy(v) for k, v in
                        synth.synth_params(synth.fastdiff_param_shapes(), seed + 1).items()})
    fd.remove_weight_norm()
    dh = fd_util.compute_hyperparams_given_schedule(torch.linspace(1e-6, 0.01, 1000))
    return gd, fd.eval(), dh


def timed(fn, repeats):
    fn()                                   # warm-up
    ts = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_ref_cpu.json"))
    ap.add_argument("--configs", default="C3,C2,C5,PITCH")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    want = set(args.configs.split(","))
    res = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            res = json.load(f).get("configs", {})
    if "C5" in want:
        res["C5"] = bench_c5(args.repeats)
        print("C5", res["C5"], flush=True)
    if "PITCH" in want:
        res["PITCH"] = bench_pitch(args.repeats)
        print("PITCH", res["PITCH"], flush=True)
    if not want & {"C3", "C2"}:
        return write(args, res)
    gd, fd, dh = build()

    # C3: 8 x 10 s, ProDiff 2-iter + FastDiff 4-iter
    B, T = 8, 861
    cond = torch.from_numpy(synth.synth_inputs(0, (B, T, 256)))
    split = {}

    @torch.no_grad()
    def c3():
        t0 = time.perf_counter()
        mel = gd(cond, infer=True)                                   # [B,T,80]
        t1 = time.perf_counter()
        fd_util.sampling_given_noise_schedule(fd, (B, 1, T * HOP), dh, torch.FloatTensor(SCHED4),
                                              condition=mel.transpose(1, 2).contiguous())
        split.setdefault("prodiff", []).append(t1 - t0)
        split.setdefault("fastdiff", []).append(time.perf_counter() - t1)

    med, ts = timed(c3, args.repeats)
    audio = B * T * HOP / SR
    res["C3"] = {"mel_frames_per_s": round(B * T / med, 2), "seconds_median": round(med, 3), "repeats": args.repeats,
                 "seconds_all": [round(t, 3) for t in ts], "rtf": round(med / audio, 4),
                 "x_realtime": round(audio / med, 3),
                 "prodiff_s_median": round(float(np.median(split["prodiff"][1:])), 3),
                 "fastdiff_s_median": round(float(np.median(split["fastdiff"][1:])), 3),
                 "sample": f"reference modules, B={B} x {T} frames ({audio:.1f} s audio), ProDiff 2-iter + "
                           f"FastDiff 4-iter, fp32"}
    print("C3", res["C3"], flush=True)

    # C2: ProDiff 2-iter, B=1, T=1000
    cond2 = torch.from_numpy(synth.synth_inputs(0, (1, 1000, 256)))
    med2, ts2 = timed(torch.no_grad()(lambda: gd(cond2, infer=True)), args.repeats)
    res["C2"] = {"mel_frames_per_s": round(1000 / med2, 2), "seconds_median": round(med2, 4), "repeats": args.repeats,
                 "seconds_all": [round(t, 4) for t in ts2], "rtf": round(med2 / (1000 * 512 / 44100), 4),
                 "sample": "reference modules, ProDiff 2-iter, B=1 x 1000 frames, M=80, fp32, mel only"}
    print("C2", res["C2"], flush=True)
    write(args, res)


def bench_c5(repeats, B=2, T=861, tokens=120):
    """Segments one at a time (B=1), as the inference handler runs them (handler/infer/handler.py:
    373-388); the reference SineGen only takes B=1 (models.py:160-166 concatenates a [1,dim] draw)."""
    from modules.svs.prodiff_teacher import ProDiffTeacher
    from modules.nsf_hifigan.env import AttrDict
    from modules.nsf_hifigan.models import Generator
    from prodiff_amd.pipeline import SVS_TEACHER, SVS_VOCAB, TOKEN_KEYS
    hp = dict(SVS_TEACHER)
    t = ProDiffTeacher(SVS_VOCAB, hp).eval()
    cp = synth.synth_cond_params(synth.cond_param_shapes(SVS_VOCAB, num_langs=len(hp["languages"]) + 1,
                                                         **{k: v for k, v in hp.items() if k != "num_langs"}), 0)
    wn = synth.synth_params(synth.wavenet_param_shapes(128, 256, 20, 256), 1)
    sd = {k: torch.from_numpy(v) for k, v in cp.items()}
    sd.update({"diffusion.denoise_fn." + k: torch.from_numpy(v) for k, v in wn.items()})
    t.load_state_dict(sd, strict=False)
    h = AttrDict(dict(synth.NSF_DEFAULTS))
    g = Generator(h)
    g.remove_weight_norm()
    g.load_state_dict({k: torch.from_numpy(v) for k, v in
                       synth.synth_params(synth.nsf_param_shapes(**synth.NSF_DEFAULTS), 2).items()})
    g.eval()
    utts = [synth.synth_svs_utterance(100 + i, T, tokens, SVS_VOCAB) for i in range(B)]
    batches = [{k: torch.from_numpy(v)[None] for k, v in u.items()} for u in utts]
    split = {}

    @torch.no_grad()
    def c5():
        tt, tn = 0.0, 0.0
        for b in batches:
            t0 = time.perf_counter()
            mel = t(b["txt_tokens"], b["mel2ph"], b["f0"], lang_seq=b["lang_seq"],
                    spk_mix_embed=b["spk_mix_embed"], voicing=b["voicing"], breath=b["breath"], infer=True)
            t1 = time.perf_counter()
            g(mel.transpose(1, 2) * 2.30259, b["f0"])       # spec2wav_torch, nsf_hifigan.py:50-54
            tt += t1 - t0
            tn += time.perf_counter() - t1
        split.setdefault("teacher", []).append(tt)
        split.setdefault("nsf", []).append(tn)

    med, ts = timed(c5, repeats)
    audio = B * T * 512 / 44100
    return {"mel_frames_per_s": round(B * T / med, 2), "seconds_median": round(med, 3), "repeats": repeats,
            "seconds_all": [round(x, 3) for x in ts], "rtf": round(med / audio, 4), "x_realtime": round(audio / med, 3),
            "teacher_s_median": round(float(np.median(split["teacher"][1:])), 3),
            "nsf_s_median": round(float(np.median(split["nsf"][1:])), 3),
            "sample": f"reference modules, {B} segments one at a time (B=1) x {T} frames ({audio:.1f} s audio "
                      f"at 44.1 kHz), "
                      f"{tokens} phonemes each: ProDiffTeacher.forward(infer=True) (encoder condition + "
                      f"4-iter ProDiff, M=128) + NSF-HiFiGAN Generator, fp32"}


def bench_pitch(repeats, B=2, T=861):
    """The pitch predictor's diffusion sampler, one segment at a time (B=1, as the handler runs
    them): PitchRectifiedFlow.forward(cond, infer_step=20, infer=True) -> pitch [1, T]."""
    from modules.diffusion.reflow import PitchRectifiedFlow
    net = WaveNet(64, 256, 20, 256, 5)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in
                         synth.synth_params(synth.wavenet_param_shapes(64, 256, 20, 256), 0).items()})
    rf = PitchRectifiedFlow(repeat_bins=64, denoise_fn=net, time_scale=1000, sampling_algorithm="euler",
                            spec_min=-8.0, spec_max=8.0, clamp_min=-12.0, clamp_max=12.0).eval()
    conds = [torch.from_numpy(synth.synth_inputs(i, (1, T, 256))) for i in range(B)]

    @torch.no_grad()
    def run():
        for c in conds:
            rf(c, infer_step=20, infer=True)

    med, ts = timed(run, repeats)
    audio = B * T * 512 / 44100
    return {"mel_frames_per_s": round(B * T / med, 2), "seconds_median": round(med, 3), "repeats": repeats,
            "seconds_all": [round(x, 3) for x in ts], "rtf": round(med / audio, 4),
            "sample": f"reference modules, {B} segments one at a time (B=1) x {T} frames: PitchRectifiedFlow "
                      f"(20 Euler steps, WaveNet 20x256, M=64 repeat bins, dilation cycle 5) + denorm_spec, fp32"}


def write(args, res):
    out = {"host": f"{cpu_model()}, {os.cpu_count()} vCPUs (survey container, no GPU)",
           "threads": args.threads, "repeats": args.repeats, "torch": torch.__version__,
           "reference": REF, "script": "tools/ref_cpu_bench.py", "configs": res}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
