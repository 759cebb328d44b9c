"""Diagnostic: FastDiff bf16 forward error vs the oracle under LVC mode switches."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_one(env):
    code = r'''
import sys, numpy as np, torch
sys.path.insert(0, "%s")
from oracle import oracle_fastdiff as OF
from prodiff_amd import FastDiff, synth
from tests import golden_io as G
p = G.fastdiff_params(31)
for B, Tc in [(1, 1), (1, 5), (3, 5), (1, 2)]:
    m = FastDiff(); m.load_state_dict({k: torch.from_numpy(v) for k, v in p.items()})
    m = m.to("cuda:0").set_compute_dtype("bf16")
    audio = synth.synth_inputs(B + 50 * Tc, (B, 1, Tc * 256))
    c = synth.synth_inputs(B + 50 * Tc + 1, (B, 80, Tc), loc=-5.0, scale=2.0)
    st = np.full((B, 1), 23.4676, np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    eps = m((t(audio), t(c), t(st))).cpu().numpy().astype(np.float64)
    ref = OF.fastdiff_forward(OF.fold_weight_norm(p), audio, c, st)
    d = eps - ref
    per_b = [float(np.linalg.norm(d[i]) / np.linalg.norm(ref[i])) for i in range(B)]
    print(B, Tc, "rel", round(float(np.linalg.norm(d) / np.linalg.norm(ref)), 5), "per-utt", [round(x, 5) for x in per_b],
          "worst t", int(np.abs(d).reshape(B, -1).max(0).argmax()))
''' % ROOT
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=300)
    print(env, "\n", r.stdout, r.stderr[-2000:] if r.returncode else "")


for env in [{"PRODIFF_LVC_SUB": "0"}, {"PRODIFF_LVC_SUB": "1"}, {"PRODIFF_LVC_SUB": "1", "PRODIFF_LVC_FUSE": "0"},
            {"PRODIFF_LVC_TS": "0"}]:
    run_one(env)
