"""Helpers to load the committed golden vectors and regenerate their weights."""
import os

import numpy as np

from prodiff_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as d:
        return {k: d[k] for k in d.files}


def wavenet_params(dims, seed):
    M, H, L, C, _ = [int(v) for v in dims]
    return synth.synth_params(synth.wavenet_param_shapes(M, H, L, C), int(seed))


def fastdiff_params(seed):
    return synth.synth_params(synth.fastdiff_param_shapes(), int(seed))


PRODIFF_SEEDS = {"prodiff_t2_m80": (80, 21), "prodiff_t4_m80": (80, 22), "prodiff_t4_m128": (128, 23)}


def prodiff_params(name):
    M, seed = PRODIFF_SEEDS[name]
    return synth.synth_params(synth.wavenet_param_shapes(M, 256, 20, 256), seed)


def prodiff_buffers(d):
    return {k[4:]: v for k, v in d.items() if k.startswith("buf_")}


COND_INPUTS = ("lang_seq", "spk_embed_id", "spk_mix_embed", "gender_embed_id", "voicing", "breath")


def cond_case(name):
    """(hparams, params, inputs, golden) of a tests/golden/cond_*.npz fixture (gen_golden.gen_cond)."""
    d = load(name)
    over = {str(k): int(v) for k, v in zip(d["hp_keys"], d["hp_vals"])}
    hp = dict(synth.COND_DEFAULTS)
    hp.update(over)
    if int(d.get("grow", 0)):   # the reference's RelPositionalEncoding table had grown to this many rows
        hp["rel_pos_len"] = int(d["grow"])
    P = synth.synth_cond_params(synth.cond_param_shapes(int(d["vocab"]), **hp), int(d["param_seed"]))
    ins = {k: d[k] for k in ("txt_tokens", "mel2ph", "f0") + COND_INPUTS if k in d}
    if str(d["spk_mode"]) != "id":
        ins.pop("spk_embed_id")
    if not hp["use_voicing_embed"]:
        ins.pop("voicing", None)
    if not hp["use_breath_embed"]:
        ins.pop("breath", None)
    return hp, P, ins, d


COND_CASES = ("cond_small", "cond_handler", "cond_mix_gender", "cond_long", "cond_relpos", "cond_relpos_grown")
