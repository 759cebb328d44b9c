"""Frame and phoneme counts of the reference's sample song, for the C5 real-length runs.

    python tests/golden/gen_ds_lengths.py  ->  tests/golden/ds_lengths.json

Reads /root/reference/samples/00_我多想说再见啊.ds (JSON data, 30 segments) and applies the
handler's duration -> frame rule (handler/infer/handler.py:236-241, timestep = hop / sr :40):
ph_acc = round(cumsum(ph_dur) / timestep + 0.5) in float32, mel_len = ph_acc[-1].  Only the
counts are committed (the fixture is data, not the .ds file)."""
import json
import os

import numpy as np
import torch

SRC = "/root/reference/samples/00_我多想说再见啊.ds"
HOP, SR = 512, 44100   # handler/base_config.yaml: hop_size, audio_sample_rate


def main():
    segs = json.load(open(SRC, encoding="utf-8"))
    timestep = HOP / SR
    frames, phones = [], []
    for s in segs:
        d = torch.from_numpy(np.array(s["ph_dur"].split(), np.float32))
        acc = torch.round(torch.cumsum(d, dim=0) / timestep + 0.5).long()
        frames.append(int(acc[-1]))
        phones.append(len(s["ph_seq"].split()))
    out = {"source": os.path.basename(SRC), "rule": "handler/infer/handler.py:236-241", "hop": HOP, "sr": SR,
           "frames": frames, "phonemes": phones}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ds_lengths.json")
    json.dump(out, open(path, "w"), indent=1)
    print(len(frames), "segments", min(frames), max(frames), sum(frames), "frames; phonemes", min(phones), max(phones))


if __name__ == "__main__":
    main()
