"""MMS-TTS-shaped VITS (transformers' VitsConfig defaults, random weights,
16 kHz, stochastic duration predictor) through our checkpoint loader + HIP
engine vs transformers' own VitsModel on the same GPU (fp32 eager, the way a
Hugging Face user runs it): ms per phrase batch.

    python scripts/exp/vits_mms_bench.py [--iters 10]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from transformers import VitsConfig, VitsModel as HFVits
    from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = HFVits(VitsConfig()).eval()
    d = tempfile.mkdtemp()
    m.save_pretrained(d, safe_serialization=True)
    vocab = {c: i for i, c in enumerate("_ '-abcdefghijklmnopqrstuvwxyz0123456")}
    with open(os.path.join(d, "vocab.json"), "w") as f:
        json.dump(vocab, f)
    eng = VitsTTSEngine(None, dev, checkpoint=d)
    caps = eng.warmup_graphs()
    print(json.dumps({"warmup_captures": caps}), flush=True)
    phrase = "turning on the kitchen lights now"
    from loqa_hub_amd.models.vits import text_to_ids
    m = m.to(dev)
    for B in (1, 2, 8):
        texts = [phrase] * B
        eng.synthesize_batch(texts)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            out = eng.synthesize_batch(texts)
        ours = (time.perf_counter() - t0) / a.iters * 1e3
        ids = torch.tensor([text_to_ids(phrase, 0, vocab)] * B, device=dev)
        with torch.no_grad():
            m(input_ids=ids)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                wav = m(input_ids=ids).waveform
            torch.cuda.synchronize()
            hf = (time.perf_counter() - t0) / a.iters * 1e3
        print(json.dumps({"phrases": B, "ours_ms": round(ours, 2), "transformers_fp32_ms": round(hf, 2),
                          "ours_audio_s": round(len(out[0]) / 16000, 2),
                          "hf_audio_s": round(wav.shape[-1] / 16000, 2)}), flush=True)


if __name__ == "__main__":
    main()
