"""VITS (vits-ljs) phrase batches on one MI355X, for rocprofv3 kernel traces and
PMC passes: 8-phrase batches through the TTS engine (graph replays after the
first call per bucket), then one eager batch for the per-kernel view.

    python scripts/exp/vits_prof.py [--iters 6] [--eager]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

PHRASES = ["Turning on the kitchen lights.", "Playing some jazz in the living room.",
           "Okay, dimming the bedroom lights to thirty percent.", "Done.",
           "The garage door is now closed.", "Good morning! It is sunny today.",
           "Locking the front door.", "Setting the thermostat to twenty one degrees."]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--eager", action="store_true", help="no graph replay")
    ap.add_argument("--phrases", type=int, default=8, help="phrases per batch (the served hub: 1-2)")
    a = ap.parse_args()
    phrases = (PHRASES * 4)[: a.phrases]
    import torch
    from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
    from loqa_hub_amd.models.configs import VITS_CONFIGS
    e = VitsTTSEngine(VITS_CONFIGS["vits-ljs"], "cuda", use_graphs=not a.eager)
    e.synthesize_batch(phrases)                      # capture / warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in range(a.iters):
        n += sum(o.size for o in e.synthesize_batch(phrases))
    dt = time.perf_counter() - t0
    print(json.dumps({"batches": a.iters, "phrases_per_batch": len(phrases),
                      "ms_per_batch": round(1e3 * dt / a.iters, 2),
                      "audio_s_per_wall_s": round(n / 22050 / dt, 1),
                      "host_launch_ms_per_batch": round(1e3 * e.stats["launch_s"] / e.stats["batches"], 3),
                      "graphs": not a.eager, "stats": e.stats}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
