"""Synthetic relay traffic: multi-command utterances as PCM16 @ 16 kHz plus their
ground-truth transcript (used to teacher-force the random-init Whisper).

Audio is deterministic per (seed, index): a wake-word burst followed by
voiced-like segments (harmonic stacks with a syllable envelope and noise), ~0.32 s
per word, so RMS-based arbitration and the log-mel front end see speech-shaped
signal energy.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

DEVICES = ["lights", "music", "tv", "lamp", "fan"]
LOCATIONS = ["kitchen", "bedroom", "living room", "bathroom", "office", "garage"]
CLAUSES = [
    "turn on the {loc} {dev}", "turn off the {loc} {dev}", "turn on the {dev} in the {loc}",
    "turn off the {dev}", "dim the {loc} lights", "play music in the {loc}",
]
JOINERS = [" and ", " and then ", " then ", ", and ", " after that ", " also "]
WAKE = ["hey loqa", "loqa", "hey loqa,"]
# a long run (make_unique past ~300 one-command utterances per rank) draws from
# a wider pool once the base one is nearly used up: more rooms and devices and
# a closing word, same clause shapes
EXTRA_DEVICES = ["heater", "speaker", "radio", "ceiling fan"]
EXTRA_LOCATIONS = ["hallway", "dining room", "basement", "porch", "attic", "study"]
CLOSERS = ["", " please", " now", " thanks", " right now"]


@dataclass
class SyntheticUtterance:
    relay_id: str
    text: str           # full transcript (with wake word)
    n_commands: int
    pcm: np.ndarray     # int16
    wake_pcm: np.ndarray


def utterance_text(rng: np.random.Generator, n_commands: int, wide: bool = False) -> str:
    devs = DEVICES + EXTRA_DEVICES if wide else DEVICES
    locs = LOCATIONS + EXTRA_LOCATIONS if wide else LOCATIONS
    parts = []
    for _ in range(n_commands):
        c = CLAUSES[rng.integers(len(CLAUSES))]
        parts.append(c.format(loc=locs[rng.integers(len(locs))],
                              dev=devs[rng.integers(len(devs))]))
    s = parts[0]
    for p in parts[1:]:
        s += JOINERS[rng.integers(len(JOINERS))] + p
    if wide:
        s += CLOSERS[rng.integers(len(CLOSERS))]
    return WAKE[rng.integers(len(WAKE))] + " " + s


def speechlike(rng: np.random.Generator, n_words: int, sr: int = 16000, amp: float = 0.3) -> np.ndarray:
    out = []
    for _ in range(n_words):
        dur = rng.uniform(0.22, 0.42)
        n = int(dur * sr)
        t = np.arange(n) / sr
        f0 = rng.uniform(95, 220)
        sig = sum((0.6 / k) * np.sin(2 * np.pi * f0 * k * t + rng.uniform(0, 6.28)) for k in range(1, 6))
        env = np.sin(np.pi * np.linspace(0, 1, n)) ** 1.5
        sig = sig * env + 0.05 * rng.standard_normal(n)
        out.append(sig)
        out.append(0.01 * rng.standard_normal(int(rng.uniform(0.03, 0.09) * sr)))
    x = np.concatenate(out) if out else np.zeros(0)
    x = amp * x / (np.abs(x).max() + 1e-9)
    return x


def to_pcm16(x: np.ndarray) -> np.ndarray:
    return np.clip(np.round(x * 32767.0), -32768, 32767).astype(np.int16)


def make_utterance(seed: int, index: int, n_commands: int, relay_id: str | None = None,
                   amp: float = 0.3, wide: bool = False) -> SyntheticUtterance:
    rng = np.random.default_rng(seed * 100003 + index)
    text = utterance_text(rng, n_commands, wide)
    return _voice(rng, text, n_commands, relay_id or f"relay-{index}", amp)


def _voice(rng: np.random.Generator, text: str, n_commands: int, relay_id: str,
           amp: float = 0.3) -> SyntheticUtterance:
    """The audio of ``text``, drawn from ``rng`` right after the text was."""
    words = text.split()
    wake = to_pcm16(speechlike(rng, 2, amp=amp))
    body = to_pcm16(speechlike(rng, max(1, len(words) - 2), amp=amp))
    return SyntheticUtterance(relay_id, text, n_commands, np.concatenate([wake, body]), wake)


def make_batch(seed: int, n: int, commands_mix: list[int], offset: int = 0) -> list[SyntheticUtterance]:
    return [make_utterance(seed, offset + i, commands_mix[(offset + i) % len(commands_mix)])
            for i in range(n)]


def make_unique(seed: int, counts: list[int], offset: int = 0,
                seen: set[str] | None = None, max_tries: int = 64) -> list[SyntheticUtterance]:
    """Utterances with ``counts[i]`` commands each, no two of which (here or in
    ``seen``) share a transcript: every LLM prompt is then distinct, so the
    prefix cache can only reuse the template text before the transcript, as
    with real traffic (a cycled set of utterances would let whole prompts hit
    the cache). The base pool holds ~320 one-command transcripts; once draws
    from it keep colliding, the utterance comes from the wider pool
    (``utterance_text(wide=True)``), so a long run never runs out."""
    seen = set() if seen is None else seen
    out = []
    for i, nc in enumerate(counts):
        for t in range(2 * max_tries):
            # the text alone first (cheap); the audio only for the accepted draw,
            # from the same generator (as make_utterance draws it)
            rng = np.random.default_rng((seed + 7919 * t) * 100003 + offset + i)
            text = utterance_text(rng, nc, wide=t >= max_tries)
            if text not in seen:
                break
        else:
            raise RuntimeError("could not draw a distinct utterance")
        seen.add(text)
        out.append(_voice(rng, text, nc, f"relay-{offset + i}"))
    return out


@dataclass
class LongUtterance:
    relay_id: str
    text: str                 # full transcript
    window_texts: list        # transcript per 30 s window (teacher forcing)
    n_commands: int
    pcm: np.ndarray
    last_command_start_s: float


def make_long_utterance(seed: int, n_commands: int = 3, seconds: float = 45.0,
                        relay_id: str = "relay-long", sr: int = 16000) -> LongUtterance:
    """A long-form utterance: the wake word and the first
    commands, a long pause (low-level noise), then the LAST command after the
    30 s mark, padded to ``seconds``. Each word's samples are known, so every
    word is assigned to the 30 s window it starts in (``window_texts``)."""
    rng = np.random.default_rng(seed * 7907 + 11)
    text = utterance_text(rng, n_commands)
    words = text.split()
    # the last command: from the last joiner on (e.g. "and then turn off ...")
    last = max(text.rfind(j.strip() + " ") for j in JOINERS if j.strip())
    n_last = len(text[last:].split())
    head, tail = words[:-n_last], words[-n_last:]
    segs, starts = [], []
    pos = 0
    for w in head:
        a = to_pcm16(speechlike(rng, 1))
        starts.append(pos)
        segs.append(a)
        pos += len(a)
    gap = int(31.5 * sr) - pos
    if gap > 0:
        segs.append(to_pcm16(0.003 * rng.standard_normal(gap)))
        pos += gap
    t_last = pos / sr
    for w in tail:
        a = to_pcm16(speechlike(rng, 1))
        starts.append(pos)
        segs.append(a)
        pos += len(a)
    if pos < int(seconds * sr):
        segs.append(to_pcm16(0.003 * rng.standard_normal(int(seconds * sr) - pos)))
    pcm = np.concatenate(segs)
    n_win = -(-len(pcm) // (30 * sr))
    win = [[] for _ in range(n_win)]
    for w, st in zip(words, starts):
        win[st // (30 * sr)].append(w)
    return LongUtterance(relay_id, text, [" ".join(x) for x in win], n_commands, pcm, t_last)
