"""Transcriber interface + transcript post-processing (wake-word stripping and
heuristic confidence).

Behavioural spec: ``internal/llm/transcriber.go:11-29`` (interface/result),
``internal/llm/stt_client.go:401-458`` (postProcessTranscription: 10 wake-word
variants most-specific first, separator stripping, NeedsConfirmation when
confidence < 0.6 or only the wake word was spoken) and ``:461-513``
(estimateConfidence: base 0.8, -0.3 if < 3 chars, -0.2 for ``...``/``???``,
-0.3 per word with a character > 60 %, +0.1 for hey/loqa, clamp [0, 1]).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Protocol

import numpy as np

WAKE_WORD_PATTERNS = ["hey loqa", "hey loca", "hey luka", "hey luca", "hey logic", "hey local",
                      "loqa", "loca", "luka", "luca"]
CONFIRMATION_THRESHOLD = 0.6


@dataclass
class TranscriptionResult:
    text: str = ""
    confidence_estimate: float = 0.0
    wake_word_detected: bool = False
    wake_word_variant: str = ""
    needs_confirmation: bool = False


@dataclass
class PostProcessingResult:
    original_text: str
    cleaned_text: str
    wake_word_detected: bool
    wake_word_variant: str
    confidence_estimate: float
    needs_confirmation: bool


class Transcriber(Protocol):
    async def transcribe(self, audio: np.ndarray, sample_rate: int) -> str: ...

    async def transcribe_with_confidence(self, audio: np.ndarray,
                                         sample_rate: int) -> TranscriptionResult: ...

    async def close(self) -> None: ...


def estimate_confidence(text: str) -> float:
    if text == "":
        return 0.0
    c = 0.8
    # Go len() counts bytes
    if len(text.encode("utf-8")) < 3:
        c -= 0.3
    if "..." in text or "???" in text:
        c -= 0.2
    for word in text.split():
        wl = len(word.encode("utf-8"))
        if wl > 2:
            counts: dict[str, int] = {}
            for ch in word:
                counts[ch] = counts.get(ch, 0) + 1
            if any(n / wl > 0.6 for n in counts.values()):
                c -= 0.3
    low = text.lower()
    if "hey" in low or "loqa" in low:
        c += 0.1
    return min(1.0, max(0.0, c))


def post_process_transcription(raw: str) -> PostProcessingResult:
    res = PostProcessingResult(raw, raw, False, "", estimate_confidence(raw), False)
    low = raw.strip().lower()
    for pat in WAKE_WORD_PATTERNS:
        if low.startswith(pat):
            res.wake_word_detected = True
            res.wake_word_variant = pat
            # the reference slices the *untrimmed* text by the pattern length
            remaining = raw[len(pat):].strip()
            res.cleaned_text = remaining.lstrip(" ,.!?")
            break
    res.needs_confirmation = res.confidence_estimate < CONFIRMATION_THRESHOLD
    if res.wake_word_detected and res.cleaned_text.strip() == "":
        res.cleaned_text = ""
        res.needs_confirmation = True
    return res


def to_transcription_result(raw: str) -> TranscriptionResult:
    p = post_process_transcription(raw)
    return TranscriptionResult(p.cleaned_text, p.confidence_estimate, p.wake_word_detected,
                               p.wake_word_variant, p.needs_confirmation)
