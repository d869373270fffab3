"""Streaming parse + progressive TTS subsystem (``internal/llm/streaming_*.go``)."""
from .audio_pipeline import AudioChunk, PipelineContext, StreamingAudioPipeline
from .chan import Chan, ChannelClosed
from .components import StreamingComponents
from .interrupt import StreamingInterruptHandler
from .metrics import StreamingMetricsCollector
from .parser import (GPUStreamingBackend, OllamaStreamingBackend, PhraseBuffer,
                     StreamingCommandParser, StreamingMetrics, StreamingResult)

__all__ = [n for n in dir() if not n.startswith("_")]
