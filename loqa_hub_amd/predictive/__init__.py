"""Predictive response subsystem: classifier, instant-ack engine, async skill
execution, status manager and the streaming-predictive bridge
(``internal/llm/{command_classifier,predictive_response,async_execution,
status_manager,streaming_predictive_bridge}.go``)."""
from .async_execution import AsyncExecutionPipeline
from .bridge import HYBRID, PREDICTIVE_ONLY, STREAMING_ONLY, StreamingPredictiveBridge
from .classifier import CommandClassifier
from .engine import PredictiveResponse, PredictiveResponseEngine
from .reliability import DeviceReliabilityTracker, extract_device_id
from .skill_adapter import NullSkillManager, SkillManagerAdapter
from .status_manager import StatusManager
from .types import CommandClassification, StatusUpdate

__all__ = [n for n in dir() if not n.startswith("_")]
