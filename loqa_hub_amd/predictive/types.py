"""Shared predictive-response types (``internal/llm/predictive_response.go:32-126``)."""
from __future__ import annotations

import time
from dataclasses import dataclass, field

# StatusType
STATUS_SUCCESS = "success"
STATUS_PROGRESS = "progress"
STATUS_ERROR = "error"
STATUS_CORRECTION = "correction"
STATUS_TIMEOUT = "timeout"

# UpdateStrategy
UPDATE_SILENT = "silent"
UPDATE_ERROR_ONLY = "error_only"
UPDATE_VERBOSE = "verbose"
UPDATE_PROGRESS = "progress"

# PredictiveType
PREDICTIVE_OPTIMISTIC = "optimistic"
PREDICTIVE_CAUTIOUS = "cautious"
PREDICTIVE_CONFIRM = "confirm"
PREDICTIVE_PROGRESS = "progress"


@dataclass
class StatusUpdate:
    type: str
    message: str
    success: bool
    execution_id: str
    timestamp: float = field(default_factory=time.time)
    error: str = ""

    def to_json(self) -> dict:
        from datetime import datetime, timezone
        from ..events import rfc3339
        d = {"type": self.type, "message": self.message, "success": self.success,
             "execution_id": self.execution_id,
             "timestamp": rfc3339(datetime.fromtimestamp(self.timestamp, timezone.utc))}
        if self.error:
            d["error"] = self.error
        return d


@dataclass
class CommandClassification:
    intent: str
    entities: dict[str, str]
    confidence: float
    device_reliability: float
    execution_time: float          # seconds (json: estimated_execution_time, ns)
    response_type: str
    update_strategy: str
    category: str = "general"
    operation: str = "control"
    target_id: str = "general_request"
    response: str = ""             # the parser's natural-language response

    def to_json(self) -> dict:
        return {"intent": self.intent, "entities": dict(self.entities),
                "confidence": self.confidence, "device_reliability": self.device_reliability,
                "estimated_execution_time": int(self.execution_time * 1e9),
                "response_type": self.response_type, "update_strategy": self.update_strategy}
