"""Per-device success-ratio tracker (``predictive_response.go:129-142,367-419``):
score = successes / requests, 0.5 for unknown devices, pairwise-average latency."""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass


@dataclass
class DeviceStats:
    total_requests: int = 0
    successful_ops: int = 0
    failed_ops: int = 0
    avg_response_time: float = 0.0
    last_updated: float = 0.0
    reliability_score: float = 0.0


class DeviceReliabilityTracker:
    def __init__(self):
        self.devices: dict[str, DeviceStats] = {}
        self._lock = threading.Lock()

    def update_stats(self, device_id: str, success: bool, response_time: float) -> None:
        with self._lock:
            s = self.devices.setdefault(device_id, DeviceStats())
            s.total_requests += 1
            if success:
                s.successful_ops += 1
            else:
                s.failed_ops += 1
            s.avg_response_time = response_time if s.total_requests == 1 else \
                (s.avg_response_time + response_time) / 2
            s.reliability_score = s.successful_ops / s.total_requests
            s.last_updated = time.time()

    def get_reliability_score(self, device_id: str) -> float:
        with self._lock:
            s = self.devices.get(device_id)
            return s.reliability_score if s is not None else 0.5


def extract_device_id(entities: dict[str, str]) -> str:
    if "location" in entities:
        if "device" in entities:
            return f"{entities['location']}_{entities['device']}"
        return f"{entities['location']}_lights"
    return "unknown_device"
