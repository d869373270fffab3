"""CRUD/list/count over ``voice_events`` (``internal/storage/voice_events_store.go``).

* ``insert`` validates the event first (:43-80);
* ``get_by_uuid`` raises ``NotFound("voice event not found")`` (:83-94, :277);
* ``list``/``count`` share one query builder: filters relay_id / intent /
  success / start-end time, whitelisted sort column + ASC/DESC (default
  ``timestamp DESC``), LIMIT/OFFSET (:193-247); count wraps the list query
  (:127-143);
* ``delete`` raises NotFound when no row matched (:155-172).

The sort whitelist accepts ``processing_time`` like the reference but maps it
to the real column ``processing_time_ms`` (the reference would emit an invalid
ORDER BY for it).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from datetime import datetime, timezone

from ..events import VoiceEvent
from ..utils.security import sanitize_log_input
from .database import Database
from .schema import COLUMNS

log = logging.getLogger("loqa.storage")

_SORT = {"timestamp": "timestamp", "confidence": "confidence", "processing_time": "processing_time_ms",
         "processing_time_ms": "processing_time_ms", "uuid": "uuid", "relay_id": "relay_id",
         "intent": "intent", "success": "success", "audio_duration": "audio_duration",
         "sample_rate": "sample_rate"}


class NotFound(LookupError):
    pass


def encode_time(dt: datetime) -> str:
    """UTC, fixed width -> lexicographic order == time order."""
    return dt.astimezone(timezone.utc).strftime("%Y-%m-%d %H:%M:%S.%f+00:00")


def decode_time(s) -> datetime:
    if isinstance(s, datetime):
        return s
    s = str(s).strip()
    for fmt in ("%Y-%m-%d %H:%M:%S.%f%z", "%Y-%m-%d %H:%M:%S%z", "%Y-%m-%dT%H:%M:%S.%f%z",
                "%Y-%m-%dT%H:%M:%S%z", "%Y-%m-%d %H:%M:%S"):
        try:
            dt = datetime.strptime(s.replace("Z", "+0000"), fmt)
            return dt if dt.tzinfo else dt.replace(tzinfo=timezone.utc)
        except ValueError:
            continue
    # Go driver format may carry nanoseconds and a zone name suffix
    head = s.split(" m=")[0]
    if "." in head:
        a, b = head.split(".", 1)
        digits = "".join(ch for ch in b if ch.isdigit())
        rest = b[len(digits):].strip().split(" ")[0]
        return decode_time(f"{a}.{digits[:6]}{rest}")
    raise ValueError(f"unparseable timestamp {s!r}")


def validate_sort_by(sort_by: str) -> str:
    return _SORT.get(sort_by, "timestamp") if sort_by else "timestamp"


def validate_sort_order(order: str) -> str:
    return order if order in ("ASC", "DESC") else "DESC"


@dataclass
class ListOptions:
    relay_id: str = ""
    intent: str = ""
    success: bool | None = None
    start_time: datetime | None = None
    end_time: datetime | None = None
    limit: int = 0
    offset: int = 0
    sort_by: str = ""
    sort_order: str = ""


class VoiceEventsStore:
    def __init__(self, db: Database):
        self.db = db

    def insert(self, ev: VoiceEvent) -> None:
        try:
            ev.is_valid()
        except ValueError as e:
            raise ValueError(f"invalid voice event: {e}") from e
        self.db.execute(
            f"INSERT INTO voice_events ({', '.join(COLUMNS)}) VALUES ({', '.join('?' * len(COLUMNS))})",
            (ev.uuid, ev.request_id, ev.relay_id, encode_time(ev.timestamp), ev.audio_duration,
             ev.sample_rate, ev.wake_word_detected, ev.transcription, ev.intent, ev.entities_json(),
             ev.confidence, ev.response_text, ev.processing_time_ms, ev.success, ev.error_message))
        log.info("stored voice event: %s (relay: %s, intent: %s)", sanitize_log_input(ev.uuid),
                 sanitize_log_input(ev.relay_id), sanitize_log_input(ev.intent))

    def get_by_uuid(self, uuid: str) -> VoiceEvent:
        rows = self.db.query(f"SELECT {', '.join(COLUMNS)} FROM voice_events WHERE uuid = ?", (uuid,))
        if not rows:
            raise NotFound("voice event not found")
        return self._scan(rows[0])

    def build_list_query(self, o: ListOptions) -> tuple[str, list]:
        q = f"SELECT {', '.join(COLUMNS)} FROM voice_events WHERE 1=1"
        args: list = []
        if o.relay_id:
            q += " AND relay_id = ?"
            args.append(o.relay_id)
        if o.intent:
            q += " AND intent = ?"
            args.append(o.intent)
        if o.success is not None:
            q += " AND success = ?"
            args.append(bool(o.success))
        if o.start_time is not None:
            q += " AND timestamp >= ?"
            args.append(encode_time(o.start_time))
        if o.end_time is not None:
            q += " AND timestamp <= ?"
            args.append(encode_time(o.end_time))
        q += f" ORDER BY {validate_sort_by(o.sort_by)} {validate_sort_order(o.sort_order)}"
        if o.limit > 0:
            q += " LIMIT ?"
            args.append(o.limit)
            if o.offset > 0:
                q += " OFFSET ?"
                args.append(o.offset)
        return q, args

    def list(self, o: ListOptions) -> list[VoiceEvent]:
        q, args = self.build_list_query(o)
        return [self._scan(r) for r in self.db.query(q, args)]

    def count(self, o: ListOptions) -> int:
        o2 = ListOptions(**{**vars(o), "limit": 0, "offset": 0})
        q, args = self.build_list_query(o2)
        return int(self.db.query(f"SELECT COUNT(*) FROM ({q}) as filtered", args)[0][0])

    def get_recent_by_relay(self, relay_id: str, limit: int) -> list[VoiceEvent]:
        return self.list(ListOptions(relay_id=relay_id, limit=limit))

    def delete(self, uuid: str) -> None:
        cur = self.db.execute("DELETE FROM voice_events WHERE uuid = ?", (uuid,))
        if cur.rowcount == 0:
            raise NotFound(f"voice event not found: {uuid}")

    @staticmethod
    def _scan(r: tuple) -> VoiceEvent:
        ev = VoiceEvent(uuid=r[0], request_id=r[1], relay_id=r[2], timestamp=decode_time(r[3]),
                        audio_duration=float(r[4]), sample_rate=int(r[5]),
                        wake_word_detected=bool(r[6]), transcription=r[7], intent=r[8],
                        confidence=float(r[10]), response_text=r[11], processing_time_ms=int(r[12]),
                        success=bool(r[13]), error_message=r[14] or "")
        ev.set_entities_from_json(r[9])
        return ev
