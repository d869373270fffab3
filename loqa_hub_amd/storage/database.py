"""SQLite database (``internal/storage/database.go``): parent dir created with
mode 0750, pragmas (WAL, synchronous=NORMAL, cache_size=10000, temp_store=memory,
mmap 256 MiB, foreign_keys, busy_timeout 5 s), schema + migrations at open,
``vacuum`` / ``checkpoint(TRUNCATE)`` / ``stats``; plus the privacy retention
sweep (``LOQA_DATA_RETENTION`` / ``LOQA_AUTO_CLEANUP``) that the reference only
validates.

One connection guarded by a lock (sqlite3 objects are not thread-safe); the
async API wraps calls with ``asyncio.to_thread`` where used from the loop.
"""
from __future__ import annotations

import logging
import os
import sqlite3
import threading
from datetime import datetime, timedelta, timezone

from ..utils.security import sanitize_log_input
from . import schema

log = logging.getLogger("loqa.storage")

PRAGMAS = [
    "PRAGMA journal_mode = WAL",
    "PRAGMA synchronous = NORMAL",
    "PRAGMA cache_size = 10000",
    "PRAGMA temp_store = memory",
    "PRAGMA mmap_size = 268435456",
    "PRAGMA foreign_keys = ON",
    "PRAGMA busy_timeout = 5000",
]


def default_db_path() -> str:
    return os.environ.get("DB_PATH") or "./data/loqa-hub.db"


class Database:
    def __init__(self, path: str = ""):
        self.path = path or default_db_path()
        if self.path != ":memory:":
            d = os.path.dirname(self.path)
            if d and d != ".":
                os.makedirs(d, mode=0o750, exist_ok=True)
        self.conn = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None,
                                    detect_types=0)
        self.lock = threading.RLock()
        self.ops = 0
        try:
            for p in PRAGMAS:
                self.conn.execute(p)
            self._migrate()
        except Exception:
            self.conn.close()
            raise
        log.info("database connected: %s", sanitize_log_input(self.path))

    def _migrate(self) -> None:
        with self.lock:
            cols = [r[1] for r in self.conn.execute("PRAGMA table_info(voice_events)")]
            if cols and "audio_hash" in cols:
                self.conn.execute("BEGIN")
                for stmt in schema.MIGRATION_001:
                    self.conn.execute(stmt)
                self.conn.execute("COMMIT")
                log.info("applied migration 001_remove_audio_hash")
            self.conn.execute(schema.VOICE_EVENTS_DDL)
            for ix in schema.INDEXES:
                self.conn.execute(ix)
            self.conn.execute(f"PRAGMA user_version = {schema.SCHEMA_VERSION}")

    def execute(self, sql: str, args=()) -> sqlite3.Cursor:
        with self.lock:
            self.ops += 1
            return self.conn.execute(sql, args)

    def query(self, sql: str, args=()) -> list[tuple]:
        with self.lock:
            self.ops += 1
            return self.conn.execute(sql, args).fetchall()

    def ping(self) -> None:
        self.query("SELECT 1")

    def vacuum(self) -> None:
        self.execute("VACUUM")

    def checkpoint(self) -> None:
        self.execute("PRAGMA wal_checkpoint(TRUNCATE)")

    def stats(self) -> dict:
        return {"path": self.path, "operations": self.ops,
                "page_count": self.query("PRAGMA page_count")[0][0],
                "journal_mode": self.query("PRAGMA journal_mode")[0][0]}

    def cleanup_older_than(self, retention_s: float) -> int:
        """Delete voice events older than the retention window; returns rows removed."""
        cutoff = datetime.now(timezone.utc) - timedelta(seconds=retention_s)
        from .voice_events_store import encode_time
        cur = self.execute("DELETE FROM voice_events WHERE timestamp < ?", (encode_time(cutoff),))
        return cur.rowcount

    def close(self) -> None:
        with self.lock:
            self.conn.close()
        log.info("closing database connection: %s", sanitize_log_input(self.path))
