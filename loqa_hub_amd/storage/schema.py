"""SQLite schema of the voice-event store.

Column set, defaults, CHECK constraints and indexes are those of the
reference's ``internal/storage/schema.sql:4-46`` (so a database file written by
either implementation is readable by the other). The reference's
``migrations/001_remove_audio_hash.sql`` is never embedded or executed there
(SURVEY §3.7 #7); here migrations are versioned through ``PRAGMA user_version``
and applied idempotently - 001 (drop ``audio_hash``) only runs when an old
table still has that column.
"""

SCHEMA_VERSION = 1

VOICE_EVENTS_DDL = """
CREATE TABLE IF NOT EXISTS voice_events (
    uuid               TEXT     PRIMARY KEY NOT NULL,
    request_id         TEXT     NOT NULL,
    relay_id           TEXT     NOT NULL,
    timestamp          DATETIME NOT NULL DEFAULT CURRENT_TIMESTAMP,
    audio_duration     REAL     NOT NULL DEFAULT 0.0,
    sample_rate        INTEGER  NOT NULL DEFAULT 16000,
    wake_word_detected BOOLEAN  NOT NULL DEFAULT FALSE,
    transcription      TEXT     NOT NULL DEFAULT '',
    intent             TEXT     NOT NULL DEFAULT 'unknown',
    entities           TEXT     NOT NULL DEFAULT '{}',
    confidence         REAL     NOT NULL DEFAULT 0.0,
    response_text      TEXT     NOT NULL DEFAULT '',
    processing_time_ms INTEGER  NOT NULL DEFAULT 0,
    success            BOOLEAN  NOT NULL DEFAULT TRUE,
    error_message      TEXT     DEFAULT NULL,
    created_at         DATETIME NOT NULL DEFAULT CURRENT_TIMESTAMP,
    CONSTRAINT chk_confidence      CHECK (confidence >= 0.0 AND confidence <= 1.0),
    CONSTRAINT chk_processing_time CHECK (processing_time_ms >= 0),
    CONSTRAINT chk_audio_duration  CHECK (audio_duration >= 0.0)
)"""

INDEXES = [
    "CREATE INDEX IF NOT EXISTS idx_voice_events_timestamp ON voice_events(timestamp DESC)",
    "CREATE INDEX IF NOT EXISTS idx_voice_events_relay_id ON voice_events(relay_id)",
    "CREATE INDEX IF NOT EXISTS idx_voice_events_intent ON voice_events(intent)",
    "CREATE INDEX IF NOT EXISTS idx_voice_events_success ON voice_events(success)",
    "CREATE INDEX IF NOT EXISTS idx_voice_events_created_at ON voice_events(created_at DESC)",
    "CREATE INDEX IF NOT EXISTS idx_voice_events_relay_timestamp ON voice_events(relay_id, timestamp DESC)",
    "CREATE INDEX IF NOT EXISTS idx_voice_events_intent_confidence ON voice_events(intent, confidence DESC)",
]

COLUMNS = ["uuid", "request_id", "relay_id", "timestamp", "audio_duration", "sample_rate",
           "wake_word_detected", "transcription", "intent", "entities", "confidence",
           "response_text", "processing_time_ms", "success", "error_message"]

# migration 001: rebuild the table without the legacy audio_hash column
MIGRATION_001 = [
    "DROP INDEX IF EXISTS idx_voice_events_audio_hash",
    VOICE_EVENTS_DDL.replace("voice_events (", "voice_events_new (", 1),
    "INSERT INTO voice_events_new (" + ", ".join(COLUMNS + ["created_at"]) + ") SELECT "
    + ", ".join(COLUMNS + ["created_at"]) + " FROM voice_events",
    "DROP TABLE voice_events",
    "ALTER TABLE voice_events_new RENAME TO voice_events",
]
