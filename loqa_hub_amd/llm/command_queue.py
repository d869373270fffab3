"""Sequential multi-command execution with rollback - the benchmark path.

Behavioural spec: ``internal/llm/command_queue.go`` (``Execute`` :77-170,
``rollbackCommands`` :173-195, ``createRollbackCommand`` :198-220,
``combinedResponse`` :223-234). Kept verbatim in behaviour: per-item
start/end/duration, the >200 ms slow-command warning, reverse-order rollback of
completed items with turn_on<->turn_off inverses, and the three combined
response strings. In the reference this path only runs under tests; here the
audio pipeline drives it after every multi-command parse.

``CommandQueueItem.duration`` of items with index >= 1 is the
"ms per added command (reference-equivalent)" of BASELINE.md.
"""
from __future__ import annotations

import asyncio
import logging
import time
from dataclasses import dataclass, field
from typing import Protocol

from .commands import Command

log = logging.getLogger("loqa.command_queue")

SLOW_COMMAND_S = 0.200


class CommandExecutor(Protocol):
    async def execute_command(self, cmd: Command) -> None: ...


@dataclass
class CommandQueueItem:
    command: Command
    index: int
    executed: bool = False
    success: bool = False
    error: BaseException | None = None
    start_time: float = 0.0
    end_time: float = 0.0
    duration: float = 0.0  # seconds

    def to_dict(self) -> dict:
        return {"command": self.command.to_dict(), "index": self.index, "executed": self.executed,
                "success": self.success, "duration_ms": self.duration * 1e3}


@dataclass
class ExecutionResult:
    success: bool = True
    completed_items: list[CommandQueueItem] = field(default_factory=list)
    failed_item: CommandQueueItem | None = None
    total_duration: float = 0.0
    rollback_occurred: bool = False
    combined_response: str = ""
    responses: list[str] = field(default_factory=list)
    error: BaseException | None = None
    cancelled: bool = False


class QueueTimeout(Exception):
    pass


class CommandQueue:
    def __init__(self, commands: list[Command], max_duration: float = 0.0,
                 rollback_enabled: bool = True):
        self.items = [CommandQueueItem(command=c, index=i) for i, c in enumerate(commands)]
        self.max_duration = max_duration
        self.rollback_enabled = rollback_enabled
        self._lock = asyncio.Lock()

    async def execute(self, executor: CommandExecutor) -> ExecutionResult:
        async with self._lock:
            t0 = time.perf_counter()
            deadline = t0 + self.max_duration if self.max_duration > 0 else None
            res = ExecutionResult()
            log.info("executing command queue with %d commands", len(self.items))
            for i, item in enumerate(self.items):
                if deadline is not None and time.perf_counter() >= deadline:
                    res.success = False
                    res.error = QueueTimeout(
                        f"command queue execution timeout or cancelled at command {i}")
                    res.cancelled = True
                    res.total_duration = time.perf_counter() - t0
                    return res
                item.start_time = time.perf_counter()
                err: BaseException | None = None
                try:
                    if deadline is not None:
                        await asyncio.wait_for(executor.execute_command(item.command),
                                               max(0.0, deadline - item.start_time))
                    else:
                        await executor.execute_command(item.command)
                except asyncio.TimeoutError as e:
                    err = QueueTimeout(f"command {i} exceeded the queue deadline")
                    err.__cause__ = e
                except Exception as e:  # executor failure
                    err = e
                item.end_time = time.perf_counter()
                item.duration = item.end_time - item.start_time
                item.executed = True
                if err is not None:
                    item.success = False
                    item.error = err
                    res.success = False
                    res.failed_item = item
                    if isinstance(err, QueueTimeout):  # deadline hit mid-command
                        res.error, res.cancelled = err, True
                    log.warning("command %d failed: %s", i + 1, err)
                    if self.rollback_enabled and res.completed_items:
                        rb_err = await self._rollback(executor, res.completed_items)
                        if rb_err is None:
                            res.rollback_occurred = True
                        else:
                            log.warning("rollback failed: %s", rb_err)
                    break
                item.success = True
                res.completed_items.append(item)
                res.responses.append(item.command.response)
                if item.duration > SLOW_COMMAND_S:
                    log.warning("command %d took longer than 200ms: %.1f ms", i + 1,
                                item.duration * 1e3)
            res.total_duration = time.perf_counter() - t0
            res.combined_response = combined_response(res.responses)
            return res

    async def run(self, executor: CommandExecutor) -> tuple[ExecutionResult, BaseException | None]:
        """Execute and return (result, error) like the reference's (result, err) pair:
        error is set only when the queue deadline cancelled execution."""
        res = await self.execute(executor)
        return res, (res.error if res.cancelled else None)

    async def _rollback(self, executor: CommandExecutor,
                        completed: list[CommandQueueItem]) -> BaseException | None:
        errors = []
        for item in reversed(completed):
            rb = create_rollback_command(item.command)
            if rb is None:
                log.info("no rollback available for command: %s", item.command.intent)
                continue
            try:
                await executor.execute_command(rb)
            except Exception as e:
                errors.append(f"rollback failed for command {item.index}: {e}")
        if errors:
            return RuntimeError(f"rollback completed with {len(errors)} errors: {errors}")
        return None

    def get_status(self) -> list[CommandQueueItem]:
        return [CommandQueueItem(**vars(i)) for i in self.items]

    def size(self) -> int:
        return len(self.items)

    def is_empty(self) -> bool:
        return not self.items


def create_rollback_command(cmd: Command) -> Command | None:
    if cmd.intent == "turn_on":
        return Command("turn_off", cmd.entities, cmd.confidence,
                       f"Rolling back: turning off {cmd.entities.get('device', '')}")
    if cmd.intent == "turn_off":
        return Command("turn_on", cmd.entities, cmd.confidence,
                       f"Rolling back: turning on {cmd.entities.get('device', '')}")
    return None


def combined_response(responses: list[str]) -> str:
    if not responses:
        return "No commands were executed."
    if len(responses) == 1:
        return responses[0]
    return f"I've completed {len(responses)} commands for you."
