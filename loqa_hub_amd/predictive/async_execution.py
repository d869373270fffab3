"""Async skill-execution worker pool (``internal/llm/async_execution.go``).

5 workers, a 50-slot queue with non-blocking submit ("execution queue is full",
:118-162), 30 s timeout, 2 retries with linear backoff (1 s x attempt) and a
progress update before each retry (:247-289), result status per update
strategy (:292-334), pairwise-average metrics (:337-380).
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field

from ..skills.interfaces import SkillResponse, VoiceIntent
from .types import (STATUS_ERROR, STATUS_PROGRESS, STATUS_SUCCESS, UPDATE_PROGRESS,
                    UPDATE_VERBOSE, CommandClassification, StatusUpdate)


@dataclass
class ExecutionTask:
    execution_id: str
    intent: VoiceIntent
    classification: CommandClassification
    status: asyncio.Queue
    start_time: float = field(default_factory=time.monotonic)
    retry_count: int = 0


@dataclass
class AsyncExecutionResult:
    execution_id: str
    success: bool = False
    response: SkillResponse | None = None
    error: Exception | None = None
    execution_time: float = 0.0
    queue_time: float = 0.0
    retry_count: int = 0
    timestamp: float = field(default_factory=time.time)


@dataclass
class ExecutionMetrics:
    total_executions: int = 0
    successful_executions: int = 0
    failed_executions: int = 0
    retried_executions: int = 0
    average_execution_time: float = 0.0
    average_queue_time: float = 0.0
    concurrent_executions: int = 0
    queue_depth: int = 0
    last_execution_time: float = 0.0


class AsyncExecutionPipeline:
    def __init__(self, skill_manager, *, max_concurrency: int = 5, queue_size: int = 50,
                 execution_timeout: float = 30.0, retry_attempts: int = 2,
                 retry_delay: float = 1.0):
        self.skill_manager = skill_manager
        self.max_concurrency = max_concurrency
        self.execution_timeout = execution_timeout
        self.retry_attempts = retry_attempts
        self.retry_delay = retry_delay
        self.metrics = ExecutionMetrics()
        self.active: dict[str, ExecutionTask] = {}
        self.queue: asyncio.Queue = asyncio.Queue(queue_size)
        self._workers: list[asyncio.Task] = []
        self._closed = False

    def _ensure_workers(self) -> None:
        if not self._workers:
            loop = asyncio.get_running_loop()
            self._workers = [loop.create_task(self._worker()) for _ in range(self.max_concurrency)]

    def submit_execution(self, execution_id: str, intent: VoiceIntent,
                         classification: CommandClassification, status: asyncio.Queue) -> None:
        if self._closed:
            raise RuntimeError("execution pipeline is shut down")
        self._ensure_workers()
        task = ExecutionTask(execution_id, intent, classification, status)
        self.active[execution_id] = task
        self.metrics.queue_depth += 1
        try:
            self.queue.put_nowait(task)
        except asyncio.QueueFull:
            self.active.pop(execution_id, None)
            self.metrics.queue_depth -= 1
            raise RuntimeError("execution queue is full, cannot process request") from None

    async def _worker(self) -> None:
        while True:
            task = await self.queue.get()
            m = self.metrics
            m.total_executions += 1
            m.concurrent_executions += 1
            m.queue_depth -= 1
            m.last_execution_time = time.time()
            try:
                res = await self._execute(task)
            finally:
                m.concurrent_executions -= 1
            if res.success:
                m.successful_executions += 1
            else:
                m.failed_executions += 1
            if m.total_executions == 1:
                m.average_execution_time, m.average_queue_time = res.execution_time, res.queue_time
            else:
                m.average_execution_time = (m.average_execution_time + res.execution_time) / 2
                m.average_queue_time = (m.average_queue_time + res.queue_time) / 2
            self._send_result(task, res)
            self.active.pop(task.execution_id, None)
            self.queue.task_done()

    async def _execute(self, task: ExecutionTask) -> AsyncExecutionResult:
        t0 = time.monotonic()
        res = AsyncExecutionResult(task.execution_id, queue_time=t0 - task.start_time)
        try:
            skill = self.skill_manager.find_skill_for_intent(task.intent)
        except Exception as e:  # noqa: BLE001
            res.error = LookupError(f"no skill found for intent: {e}")
            res.execution_time = time.monotonic() - t0
            return res
        try:
            resp = await asyncio.wait_for(self._with_retry(task, skill), self.execution_timeout)
            res.success, res.response = resp.success, resp
        except asyncio.TimeoutError:
            res.error = TimeoutError("context deadline exceeded")
        except Exception as e:  # noqa: BLE001
            res.error = e
        res.retry_count = task.retry_count
        res.execution_time = time.monotonic() - t0
        return res

    async def _with_retry(self, task: ExecutionTask, skill) -> SkillResponse:
        last: Exception | None = None
        for attempt in range(self.retry_attempts + 1):
            if attempt > 0:
                task.retry_count = attempt
                self.metrics.retried_executions += 1
                await asyncio.sleep(self.retry_delay * attempt)
            try:
                resp = await self.skill_manager.execute_skill(skill, task.intent)
                if resp.success:
                    return resp
                last = RuntimeError(f"skill execution failed: {resp.error}")
            except Exception as e:  # noqa: BLE001
                last = e
            if attempt < self.retry_attempts:
                self._put(task, StatusUpdate(STATUS_PROGRESS,
                                             f"Retrying operation (attempt {attempt + 2})",
                                             False, task.execution_id))
        raise RuntimeError(f"execution failed after {self.retry_attempts} retries: {last}")

    @staticmethod
    def _put(task: ExecutionTask, upd: StatusUpdate) -> None:
        try:
            task.status.put_nowait(upd)
        except asyncio.QueueFull:
            pass

    def _send_result(self, task: ExecutionTask, res: AsyncExecutionResult) -> None:
        if res.success:
            if task.classification.update_strategy not in (UPDATE_VERBOSE, UPDATE_PROGRESS):
                return
            self._put(task, StatusUpdate(STATUS_SUCCESS, success_message(task, res.response),
                                         True, task.execution_id))
        else:
            self._put(task, StatusUpdate(STATUS_ERROR, error_message(task), False,
                                         task.execution_id, error=str(res.error)))

    def get_metrics(self) -> ExecutionMetrics:
        return ExecutionMetrics(**vars(self.metrics))

    def get_active_executions(self) -> dict[str, ExecutionTask]:
        return dict(self.active)

    async def shutdown(self, timeout: float = 5.0) -> None:
        self._closed = True
        for w in self._workers:
            w.cancel()
        if self._workers:
            await asyncio.wait(self._workers, timeout=timeout)
        self._workers = []


def success_message(task: ExecutionTask, resp: SkillResponse) -> str:
    if resp.speech_text:
        return resp.speech_text
    if resp.message:
        return resp.message
    ents = task.intent.entities
    if "action" in ents:
        if "location" in ents:
            return f"{ents['action']} {ents['location']} completed successfully"
        return f"{ents['action']} completed successfully"
    return f"{task.intent.intent} operation completed"


def error_message(task: ExecutionTask) -> str:
    ents = task.intent.entities
    if "location" in ents:
        if "device" in ents:
            return f"Sorry, I couldn't reach the {ents['location']} {ents['device']}"
        return f"Sorry, I couldn't reach the {ents['location']} device"
    return "Sorry, I couldn't complete that operation"
