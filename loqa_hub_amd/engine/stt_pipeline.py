"""Pipelined (two steps in flight) Whisper decoder for ``STTEngine``.

A synchronous decoder step is a round trip: the host waits for step j's
tokens, builds step j+1's metadata and only then launches it - a host gap of
~0.3 ms per ~4 ms step beside the LLM decode (docs/PERF.md). Here step j+1 is
launched while step j still runs, as the LLM engine does
(``engine/llm_pipeline.py``):

* a teacher-forced request (synthetic traffic) knows every fed token in
  advance - target[k-1] at step k - so its steps need no device feedback;
* a greedy request feeds, while its previous step is still in flight, the
  token that step sampled, straight from ``last_tok[slot]`` on the device
  (``STTEngine._graph``'s fetch node); its end (EOT / max tokens) is known only
  when that step retires, so at most one speculative step past the end runs
  and is discarded (its KV / last-token writes are stream-ordered before any
  reuse of the blocks or the slot).

Step I/O is the engine's pinned staging / result rings and device counter.
"""
from __future__ import annotations

import collections
import time

import numpy as np
import torch

from .. import ops

DEV = -1   # feed placeholder: the token this request sampled in its previous step


class _Step:
    __slots__ = ("rows", "B", "out", "event", "entries")

    def __init__(self, rows, B, out, event, entries):
        self.rows, self.B, self.out, self.event, self.entries = rows, B, out, event, entries


class STTPipeline:
    DEPTH = 2

    def __init__(self, eng):
        self.eng = eng
        self.inflight: collections.deque[_Step] = collections.deque()
        self.stats = eng.stats
        for k in ("pl_steps", "pl_spec", "pl_discard", "pl_empty"):
            self.stats.setdefault(k, 0)
        # host time of the launch path (metadata + graph replay) and of the
        # replay call alone: where a step-to-step gap on the STT stream comes from
        for k in ("pl_launch_s", "pl_replay_s"):
            self.stats.setdefault(k, 0.0)
        assert eng.RES_SLOTS >= self.DEPTH + 1

    # -------------------------------------------------------------- helpers
    @staticmethod
    def admit(r) -> None:
        """A request whose encoder output is ready (``feed`` = its SOT prompt)."""
        r.pl_launched = 0          # decoder steps launched (step 0 feeds the prompt)
        r.pl_fl = 0                # of which still in flight
        r.pl_end = False           # greedy: the last decided token ended the sequence

    def _feed(self, r):
        """(tokens with DEV placeholders, speculative) of r's next step, or None.
        The first ``r.prompt_steps`` steps feed the prompt (the SOT tokens, after
        a long-form window's previous-text prompt) at most len(SOT) tokens at a
        time - the captured graphs' per-sequence query limit."""
        c = self.eng.n_prompt_tokens_per_step
        ps = r.prompt_steps
        k = r.pl_launched
        if k < ps:
            return list(r.feed[k * c:(k + 1) * c]), False
        k = k - ps + 1                            # 1 = the first step feeding a decoded token
        if r.target is not None:
            if k >= len(r.target):
                return None                       # every target token is in flight / done
            return [int(r.target[k - 1])], False
        if r.pl_end or k >= r.max_new_tokens or r.pl_fl >= self.DEPTH:
            return None
        if r.pl_fl:
            return [DEV], True
        return [int(r.tokens[-1])], False

    # ---------------------------------------------------------------- pump
    def pump(self, live: list) -> list:
        """Retire the oldest step if the pipeline is full, launch the next one
        (or retire when nothing can be launched); returns finished requests."""
        done = []
        if len(self.inflight) >= self.DEPTH:
            done += self._retire(self.inflight.popleft())
        t0 = time.perf_counter()
        launched = self._launch(live)
        self.stats["pl_launch_s"] += time.perf_counter() - t0
        if not launched:
            if self.inflight:
                done += self._retire(self.inflight.popleft())
            else:
                self.stats["pl_empty"] += 1     # nothing to launch and nothing in flight
        return done

    def drain(self) -> list:
        done = []
        while self.inflight:
            done += self._retire(self.inflight.popleft())
        return done

    def abort(self) -> None:
        for st in self.inflight:
            try:
                st.event.synchronize()
            except Exception:  # noqa: BLE001
                pass
        self.inflight.clear()

    # -------------------------------------------------------------- launch
    def _launch(self, live: list) -> bool:
        eng = self.eng
        cands = [(r, f) for r in live if r.t_done == 0.0 for f in [self._feed(r)] if f is not None]
        if not cands:
            return False
        rows, feeds, spec = [], [], []
        T = 0
        for r, (f, sp) in cands:            # prompts first fill the step-token budget
            if T + len(f) > eng.step_tokens:
                continue
            rows.append(r)
            feeds.append(f)
            spec.append(sp)
            T += len(f)
        if not rows:
            return False
        B = len(rows)
        B_pad = next((b for b in eng.SEQ_BUCKETS if b >= B), B)
        T_pad = ops.mpad_for(T)
        ctx = max(eng.kv.pool.seq_len(r.seq_id) + len(f) for r, f in zip(rows, feeds))
        C = min(eng.cfg.n_text_ctx, -(-ctx // eng.SPLIT_KEYS) * eng.SPLIT_KEYS)
        if (B_pad, T_pad, C) not in eng._graphs and eng._graphs_frozen:
            return self._launch_sync(rows, feeds)
        g = eng._graph(B_pad, T_pad, C)
        hb = eng._stage(g)
        saved = [r.feed for r in rows]
        for r, f in zip(rows, feeds):
            r.feed = [0 if t == DEV else t for t in f]
        eng._host_meta(rows, B_pad, T_pad, out=hb)
        for r, f in zip(rows, saved):
            r.feed = f
        src = hb["src"]
        src.fill(-1)
        i = 0
        for r, f in zip(rows, feeds):
            for t in f:
                if t == DEV:
                    src[i] = r.slot
                i += 1
        hb["row_slot"].fill(eng.max_batch)
        hb["row_slot"][:B] = [r.slot for r in rows]
        t_r = time.perf_counter()
        rslot = eng._replay(g)
        self.stats["pl_replay_s"] += time.perf_counter() - t_r
        ev = torch.cuda.Event()
        ev.record()
        entries = []
        for r, sp in zip(rows, spec):
            entries.append((r.pl_launched, sp))
            r.pl_launched += 1
            r.pl_fl += 1
            if sp:
                self.stats["pl_spec"] += 1
        self.inflight.append(_Step(rows, B, eng._res_ring[rslot], ev, entries))
        self.stats["pl_steps"] += 1
        eng.stats["decode_steps"] += 1
        return True

    def _launch_sync(self, rows, feeds) -> bool:
        """Bucket without a captured graph (serving never captures): finish
        what is in flight, then one synchronous step through ``STTEngine._step``."""
        if any(DEV in f for f in feeds):
            return False                     # wait for the in-flight step instead
        saved = [r.feed for r in rows]
        for r, f in zip(rows, feeds):
            r.feed = f
        out = self.eng._step(rows)
        for r, f in zip(rows, saved):
            r.feed = f
        # the eager step does not run the graphs' publish node: keep last_tok
        # current for a following device-fed step
        idx = torch.tensor([r.slot for r in rows], dtype=torch.long, device=self.eng.device)
        self.eng.last_tok[idx] = torch.as_tensor(np.asarray(out, np.int32)[: len(rows)],
                                                 device=self.eng.device)
        entries = []
        for r in rows:
            entries.append((r.pl_launched, False))
            r.pl_launched += 1
            r.pl_fl += 1
        self.inflight.append(_Step(rows, len(rows), torch.from_numpy(np.asarray(out, np.int32)),
                                   None, entries))
        self.eng.stats["decode_steps"] += 1
        return True

    # -------------------------------------------------------------- retire
    def _retire(self, st: _Step) -> list:
        eng = self.eng
        t0 = time.perf_counter()
        if st.event is not None:
            st.event.synchronize()
        nxt = st.out[: st.B].numpy().copy()
        eng.stats["gpu_wait_s"] += time.perf_counter() - t0
        done = []
        for b, (r, (k, sp)) in enumerate(zip(st.rows, st.entries)):
            r.pl_fl -= 1
            if r.t_done != 0.0 or r.pl_end:
                if sp:
                    self.stats["pl_discard"] += 1
                continue
            k -= r.prompt_steps - 1              # token index; < 0: a prompt chunk (logits unused)
            if k < 0:
                continue
            t = int(r.target[k]) if r.target is not None else int(nxt[b])
            r.tokens.append(t)
            r.step += 1
            end = (t == eng.eot or len(r.tokens) >= r.max_new_tokens
                   or (r.target is not None and r.step >= len(r.target)))
            if end:
                r.pl_end = True
                if r.pl_fl == 0:
                    self._window_end(r, done)
        # a greedy request that ended while a discarded step was in flight
        for r in st.rows:
            if r.pl_end and r.pl_fl == 0 and r.t_done == 0.0 and r not in done:
                self._window_end(r, done)
        return done

    def _window_end(self, r, done: list) -> None:
        """r's current window is decoded: r completes, or (long-form) its next
        window starts as a fresh pipelined sequence."""
        f = self.eng._finish(r)
        if f is not None:
            done.append(f)
        else:
            self.admit(r)
