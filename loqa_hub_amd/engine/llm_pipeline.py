"""Pipelined (two steps in flight) constrained decode for ``LLMEngine``.

A plain decode step is a round trip: the host waits for step j's sampled
tokens, advances every sequence's grammar, builds step j+1's metadata and only
then launches it, so the GPU idles (or only runs the concurrent Whisper
decoder) for the host's turnaround - measured 0.3-0.5 ms per 4 ms step in the
serving pipeline. Here step j+1 is launched while step j still runs:

* the token a sequence sampled in step j is not known to the host yet, so
  step j+1 takes it on the device: the step graph gathers it from
  ``last_tok[seq slot]``, which every step's epilogue writes
  (``LLMEngine._step_body``);
* what FOLLOWS that token - the jump-forward literal, the next mask row,
  whether the grammar completes - comes from ``GrammarState.predict``, exact
  for every token except a Free field's closing quote (and undefined at a
  Choice node with multi-token options, where the sequence sits the step out);
* when step j's results arrive the host commits them; a sequence whose token
  broke the prediction (it closed a string early) has its step j+1 work
  discarded: its KV length is rolled back (``pool.truncate``) and the correct
  tokens are fed in step j+2 at the same positions, overwriting the garbage.

Streams order everything else: a step's H2D metadata copy runs after the
previous step, its result copy before the next one, so two pinned staging
buffers per graph and one result buffer per in-flight step suffice.
"""
from __future__ import annotations

import collections
import time

import numpy as np
import torch

from .. import ops
from .batching import MPAD_PLAN, plan_step, plan_step_mpad

DEV = -1   # feed placeholder: "the token this sequence sampled in its previous step"


class _Step:
    __slots__ = ("id", "rows", "B", "out", "event", "g", "entries")

    def __init__(self, sid, rows, B, out, event, g, entries):
        self.id, self.rows, self.B, self.out, self.event, self.g = sid, rows, B, out, event, g
        self.entries = entries


class DecodePipeline:
    DEPTH = 2

    def __init__(self, eng):
        self.eng = eng
        self.inflight: collections.deque[_Step] = collections.deque()
        self.next_id = 0
        self.rr = 0
        self.stats = eng.stats          # pipeline counters live with the engine's
        for k in ("pl_steps", "pl_spec", "pl_discard", "pl_sitout", "pl_sitout_long",
                  "pl_sitout_pred"):
            self.stats.setdefault(k, 0)
        # test hook: treat this fraction of generic tokens as mispredicted
        self.force_mispredict = 0.0
        self._rng = np.random.default_rng(0)
        assert not eng.use_graphs or eng.RES_SLOTS >= self.DEPTH + 1

    # ----------------------------------------------------------- helpers
    def admit(self, r) -> None:
        """A request that finished its prefill joins (its first sampled token
        and forced literal are host-known in ``r.feed``)."""
        eng = self.eng
        r.pl_slot = eng._free_seq_slots.pop(0)
        r.pl_host = list(r.feed)
        r.pl_fl = []                 # in-flight entries, oldest first

    def release(self, r) -> None:
        if getattr(r, "pl_slot", -1) >= 0:
            self.eng._free_seq_slots.append(r.pl_slot)
            self.eng._free_seq_slots.sort()
            r.pl_slot = -1

    # -------------------------------------------------------------- pump
    def pump(self, live: list) -> None:
        """Advance the pipeline by one step: retire the oldest step if the
        pipeline is full, then launch the next one (or, if no sequence can be
        fed yet, retire the oldest in-flight step instead)."""
        if len(self.inflight) >= self.DEPTH:
            self._retire(self.inflight.popleft())
        if not self._launch(live) and self.inflight:
            self._retire(self.inflight.popleft())

    def drain(self) -> None:
        while self.inflight:
            self._retire(self.inflight.popleft())

    def abort(self) -> None:
        """After an error: wait for in-flight GPU work, forget it."""
        for st in self.inflight:
            try:
                if st.event is not None:
                    st.event.synchronize()
            except Exception:  # noqa: BLE001
                pass
        self.inflight.clear()

    # ------------------------------------------------------------ launch
    def _intended(self, r):
        """(feed tokens with DEV placeholders, speculative, mask row after the
        whole feed) for the next step, or None when ``r`` sits it out."""
        if r.done:
            return None
        last = r.pl_fl[-1] if r.pl_fl else None
        if last is not None and last["sample"] and not last["discard"]:
            if len(r.pl_fl) >= self.DEPTH:
                return None
            pred = r.grammar.predict()
            if pred is None:
                self.stats["pl_sitout_pred"] += 1
                return None
            forced, row, done = pred
            if done:
                return None            # completes with the in-flight token
            feed = [DEV] + forced
            if len(feed) > self.eng.max_decode_q:
                self.stats["pl_sitout_long"] += 1
                return None            # never split a speculative feed
            return feed, True, row
        if not r.pl_host:
            return None
        return list(r.pl_host), False, r.grammar.mask_row()

    def _launch(self, live: list) -> bool:
        eng = self.eng
        cands = []
        for r in live:
            it = self._intended(r)
            if it is not None:
                cands.append((r, it))
        if not cands:
            return False
        lens = [len(it[0]) for _, it in cands]
        if MPAD_PLAN:
            take = plan_step_mpad(lens, eng.step_tokens, eng.max_decode_q, self.rr,
                                  whole=[it[1] for _, it in cands])
        else:
            take = plan_step(lens, eng.step_tokens, eng.max_decode_q, self.rr)
        n_c = len(cands)
        self.rr = (self.rr + eng.step_tokens) % n_c if n_c > eng.step_tokens else 0
        rows, feeds, entries = [], [], []
        pool = eng.kv.pool
        for (r, (feed, spec, row)), n in zip(cands, take):
            if n == 0 or (spec and n < len(feed)):
                continue
            sample = n == len(feed)
            pos0 = pool.seq_len(r.seq_id)
            e = {"step": self.next_id, "sample": sample, "spec": spec, "pos0": pos0,
                 "discard": False, "row": row if sample else 0}
            if not spec:
                r.pl_host = r.pl_host[n:]
            rows.append(r)
            feeds.append(feed[:n])
            entries.append(e)
        if not rows:
            return False
        B = len(rows)
        T = sum(len(f) for f in feeds)
        t0 = time.perf_counter()
        ctx = max(e["pos0"] + len(f) for e, f in zip(entries, feeds))
        B_pad = eng._bucket_seqs(B)
        T_pad = ops.mpad_for(T)
        C = min(eng.max_seq_len, -(-ctx // eng.CTX_BUCKET) * eng.CTX_BUCKET)
        g = eng._graphs.get((B_pad, T_pad, C)) if eng.use_graphs else None
        if eng.use_graphs and g is None:
            if eng._graphs_frozen:
                # uncaptured bucket while serving: finish what is in flight and
                # run this step eagerly (no capture while other threads launch)
                for r, e, f in zip(rows, entries, feeds):
                    if not e["spec"]:
                        r.pl_host = list(f) + r.pl_host
                self.drain()
                return self._launch_eager(live)
            g = eng._decode_graph(B_pad, T_pad, C)
        sid = self.next_id
        self.next_id += 1
        slot_of = [r.pl_slot for r in rows]
        toks = [0 if t == DEV else t for f in feeds for t in f]
        src = []
        for f, sl in zip(feeds, slot_of):
            src += [sl if t == DEV else -1 for t in f]
        mrows = [e["row"] for e in entries]
        if g is not None:
            # the staging slot written here was last read by the step two
            # launches back, which has retired
            host = eng._stage(g)
            eng._meta(rows, [[0] * len(f) for f in feeds], True, B_pad, T_pad, out=host)
            host["tokens"][:T] = toks
            host["src"].fill(-1)
            host["src"][:T] = src
            host["mask_rows"].fill(0)
            host["mask_rows"][:B] = mrows
            host["row_slot"].fill(eng.max_seqs)
            host["row_slot"][:B] = slot_of
            t1 = time.perf_counter()
            rslot = eng._replay(g)
            ev = torch.cuda.Event()
            ev.record()
            eng.stats["host_pre_s"] += t1 - t0
            st = _Step(sid, rows, B, eng._res_ring[rslot], ev, g, entries)
        else:
            st = self._run_eager(sid, rows, feeds, toks, src, mrows, slot_of, entries, B_pad, T_pad)
        for r, e in zip(rows, entries):
            r.pl_fl.append(e)
            if e["spec"]:
                self.stats["pl_spec"] += 1
        eng.stats["decode_steps"] += 1
        eng.stats["decode_tokens"] += T
        self.stats["pl_steps"] += 1
        self.inflight.append(st)
        return True

    def _launch_eager(self, live: list) -> bool:
        """Bucket without a captured graph: one synchronous eager step."""
        eng = self.eng
        use = eng.use_graphs
        eng.use_graphs = False
        try:
            return self._launch(live)
        finally:
            eng.use_graphs = use

    def _run_eager(self, sid, rows, feeds, toks, src, mrows, slot_of, entries, B_pad, T_pad):
        eng = self.eng
        max_q, max_ctx, host = eng._meta(rows, [[0] * len(f) for f in feeds], True, B_pad, T_pad)
        T = len(toks)
        host["tokens"][:T] = toks
        s = np.full(T_pad, -1, np.int32)
        s[:T] = src
        host["src"] = s
        mr = np.zeros(B_pad, np.int32)
        mr[:len(mrows)] = mrows
        host["mask_rows"] = mr
        rs = np.full(B_pad, eng.max_seqs, np.int32)
        rs[:len(slot_of)] = slot_of
        host["row_slot"] = rs
        dev = eng._to_device(host)
        meta = eng._build_meta(dev, max_q, max_ctx, True)
        out = eng._step_body(meta, dev)
        res = out[:B_pad].to("cpu", torch.int32)
        return _Step(sid, rows, len(rows), res, None, None, entries)

    # ------------------------------------------------------------ retire
    def _retire(self, st: _Step) -> None:
        eng = self.eng
        t0 = time.perf_counter()
        if st.event is not None:
            st.event.synchronize()
        t1 = time.perf_counter()
        nxt = st.out[: st.B].numpy().copy()
        eng.stats["gpu_wait_s"] += t1 - t0
        now = time.perf_counter()
        for b, r in enumerate(st.rows):
            e = r.pl_fl.pop(0)
            assert e["step"] == st.id, "pipeline entry order"
            if e["discard"] or not e["sample"] or r.done:
                continue
            t = int(nxt[b])
            nxt_e = r.pl_fl[0] if r.pl_fl else None
            generic = r.grammar.is_generic(t)
            if generic and self.force_mispredict and self._rng.random() < self.force_mispredict:
                generic = False
            forced = eng._commit(r, t, now)
            if r.done:
                if nxt_e is not None:
                    nxt_e["discard"] = True
                continue
            if nxt_e is not None and nxt_e["spec"]:
                if generic:
                    continue           # step j+1 fed exactly [t] + forced
                nxt_e["discard"] = True
                eng.kv.pool.truncate(r.seq_id, nxt_e["pos0"])
                self.stats["pl_discard"] += 1
            r.pl_host = [t] + forced
        eng.stats["host_post_s"] += time.perf_counter() - now
