"""Continuous-batching, grammar-constrained LLM engine (one per GPU).

Replaces the up-to-five Ollama HTTP calls per utterance of the reference
(SURVEY §3.2 observation 2) with ONE constrained multi-command decode whose
result is shared by the classifier, the bridge, the fallback parser and the
command queue.

Step anatomy (all on the compute stream):
  prefill : prompts (+ the schema's opening literal, jump-forwarded) as one
            flat batch -> flash attention over the paged cache (prefix blocks
            shared through the native block pool's prefix cache).
  decode  : every live sequence feeds [sampled token + forced literal tokens]
            -> grouped split-K paged attention -> lm_head -> fused
            grammar-masked argmax (one mask row per sequence).  Decode steps
            are replayed from HIP graphs bucketed by (seqs, tokens).
Host work per step is the grammar cursor advance (a few dict lookups per
sequence) plus one small pinned H2D copy of the step metadata.
"""
from __future__ import annotations

import logging
import os
import queue
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..models.configs import LlamaConfig
from .batching import MPAD_PLAN, join_futures, plan_step, plan_step_mpad
from ..models.llama import LlamaModel, LlamaWeights, StepMeta, TPGroup
from .grammar import GrammarState, GrammarTables
from .kv_cache import PagedKVCache
from .tokenizer import get_tokenizer
from ..parallel.custom_allreduce import ERR_TOKEN, CollectiveError

log = logging.getLogger("loqa.llm")


@dataclass
class GenRequest:
    prompt: list[int]
    schema: list
    seq_id: int = -1
    # filled by the engine
    grammar: GrammarState | None = None
    feed: list[int] = field(default_factory=list)
    output: str = ""
    t_submit: float = 0.0
    t_first: float = 0.0
    t_done: float = 0.0
    steps: int = 0
    token_times: list[float] = field(default_factory=list)
    done: bool = False
    # optional streaming hook: called from the engine thread with each step's
    # newly emitted token ids (sampled token + jump-forward literal)
    on_tokens: object = None
    # optional completion hook (continuous-batching scheduler), engine thread
    on_done: object = None


def _bucket(n: int, buckets: list[int]) -> int:
    for b in buckets:
        if n <= b:
            return b
    return n


class LLMEngine:
    SEQ_BUCKETS = [1, 2, 4, 8, 16, 32, 64, 128]
    RES_SLOTS = 3       # result ring slots (>= steps in flight + 1)

    def __init__(self, cfg: LlamaConfig, device, *, seed: int = 0, max_seqs: int = 64,
                 max_seq_len: int = 1024, block_size: int = 16, num_blocks: int | None = None,
                 tp: TPGroup | None = None, use_graphs: bool = True, prefill_chunk: int = 8192,
                 weights: LlamaWeights | None = None, fused_decode: bool = True,
                 compact: bool = False, tokenizer=None):
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.tp = tp or TPGroup()
        from ..utils.streams import decode_cap, init_pools
        init_pools(self.device)       # fixed stream -> hardware-queue placement
        self.max_wgs = decode_cap("LOQA_LLM_MAX_WGS")
        with ops.decode_cap(self.max_wgs):
            self.weights = weights or LlamaWeights(cfg, self.device, seed=seed, tp=self.tp,
                                                   compact=compact)
        self.weights.max_wgs = self.max_wgs or ops.MAX_DECODE_WGS
        self.model = LlamaModel(self.weights)
        # a checkpoint's own tokenizer (tokenizer.HFTokenizer), else the
        # synthetic one of the random-init weights
        self.tok = tokenizer or get_tokenizer(cfg.vocab_size)
        self.grammar = GrammarTables(self.tok, self.device)
        from .grammar import INTENTS
        self.grammar.trie(INTENTS)
        self.grammar.trie(["true", "false"])
        self.masks = self.grammar.mask_table(self.device)
        self.max_seqs, self.max_seq_len = max_seqs, max_seq_len
        self.block_size = block_size
        self.max_blocks = (max_seq_len + block_size - 1) // block_size
        if num_blocks is None:
            num_blocks = max_seqs * self.max_blocks + 64
        self.kv = PagedKVCache(cfg.n_layers, self.weights.hkv, cfg.head_dim, num_blocks, block_size,
                               self.device)
        self.is_gpu = self.device.type == "cuda"
        # grouped decode attention holds G * q_len <= 32 query rows per kv head
        self.max_decode_q = max(1, 32 // (self.weights.h // self.weights.hkv))
        self.attn_ws = ops.AttnWorkspace(self.device, 128, self.weights.h, cfg.head_dim,
                                         (max_seq_len + 127) // 128) if self.is_gpu else None
        # decode-attention keys per split (>= 128: the workspace holds max_seq_len / 128 splits)
        self.attn_split_keys = max(128, int(os.environ.get("LOQA_LLM_ATTN_SPLIT_KEYS", "128")) // 32 * 32)
        self.use_graphs = use_graphs and self.is_gpu
        # fused-epilogue decode GEMMs (single GPU, <= 32 tokens per step)
        self.fused_decode = fused_decode and self.weights.fused
        self.scratch = ops.FusedScratch(self.device)
        self.prefill_chunk = prefill_chunk
        # inline prefill: a new request whose uncached prompt tail is at most
        # this many tokens skips the separate prefill pass and joins the decode
        # batch directly, its tail fed max_decode_q tokens per step (it shares
        # the decode steps' weight reads instead of a whole pass of its own)
        self.inline_prefill = int(os.environ.get("LOQA_INLINE_PREFILL", "64"))
        # chunked prompt passes (0: whole-prompt passes between decode steps):
        # while sequences are decoding, a new prompt goes in chunks of this many
        # tokens, each chunk in ONE pass together with every live sequence's
        # next feed (a mixed step: the live sequences advance during the prompt
        # pass instead of stalling for it); with nothing decoding the whole
        # prompt is one pass (_mixed_step). Measured (docs/PERF.md "Round 4"):
        # 256 -> 19.49-19.64 vs 18.58-19.30 utt/s (4 interleaved pairs); chunk
        # sweep 192 / 256 / 320 / 384 / 512 -> 320 best; 128 loses (a pass is
        # expensive at any row count, so more passes cost more)
        self.chunk_prefill = int(os.environ.get("LOQA_CHUNK_PREFILL", "320"))
        # token budget of one decode step: every live sequence feeds its sampled
        # token plus a jump-forward literal, so without a cap 17+ sequences in a
        # forced run would exceed the fused GEMMs' row limit (ops.MPADS);
        # leftovers carry to the next step (batching.plan_step)
        self.step_tokens = max(1, min(int(os.environ.get("LOQA_LLM_STEP_TOKENS", "64")),
                                      ops.MPADS[-2]))
        self._rr = 0
        self._graphs: dict[tuple[int, int], dict] = {}
        # pipelined decode (GPU graphs): last sampled token per sequence slot
        # (+ one trash slot for padding rows), free sequence slots
        self.last_tok = torch.zeros(max_seqs + 1, dtype=torch.int32, device=self.device)
        self._free_seq_slots = list(range(max_seqs))
        if self.use_graphs:
            # step I/O without copy-engine operations between step graphs
            # (elementwise.hip step_fetch / step_publish): a 2-slot pinned
            # staging ring for step metadata, a 3-slot pinned result ring, and
            # a device counter of launched step graphs that picks the slots
            b_max = _bucket(max(1, max_seqs), self.SEQ_BUCKETS)
            self._n32_max = 4 * ops.MPADS[-1] + 4 * b_max + 1 + b_max * self.max_blocks
            self._n64_max = max(16, b_max)
            self._stage32 = torch.zeros(2, self._n32_max, dtype=torch.int32).pin_memory()
            self._stage64 = torch.zeros(2, self._n64_max, dtype=torch.int64).pin_memory()
            self._res_ring = torch.zeros(self.RES_SLOTS, 256, dtype=torch.int32).pin_memory()
            self._step_ctr = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._step_no = 0
        self.pipelined = self.use_graphs and os.environ.get("LOQA_LLM_PIPELINE", "1") != "0"
        self._pl = None
        # set once warmup_graphs() has captured every reachable bucket: from
        # then on an uncaptured shape runs eagerly instead of capturing while
        # the other worker threads issue HIP work
        self._graphs_frozen = False
        self._next_id = 1
        self._on_done = None
        # tensor parallel: the lock-step control ring (parallel/tp_control.py);
        # rank 0 publishes each scheduler iteration's arrivals, followers replay
        self.tp_ctl = None
        self._cells_lock = threading.Lock()
        # prompt placement (continuous-batching scheduler): prompt passes run on
        # the decode stream, serialised with the decode steps; while sequences
        # decode they are the chunked mixed steps above. Removed in round 4
        # after measuring (docs/PERF.md): a prefill worker stream overlapped
        # with the decode steps (its GEMMs slowed every concurrent step,
        # 17.9-18.0 vs 18.3-18.5 utt/s), round 3's rider variant (one
        # jump-forward slice per live sequence on a hipBLASLt pass: the drain
        # cost what the riders saved) and coalescing holds.
        self.stats = {"prefill_tokens": 0, "decode_steps": 0, "decode_tokens": 0,
                      "forced_tokens": 0, "sampled_tokens": 0, "prefix_hit_tokens": 0,
                      "prefill_s": 0.0, "decode_s": 0.0, "host_pre_s": 0.0, "gpu_wait_s": 0.0,
                      "host_post_s": 0.0, "replay_call_s": 0.0, "sched_s": 0.0}

    # ------------------------------------------------------------- metadata
    def _meta(self, seqs: list[GenRequest], feeds: list[list[int]], decode: bool,
              B_pad: int | None = None, T_pad: int | None = None,
              out: dict | None = None) -> tuple[StepMeta, dict]:
        """Host metadata of one step; ``out`` = preallocated (pinned) numpy views
        to fill in place (the graph path: one H2D copy per step, no allocation)."""
        B = len(seqs)
        T = sum(len(f) for f in feeds)
        B_pad = B_pad or B
        T_pad = T_pad or T
        if out is not None:
            tokens, positions, slots = out["tokens"], out["positions"], out["slots"]
            cu, ctx, bt, lidx = out["cu_q"], out["ctx_lens"], out["block_tables"], out["logit_idx"]
        else:
            tokens = np.zeros(T_pad, np.int32)
            positions = np.zeros(T_pad, np.int32)
            slots = np.full(T_pad, -1, np.int32)
            cu = np.zeros(B_pad + 1, np.int32)
            ctx = np.zeros(B_pad, np.int32)
            bt = np.zeros((B_pad, self.max_blocks), np.int32)
            lidx = np.zeros(max(16, B_pad) if decode else B_pad, np.int64)
        tokens.fill(0)
        if T:
            tokens[:T] = [t for f in feeds for t in f]
        rc = self.kv.pool.step_meta([r.seq_id for r in seqs], [len(f) for f in feeds], B_pad,
                                    T_pad, self.max_blocks, positions, slots, cu, ctx, bt, lidx)
        if rc == -2:
            raise RuntimeError("KV cache exhausted")
        if rc != 0:
            raise RuntimeError(f"step metadata failed ({rc})")
        max_q = max([len(f) for f in feeds] + [1])
        max_ctx = max(int(ctx[:B].max()) if B else 1, 1)
        host = {"tokens": tokens, "positions": positions, "slots": slots, "cu_q": cu,
                "ctx_lens": ctx, "block_tables": bt, "logit_idx": lidx}
        return max_q, max_ctx, host

    def _to_device(self, host: dict, dst: dict | None = None) -> dict:
        out = {}
        for k, a in host.items():
            t = torch.from_numpy(a)
            if self.is_gpu:
                t = t.pin_memory()
            if dst is not None:
                dst[k].copy_(t, non_blocking=True)
                out[k] = dst[k]
            else:
                out[k] = t.to(self.device, non_blocking=True)
        return out

    # ------------------------------------------------------------ forward
    def _forward_sample(self, meta: StepMeta, mask_rows: torch.Tensor) -> torch.Tensor:
        if meta.decode:
            if self.fused_decode and meta.tokens.numel() <= 64:
                logits = self.model.forward_decode_fused(meta, self.kv.k, self.kv.v, self.attn_ws,
                                                         self.scratch, self.attn_split_keys)
            else:
                logits = self.model.forward_decode(meta, self.kv.k, self.kv.v, self.attn_ws)
            logits = logits[: mask_rows.numel()]
        else:
            hid = self.model.forward(meta, self.kv.k, self.kv.v, self.attn_ws)
            logits = self.model.logits(hid)
        if self.tp.world == 1:
            return ops.masked_argmax(logits, self.masks, mask_rows)
        return self._tp_argmax(logits, mask_rows)

    def _tp_argmax(self, logits: torch.Tensor, mask_rows: torch.Tensor) -> torch.Tensor:
        """Vocab-parallel masked argmax (D5): this rank's masked argmax over its
        vocab slice, then one combine - the custom all-reduce's argmax kernel
        on GPUs (one 64-bit record per row and rank), all_gather otherwise."""
        V = self.weights.v
        lo = self.tp.rank * V
        if getattr(self, "_local_mask", None) is None:
            assert lo % 32 == 0, "vocab shard must start on a mask word"
            w0 = lo // 32
            self._local_mask = self.masks[:, w0:w0 + (V + 31) // 32].contiguous()
        idx = ops.masked_argmax(logits, self._local_mask, mask_rows)
        if self.tp.car is not None and logits.is_cuda and self.tp.car.argmax_fits(lo, V):
            if logits.dtype != torch.float32:
                logits = logits.float()
            return self.tp.car.argmax(logits, idx, lo)
        import torch.distributed as dist
        val = logits.float().gather(1, idx.clamp(min=0).long()[:, None])[:, 0]
        val = torch.where(idx >= 0, val, torch.full_like(val, -float("inf")))
        pair = torch.stack([val, (idx + lo).float()], dim=1)  # idx < 2^24 exact in fp32
        gathered = [torch.empty_like(pair) for _ in range(self.tp.world)]
        dist.all_gather(gathered, pair, group=self.tp.group)
        allp = torch.stack(gathered, 0)  # [W, B, 2]
        best = allp[:, :, 0].argmax(0)
        return allp[best, torch.arange(allp.shape[1], device=allp.device), 1].to(torch.int32)

    def _build_meta(self, dev: dict, max_q: int, max_ctx: int, decode: bool) -> StepMeta:
        return StepMeta(tokens=dev["tokens"], positions=dev["positions"], slots=dev["slots"],
                        cu_q=dev["cu_q"], ctx_lens=dev["ctx_lens"], block_tables=dev["block_tables"],
                        logit_idx=dev["logit_idx"], max_q=max_q, max_ctx=max_ctx, decode=decode)

    CTX_BUCKET = 256

    def _decode_graph(self, B_pad: int, T_pad: int, ctx: int | None = None) -> dict:
        """Captured decode step per (sequence, token, context) bucket; the
        context bucket sizes the attention split grid (no empty splits)."""
        ctx = ctx or self.max_seq_len
        key = (B_pad, T_pad, ctx)
        g = self._graphs.get(key)
        if g is not None:
            return g
        # all int32 metadata lives in ONE device buffer, int64 logit rows in a
        # second; the graph's first node fills both from the pinned staging ring
        shapes = {"tokens": (T_pad,), "positions": (T_pad,), "slots": (T_pad,),
                  "cu_q": (B_pad + 1,), "ctx_lens": (B_pad,),
                  "block_tables": (B_pad, self.max_blocks), "mask_rows": (B_pad,),
                  "src": (T_pad,), "row_slot": (B_pad,)}
        n32 = sum(int(np.prod(v)) for v in shapes.values())
        L = max(16, B_pad)
        assert n32 <= self._n32_max and L <= self._n64_max and B_pad <= 256
        d32 = torch.zeros(n32, dtype=torch.int32, device=self.device)
        d64 = torch.zeros(L, dtype=torch.int64, device=self.device)
        dev, off = {}, 0
        for k, shp in shapes.items():
            n = int(np.prod(shp))
            dev[k] = d32[off:off + n].view(*shp)
            off += n
        dev["slots"].fill_(-1)
        dev["src"].fill_(-1)
        dev["row_slot"].fill_(self.max_seqs)
        dev["logit_idx"] = d64
        meta = self._build_meta(dev, self.max_decode_q, ctx, True)
        # warm up (allocator + kernels) on a side stream, then capture; the
        # warm-up runs the body only (the I/O nodes would advance the counter)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            out = self._step_body(meta, dev)
        torch.cuda.current_stream(self.device).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        k = ops._lib.kernels()
        # thread-local capture: the other GPU worker thread keeps running
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            st = ops._lib.stream_ptr(d32)
            src_off = dev["src"].data_ptr() // 4 - d32.data_ptr() // 4
            ops._lib.check(k.loqa_step_fetch(
                ops._lib.ptr(d32), self._stage32.data_ptr(), n32, self._n32_max, ops._lib.ptr(d64),
                self._stage64.data_ptr(), L, self._n64_max, ops._lib.ptr(self._step_ctr), T_pad,
                src_off, ops._lib.ptr(self.last_tok), st), "step_fetch")
            out = self._step_body(meta, dev, device_io=True)
            ops._lib.check(k.loqa_step_publish(
                ops._lib.ptr(out), B_pad, self._res_ring.data_ptr(), self._res_ring.shape[1],
                self.RES_SLOTS, ops._lib.ptr(self._step_ctr), ops._lib.ptr(dev["row_slot"]),
                ops._lib.ptr(self.last_tok), st), "step_publish")
        g = {"graph": graph, "dev": dev, "out": out, "shapes": shapes, "n32": n32, "L": L}
        self._graphs[key] = g
        return g

    def _stage(self, g: dict) -> dict:
        """Numpy views of the staging slot of the NEXT step graph launch, in
        graph ``g``'s metadata layout."""
        slot = self._step_no % 2
        hn, out, off = self._stage32[slot].numpy(), {}, 0
        for k, shp in g["shapes"].items():
            n = int(np.prod(shp))
            out[k] = hn[off:off + n].reshape(shp)
            off += n
        out["logit_idx"] = self._stage64[slot].numpy()[: g["L"]]
        return out

    def _replay(self, g: dict) -> int:
        """Launch a step graph whose staging slot is filled; returns the result
        ring slot its sampled tokens will land in."""
        rslot = self._step_no % self.RES_SLOTS
        g["graph"].replay()
        # wraps like the device counter (step_publish): 2 staging x RES_SLOTS
        self._step_no = (self._step_no + 1) % (2 * self.RES_SLOTS)
        return rslot

    def _step_body(self, meta: StepMeta, dev: dict, device_io: bool = False) -> torch.Tensor:
        """One captured decode step: tokens whose ``src`` >= 0 are taken from
        the device-resident last sampled token of that sequence slot (the
        pipelined decode launches a step before the host has seen the previous
        step's tokens), then forward + masked argmax, then each row's sampled
        token is stored under its sequence slot (``row_slot``; padding rows
        write a trash slot). ``device_io``: the graph's fetch / publish nodes
        do the gather and the store (LLMEngine._decode_graph)."""
        if device_io:
            return self._forward_sample(meta, dev["mask_rows"])
        src = dev["src"]
        # (a failed step's negative sentinel never becomes an embedding index)
        tok = torch.where(src >= 0, self.last_tok[src.clamp(min=0).long()].clamp(min=0),
                          dev["tokens"])
        meta = StepMeta(tokens=tok, positions=meta.positions, slots=meta.slots, cu_q=meta.cu_q,
                        ctx_lens=meta.ctx_lens, block_tables=meta.block_tables,
                        logit_idx=meta.logit_idx, max_q=meta.max_q, max_ctx=meta.max_ctx,
                        decode=meta.decode)
        out = self._forward_sample(meta, dev["mask_rows"])
        self.last_tok.index_copy_(0, dev["row_slot"].long(), out[: dev["row_slot"].numel()])
        return out

    def warmup_graphs(self) -> int:
        """Capture every decode-step graph bucket up front (sequence x token x
        context buckets). Serving then never captures: a capture on one worker
        thread while another thread issues HIP calls can be invalidated, and a
        first-time capture would stall that step by tens of ms."""
        if not self.use_graphs:
            return 0
        if self.tp.world > 1:
            # the captures' warm-up runs collectives: every rank must arrive
            # here before any of them spins on a peer (the leader's STT warm-up
            # can take longer than a bounded collective wait)
            import torch.distributed as dist
            dist.barrier(group=self.tp.group)
        n = 0
        b_max = _bucket(max(1, self.max_seqs), self.SEQ_BUCKETS)
        for b in self.SEQ_BUCKETS:
            if b > b_max:
                break
            t_min = ops.mpad_for(min(self.step_tokens, b // 2 + 1))   # T >= B > b/2
            t_max = ops.mpad_for(min(self.step_tokens, b * self.max_decode_q))
            for t in ops.MPADS:
                if t > t_max:
                    break
                if t < t_min:
                    continue
                for c in range(self.CTX_BUCKET, self.max_seq_len + self.CTX_BUCKET, self.CTX_BUCKET):
                    self._decode_graph(b, t, min(c, self.max_seq_len))
                    n += 1
        self._graphs_frozen = True
        return n

    # ------------------------------------------------------------ generate
    def submit(self, req: GenRequest) -> GenRequest:
        req.seq_id = self._next_id
        self._next_id += 1
        req.grammar = GrammarState(self.grammar, req.schema)
        start = req.grammar.start()
        req.feed = list(req.prompt) + start
        if req.on_tokens is not None and start:
            req.on_tokens(list(start))
        req.t_submit = time.perf_counter()
        hit = self.kv.pool.add_seq(req.seq_id, req.feed)
        if hit < 0:
            raise RuntimeError("duplicate sequence id")
        self.stats["prefix_hit_tokens"] += hit
        req.feed = req.feed[hit:]
        req._prompt_full = list(req.prompt) + req.grammar.emitted  # type: ignore[attr-defined]
        return req

    def _commit(self, r: GenRequest, t: int, now: float) -> list[int]:
        """Consume one sampled token of ``r``: grammar advance, streaming hook,
        completion. Returns the forced tokens that follow it."""
        if r.t_first == 0.0:
            r.t_first = now
            if getattr(r, "inline", False):   # prompt fed through decode steps
                self.stats["prefill_tokens"] += r.inline   # type: ignore[attr-defined]
                self.kv.pool.cache_prefix(r.seq_id, r._prompt_full)  # type: ignore[attr-defined]
        if t < 0:
            if self.tp.world > 1 and t == ERR_TOKEN:
                raise CollectiveError(f"TP rank {self.tp.rank}: a collective timed out "
                                      "(a peer rank is gone or hung)")
            raise RuntimeError(f"no token allowed for sequence {r.seq_id} (sampled {t})")
        r.token_times.append(now)
        r.steps += 1
        forced = r.grammar.advance(int(t))
        self.stats["sampled_tokens"] += 1
        self.stats["forced_tokens"] += len(forced)
        if r.on_tokens is not None:
            try:
                r.on_tokens([int(t)] + forced)
            except Exception:  # noqa: BLE001 - a consumer's hook never reaches the scheduler
                log.exception("on_tokens hook of sequence %d failed", r.seq_id)
        if r.grammar.done:
            r.done = True
            r.t_done = now
            r.output = r.grammar.text()
            r.feed = []
            if self._pl is not None:
                self._pl.release(r)
            if r.on_done is not None:
                r.on_done(r)
            elif self._on_done is not None:
                self._on_done(r)
        else:
            r.feed = [int(t)] + forced
        return forced

    def _bucket_seqs(self, B: int) -> int:
        return _bucket(B, self.SEQ_BUCKETS)

    def _sample_and_advance(self, live: list[GenRequest], nxt: np.ndarray, now: float,
                            carry: list[bool] | None = None) -> None:
        for i, (r, t) in enumerate(zip(live, nxt.tolist())):
            if carry is not None and carry[i]:
                continue  # long forced run split across steps: logits of this step unused
            self._commit(r, int(t), now)

    def prefill(self, reqs: list[GenRequest]) -> None:
        """Run the prompts (chunked) and sample each sequence's first token."""
        if getattr(self.weights, "compact", False):
            return self._prefill_fused(reqs)
        i = 0
        while i < len(reqs):
            batch, T = [], 0
            while i < len(reqs) and (not batch or T + len(reqs[i].feed) <= self.prefill_chunk):
                batch.append(reqs[i])
                T += len(reqs[i].feed)
                i += 1
            feeds = [r.feed for r in batch]
            max_q, max_ctx, host = self._meta(batch, feeds, decode=False)
            rows = np.array([r.grammar.mask_row() for r in batch], np.int32)
            host["mask_rows"] = rows
            dev = self._to_device(host)
            meta = self._build_meta(dev, max_q, max_ctx, False)
            nxt = self._forward_sample(meta, dev["mask_rows"]).cpu().numpy()
            self.stats["prefill_tokens"] += T
            for r in batch:
                self.kv.pool.cache_prefix(r.seq_id, r._prompt_full)  # type: ignore[attr-defined]
            self._sample_and_advance(batch, nxt, time.perf_counter())

    PREFILL_CHUNK_FUSED = 64

    def _prefill_fused(self, reqs: list[GenRequest]) -> None:
        """Prefill through the fused decode GEMMs (compact single-copy weights):
        each prompt in <= 64-token chunks (one weight pass per chunk; attention
        falls back to the varlen flash kernel past the decode kernel's row
        limit). Prompts mostly hit the prefix cache, so a request typically
        costs one chunk."""
        C = self.PREFILL_CHUNK_FUSED
        for r in reqs:
            feed = r.feed
            nxt = None
            for c0 in range(0, len(feed), C):
                chunk = feed[c0:c0 + C]
                T_pad = ops.mpad_for(len(chunk))
                max_q, max_ctx, host = self._meta([r], [chunk], True, 1, T_pad)
                host["mask_rows"] = np.array([r.grammar.mask_row()], np.int32)
                dev = self._to_device(host)
                meta = self._build_meta(dev, max_q, max_ctx, True)
                nxt = self._forward_sample(meta, dev["mask_rows"])
            self.stats["prefill_tokens"] += len(feed)
            self.kv.pool.cache_prefix(r.seq_id, r._prompt_full)  # type: ignore[attr-defined]
            self._sample_and_advance([r], nxt.cpu().numpy(), time.perf_counter())

    def decode_step(self, live: list[GenRequest]) -> None:
        """One decode step over (a budgeted subset of) ``live``: at most
        ``step_tokens`` tokens in total and ``max_decode_q`` per sequence; a
        sequence fed only part of its pending tokens carries the rest (its
        logits this step are unused), one left out entirely waits a step."""
        plan = plan_step_mpad if MPAD_PLAN else plan_step
        take = plan([len(r.feed) for r in live], self.step_tokens, self.max_decode_q, self._rr)
        self._rr = (self._rr + self.step_tokens) % len(live) if len(live) > self.step_tokens else 0
        step, feeds, carry = [], [], []
        for r, n in zip(live, take):
            if n == 0:
                continue
            f = r.feed
            step.append(r)
            feeds.append(f[:n])
            carry.append(n < len(f))
            if n < len(f):
                r.feed = f[n:]
        live = step
        t0 = time.perf_counter()
        B = len(live)
        T = sum(len(f) for f in feeds)
        rows = np.array([r.grammar.mask_row() for r in live], np.int32)
        if self.use_graphs:
            B_pad = _bucket(B, self.SEQ_BUCKETS)
            T_pad = ops.mpad_for(T)
            ctx = max(self.kv.pool.seq_len(r.seq_id) + len(f) for r, f in zip(live, feeds))
            C = min(self.max_seq_len, -(-ctx // self.CTX_BUCKET) * self.CTX_BUCKET)
            g = self._graphs.get((B_pad, T_pad, C))
            if g is None and self._graphs_frozen:
                g = False                 # uncaptured shape while serving: eager
            elif g is None:
                g = self._decode_graph(B_pad, T_pad, C)
        if self.use_graphs and g is not False:
            hb = self._stage(g)
            self._meta(live, feeds, True, B_pad, T_pad, out=hb)
            hb["mask_rows"].fill(0)
            hb["mask_rows"][:B] = rows
            hb["src"].fill(-1)
            hb["row_slot"].fill(self.max_seqs)
            t1 = time.perf_counter()
            rslot = self._replay(g)
            t15 = time.perf_counter()
            torch.cuda.current_stream(self.device).synchronize()
            nxt = self._res_ring[rslot, :B].numpy().copy()
            t2 = time.perf_counter()
            self.stats["host_pre_s"] += t1 - t0
            self.stats["replay_call_s"] += t15 - t1
            self.stats["gpu_wait_s"] += t2 - t1
        else:
            max_q, max_ctx, host = self._meta(live, feeds, True, B, ops.mpad_for(T))
            host["mask_rows"] = rows
            dev = self._to_device(host)
            meta = self._build_meta(dev, max_q, max_ctx, True)
            nxt = self._forward_sample(meta, dev["mask_rows"]).cpu().numpy()
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += T
        t3 = time.perf_counter()
        self._sample_and_advance(live, nxt, t3, carry)
        self.stats["host_post_s"] += time.perf_counter() - t3

    # --------------------------------------------- continuous batching
    def start(self, stream_priority: int = 0) -> None:
        """Start the scheduler thread: requests submitted with ``submit_batch``
        join the running decode batch at the next step boundary (their prompts
        are prefilled first), so utterances arriving while others decode share
        every weight read of the decode steps."""
        if getattr(self, "_sched", None) is not None:
            return
        from ..utils.gil import tune_switch_interval
        tune_switch_interval()
        self._inbox: queue.Queue = queue.Queue()
        self._running = True
        self._sched = threading.Thread(target=self._schedule, args=(stream_priority,),
                                       name="llm-scheduler", daemon=True)
        self._sched.start()

    def stop(self) -> None:
        if getattr(self, "_sched", None) is None:
            return
        self._running = False
        self._inbox.put(None)
        self._sched.join(timeout=60)
        self._sched = None

    def submit_batch(self, reqs: list[GenRequest], on_done=None) -> Future:
        """Queue requests for the scheduler; ``on_done(req)`` fires on the
        engine thread as each finishes; the returned future resolves with
        ``reqs`` when all of them are done."""
        self.start()
        fut: Future = Future()
        if getattr(self, "_fatal", None) is not None:
            fut.set_exception(self._fatal)
            return fut
        reqs = list(reqs)
        cap = max(1, self.max_seqs)
        if len(reqs) > cap:
            # admission holds an inbox item until it fits under max_seqs: an
            # oversize item would wait forever, so it goes in max_seqs chunks
            return join_futures([self.submit_batch(reqs[i:i + cap], on_done)
                                 for i in range(0, len(reqs), cap)], reqs)
        self._inbox.put((reqs, on_done, fut))
        if getattr(self, "_fatal", None) is not None:
            self._fail_inbox()         # raced a TP failure: the scheduler is gone
        return fut

    def _fail_inbox(self) -> None:
        while True:
            try:
                it = self._inbox.get_nowait()
            except queue.Empty:
                return
            if it is not None and not it[2].done():
                it[2].set_exception(self._fatal)

    def _schedule(self, stream_priority: int) -> None:
        try:
            if self.is_gpu:
                from ..utils.streams import placed_stream
                torch.cuda.set_device(self.device)
                torch.cuda.set_stream(placed_stream(self.device, "llm", stream_priority))
        except Exception as e:  # noqa: BLE001 - never leave submitters waiting
            self._fatal = e
            while True:
                try:
                    it = self._inbox.get_nowait()
                except queue.Empty:
                    return
                if it is not None and not it[2].done():
                    it[2].set_exception(e)
        live: list[GenRequest] = []
        prefilling: list[GenRequest] = []   # chunked prompts not yet through (chunk_prefill)
        cells: dict[int, list] = {}   # id(cell) -> [remaining, future, reqs]
        # inbox items not yet admitted: at most max_seqs sequences are live or
        # prefilling at once (the KV pool and the captured graph buckets are
        # sized for that many)
        waiting: list[tuple] = []
        cap = max(1, self.max_seqs)
        if self.pipelined:
            from .llm_pipeline import DecodePipeline
            self._pl = DecodePipeline(self)
        pl = self._pl
        t_end = 0.0
        while self._running:
            idle = not live and not waiting and not prefilling
            try:
                # inside the try: a leader's heartbeat check or control-ring
                # publish raises CollectiveError here, and that must reach the
                # fail-all + _tp_fail path below (an idle hub's follower death)
                items = self._next_items(idle)
                if items is None:          # TP follower: the leader stopped
                    break
                waiting += [it for it in items if it is not None]
                new: list[GenRequest] = []
                active = len(live) + len(prefilling)
                while waiting and active + len(new) + len(waiting[0][0]) <= cap:
                    reqs, cb, fut = waiting.pop(0)
                    if not reqs:
                        fut.set_result(reqs)
                        continue
                    cell = [len(reqs), fut, reqs]
                    with self._cells_lock:
                        cells[id(cell)] = cell
                    for r in reqs:
                        r.on_done = self._completion(cb, cell, cells)
                        self.submit(r)
                    new += reqs
                if new and self.inline_prefill > 0:
                    inl = [r for r in new if len(r.feed) <= self.inline_prefill]
                    for r in inl:
                        r.inline = len(r.feed)   # type: ignore[attr-defined]
                        if pl is not None:
                            pl.admit(r)
                    live += inl
                    new = [r for r in new if len(r.feed) > self.inline_prefill]
                if new and self.chunk_prefill > 0 and not getattr(self.weights, "compact", False):
                    # (compact weights keep only the fused decode copies: their
                    # prompts go through _prefill_fused below, not a mixed pass)
                    for r in new:
                        r.chunk_total = len(r.feed)   # type: ignore[attr-defined]
                    prefilling += new
                    new = []
                if new:
                    self._prefill_timed(new)
                    live = [r for r in live if not r.done]
                    joined = [r for r in new if not r.done]
                    if pl is not None:
                        for r in joined:
                            pl.admit(r)
                    live += joined
                if prefilling:
                    t0 = time.perf_counter()
                    live += self._mixed_step([r for r in live if not r.done], prefilling)
                    prefilling = [r for r in prefilling
                                  if not getattr(r, "chunk_done", False) and not r.done]
                    live = [r for r in live if not r.done]
                    t_end = time.perf_counter()
                    self.stats["mixed_s"] = self.stats.get("mixed_s", 0.0) + t_end - t0
                elif live:
                    t0 = time.perf_counter()
                    if t_end:
                        self.stats["sched_s"] += t0 - t_end   # loop work between steps
                    if pl is not None:
                        pl.pump(live)
                    else:
                        self.decode_step(live)
                    t_end = time.perf_counter()
                    self.stats["decode_s"] += t_end - t0
                    live = [r for r in live if not r.done]
                    if not live and pl is not None:
                        pl.drain()          # speculative steps of finished sequences
                else:
                    t_end = 0.0
            except Exception as e:  # noqa: BLE001 - fail every waiting batch loudly
                if isinstance(e, CollectiveError):
                    log.error("%s", e)
                else:
                    log.exception("LLM scheduler iteration failed")
                # in-flight pipelined steps still write KV into their sequences'
                # blocks: let them finish before the blocks go back
                if pl is not None:
                    pl.abort()
                    self._free_seq_slots = list(range(self.max_seqs))
                with self._cells_lock:
                    for cell in list(cells.values()):
                        if not cell[1].done():
                            cell[1].set_exception(e)
                        for r in cell[2]:
                            if not r.done:
                                r.done = True
                                try:
                                    self.kv.pool.free_seq(r.seq_id)
                                except KeyError:
                                    pass        # never registered
                    cells.clear()
                for _, _, fut in waiting:
                    if not fut.done():
                        fut.set_exception(e)
                live, waiting, prefilling = [], [], []
                if self.tp_ctl is not None:
                    # lock-step TP: the ranks' scheduler states may now differ
                    # (this rank reset, the others did not), so the group
                    # cannot continue - stop it and report
                    self._tp_fail(e)
                    break

        if self.tp_ctl is not None and self.tp_ctl.leader:
            try:
                self.tp_ctl.publish([], stop=True, timeout_s=2.0)
            except Exception as e:  # noqa: BLE001 - a follower is gone: nothing to stop
                log.warning("TP stop record not delivered: %s", e)

    def _tp_fail(self, e: Exception) -> None:
        """The TP group failed: later submissions fail at once, followers get
        the stop record, and the owner's ``on_tp_failure`` hook (the hub's
        degradation to a single-GPU engine) runs."""
        self._fatal = e if isinstance(e, CollectiveError) else CollectiveError(
            f"TP group stopped after a scheduler failure on rank {self.tp.rank}: {e}")
        self._running = False
        self.stats["tp_failed"] = 1
        self._fail_inbox()         # submissions that raced the failure
        hook = getattr(self, "on_tp_failure", None)
        if hook is not None:
            try:
                hook(self._fatal)
            except Exception:  # noqa: BLE001
                log.exception("on_tp_failure hook failed")

    def _next_items(self, idle: bool) -> list | None:
        """This scheduler iteration's new inbox items (blocking when idle).
        TP leader: also publishes them; TP follower: replays the leader's
        record instead of reading an inbox (None once the leader stopped)."""
        ctl = self.tp_ctl
        if ctl is None:
            items = [self._inbox.get()] if idle else []   # idle: block for work
            while True:
                try:
                    items.append(self._inbox.get_nowait())
                except queue.Empty:
                    break
            return items
        if ctl.leader:
            items = []
            while True:
                # idle: block for work, waking up to check the followers' heartbeats
                self._check_followers()
                if not idle:
                    break
                try:
                    items.append(self._inbox.get(timeout=0.25))
                    break
                except queue.Empty:
                    continue
            while True:
                try:
                    items.append(self._inbox.get_nowait())
                except queue.Empty:
                    break
            try:
                ctl.publish([[(r.prompt, r.schema) for r in it[0]] for it in items if it is not None],
                            timeout_s=self.tp_follower_timeout)
            except RuntimeError as e:
                for it in items:
                    if it is not None and not it[2].done():
                        it[2].set_exception(CollectiveError(str(e)))
                raise CollectiveError(str(e)) from e
            return items
        while True:
            rec, stop = ctl.recv(timeout_s=0.5)
            if stop:
                self._running = False
                return None
            if rec is not None:
                break
        self.stats["tp_records"] = self.stats.get("tp_records", 0) + 1
        return [([GenRequest(list(p), sch) for p, sch in batch], None, Future()) for batch in rec]

    # a follower whose heartbeat is this old is gone (its process died)
    tp_follower_timeout = float(os.environ.get("LOQA_TP_FOLLOWER_TIMEOUT", "10"))

    def _check_followers(self) -> None:
        lost = self.tp_ctl.lost_followers(self.tp_follower_timeout)
        if lost:
            raise CollectiveError(f"TP followers {lost} stopped heart-beating "
                                  f"for {self.tp_follower_timeout:.0f} s")

    def follow(self, stream_priority: int = 0) -> None:
        """TP follower rank: run the scheduler on the calling thread, replaying
        the leader's iterations until it stops."""
        assert self.tp_ctl is not None and not self.tp_ctl.leader
        from ..utils.gil import tune_switch_interval
        tune_switch_interval()
        self._inbox = queue.Queue()
        self._running = True
        self._schedule(stream_priority)

    MIXED_SPLIT = os.environ.get("LOQA_MIXED_SPLIT_ATTN", "1") != "0"
    CHUNK_FIT = os.environ.get("LOQA_CHUNK_FIT", "0") == "1"

    def _mixed_split(self, kinds: list[int], feeds: list[list[int]], host: dict):
        """(live sequences, their rows, longest feed, longest context) when a
        mixed pass's attention can run as grouped decode attention for the
        leading live sequences + flash prefill for the prompt chunks (adds
        ``cu_tail`` to ``host``), else None."""
        nd = sum(1 for k in kinds if k == 0)
        if (not self.MIXED_SPLIT or nd == 0 or nd == len(kinds)
                or any(k != 0 for k in kinds[:nd])):
            return None
        dq = max(len(f) for f in feeds[:nd])
        cu = host["cu_q"]
        rd = int(cu[nd])
        ws = self.attn_ws            # None on the CPU (reference attention)
        if dq > self.max_decode_q or (ws is not None and (
                rd > ws.max_tokens or nd * self.weights.hkv > ws.counters.numel())):
            return None
        host["cu_tail"] = (cu[nd:len(kinds) + 1] - cu[nd]).astype(np.int32)
        return nd, rd, dq, max(int(host["ctx_lens"][:nd].max()), 1)

    def _mixed_step(self, live: list[GenRequest], prefilling: list[GenRequest]
                    ) -> list[GenRequest]:
        """One pass over every live sequence's whole next feed plus the next
        chunk (``chunk_prefill`` tokens) of the waiting prompts, on the prompt
        pass's hand-written GEMMs: the chunk shares the decode step's weight
        reads. The live sequences sample as in a decode step; a prompt whose
        last chunk went in samples its first token and joins. With no live
        sequence the prompts go in whole (one pass). The pipelined decode is
        drained first (its in-flight steps retired), so every feed is
        host-known. Returns the requests that finished their prompt."""
        pl = self._pl
        t_a = time.perf_counter()
        if pl is not None:
            pl.drain()
            live = [r for r in live if not r.done]
        t_b = time.perf_counter()
        rows: list[GenRequest] = []
        feeds: list[list[int]] = []
        kinds: list[int] = []          # 0 live sequence, 1 last prompt chunk, 2 prompt chunk
        for r in live:
            f = r.pl_host if pl is not None else r.feed   # type: ignore[attr-defined]
            if f:
                rows.append(r)
                feeds.append(list(f))
                kinds.append(0)
        budget = self.chunk_prefill if rows else self.prefill_chunk
        if rows and self.CHUNK_FIT:
            # the pass's row count (live feeds + chunk) = the chunk size, a
            # multiple of 64: the prompt GEMMs' row blocks carry no padding
            budget = max(64, budget - sum(len(f) for f in feeds))
        for r in prefilling:
            if budget <= 0:
                break
            n = min(len(r.feed), budget)
            rows.append(r)
            feeds.append(r.feed[:n])
            kinds.append(1 if n == len(r.feed) else 2)
            budget -= n
        max_q, max_ctx, host = self._meta(rows, feeds, decode=False)
        host["mask_rows"] = np.array([r.grammar.mask_row() for r in rows], np.int32)
        split = self._mixed_split(kinds, feeds, host)
        dev = self._to_device(host)
        meta = self._build_meta(dev, max_q, max_ctx, False)
        if split is not None:
            meta.split = split + (dev["cu_tail"],)
            self.stats["mixed_split"] = self.stats.get("mixed_split", 0) + 1
        t_c = time.perf_counter()
        nxt = self._forward_sample(meta, dev["mask_rows"])
        t_d = time.perf_counter()
        nxt = nxt.cpu().numpy()
        t_e = time.perf_counter()
        # where a mixed pass's wall time goes: draining the pipelined steps,
        # host metadata, host-side launches, waiting for the GPU
        for k, v in (("mixed_drain_s", t_b - t_a), ("mixed_meta_s", t_c - t_b),
                     ("mixed_launch_s", t_d - t_c), ("mixed_wait_s", t_e - t_d)):
            self.stats[k] = self.stats.get(k, 0.0) + v
        now = time.perf_counter()
        joined: list[GenRequest] = []
        n_dec = 0
        for r, f, k, t in zip(rows, feeds, kinds, nxt.tolist()):
            if k == 2:                 # a prompt's inner chunk: logits unused
                r.feed = r.feed[len(f):]
                continue
            if k == 1:                 # the prompt is in: first sampled token
                r.feed = []
                r.chunk_done = True    # type: ignore[attr-defined]
                self.stats["prefill_tokens"] += r.chunk_total   # type: ignore[attr-defined]
                self.kv.pool.cache_prefix(r.seq_id, r._prompt_full)  # type: ignore[attr-defined]
                self._commit(r, int(t), now)
                if not r.done:
                    if pl is not None:
                        pl.admit(r)
                    joined.append(r)
                continue
            n_dec += len(f)
            forced = self._commit(r, int(t), now)
            if pl is not None and not r.done:
                r.pl_host = [int(t)] + forced   # type: ignore[attr-defined]
        self.stats["mixed_steps"] = self.stats.get("mixed_steps", 0) + 1
        self.stats["decode_tokens"] += n_dec
        return joined

    def _prefill_timed(self, reqs: list[GenRequest]) -> None:
        t0 = time.perf_counter()
        self.prefill(reqs)
        self.stats["prefill_s"] += time.perf_counter() - t0
        self.stats["prefill_passes"] = self.stats.get("prefill_passes", 0) + 1

    def _completion(self, cb, cell, cells):
        def done(r: GenRequest) -> None:   # scheduler or prefill thread
            self.kv.pool.free_seq(r.seq_id)
            if cb is not None:
                try:
                    cb(r)
                except Exception:  # noqa: BLE001 - the caller's callback, not the scheduler's
                    log.exception("completion callback of sequence %d failed", r.seq_id)
            with self._cells_lock:
                cell[0] -= 1
                last = cell[0] == 0
                if last:
                    cells.pop(id(cell), None)
            if last and not cell[1].done():
                cell[1].set_result(cell[2])
        return done

    def generate(self, reqs: list[GenRequest], on_done=None) -> list[GenRequest]:
        """Run the requests to completion. ``on_done(req)`` fires as soon as each
        sequence finishes (its command queue can start while others decode)."""
        self._on_done = on_done
        t0 = time.perf_counter()
        for r in reqs:
            self.submit(r)
        self.prefill(reqs)
        t1 = time.perf_counter()
        live = [r for r in reqs if not r.done]
        while live:
            self.decode_step(live)
            live = [r for r in live if not r.done]
        self.stats["prefill_s"] += t1 - t0
        self.stats["decode_s"] += time.perf_counter() - t1
        for r in reqs:
            self.kv.pool.free_seq(r.seq_id)
        return reqs
