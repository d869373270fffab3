"""JSON-schema-constrained decoding with jump-forward.

The reference asks the LLM for a JSON object and then digs it out of free text
(``command_parser.go:269-303``, ``:413-473``), falling back to a second call on
failure. Here the schema of ``buildMultiCommandPrompt`` (``command_parser.go:379-410``)
is compiled into a token-level program:

* ``Lit``    - structural text (keys, quotes, braces): forced, never sampled. The
               forced tokens are appended to the *next* forward pass of that
               sequence ("jump-forward"), so a key costs no decode step.
* ``Choice`` - enum values (intent, is_multi): masked argmax over a token trie.
* ``Free``   - JSON string bodies (device, location, response): any string-safe
               token, closed by sampling ``"`` or forced at ``max_tokens``.
* ``Digits`` - fixed-width digits (confidence 0.xx).

Every decision point maps to one row of a packed uint32 mask table resident on
the GPU, consumed by the fused masked-argmax kernel (K15). The number of command
objects is fixed by the compound-utterance splitter, so the output always
parses and has the intended command count - with random-init weights this is
what makes the multi-command benchmark meaningful.
"""
from __future__ import annotations

import torch

from ..ops.reference import pack_mask
from .tokenizer import SyntheticTokenizer

INTENTS = ["turn_on", "turn_off", "greeting", "question", "unknown"]


class Lit:
    __slots__ = ("text",)

    def __init__(self, text: str):
        self.text = text


class Choice:
    __slots__ = ("options", "name")

    def __init__(self, name: str, options: list[str]):
        self.name, self.options = name, options


class Free:
    __slots__ = ("max_tokens", "name", "min_tokens")

    def __init__(self, name: str, max_tokens: int, min_tokens: int = 0):
        self.name, self.max_tokens, self.min_tokens = name, max_tokens, min_tokens


class Digits:
    __slots__ = ("n",)

    def __init__(self, n: int):
        self.n = n


def multi_command_schema(n_commands: int, *, max_entity_tokens: int = 3,
                         max_response_tokens: int = 12, max_combined_tokens: int = 16,
                         min_response_tokens: int = 0) -> list:
    """Segments of the multi-command response object with exactly n commands."""
    segs: list = [Lit('{"is_multi": '), Choice("is_multi", ["true", "false"]), Lit(', "commands": [')]
    for i in range(n_commands):
        segs += [Lit(('' if i == 0 else ', ') + '{"intent": "'), Choice("intent", INTENTS),
                 Lit('", "entities": {"device": "'), Free("device", max_entity_tokens),
                 Lit('", "location": "'), Free("location", max_entity_tokens),
                 Lit('"}, "confidence": 0.'), Digits(2), Lit(', "response": "'),
                 Free("response", max_response_tokens, min_response_tokens), Lit('"}')]
    segs += [Lit('], "combined_response": "'),
             Free("combined_response", max_combined_tokens, min_response_tokens),
             Lit('"}')]
    return segs


def single_command_schema(*, max_entity_tokens: int = 3, max_response_tokens: int = 12) -> list:
    """Segments of the single-command object of ``buildPrompt`` (command_parser.go:195-220)."""
    return [Lit('{"intent": "'), Choice("intent", INTENTS), Lit('", "entities": {"device": "'),
            Free("device", max_entity_tokens), Lit('", "location": "'),
            Free("location", max_entity_tokens), Lit('"}, "confidence": 0.'), Digits(2),
            Lit(', "response": "'), Free("response", max_response_tokens), Lit('"}')]


class _Trie:
    def __init__(self):
        self.children: dict[int, "_Trie"] = {}
        self.terminal = False
        self.row = -1


class GrammarTables:
    """Mask table shared by all sequences of an engine (one GPU copy)."""

    def __init__(self, tok: SyntheticTokenizer, device=None):
        self.tok = tok
        V = tok.vocab_size
        self.quote = tok.token_id('"')
        rows: list[torch.Tensor] = []
        safe = torch.zeros(V, dtype=torch.bool)
        for t in range(tok.n_special, tok.n_real):
            s = tok.token_text(t)
            if s and '"' not in s and "\\" not in s and all(32 <= ord(c) < 127 for c in s):
                safe[t] = True
        free = safe.clone()
        free[self.quote] = True
        self.ROW_FREE = 0
        rows.append(free)
        digits = torch.zeros(V, dtype=torch.bool)
        for c in "0123456789":
            digits[tok.token_id(c)] = True
        self.ROW_DIGIT = 1
        rows.append(digits)
        self.ROW_FREE_OPEN = 2  # string body that may not close yet (min length)
        rows.append(safe)
        # two digits in one token ("95"): a Digits field with >= 2 digits left
        # samples one of these instead of two single digits (one decode step)
        digits2 = torch.zeros(V, dtype=torch.bool)
        for t in range(tok.n_special, tok.n_real):
            s2 = tok.token_text(t)
            if len(s2) == 2 and s2.isdigit():
                digits2[t] = True
        self.ROW_DIGIT2 = 3 if bool(digits2.any()) else -1
        if self.ROW_DIGIT2 >= 0:
            rows.append(digits2)
        # stand-ins for "some allowed token" in GrammarState.predict
        self.generic_free = int(safe.nonzero()[0])
        self.generic_digit = tok.token_id("0")
        self.generic_digit2 = int(digits2.nonzero()[0]) if self.ROW_DIGIT2 >= 0 else -1
        self._rows = rows
        self._tries: dict[tuple, _Trie] = {}
        self._lit_cache: dict[str, list[int]] = {}
        self.device = device
        self._gpu = None

    def literal(self, text: str) -> list[int]:
        ids = self._lit_cache.get(text)
        if ids is None:
            ids = self.tok.encode(text)
            self._lit_cache[text] = ids
        return ids

    def trie(self, options: list[str]) -> _Trie:
        key = tuple(options)
        tr = self._tries.get(key)
        if tr is not None:
            return tr
        tr = _Trie()
        for o in options:
            node = tr
            for t in self.tok.encode(o):
                node = node.children.setdefault(t, _Trie())
            node.terminal = True
        stack = [tr]
        while stack:
            n = stack.pop()
            if n.children:
                m = torch.zeros(self.tok.vocab_size, dtype=torch.bool)
                m[list(n.children)] = True
                n.row = len(self._rows)
                self._rows.append(m)
                stack.extend(n.children.values())
        self._tries[key] = tr
        self._gpu = None
        return tr

    def mask_table(self, device=None) -> torch.Tensor:
        device = device or self.device
        want = torch.device(device or "cpu")
        if self._gpu is None or self._gpu.shape[0] != len(self._rows) or self._gpu.device != want:
            self._gpu = pack_mask(torch.stack(self._rows)).to(device or "cpu")
        return self._gpu

    def allowed(self, row: int) -> torch.Tensor:
        return self._rows[row]


class GrammarState:
    """Per-sequence cursor over a compiled schema."""

    def __init__(self, tables: GrammarTables, schema: list):
        self.t = tables
        self.segs = schema
        self.i = 0
        self.node: _Trie | None = None
        self.count = 0
        self.after_free = False
        self.done = False
        self.emitted: list[int] = []
        self.free_steps = 0  # number of sampled (non-forced) tokens

    def start(self) -> list[int]:
        """Forced tokens before the first decision (folded into the prefill)."""
        return self._run_forced()

    def _run_forced(self) -> list[int]:
        out: list[int] = []
        while self.i < len(self.segs):
            s = self.segs[self.i]
            if isinstance(s, Lit):
                text = s.text
                if self.after_free:
                    assert text.startswith('"')
                    text = text[1:]
                    self.after_free = False
                if text:
                    out.extend(self.t.literal(text))
                self.i += 1
                continue
            if isinstance(s, Choice):
                self.node = self.t.trie(s.options)
            self.count = 0
            break
        else:
            self.done = True
        self.emitted.extend(out)
        return out

    def mask_row(self) -> int:
        """Mask-table row for the next sampled token (-1 when finished)."""
        if self.done:
            return -1
        s = self.segs[self.i]
        if isinstance(s, Choice):
            return self.node.row
        if isinstance(s, Free):
            return self.t.ROW_FREE if self.count >= s.min_tokens else self.t.ROW_FREE_OPEN
        return self._digit_row(s)

    def _digit_row(self, s: "Digits") -> int:
        if s.n - self.count >= 2 and self.t.ROW_DIGIT2 >= 0:
            return self.t.ROW_DIGIT2
        return self.t.ROW_DIGIT

    def advance(self, tok: int) -> list[int]:
        """Consume a sampled token; return the forced tokens that follow it."""
        assert not self.done
        self.free_steps += 1
        self.emitted.append(tok)
        s = self.segs[self.i]
        forced: list[int] = []
        if isinstance(s, Choice):
            nxt = self.node.children.get(tok)
            if nxt is None:  # cannot happen with a correct mask; recover deterministically
                nxt = next(iter(self.node.children.values()))
            self.node = nxt
            if not nxt.children:
                self.i += 1
                forced = self._run_forced()
            return forced
        if isinstance(s, Free):
            self.count += 1
            if tok == self.t.quote:
                self.after_free = True
                self.i += 1
                return self._run_forced()
            if self.count >= s.max_tokens:
                self.after_free = True
                self.i += 1
                forced = [self.t.quote]
                self.emitted.append(self.t.quote)
                return forced + self._run_forced()
            return forced
        # Digits: one or two digits per token
        self.count += max(1, len(self.t.tok.token_text(tok)))
        if self.count >= s.n:
            self.i += 1
            forced = self._run_forced()
        return forced

    def text(self) -> str:
        return self.t.tok.decode(self.emitted)

    # ---- speculation support (pipelined decode, LLMEngine._pl_*)
    def fork(self) -> "GrammarState":
        """Cursor copy without the emitted text (segments / tries are shared)."""
        g = GrammarState.__new__(GrammarState)
        g.t, g.segs, g.i, g.node, g.count = self.t, self.segs, self.i, self.node, self.count
        g.after_free, g.done, g.emitted, g.free_steps = self.after_free, self.done, [], 0
        return g

    def is_generic(self, tok: int) -> bool:
        """Whether ``tok`` (about to be consumed) takes the path ``predict``
        assumes: anything but a Free field's closing quote."""
        return self.done or not (isinstance(self.segs[self.i], Free) and tok == self.t.quote)

    def predict(self):
        """(forced tokens, next mask row, done) after the NEXT sampled token,
        for any generic token (see ``is_generic``), or None when the outcome
        depends on which token is sampled (a Choice node with a non-terminal
        child). The pipelined decode feeds these forced tokens before the
        sampled token itself is known."""
        if self.done:
            return None
        s = self.segs[self.i]
        if isinstance(s, Choice):
            if any(c.children for c in self.node.children.values()):
                return None
            tok = next(iter(self.node.children))
        elif isinstance(s, Free):
            tok = self.t.generic_free
        else:
            tok = (self.t.generic_digit2 if self._digit_row(s) == self.t.ROW_DIGIT2
                   else self.t.generic_digit)
        f = self.fork()
        forced = f.advance(tok)
        return forced, f.mask_row(), f.done
