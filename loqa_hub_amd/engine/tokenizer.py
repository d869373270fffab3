"""Deterministic synthetic tokenizer.

There is no network and no tokenizer file in this image, and the models run on
seeded random weights, so the tokenizer only has to be *consistent* (encode ->
ids -> decode round-trips) and produce realistic token counts (~4-5 characters
per token on English text, so the reference's ~1.5 kB parser prompt becomes
~330 tokens as it would with a real BPE). Layout of the id space:

    [specials][256 byte tokens][word/fragment tokens][reserved filler ...]

Encoding is greedy longest-match over the known strings (byte tokens guarantee
coverage); reserved filler ids are never produced by ``encode`` and are
excluded from every grammar mask, but they exist so the embedding/lm-head have
the real vocabulary size of the target model (e.g. 128256 for Llama-3).
"""
from __future__ import annotations

import functools
import re

SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|pad|>", "<|startoftranscript|>", "<|en|>",
            "<|transcribe|>", "<|notimestamps|>", "<|endoftext|>"]

_COMMON = """
the be to of and a in that have i it for not on with he as you do at this but his by from they we
say her she or an will my one all would there their what so up out if about who get which go me when
make can like time no just him know take people into year your good some could them see other than
then now look only come its over think also back after use two how our work first well way even new
want because any these give day most us is are was were been has had did said does doing done please
turn on off lights light lamp music tv television kitchen bedroom living room bathroom office garage
hallway dining main all play stop pause volume up down dim brighten set timer alarm weather today
tomorrow morning evening night hello hi hey good thanks thank okay sure done doing turning turned
switch open close lock unlock temperature degrees percent minutes seconds hours next also after that
voice assistant command parser analyze following respond json object classify only exact format one
intent entities device location etc empty string none if confidence response natural user rules
wants something someone saying asking question unknown unclear unrecognized should be based clear
conversational other text handles compound utterances multiple commands distinct connected break them
separate single return it true false is_multi combined_response combining acknowledging each specific
individual commands contains connected message messages right away will i'll i've ive let me here
turning_on turning_off now lights. rolling back completed sorry couldn't understand hear clearly try
again didn't anything not sure help with what want do having trouble understanding right
""".split()

_FRAGMENTS = [
    "{", "}", "[", "]", ":", ",", '"', "\n", "  ", "    ", "      ", "        ", "\n  ", "\n    ",
    "\n      ", "\n        ", '{"', '"}', '":', '": ', '": "', '",', '", "', '"\n', "},", "}]", "]}",
    "}\n", "},\n", '  "', '    "', '      "', '        "', ', "', '", "', ': "', ', {"', '"}, "',
    '}, {"', '"}],', '], "', ': 0.', ': [', ': {', '": {"', '": [', '": 0.', '"},', '"}]',
    "0.", "1.", "0", "1", "2", "3", "4", "5",
    "6", "7", "8", "9", "00", "95", "90", "85", "80", "75", "50", ".", "!", "?", "'", "-", "_",
    "...", "(", ")", "/", "turn_on", "turn_off", "greeting", "question", "unknown", "true", "false",
    "intent", "entities", "device", "location", "confidence", "response", "commands", "is_multi",
    "combined_response", '"intent"', '"entities"', '"device"', '"location"', '"confidence"',
    '"response"', '"commands"', '"is_multi"', '"combined_response"', "living room", "hey loqa",
    "loqa", "Loqa", "Hey", "OK", "I", "I'm", "I'll", "I've", "You", "The", "Turn", "Turning",
    "Rules", "Voice", "Classify", "Respond", "Analyze", "If", "For", "Only", "\n- ", "- ",
]


@functools.lru_cache(maxsize=8)
def get_tokenizer(vocab_size: int) -> "SyntheticTokenizer":
    return SyntheticTokenizer(vocab_size)


class SyntheticTokenizer:
    def __init__(self, vocab_size: int):
        strings: list[str] = []
        seen: set[str] = set()

        def add(s: str) -> None:
            if s not in seen:
                seen.add(s)
                strings.append(s)

        for s in SPECIALS:
            add(s)
        self.n_special = len(strings)
        self.byte_base = len(strings)
        byte_tokens = []
        for b in range(256):
            s = chr(b) if 32 <= b < 127 else f"<0x{b:02X}>"
            byte_tokens.append(s)
            strings.append(s)  # byte tokens may duplicate fragment text; keep ids fixed
            seen.add(s)
        for f in _FRAGMENTS:
            add(f)
        for w in _COMMON:
            add(w)
            add(" " + w)
            add(w.capitalize())
            add(" " + w.capitalize())
        # every two-digit number is one token, as in Llama-3's BPE (digits are
        # pre-split into runs of up to three); appended last so earlier ids stay
        for n in range(100):
            add(f"{n:02d}")
        # Whisper's previous-text prompt marker (long-form windows), appended
        # after everything else so no earlier id moves
        add("<|startofprev|>")
        if len(strings) > vocab_size:
            raise ValueError(f"vocab_size {vocab_size} too small for the synthetic tokenizer")
        self.n_real = len(strings)
        self.vocab_size = vocab_size
        self.strings = strings + [f"<|reserved_{i}|>" for i in range(vocab_size - len(strings))]
        self.bos = 0
        self.eos = 1
        self.pad = 2
        # lookup: longest-match table (byte tokens win ties for single chars)
        self._lookup: dict[str, int] = {}
        for i in range(self.n_real - 1, self.byte_base - 1, -1):
            s = self.strings[i]
            if not (i < self.byte_base + 256 and s.startswith("<0x")):
                self._lookup[s] = i
        for b in range(32, 127):
            self._lookup[chr(b)] = self.byte_base + b
        self._maxlen = max(len(s) for s in self._lookup)
        self._special_re = re.compile("|".join(re.escape(s) for s in SPECIALS))

    def token_id(self, s: str) -> int:
        if s in SPECIALS:
            return SPECIALS.index(s)
        return self._lookup[s]

    def encode_prompt(self, text: str) -> list[int]:
        """A whole LLM prompt (no chat template for the random-init weights)."""
        return self.encode(text, bos=True)

    def encode(self, text: str, bos: bool = False) -> list[int]:
        out = [self.bos] if bos else []
        pos = 0
        for m in self._special_re.finditer(text):
            out.extend(self._encode_plain(text[pos:m.start()]))
            out.append(SPECIALS.index(m.group(0)))
            pos = m.end()
        out.extend(self._encode_plain(text[pos:]))
        return out

    def _encode_plain(self, text: str) -> list[int]:
        ids = []
        i, n = 0, len(text)
        lk, ml = self._lookup, self._maxlen
        while i < n:
            for L in range(min(ml, n - i), 0, -1):
                tid = lk.get(text[i:i + L])
                if tid is not None:
                    ids.append(tid)
                    i += L
                    break
            else:
                for b in text[i].encode("utf-8"):
                    ids.append(self.byte_base + b)
                i += 1
        return ids

    def decode(self, ids) -> str:
        out = []
        pending = bytearray()
        for t in ids:
            t = int(t)
            if self.byte_base <= t < self.byte_base + 256:
                pending.append(t - self.byte_base)
                continue
            if pending:
                out.append(pending.decode("utf-8", errors="replace"))
                pending.clear()
            if t < self.n_special or t >= self.n_real:
                continue
            out.append(self.strings[t])
        if pending:
            out.append(pending.decode("utf-8", errors="replace"))
        return "".join(out)

    def token_text(self, t: int) -> str:
        if self.byte_base <= t < self.byte_base + 256:
            b = t - self.byte_base
            return chr(b) if 32 <= b < 127 else ""
        return self.strings[t] if self.n_special <= t < self.n_real else ""


# ---------------------------------------------------------------------------
# Real checkpoints: the Hugging Face ``tokenizer.json`` shipped with them
TOKENIZER_FILE = "tokenizer.json"
_BOS_NAMES = ("<|begin_of_text|>", "<s>", "<|startoftext|>")
_EOS_NAMES = ("<|end_of_text|>", "<|eot_id|>", "</s>", "<|endoftext|>")


def find_tokenizer(path: str) -> str | None:
    """``tokenizer.json`` for a checkpoint: ``path`` itself, or the file in
    ``path`` (a checkpoint directory) or beside it (a single safetensors file)."""
    import os
    if not path:
        return None
    if os.path.isfile(path) and os.path.basename(path) == TOKENIZER_FILE:
        return path
    d = path if os.path.isdir(path) else os.path.dirname(os.path.abspath(path))
    f = os.path.join(d, TOKENIZER_FILE)
    return f if os.path.isfile(f) else None


def load_tokenizer(path: str, vocab_size: int) -> "HFTokenizer":
    f = find_tokenizer(path)
    if f is None:
        raise FileNotFoundError(f"no {TOKENIZER_FILE} at or beside {path!r}")
    return HFTokenizer(f, vocab_size)


class HFTokenizer:
    """A checkpoint's own tokenizer (``tokenizers`` library, Rust; the file is
    JSON: nothing in it executes) behind the interface the engines and the
    grammar use (``SyntheticTokenizer``'s): ``encode`` / ``decode``,
    ``token_id`` of a one-token string, and ``token_text`` - the exact text a
    token adds after any other token. ``token_text`` is what the constrained
    decoder concatenates into its JSON, so it must keep a SentencePiece
    token's leading space that ``decode([t])`` alone would strip: every token
    is decoded behind a fixed anchor token and the anchor's text is cut off.
    Special / added tokens and ids past the file's vocabulary have no text
    (the grammar never allows them)."""

    def __init__(self, file: str, vocab_size: int):
        from tokenizers import Tokenizer
        self._t = Tokenizer.from_file(file)
        n = self._t.get_vocab_size(with_added_tokens=True)
        if n > vocab_size:
            raise ValueError(f"{file}: {n} tokens exceed the model's vocabulary of {vocab_size}")
        self.vocab_size = vocab_size
        self.n_special = 0
        self.n_real = n
        self._added = {int(i): t for i, t in self._t.get_added_tokens_decoder().items()}
        self.bos = next((i for i in map(self._t.token_to_id, _BOS_NAMES) if i is not None), None)
        self.eos = next((i for i in map(self._t.token_to_id, _EOS_NAMES) if i is not None), None)
        self._chat = self._chat_template(file)
        # generation_config.json beside the file (Whisper: suppress_tokens)
        import json
        import os
        gc = os.path.join(os.path.dirname(file), "generation_config.json")
        self.generation_config = {}
        if os.path.isfile(gc):
            with open(gc, encoding="utf-8") as fh:
                self.generation_config = json.load(fh)
        anchor = self._anchor()
        a_text = self._t.decode([anchor], skip_special_tokens=False)
        texts = self._t.decode_batch([[anchor, i] for i in range(n)], skip_special_tokens=False)
        self._text = []
        for i, s in enumerate(texts):
            ok = i not in self._added and s.startswith(a_text) and "�" not in s
            self._text.append(s[len(a_text):] if ok else "")
        # text -> id for token_id: a vocabulary piece before a byte-fallback
        # token (SentencePiece "<0x22>" also decodes to '"'; a model emits
        # the piece), then the lowest id
        self._by_text: dict[str, int] = {}
        byte_fb = re.compile(r"<0x[0-9A-Fa-f]{2}>")
        for i in sorted(range(n), key=lambda i: (bool(byte_fb.fullmatch(self._t.id_to_token(i) or "")), i)):
            if self._text[i] and self._text[i] not in self._by_text:
                self._by_text[self._text[i]] = i

    def _chat_template(self, file: str):
        """The checkpoint's chat template (``tokenizer_config.json`` beside
        ``tokenizer.json``), compiled in a sandboxed Jinja environment, or None.
        The reference sends its prompts to Ollama's ``/api/generate`` without
        ``raw``, which wraps them in the model's template; a real instruct
        checkpoint here gets the same (``encode_prompt``)."""
        import json
        import os
        cfg_file = os.path.join(os.path.dirname(file), "tokenizer_config.json")
        if not os.path.isfile(cfg_file):
            return None
        with open(cfg_file, encoding="utf-8") as fh:
            cfg = json.load(fh)
        tpl = cfg.get("chat_template")
        if isinstance(tpl, list):        # named templates: the default one
            tpl = next((t.get("template") for t in tpl if t.get("name") == "default"), None)
        if not isinstance(tpl, str) or not tpl:
            return None
        from jinja2.sandbox import ImmutableSandboxedEnvironment

        def raise_exception(msg):
            raise ValueError(f"chat template: {msg}")

        env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
        env.globals["raise_exception"] = raise_exception

        def tok_str(k):
            v = cfg.get(k)
            return v.get("content", "") if isinstance(v, dict) else (v or "")
        return env.from_string(tpl), tok_str("bos_token"), tok_str("eos_token")

    def encode_prompt(self, text: str) -> list[int]:
        """A whole LLM prompt: as the user turn of the checkpoint's chat
        template (followed by the assistant header) when it has one - the
        template writes its own BOS - else the text after BOS."""
        if self._chat is None:
            return self.encode(text, bos=True)
        tpl, bos, eos = self._chat
        s = tpl.render(messages=[{"role": "user", "content": text}], add_generation_prompt=True,
                       bos_token=bos, eos_token=eos)
        return self.encode(s)

    def _anchor(self) -> int:
        for s in ("a", "x", "the", "A"):
            ids = self._t.encode(s, add_special_tokens=False).ids
            if len(ids) == 1 and ids[0] not in self._added:
                return ids[0]
        return next(i for i in range(self._t.get_vocab_size()) if i not in self._added)

    def token_id(self, s: str) -> int:
        i = self._t.token_to_id(s)
        if i is not None and (i in self._added or self._text[i] == s):
            return i
        ids = self._t.encode(s, add_special_tokens=False).ids
        if len(ids) == 1 and self._text[ids[0]] == s:
            return ids[0]
        if s in self._by_text:
            return self._by_text[s]
        raise KeyError(f"{s!r} is not one token of this tokenizer")

    def encode(self, text: str, bos: bool = False) -> list[int]:
        ids = self._t.encode(text, add_special_tokens=False).ids
        return ([self.bos] if bos and self.bos is not None else []) + ids

    def decode(self, ids) -> str:
        return self._t.decode([int(t) for t in ids if 0 <= int(t) < self.n_real],
                              skip_special_tokens=True)

    def token_text(self, t: int) -> str:
        return self._text[t] if 0 <= t < self.n_real else ""

    def sampling_mask(self, keep: tuple = ()):
        """bool [vocab_size]: the tokens free (unconstrained) sampling may
        emit: not the added / special tokens (Whisper's task, language and
        timestamp tokens) except ``keep``, not the ``suppress_tokens`` of the
        checkpoint's generation config, not the padding ids past the file."""
        import torch
        m = torch.zeros(self.vocab_size, dtype=torch.bool)
        m[: self.n_real] = True
        for i in self._added:
            m[i] = False
        for i in self.generation_config.get("suppress_tokens") or ():
            if 0 <= int(i) < self.vocab_size:
                m[int(i)] = False
        for i in keep:
            m[i] = True
        return m
