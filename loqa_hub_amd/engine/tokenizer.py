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
