"""Control-plane parity tests: config (C4), command parsing (C17), command queue
(C18), STT post-processing (C14), parser backends. Cases mirror the reference's
``config_test.go``, ``command_parser_test.go``, ``command_queue_test.go`` and
``stt_client_test.go`` tables."""
import asyncio
import json

import pytest

from loqa_hub_amd import config as cfgmod
from loqa_hub_amd.llm.command_parser import CommandParser, OllamaBackend
from loqa_hub_amd.llm.command_queue import (CommandQueue, combined_response,
                                            create_rollback_command)
from loqa_hub_amd.llm.commands import (Command, MultiCommand, ParseError, create_combined_command,
                                       detect_compound_utterance, parse_multi_command_response,
                                       parse_response, split_compound_utterance)
from loqa_hub_amd.llm.http import create_mock_ollama
from loqa_hub_amd.llm.prompts import build_multi_command_prompt, build_prompt
from loqa_hub_amd.llm.transcriber import estimate_confidence, post_process_transcription


# -- config --------------------------------------------------------------------------------------
def test_config_defaults():
    c = cfgmod.load({})
    assert (c.server.host, c.server.port, c.server.grpc_port) == ("0.0.0.0", 8080, 50051)
    assert c.server.db_path == "./data/loqa-hub.db"
    assert (c.stt.url, c.stt.language, c.stt.temperature) == ("http://stt:8000", "en", 0.0)
    assert (c.tts.url, c.tts.voice, c.tts.speed) == ("http://localhost:8880/v1", "af_bella", 1.0)


def test_config_env_overrides():
    c = cfgmod.load({"STT_LANGUAGE": "es", "STT_URL": "http://custom-stt:9000",
                     "LOQA_HOST": "127.0.0.1", "LOQA_PORT": "3000", "LOQA_GRPC_PORT": "50052",
                     "LOQA_DB_PATH": "/custom/path/db.sqlite", "TTS_URL": "http://custom-tts:8881/v1",
                     "TTS_VOICE": "en_male", "TTS_SPEED": "1.5", "TTS_FORMAT": "wav",
                     "TTS_MAX_CONCURRENT": "15", "TTS_NORMALIZE": "false", "TTS_TIMEOUT": "15s",
                     "TTS_FALLBACK_ENABLED": "false"})
    assert c.stt.language == "es" and c.stt.url == "http://custom-stt:9000"
    assert (c.server.host, c.server.port, c.server.grpc_port) == ("127.0.0.1", 3000, 50052)
    assert c.server.db_path == "/custom/path/db.sqlite"
    assert (c.tts.voice, c.tts.speed, c.tts.response_format) == ("en_male", 1.5, "wav")
    assert c.tts.max_concurrent == 15 and c.tts.normalize is False and c.tts.timeout == 15.0
    assert c.tts.fallback_enabled is False


@pytest.mark.parametrize("env,msg", [({"LOQA_PORT": "0"}, "invalid server port"),
                                     ({"LOQA_GRPC_PORT": "99999"}, "invalid gRPC port")])
def test_config_invalid(env, msg):
    with pytest.raises(cfgmod.ConfigError, match=msg):
        cfgmod.load(env)


def test_config_parse_errors_fall_back_and_durations():
    c = cfgmod.load({"LOQA_PORT": "notanumber", "TTS_SPEED": "fast", "TTS_NORMALIZE": "maybe"})
    assert c.server.port == 8080 and c.tts.speed == 1.0 and c.tts.normalize is True
    assert cfgmod.parse_go_duration("1h30m") == 5400.0
    assert cfgmod.parse_go_duration("250ms") == 0.25
    assert cfgmod.format_go_duration(15.0) == "15s"


# -- command parsing -----------------------------------------------------------------------------
@pytest.mark.parametrize("utt,exp", [
    ("turn on the lights and play music", True),
    ("turn off the tv then dim the bedroom lights", True),
    ("turn on the lights, after that play some music", True),
    ("turn on the lights", False),
    ("play rock and roll music", False),
    ("turn on the lights and play music and set the temperature", True),
    ("turn on the lights, and play music", True),
    ("turn off the lights next turn on the fan", True),
    ("turn on the lights also play music", True),
    ("", False)])
def test_detect_compound(utt, exp):
    assert detect_compound_utterance(utt) is exp


def test_split_compound():
    assert split_compound_utterance("turn on the lights and play music, then lock the door") == [
        "turn on the lights", "play music", "lock the door"]
    assert split_compound_utterance("turn on the lights") == ["turn on the lights"]


def test_prompts_contain_transcription():
    p = build_prompt("turn on the lights")
    assert "turn on the lights" in p and "intent" in p
    mp = build_multi_command_prompt("a and b")
    for kw in ("commands", "is_multi", "combined_response"):
        assert kw in mp


def test_parse_response_defaults():
    c = parse_response('Sure! {"intent": "", "entities": {"device": "lights"}, "confidence": 7}')
    assert c.intent == "unknown" and c.confidence == 0.5
    assert c.response == "I'm not sure what you want me to do."
    with pytest.raises(ParseError):
        parse_response("no json here")


def test_parse_multi_command_response():
    raw = json.dumps({"commands": [
        {"intent": "turn_on", "entities": {"device": "lights"}, "confidence": 0.9,
         "response": "on"},
        {"intent": "play", "entities": {"device": "music"}, "confidence": 0.8,
         "response": "playing"}], "is_multi": True, "combined_response": "ok"})
    mc = parse_multi_command_response(raw, "turn on the lights and play music")
    assert mc.is_multi and len(mc.commands) == 2
    assert mc.original_text == "turn on the lights and play music"
    mc1 = parse_multi_command_response(json.dumps({"commands": [
        {"intent": "turn_on", "entities": {"device": "lights"}, "confidence": 0.9}],
        "is_multi": False}), "x")
    assert not mc1.is_multi and len(mc1.commands) == 1
    mc0 = parse_multi_command_response('{"commands": [], "is_multi": false}', "x")
    assert len(mc0.commands) == 0


def test_create_combined_command():
    assert create_combined_command(MultiCommand([], False, "", "")).intent == "unknown"
    one = Command("turn_on", {"device": "lights"}, 0.9, "ok")
    assert create_combined_command(MultiCommand([one], False, "", "")).intent == "turn_on"
    two = Command("play", {"device": "music"}, 0.7, "p")
    c = create_combined_command(MultiCommand([one, two], True, "", "both"))
    assert c.intent == "multi_turn_on" and c.entities == {"device": "lights, music"}
    assert c.confidence == pytest.approx(0.8) and c.response == "both"


def test_parser_with_mock_ollama():
    async def go():
        single = json.dumps({"intent": "turn_on", "entities": {"device": "lights"},
                             "confidence": 0.9, "response": "Turning on"})
        multi = json.dumps({"commands": [
            {"intent": "turn_on", "entities": {"device": "lights"}, "confidence": 0.9,
             "response": "a"},
            {"intent": "turn_off", "entities": {"device": "fan"}, "confidence": 0.7,
             "response": "b"}], "is_multi": True, "combined_response": "done both"})

        def responder(prompt):
            return multi if "commands" in prompt and "is_multi" in prompt else single
        p = CommandParser(OllamaBackend(client=create_mock_ollama(responder)))
        c = await p.parse_command("turn on the lights")
        assert c.intent == "turn_on"
        c = await p.parse_command("turn on the lights and turn off the fan")
        assert c.intent == "multi_turn_on" and c.response == "done both"
        # backend down -> reference fallback text
        bad = CommandParser(OllamaBackend(client=create_mock_ollama("", status=500)))
        c = await bad.parse_command("turn on the lights")
        assert c.intent == "unknown"
        assert c.response == "I'm having trouble understanding you right now."
        assert (await bad.parse_command("")).response == "I didn't hear anything."
    asyncio.run(go())


# -- command queue -------------------------------------------------------------------------------
class RecExec:
    def __init__(self, fail_on=None, delay=0.0):
        self.calls, self.fail_on, self.delay = [], fail_on, delay

    async def execute_command(self, cmd):
        self.calls.append((cmd.intent, cmd.entities.get("device")))
        if self.delay:
            await asyncio.sleep(self.delay)
        if self.fail_on and cmd.entities.get("device") == self.fail_on:
            raise RuntimeError("device offline")


def cmds():
    return [Command("turn_on", {"device": "lights"}, 0.9, "Lights on"),
            Command("turn_off", {"device": "fan"}, 0.9, "Fan off"),
            Command("turn_on", {"device": "tv"}, 0.9, "TV on")]


def test_queue_success():
    q = CommandQueue(cmds())
    assert q.size() == 3 and not q.is_empty()
    r = asyncio.run(q.execute(RecExec()))
    assert r.success and len(r.completed_items) == 3 and not r.rollback_occurred
    assert r.combined_response == "I've completed 3 commands for you."
    assert all(i.executed and i.success and i.duration >= 0 for i in q.get_status())


def test_queue_failure_rolls_back_in_reverse():
    ex = RecExec(fail_on="tv")
    r = asyncio.run(CommandQueue(cmds()).execute(ex))
    assert not r.success and r.failed_item.index == 2 and r.rollback_occurred
    assert ex.calls[3:] == [("turn_on", "fan"), ("turn_off", "lights")]
    ex2 = RecExec(fail_on="tv")
    r2 = asyncio.run(CommandQueue(cmds(), rollback_enabled=False).execute(ex2))
    assert not r2.rollback_occurred and len(ex2.calls) == 3


def test_queue_timeout():
    r, err = asyncio.run(CommandQueue(cmds(), max_duration=0.05).run(RecExec(delay=0.04)))
    assert err is not None and not r.success


def test_rollback_and_combined_response():
    assert create_rollback_command(Command("turn_on", {"device": "x"})).intent == "turn_off"
    assert create_rollback_command(Command("turn_off", {"device": "x"})).intent == "turn_on"
    assert create_rollback_command(Command("play", {})) is None
    assert combined_response([]) == "No commands were executed."
    assert combined_response(["a"]) == "a"
    assert combined_response(["a", "b"]) == "I've completed 2 commands for you."


# -- STT post-processing -------------------------------------------------------------------------
@pytest.mark.parametrize("inp,clean,wake,variant,confirm", [
    ("Hey Loqa turn on the lights", "turn on the lights", True, "hey loqa", False),
    ("Hey Luca turn off the music", "turn off the music", True, "hey luca", False),
    ("Hey Luka what time is it", "what time is it", True, "hey luka", False),
    ("Hey Loqa", "", True, "hey loqa", True),
    ("turn on the lights", "turn on the lights", False, "", False),
    ("on", "on", False, "", True),
    ("???", "???", False, "", True),
    ("Hey Loqa aaaaaah", "aaaaaah", True, "hey loqa", False),
    ("HEY LOQA TURN ON LIGHTS", "TURN ON LIGHTS", True, "hey loqa", False),
    ("Hey Loqa, turn on the lights", "turn on the lights", True, "hey loqa", False)])
def test_post_process(inp, clean, wake, variant, confirm):
    r = post_process_transcription(inp)
    assert (r.cleaned_text, r.wake_word_detected, r.wake_word_variant,
            r.needs_confirmation) == (clean, wake, variant, confirm)


@pytest.mark.parametrize("inp,lo,hi", [("", 0, 0), ("turn on the lights", 0.7, 1.0),
                                       ("on", 0, 0.6), ("Hey Loqa turn on lights", 0.8, 1.0),
                                       ("...", 0, 0.7), ("aaaaaah", 0, 0.6)])
def test_estimate_confidence(inp, lo, hi):
    assert lo <= estimate_confidence(inp) <= hi
