"""Prompt templates of the intent parser.

The prompt text is part of the observable behaviour of the reference (it shapes
what the model returns), so the three templates are reproduced exactly:

* single command  - ``internal/llm/command_parser.go:195-220`` (buildPrompt)
* multi command   - ``internal/llm/command_parser.go:379-410`` (buildMultiCommandPrompt)
* streaming       - ``internal/llm/streaming_command_parser.go:388-413``
"""
from __future__ import annotations

DEFAULT_UNCLEAR_RESPONSE = "I'm not sure what you want me to do."

_SINGLE = (
    "You are a voice assistant command parser. Analyze the following voice command and respond "
    "with a JSON object.\n\n"
    'Voice command: "{t}"\n\n'
    "Classify this command and respond with ONLY a JSON object in this exact format:\n"
    "{{\n"
    '  "intent": "one of: turn_on, turn_off, greeting, question, unknown",\n'
    '  "entities": {{\n'
    '    "device": "lights, music, tv, etc. or empty string if none",\n'
    '    "location": "bedroom, kitchen, living room, etc. or empty string if none"\n'
    "  }},\n"
    '  "confidence": 0.95,\n'
    '  "response": "A natural response to the user"\n'
    "}}\n\n"
    "Rules:\n"
    "- turn_on: user wants to turn something on (lights, music, etc.)\n"
    "- turn_off: user wants to turn something off \n"
    "- greeting: user is saying hello, hi, good morning, etc.\n"
    "- question: user is asking a question\n"
    "- unknown: unclear or unrecognized command\n"
    "- confidence should be 0.0-1.0 based on how clear the intent is\n"
    "- response should be natural and conversational\n"
    "- Only respond with the JSON object, no other text"
)

_MULTI = (
    "You are a voice assistant command parser that handles compound utterances with multiple "
    "commands. Analyze the following voice command and respond with a JSON object.\n\n"
    'Voice command: "{t}"\n\n'
    'If this contains multiple distinct commands (connected by "and", "then", "after that", '
    "etc.), break them down into separate commands. If it's just one command, return it as a "
    "single command.\n\n"
    "Respond with ONLY a JSON object in this exact format:\n"
    "{{\n"
    '  "is_multi": true/false,\n'
    '  "commands": [\n'
    "    {{\n"
    '      "intent": "one of: turn_on, turn_off, greeting, question, unknown",\n'
    '      "entities": {{\n'
    '        "device": "lights, music, tv, etc. or empty string if none",\n'
    '        "location": "bedroom, kitchen, living room, etc. or empty string if none"\n'
    "      }},\n"
    '      "confidence": 0.95,\n'
    '      "response": "A natural response for this specific command"\n'
    "    }}\n"
    "  ],\n"
    '  "combined_response": "A single natural response combining all commands"\n'
    "}}\n\n"
    "Rules:\n"
    "- is_multi: true if there are multiple distinct commands, false otherwise\n"
    "- For each command: turn_on (turn something on), turn_off (turn something off), greeting "
    "(hello/hi), question (asking something), unknown (unclear)\n"
    "- confidence should be 0.0-1.0 based on how clear each intent is\n"
    "- response should be natural and conversational for each individual command\n"
    "- combined_response should be a single natural response acknowledging all commands\n"
    "- Only respond with the JSON object, no other text"
)

_STREAMING = _SINGLE.replace(
    "respond with a JSON object.\n\n",
    "respond with a JSON object. Respond progressively as you process the command.\n\n", 1,
).replace("turn something off \n", "turn something off\n", 1)


def build_prompt(transcription: str) -> str:
    return _SINGLE.format(t=transcription)


def build_multi_command_prompt(transcription: str) -> str:
    return _MULTI.format(t=transcription)


def build_streaming_prompt(transcription: str) -> str:
    return _STREAMING.format(t=transcription)
