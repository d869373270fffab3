"""``audio.AudioService`` protobuf + gRPC definitions, built at runtime.

The reference imports ``github.com/loqalabs/loqa-proto/go/audio`` (``go.mod:6``);
the .proto is not in the reference tree and ``grpc_tools`` is not installed, so
the descriptors are constructed with ``descriptor_pb2`` from the field usage in
``audio_service.go:694-699,733-734,765-769,864-870,953-1008``.

ASSUMPTION (documented): field numbers follow declaration
order; override with ``LOQA_PROTO_FIELDS`` (JSON ``{"AudioChunk": {"relay_id": 1,
...}}``) if a real relay uses different numbers.

    service AudioService { rpc StreamAudio(stream AudioChunk) returns (stream AudioResponse); }
    message AudioChunk    { string relay_id=1; bytes audio_data=2; int32 sample_rate=3;
                            bool is_wake_word=4; bool is_end_of_speech=5; int64 timestamp=6; }
    message AudioResponse { string request_id=1; string transcription=2; string command=3;
                            string response_text=4; bool success=5; bytes response_audio=6;
                            string audio_format=7; float audio_duration=8; }
"""
from __future__ import annotations

import json
import os

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "audio"
SERVICE = "AudioService"
METHOD = "StreamAudio"
FULL_METHOD = f"/{PACKAGE}.{SERVICE}/{METHOD}"

_T = descriptor_pb2.FieldDescriptorProto
_CHUNK = [("relay_id", _T.TYPE_STRING), ("audio_data", _T.TYPE_BYTES), ("sample_rate", _T.TYPE_INT32),
          ("is_wake_word", _T.TYPE_BOOL), ("is_end_of_speech", _T.TYPE_BOOL),
          ("timestamp", _T.TYPE_INT64)]
_RESP = [("request_id", _T.TYPE_STRING), ("transcription", _T.TYPE_STRING), ("command", _T.TYPE_STRING),
         ("response_text", _T.TYPE_STRING), ("success", _T.TYPE_BOOL),
         ("response_audio", _T.TYPE_BYTES), ("audio_format", _T.TYPE_STRING),
         ("audio_duration", _T.TYPE_FLOAT)]


def _build():
    overrides = json.loads(os.environ.get("LOQA_PROTO_FIELDS", "{}") or "{}")
    fd = descriptor_pb2.FileDescriptorProto(name="loqa_audio.proto", package=PACKAGE, syntax="proto3")
    for name, fields in (("AudioChunk", _CHUNK), ("AudioResponse", _RESP)):
        m = fd.message_type.add(name=name)
        numbers = overrides.get(name, {})
        for i, (fname, ftype) in enumerate(fields, start=1):
            m.field.add(name=fname, number=int(numbers.get(fname, i)), type=ftype,
                        label=_T.LABEL_OPTIONAL, json_name=_camel(fname))
    svc = fd.service.add(name=SERVICE)
    svc.method.add(name=METHOD, input_type=f".{PACKAGE}.AudioChunk",
                   output_type=f".{PACKAGE}.AudioResponse", client_streaming=True,
                   server_streaming=True)
    pool = descriptor_pool.DescriptorPool()
    fdesc = pool.Add(fd)
    f = pool.FindFileByName(fd.name)
    chunk = message_factory.GetMessageClass(f.message_types_by_name["AudioChunk"])
    resp = message_factory.GetMessageClass(f.message_types_by_name["AudioResponse"])
    return fdesc, chunk, resp


def _camel(s: str) -> str:
    p = s.split("_")
    return p[0] + "".join(x.capitalize() for x in p[1:])


_FILE, AudioChunk, AudioResponse = _build()


def add_audio_service(server, servicer) -> None:
    """Register ``servicer.StreamAudio(request_iterator, context)`` (async
    generator) on a ``grpc.aio`` server."""
    import grpc
    handler = grpc.method_handlers_generic_handler(f"{PACKAGE}.{SERVICE}", {
        METHOD: grpc.stream_stream_rpc_method_handler(
            servicer.StreamAudio, request_deserializer=AudioChunk.FromString,
            response_serializer=AudioResponse.SerializeToString),
    })
    server.add_generic_rpc_handlers((handler,))


def stream_audio_stub(channel):
    """Client-side callable for StreamAudio (relay simulators, tests)."""
    return channel.stream_stream(FULL_METHOD, request_serializer=AudioChunk.SerializeToString,
                                 response_deserializer=AudioResponse.FromString)
