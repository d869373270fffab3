"""Long-form audio: an utterance longer than
Whisper's 30 s window is split into 30 s windows (extra encoder rows of one
batch), decoded window after window with the previous window's text as the
prompt, and the texts joined - the reference transcribes the whole
accumulated audio (``audio_service.go:965,1002`` -> ``:609`` ->
``stt_client.go:157``). A command spoken after the 30 s mark reaches the
intent parser and is published on NATS."""
import asyncio
import json

import numpy as np
import pytest
import torch

from loqa_hub_amd.engine.synthetic import make_long_utterance, make_utterance


def _stt(device, name, **kw):
    from loqa_hub_amd.engine.stt_engine import STTEngine
    from loqa_hub_amd.models.configs import whisper_config
    return STTEngine(whisper_config(name), device, seed=1, max_batch=4, **kw)


def test_stt_long_form_windows_cpu():
    from loqa_hub_amd.engine.stt_engine import STTRequest
    eng = _stt(torch.device("cpu"), "test-whisper")
    u, s = make_long_utterance(1, 3), make_utterance(0, 1, 2)
    assert len(u.pcm) == 45 * 16000 and u.last_command_start_s > 30
    assert len(u.window_texts) == 2 and u.window_texts[1]
    reqs = [STTRequest(u.pcm, transcript=u.text, transcript_windows=u.window_texts),
            STTRequest(s.pcm, transcript=s.text)]
    eng.transcribe(reqs)
    assert reqs[0].windows == 2 and reqs[0].n_samples == len(u.pcm)
    assert reqs[0].text == u.text and reqs[1].text == s.text
    assert eng.stats["long_form_windows"] == 1
    # the second window's decode was prompted with the first window's text
    assert reqs[0].prev_tokens and eng.sop is not None
    # continuous batching: the long request holds two cross-attention slots
    out = eng.submit_batch([STTRequest(u.pcm, transcript=u.text, transcript_windows=u.window_texts),
                            STTRequest(s.pcm, transcript=s.text)]).result(timeout=300)
    eng.stop()
    assert [r.text for r in out] == [u.text, s.text]
    assert sorted(eng._free_slots) == [0, 1, 2, 3]


def test_stt_long_form_free_decoding_cpu():
    """Without a transcript (real greedy decoding) every window is decoded and
    the RMS covers all the samples."""
    from loqa_hub_amd.engine.stt_engine import STTRequest
    eng = _stt(torch.device("cpu"), "test-whisper")
    u = make_long_utterance(2, 2, seconds=70)
    r = STTRequest(u.pcm, max_new_tokens=3)
    eng.transcribe([r])
    assert r.windows == 3 and r.win == 2 and r.t_done > 0
    assert len(r.win_texts) == 3
    want = float(np.sqrt(np.mean((u.pcm.astype(np.float64) / 32767) ** 2)))
    assert abs(r.rms - want) <= 1e-4 * want


def test_stt_windows_capped_by_max_batch_and_hol_bypass_cpu():
    """an utterance needing more 30 s windows than the engine has
    cross-attention slots is truncated (like one past LOQA_STT_MAX_WINDOWS),
    not rejected; and a short utterance may pass a long-form one that waits
    for free slots (bounded, so the long one is never starved)."""
    from loqa_hub_amd.engine.stt_engine import STTRequest
    eng = _stt(torch.device("cpu"), "test-whisper")        # max_batch 4
    u = make_long_utterance(2, 2, seconds=150)            # 5 windows > 4 slots
    r = STTRequest(u.pcm, max_new_tokens=2)
    assert eng.rows_needed([r]) == 4
    out = eng.submit_batch([r]).result(timeout=300)
    assert out[0].windows == 4 and out[0].t_done > 0
    assert eng.stats["long_form_dropped_samples"] == len(u.pcm) - 4 * 480000
    # a 3-window item at the head cannot start while 2 slots are held; the
    # 1-window items behind it pass it
    s = make_utterance(0, 1, 2)
    a = eng.submit_batch([STTRequest(make_long_utterance(3, 2, seconds=40).pcm, max_new_tokens=40),
                          STTRequest(s.pcm, max_new_tokens=40)])   # 3 rows, takes 3 of 4
    b = eng.submit_batch([STTRequest(make_long_utterance(4, 2, seconds=80).pcm, max_new_tokens=2)])
    c = eng.submit_batch([STTRequest(s.pcm, transcript=s.text)])
    for f in (a, b, c):
        f.result(timeout=300)
    eng.stop()
    assert sorted(eng._free_slots) == [0, 1, 2, 3]


def _long_pipeline(device, stt_name, llm_name, graphs):
    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.engine.pipeline import PipelineJob, VoicePipeline
    from loqa_hub_amd.messaging.nats_client import NATSClient
    from loqa_hub_amd.messaging.nats_server import NATSServer
    from loqa_hub_amd.messaging.nats_service import NATSService
    from loqa_hub_amd.models.configs import llama_config
    stt = _stt(device, stt_name, use_graphs=graphs)
    llm = LLMEngine(llama_config(llm_name), device, seed=0, max_seqs=8, max_seq_len=1024,
                    use_graphs=graphs)
    u = make_long_utterance(3, 3)
    short = make_utterance(4, 0, 2)

    async def main():
        broker = await NATSServer("127.0.0.1", 0).start()
        nats = NATSService(broker.url)
        await nats.connect()
        sub = NATSClient(name="test")
        await sub.connect(broker.url)
        got = []
        await sub.subscribe("loqa.>", lambda m: got.append((m.subject, json.loads(m.data))))
        await sub.flush()
        try:
            pipe = VoicePipeline(stt, llm, nats, min_response_tokens=2, continuous=True,
                                 stt_continuous=True, max_batch=4)
            if graphs:
                pipe.warmup()
            jobs = [PipelineJob(u.relay_id, "long", u.pcm, transcript_hint=u.window_texts),
                    PipelineJob(short.relay_id, "short", short.pcm, transcript_hint=short.text)]
            res = await asyncio.gather(*[pipe.submit(j) for j in jobs])
            await asyncio.sleep(0.2)
            await sub.flush()
            return res, got
        finally:
            stt.stop()
            llm.stop()
            await sub.close()
            await nats.close()
            await broker.stop()
    res, got = asyncio.run(main())
    long_job = res[0]
    assert long_job.raw_text == u.text, long_job.raw_text
    tail = u.window_texts[1].split()
    assert all(w in long_job.raw_text.split() for w in tail)
    assert long_job.n_commands == u.n_commands == 3
    assert long_job.queue is not None and long_job.queue.success
    cmds = [m for s, m in got if s == "loqa.voice.commands" and m.get("relay_id") == u.relay_id]
    assert len(cmds) >= 1, got
    # the last command (spoken after 30 s) was published with the rest
    assert res[1].n_commands == 2
    return long_job, got


def test_long_form_pipeline_publishes_last_command_cpu():
    _long_pipeline(torch.device("cpu"), "test-whisper", "test-tiny", graphs=False)


@pytest.mark.gpu
def test_long_form_pipeline_publishes_last_command_gpu():
    """The same on the GPU: pinned slot chain, stream-in copies, two encoder
    rows, the pipelined graph-replayed decoder across the window boundary."""
    _long_pipeline(torch.device("cuda", 0), "whisper-tiny", "test-tiny", graphs=True)


@pytest.mark.gpu
def test_pcm_stager_uploads_byte_identical_gpu():
    """Stream-in staging (per-chunk hipMemcpyAsync on the placed H2D stream
    while the relay speaks), slot chains past 30 s and a host-buffered tail
    (stager out of slots) all land the exact samples in HBM."""
    from loqa_hub_amd.engine.pcm_staging import PcmStager
    from loqa_hub_amd.utils.streams import placed_stream
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    cur = torch.cuda.current_stream(dev)
    for stream_in in (False, True):
        st = PcmStager(3, 480000, h2d_stream=placed_stream(dev, "h2d") if stream_in else None)
        assert st.stream_in == stream_in
        for n in (1600, 479999, 480000, 700001, 1500000):   # the last: 3 slots + a host tail
            pcm = rng.integers(-32768, 32767, n).astype("<i2")
            slot = st.acquire()
            b = pcm.tobytes()
            for i in range(0, len(b), 3200):                # 100 ms relay chunks
                slot.append(b[i:i + 3200])
            assert len(slot) == n
            assert np.array_equal(slot.numpy(), pcm)
            out = torch.empty(n, dtype=torch.int16, device=dev)
            slot.upload(out.data_ptr(), n, cur.cuda_stream)
            assert np.array_equal(out.cpu().numpy(), pcm), (stream_in, n)
            assert len(slot.slots) == min(3, -(-n // 480000))
        st.close()


@pytest.mark.gpu
def test_dp_pcm_ring_registered_upload_gpu():
    """The DP worker's side of the shared-memory PCM ring on a GPU: the ring
    is pinned with hipHostRegister and a slot uploads straight to HBM
    (RegisteredPcm), byte-identical."""
    from multiprocessing import shared_memory

    from loqa_hub_amd.parallel.dp_serving import _WorkerPcmRing
    dev = torch.device("cuda", 0)
    slot_bytes = 480000 * 2
    shm = shared_memory.SharedMemory(create=True, size=3 * slot_bytes)
    try:
        rng = np.random.default_rng(1)
        pcm = rng.integers(-32768, 32767, 123457).astype("<i2")
        b = pcm.tobytes()
        shm.buf[slot_bytes:slot_bytes + len(b)] = b        # slot 1, as the front end writes it
        ring = _WorkerPcmRing(shm.name, slot_bytes, "cuda:0")
        assert ring.registered
        view, reg = ring.samples(1, len(b))
        assert reg is not None and np.array_equal(view, pcm)
        out = torch.empty(pcm.size, dtype=torch.int16, device=dev)
        reg.upload(out.data_ptr(), pcm.size, torch.cuda.current_stream(dev).cuda_stream)
        assert np.array_equal(out.cpu().numpy(), pcm)
        del view, reg
        ring.close()
    finally:
        shm.close()
        shm.unlink()
