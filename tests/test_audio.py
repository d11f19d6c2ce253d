"""Desktop audio: G.711 mu-law, FIR decimator, capture pipeline, WebSocket
PCM transport and WebRTC PCMU transport (loopback through DTLS-SRTP)."""
import asyncio

import numpy as np
import pytest

from mxdesk.audio.pipeline import CHUNK_FRAMES, AudioPipeline, SyntheticTone, audio_message, parse_audio_message

from .test_server import free_port, make_server


def test_ulaw_codec(native):
    A = native.audio
    x = np.array([0, -1, 32767, -32768, 100, -100, 1000, -1000], np.int16)
    assert A.encode_ulaw(x)[:4] == bytes([0xFF, 0x7F, 0x80, 0x00])
    codes = bytes(c for c in range(256) if c != 0x7F)  # 0x7F and 0xFF both decode to 0
    assert A.encode_ulaw(A.decode_ulaw(codes)) == codes
    ramp = np.arange(-32768, 32768, 7, dtype=np.int16)
    dec = A.decode_ulaw(A.encode_ulaw(ramp)).astype(np.int64)
    assert np.all(np.diff(dec) >= 0)  # monotonic
    err = np.abs(dec - ramp)
    assert np.all(err <= np.maximum(8, np.abs(ramp.astype(np.int64)) // 16 + 8))  # log-segment step


def test_decimator_passband_stopband_and_chunking(native):
    A = native.audio
    t = np.arange(48000) / 48000.0

    def run(freq, chunks):
        x = np.repeat((8000 * np.sin(2 * np.pi * freq * t)).astype(np.int16), 2)
        d = A.Decimator(6, 2)
        parts = np.array_split(x.reshape(-1, 2), chunks)
        return np.concatenate([d.process(p.reshape(-1).copy()) for p in parts])

    y = run(440, 1)
    assert len(y) == 8000
    assert abs(np.sqrt(np.mean(y[1000:].astype(float) ** 2)) * np.sqrt(2) / 8000 - 1) < 0.02
    assert np.array_equal(y, run(440, 37))  # stateful: chunking does not change the output
    z = run(6000, 1)  # above the 4 kHz output Nyquist
    assert np.sqrt(np.mean(z[1000:].astype(float) ** 2)) < 8000 * 0.01


def test_audio_pipeline_and_message_roundtrip():
    pipe = AudioPipeline(SyntheticTone())

    async def go():
        sub = pipe.subscribe(asyncio.get_running_loop())
        pipe.start()
        chunks = [await asyncio.wait_for(sub.queue.get(), 5) for _ in range(5)]
        pipe.stop()
        return chunks

    chunks = asyncio.run(go())
    assert [c.seq for c in chunks] == list(range(5))
    assert all(8000 <= b.t_capture_us - a.t_capture_us <= 40000 for a, b in zip(chunks, chunks[1:]))
    ref = SyntheticTone().read(5 * CHUNK_FRAMES)
    assert np.array_equal(np.concatenate([c.pcm for c in chunks]), ref)
    m = parse_audio_message(audio_message(chunks[1]))
    assert m["rate"] == 48000 and m["channels"] == 2 and m["seq"] == 1 and np.array_equal(m["pcm"], chunks[1].pcm)


def test_websocket_transport_carries_audio():
    from mxdesk.server.app import serve
    from mxdesk.server.client import view

    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "MXDESK_AUDIO_SOURCE": "synthetic"})

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await view(f"http://127.0.0.1:{port}/mxws", 8)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert res.config["audio"] == {"codec": "pcm_s16le", "rate": 48000, "channels": 2}
    assert len(res.frames) == 8 and len(res.audio) >= 5
    seqs = [a["seq"] for a in res.audio]
    assert seqs == sorted(seqs)
    # the subscriber joined mid-stream: its samples are a contiguous slice of the tone
    pcm = np.concatenate([a["pcm"] for a in res.audio])
    ref = SyntheticTone().read((seqs[-1] + 1) * CHUNK_FRAMES)
    assert np.array_equal(pcm, ref[seqs[0] * CHUNK_FRAMES * 2:(seqs[-1] + 1) * CHUNK_FRAMES * 2])


def test_webrtc_pcmu_audio(native, monkeypatch):
    from mxdesk.server.app import serve
    from mxdesk.server.whep_client import whep_view

    monkeypatch.setenv("MXDESK_WEBRTC_HOST", "127.0.0.1")
    cfg, pipe, srv = make_server({"ENABLE_BASIC_AUTH": "false", "MXDESK_AUDIO_SOURCE": "synthetic"})

    async def go():
        port = free_port()
        runner = await serve(srv, "127.0.0.1", port)
        try:
            return await whep_view(f"http://127.0.0.1:{port}/whep", 20)
        finally:
            await runner.cleanup()

    res = asyncio.run(go())
    assert "m=audio" in res.answer and "PCMU/8000" in res.answer and "a=group:BUNDLE 0 1" in res.answer
    assert len(res.audio_payloads) >= 5 and all(len(p) == 160 for p in res.audio_payloads)
    assert all(((b - a) & 0xFFFF) == 1 for a, b in zip(res.audio_seqs, res.audio_seqs[1:]))
    x = native.audio.decode_ulaw(b"".join(res.audio_payloads)).astype(float)
    spec = np.abs(np.fft.rfft(x * np.hanning(len(x))))
    f = np.fft.rfftfreq(len(x), 1 / 8000.0)
    band = (f > 300) & (f < 1200)
    assert abs(f[band][np.argmax(spec[band])] - 440) < 20 or abs(f[band][np.argmax(spec[band])] - 1000) < 20
