"""Desktop audio: capture -> fan-out to the WebSocket (PCM) and WebRTC
(PCMU) transports.  The reference runs PulseAudio in system mode and ``pulsesrc ! opusenc
! rtpopuspay`` inside selkies (supervisord.conf:22-32); this image has no libopus, so audio
goes out as lossless 48 kHz PCM over the WebSocket transport and as G.711 mu-law (PCMU,
universally supported by browsers) over WebRTC."""
from .pipeline import AudioChunk, AudioPipeline, make_source  # noqa: F401
