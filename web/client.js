// mxdesk browser client: receives Annex-B H.264 access units over the /mxws WebSocket,
// decodes them with WebCodecs (hardware decoder on the viewer's machine) and paints a
// canvas; mouse/keyboard/clipboard events go back as selkies-style text messages.
// `?transport=webrtc` instead plays the stream through RTCPeerConnection (WHEP offer/answer
// against POST /whep; SRTP video into a <video> element); input then travels on an SCTP data
// channel named "input" (selkies' channel), with /mxws?media=0 as the fallback until it opens.
"use strict";
const mxdesk = (() => {
  const HDR = 36;
  let ws, dc = null, decoder, canvas, ctx, statsEl, msgEl, cfg = null, waitingKey = true;
  let frames = 0, bytes = 0, lastStats = performance.now(), decodeTimes = [];
  const sendQ = (m) => {
    if (dc && dc.readyState === "open") dc.send(m);
    else if (ws && ws.readyState === 1) ws.send(m);
  };

  function parse(buf) {
    const dv = new DataView(buf);
    const magic = String.fromCharCode(dv.getUint8(0), dv.getUint8(1), dv.getUint8(2), dv.getUint8(3));
    if (magic !== "MXV1") throw new Error("bad frame");
    return {
      key: (dv.getUint8(4) & 1) === 1,
      frameId: dv.getUint32(8, true),
      tCapture: Number(dv.getBigUint64(12, true)),
      tSend: Number(dv.getBigUint64(20, true)),
      width: dv.getUint16(28, true), height: dv.getUint16(30, true),
      data: new Uint8Array(buf, HDR, dv.getUint32(32, true)),
    };
  }

  // remote -> client state pushed by the server (selkies message shapes)
  function onControl(m) {
    if (m.type === "clipboard" && m.data) {
      const text = decodeURIComponent(escape(atob(m.data.content)));
      if (navigator.clipboard && navigator.clipboard.writeText) navigator.clipboard.writeText(text).catch(() => {});
    } else if (m.type === "cursor" && m.data) {
      const h = m.data.hotspot || { x: 0, y: 0 };
      canvas.style.cursor = `url(data:image/png;base64,${m.data.curdata}) ${h.x} ${h.y}, auto`;
    }
  }

  let resizeTimer = null;
  function requestResize() {
    if (!cfg || !cfg.resize) return;
    clearTimeout(resizeTimer);
    resizeTimer = setTimeout(() => sendQ(`r,${window.innerWidth}x${window.innerHeight}`), 300);
  }

  function makeDecoder() {
    decoder = new VideoDecoder({
      output: (frame) => {
        if (canvas.width !== frame.displayWidth || canvas.height !== frame.displayHeight) {
          canvas.width = frame.displayWidth; canvas.height = frame.displayHeight;
        }
        ctx.drawImage(frame, 0, 0);
        frame.close();
      },
      error: (e) => { msgEl.textContent = "decoder error: " + e; waitingKey = true; sendQ("pli"); makeDecoder(); },
    });
    decoder.configure({ codec: cfg.codec, optimizeForLatency: true, hardwareAcceleration: "prefer-hardware" });
  }

  function onFrame(buf) {
    const f = parse(buf);
    if (waitingKey && !f.key) return;
    waitingKey = false;
    const t0 = performance.now();
    decoder.decode(new EncodedVideoChunk({ type: f.key ? "key" : "delta", timestamp: f.frameId * 1000, data: f.data }));
    decodeTimes.push(performance.now() - t0);
    frames++; bytes += f.data.byteLength;
    sendQ(JSON.stringify({ type: "ack", frame_id: f.frameId }));
    const now = performance.now();
    if (now - lastStats > 1000) {
      const dt = (now - lastStats) / 1000;
      statsEl.textContent = `${cfg.width}x${cfg.height} ${cfg.codec}\n${(frames / dt).toFixed(1)} fps ` +
        `${(bytes * 8 / dt / 1000).toFixed(0)} kbps\nqueue ${decoder.decodeQueueSize}`;
      frames = 0; bytes = 0; lastStats = now; decodeTimes = [];
    }
  }

  // ---- desktop audio over the WebSocket: "MXA1" chunks of s16le PCM, scheduled on an
  // AudioContext with a ~60 ms jitter buffer (browsers need a user gesture to start audio)
  let actx = null, playAt = 0;
  const unlockAudio = () => {
    if (!actx && window.AudioContext) actx = new AudioContext({ sampleRate: 48000, latencyHint: "interactive" });
    if (actx && actx.state === "suspended") actx.resume();
  };
  function onAudio(buf) {
    if (!actx || actx.state !== "running") return;
    const dv = new DataView(buf);
    const ch = dv.getUint8(5), rate = dv.getUint16(6, true) * 100, n = dv.getUint32(20, true);
    const pcm = new Int16Array(buf, 24, n / 2);
    const frames = pcm.length / ch;
    const ab = actx.createBuffer(ch, frames, rate);
    for (let c = 0; c < ch; c++) {
      const d = ab.getChannelData(c);
      for (let i = 0; i < frames; i++) d[i] = pcm[i * ch + c] / 32768;
    }
    const src = actx.createBufferSource();
    src.buffer = ab;
    src.connect(actx.destination);
    const now = actx.currentTime;
    if (playAt < now + 0.02 || playAt > now + 0.25) playAt = now + 0.06;
    src.start(playAt);
    playAt += frames / rate;
  }

  function input() {
    canvas.addEventListener("mousedown", unlockAudio);
    window.addEventListener("keydown", unlockAudio);
    const pos = (e) => {
      const r = canvas.getBoundingClientRect();
      const sx = canvas.width / r.width, sy = canvas.height / r.height;
      const s = Math.min(1 / sx, 1 / sy);
      const ox = (r.width - canvas.width * s) / 2, oy = (r.height - canvas.height * s) / 2;
      return [Math.round((e.clientX - r.left - ox) / s), Math.round((e.clientY - r.top - oy) / s)];
    };
    let mask = 0;
    const mouse = (e, scroll = 0) => { const [x, y] = pos(e); sendQ(`m,${x},${y},${mask},${scroll}`); };
    canvas.addEventListener("mousemove", (e) => mouse(e));
    canvas.addEventListener("mousedown", (e) => { mask |= 1 << e.button; mouse(e); e.preventDefault(); canvas.focus(); });
    canvas.addEventListener("mouseup", (e) => { mask &= ~(1 << e.button); mouse(e); e.preventDefault(); });
    canvas.addEventListener("wheel", (e) => { mouse(e, e.deltaY < 0 ? 1 : -1); e.preventDefault(); }, { passive: false });
    canvas.addEventListener("contextmenu", (e) => e.preventDefault());
    const keysym = (e) => (e.key.length === 1 ? e.key.codePointAt(0) : ({
      Enter: 0xff0d, Backspace: 0xff08, Tab: 0xff09, Escape: 0xff1b, Delete: 0xffff, Home: 0xff50,
      ArrowLeft: 0xff51, ArrowUp: 0xff52, ArrowRight: 0xff53, ArrowDown: 0xff54, PageUp: 0xff55, PageDown: 0xff56,
      End: 0xff57, Shift: 0xffe1, Control: 0xffe3, Alt: 0xffe9, Meta: 0xffeb,
    }[e.key] || 0));
    canvas.addEventListener("keydown", (e) => { const k = keysym(e); if (k) sendQ(`kd,${k}`); e.preventDefault(); });
    canvas.addEventListener("keyup", (e) => { const k = keysym(e); if (k) sendQ(`ku,${k}`); e.preventDefault(); });
    window.addEventListener("blur", () => sendQ("kr"));
    document.addEventListener("paste", (e) => {
      const t = e.clipboardData.getData("text");
      if (t) sendQ("cw," + btoa(unescape(encodeURIComponent(t))));
    });
    window.addEventListener("resize", requestResize);
    gamepads();
  }

  // Gamepad API -> selkies-style js,* messages -> /dev/input/jsN in the desktop (interposer)
  function gamepads() {
    const last = {};
    window.addEventListener("gamepadconnected", (e) => {
      const g = e.gamepad;
      sendQ(`js,c,${g.index},${btoa(unescape(encodeURIComponent(g.id)))},${g.axes.length},${g.buttons.length}`);
      last[g.index] = { b: g.buttons.map(() => 0), a: g.axes.map(() => 0) };
    });
    window.addEventListener("gamepaddisconnected", (e) => { sendQ(`js,d,${e.gamepad.index}`); delete last[e.gamepad.index]; });
    const poll = () => {
      for (const g of navigator.getGamepads ? navigator.getGamepads() : []) {
        if (!g || !last[g.index]) continue;
        const s = last[g.index];
        g.buttons.forEach((b, i) => { if (b.value !== s.b[i]) { s.b[i] = b.value; sendQ(`js,b,${g.index},${i},${b.value}`); } });
        g.axes.forEach((v, i) => { const q = Math.round(v * 100) / 100; if (q !== s.a[i]) { s.a[i] = q; sendQ(`js,a,${g.index},${i},${q}`); } });
      }
      requestAnimationFrame(poll);
    };
    requestAnimationFrame(poll);
  }

  async function whep(video) {
    // RTC configuration (STUN/TURN with time-limited credentials) from the server's /turn
    let iceServers = [];
    try { iceServers = (await (await fetch("turn")).json()).iceServers || []; } catch (e) { /* no TURN */ }
    const pc = new RTCPeerConnection({ iceServers });
    pc.addTransceiver("video", { direction: "recvonly" });
    // audio: 48 kHz PCM on an unordered, no-retransmit data channel (played through WebAudio
    // like the WebSocket transport) instead of the 8 kHz PCMU RTP track
    const ach = pc.createDataChannel("audio", { ordered: false, maxRetransmits: 0 });
    ach.binaryType = "arraybuffer";
    ach.onmessage = (ev) => onAudio(ev.data);
    const ch = pc.createDataChannel("input", { ordered: true });
    ch.onopen = () => { dc = ch; };
    ch.onclose = () => { if (dc === ch) dc = null; };
    ch.onmessage = (ev) => {
      try {
        const m = JSON.parse(ev.data);
        if (m.type !== "stats") { onControl(m); return; }
        serverStats = `\nserver ${(m.encoded_fps_1s || 0).toFixed(1)} fps ` +
          `${Math.round(m.bitrate_kbps_1s || 0)} kbps qp ${m.qp || 0} rtx ${m.rtx}`;
      } catch (e) { /* not JSON */ }
    };
    let serverStats = "";
    const audioEl = new Audio();
    pc.ontrack = (ev) => {
      if (ev.track.kind === "audio") {
        audioEl.srcObject = new MediaStream([ev.track]);
        const go = () => audioEl.play().catch(() => {});
        go(); window.addEventListener("mousedown", go, { once: true });
        return;
      }
      video.srcObject = new MediaStream([ev.track]);
      video.play().catch(() => {});
    };
    pc.onconnectionstatechange = () => {
      msgEl.textContent = pc.connectionState === "connected" ? "" : "webrtc: " + pc.connectionState;
      if (pc.connectionState === "failed") { pc.close(); setTimeout(() => whep(video), 1000); }
    };
    await pc.setLocalDescription(await pc.createOffer());
    // non-trickle WHEP: wait (<= 2 s) for candidates so the offer carries them -- the server
    // turns them into TURN permissions on its relay; late candidates go out as PATCHes
    await new Promise((resolve) => {
      if (pc.iceGatheringState === "complete") return resolve();
      const t = setTimeout(resolve, 2000);
      pc.addEventListener("icegatheringstatechange", () => {
        if (pc.iceGatheringState === "complete") { clearTimeout(t); resolve(); }
      });
    });
    let whepLocation = null;
    pc.onicecandidate = (ev) => {
      if (ev.candidate && ev.candidate.candidate && whepLocation) {
        fetch(whepLocation, { method: "PATCH", headers: { "Content-Type": "application/trickle-ice-sdpfrag" },
                              body: `a=${ev.candidate.candidate}\r\n` }).catch(() => {});
      }
    };
    const r = await fetch("whep", { method: "POST", headers: { "Content-Type": "application/sdp" }, body: pc.localDescription.sdp });
    if (r.status !== 201) { msgEl.textContent = "WHEP failed: " + r.status; return; }
    const loc = r.headers.get("Location");
    whepLocation = loc;
    window.addEventListener("beforeunload", () => { fetch(loc, { method: "DELETE", keepalive: true }); });
    await pc.setRemoteDescription({ type: "answer", sdp: await r.text() });
    setInterval(async () => {
      const st = await pc.getStats();
      st.forEach((x) => {
        if (x.type === "inbound-rtp" && x.kind === "video") {
          // client statistics for the server's CSV log (SELKIES_ENABLE_WEBRTC_STATISTICS)
          sendQ(JSON.stringify({ type: "stats", fps: x.framesPerSecond || 0, frames_decoded: x.framesDecoded,
            packets_lost: x.packetsLost, jitter: x.jitter, nack: x.nackCount, pli: x.pliCount,
            bytes: x.bytesReceived, decode_s: x.totalDecodeTime, width: x.frameWidth, height: x.frameHeight }));
          statsEl.textContent = `webrtc ${x.frameWidth}x${x.frameHeight}\n${(x.framesPerSecond || 0).toFixed(1)} fps ` +
            `lost ${x.packetsLost} nack ${x.nackCount} pli ${x.pliCount}` + (dc ? " dc" : "") + serverStats;
        }
      });
    }, 1000);
  }

  function connect(media = true) {
    const proto = location.protocol === "https:" ? "wss:" : "ws:";
    ws = new WebSocket(`${proto}//${location.host}/mxws${media ? "" : "?media=0"}`);
    ws.binaryType = "arraybuffer";
    ws.onmessage = (ev) => {
      if (typeof ev.data === "string") {
        const m = JSON.parse(ev.data);
        if (m.type === "config") {
          const first = !cfg;
          cfg = m; waitingKey = true; if (ctx) makeDecoder(); msgEl.textContent = "";
          if (first) requestResize();  // follow the browser window from the start (WEBRTC_ENABLE_RESIZE)
        } else onControl(m);
        return;
      }
      if (new Uint8Array(ev.data, 0, 4).every((b, i) => b === "MXA1".charCodeAt(i))) { onAudio(ev.data); return; }
      if (cfg) onFrame(ev.data);
    };
    ws.onclose = () => { msgEl.textContent = "disconnected - retrying"; setTimeout(() => connect(media), 1000); };
  }

  return {
    start(c, s, m, video) {
      canvas = c; statsEl = s; msgEl = m;
      if (new URLSearchParams(location.search).get("transport") === "webrtc" || !("VideoDecoder" in window)) {
        // video element on top; input events still come from the canvas-sized overlay
        video.style.display = "block"; canvas.style.position = "fixed"; canvas.style.inset = "0";
        canvas.width = 1920; canvas.height = 1080; canvas.style.opacity = "0";
        video.addEventListener("resize", () => { canvas.width = video.videoWidth; canvas.height = video.videoHeight; });
        input(); connect(false); whep(video);
        return;
      }
      ctx = canvas.getContext("2d");
      input(); connect();
    },
    parse,
  };
})();
