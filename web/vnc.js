// mxdesk VNC viewer: the browser front end of NOVNC_ENABLE=true (the reference serves noVNC
// 1.4.0 on :8080 behind websockify, entrypoint.sh:120-125).  It speaks RFB 3.8 to the
// built-in server on /websockify: VNC authentication (DES challenge, RFC 6143 7.2.2), a
// 32-bpp RGBX pixel format, and ZRLE (RFC 6143 7.7.6) decoded with a small streaming inflate
// (the ZRLE zlib stream persists across rectangles, so the decoder keeps its 32 KiB window),
// plus Raw and DesktopSize.  The protocol core is transport-agnostic so it also runs under
// Node for the tests (tools/vnc_client_check.js).
"use strict";
(function (root) {
  // ------------------------------------------------------------------ DES (VNC auth only)
  const IP = [58, 50, 42, 34, 26, 18, 10, 2, 60, 52, 44, 36, 28, 20, 12, 4, 62, 54, 46, 38, 30, 22, 14, 6, 64, 56,
    48, 40, 32, 24, 16, 8, 57, 49, 41, 33, 25, 17, 9, 1, 59, 51, 43, 35, 27, 19, 11, 3, 61, 53, 45, 37, 29, 21, 13, 5,
    63, 55, 47, 39, 31, 23, 15, 7];
  const FP = [40, 8, 48, 16, 56, 24, 64, 32, 39, 7, 47, 15, 55, 23, 63, 31, 38, 6, 46, 14, 54, 22, 62, 30, 37, 5, 45,
    13, 53, 21, 61, 29, 36, 4, 44, 12, 52, 20, 60, 28, 35, 3, 43, 11, 51, 19, 59, 27, 34, 2, 42, 10, 50, 18, 58, 26,
    33, 1, 41, 9, 49, 17, 57, 25];
  const E = [32, 1, 2, 3, 4, 5, 4, 5, 6, 7, 8, 9, 8, 9, 10, 11, 12, 13, 12, 13, 14, 15, 16, 17, 16, 17, 18, 19, 20, 21,
    20, 21, 22, 23, 24, 25, 24, 25, 26, 27, 28, 29, 28, 29, 30, 31, 32, 1];
  const P = [16, 7, 20, 21, 29, 12, 28, 17, 1, 15, 23, 26, 5, 18, 31, 10, 2, 8, 24, 14, 32, 27, 3, 9, 19, 13, 30, 6,
    22, 11, 4, 25];
  const PC1 = [57, 49, 41, 33, 25, 17, 9, 1, 58, 50, 42, 34, 26, 18, 10, 2, 59, 51, 43, 35, 27, 19, 11, 3, 60, 52, 44,
    36, 63, 55, 47, 39, 31, 23, 15, 7, 62, 54, 46, 38, 30, 22, 14, 6, 61, 53, 45, 37, 29, 21, 13, 5, 28, 20, 12, 4];
  const PC2 = [14, 17, 11, 24, 1, 5, 3, 28, 15, 6, 21, 10, 23, 19, 12, 4, 26, 8, 16, 7, 27, 20, 13, 2, 41, 52, 31, 37,
    47, 55, 30, 40, 51, 45, 33, 48, 44, 49, 39, 56, 34, 53, 46, 42, 50, 36, 29, 32];
  const SHIFTS = [1, 1, 2, 2, 2, 2, 2, 2, 1, 2, 2, 2, 2, 2, 2, 1];
  const SBOX = [
    "e4d12fb83a6c5907 0f74e2d1a6cb9538 41e8d62bfc973a50 fc8249175b3ea06d",
    "f18e6b34972dc05a 3d47f28ec01a69b5 0e7ba4d158c6932f d8a13f42b67c05e9",
    "a09e63f51dc7b428 d709346a285ecbf1 d6498f30b12c5ae7 1ad069874fe3b52c",
    "7de3069a1285bc4f d8b56f03472c1ae9 a690cb7df13e5284 3f06a1d8945bc72e",
    "2c417ab6853fd0e9 eb2c47d150fa3986 421bad78f9c5630e b8c71e2d6f09a453",
    "c1af92680d34e75b af427c9561de0b38 9ef528c3704a1db6 432c95fabe17608d",
    "4b2ef08d3c975a61 d0b7491ae35c2f86 14bdc37eaf680592 6bd814a7950fe23c",
    "d2846fb1a93e50c7 1fd8a374c56b0e92 7b419ce206adf358 21e74a8dfc90356b",
  ].map((s) => Array.from(s.replace(/ /g, ""), (c) => parseInt(c, 16)));

  function desBlock(key8, block8) {
    const bits = (bytes) => { const o = []; for (const b of bytes) for (let i = 7; i >= 0; i--) o.push((b >> i) & 1); return o; };
    const perm = (v, t) => t.map((p) => v[p - 1]);
    const k = perm(bits(key8), PC1);
    let c = k.slice(0, 28), d = k.slice(28);
    const keys = [];
    for (const s of SHIFTS) {
      c = c.slice(s).concat(c.slice(0, s)); d = d.slice(s).concat(d.slice(0, s));
      keys.push(perm(c.concat(d), PC2));
    }
    const v = perm(bits(block8), IP);
    let L = v.slice(0, 32), R = v.slice(32);
    for (const K of keys) {
      const x = perm(R, E).map((b, i) => b ^ K[i]);
      const out = [];
      for (let i = 0; i < 8; i++) {
        const s = x.slice(6 * i, 6 * i + 6);
        const val = SBOX[i][((s[0] << 1) | s[5]) * 16 + ((s[1] << 3) | (s[2] << 2) | (s[3] << 1) | s[4])];
        for (let j = 3; j >= 0; j--) out.push((val >> j) & 1);
      }
      const f = perm(out, P);
      const nR = L.map((b, i) => b ^ f[i]);
      L = R; R = nR;
    }
    const o = perm(R.concat(L), FP);
    const res = new Uint8Array(8);
    for (let i = 0; i < 64; i++) res[i >> 3] |= o[i] << (7 - (i & 7));
    return res;
  }

  function vncResponse(password, challenge) {
    const key = new Uint8Array(8);
    for (let i = 0; i < 8 && i < password.length; i++) {
      let b = password.charCodeAt(i) & 0xff, r = 0;
      for (let j = 0; j < 8; j++) r |= ((b >> j) & 1) << (7 - j);
      key[i] = r;
    }
    const out = new Uint8Array(16);
    out.set(desBlock(key, challenge.subarray(0, 8)), 0);
    out.set(desBlock(key, challenge.subarray(8, 16)), 8);
    return out;
  }

  // ------------------------------------------------------------------ streaming inflate
  // RFC 1950/1951 decoder for a zlib stream delivered in sync-flushed pieces: each push()
  // holds whole deflate blocks, so only the 32 KiB history survives between pushes.
  const LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163,
    195, 227, 258];
  const LEXT = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0];
  const DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
    4097, 6145, 8193, 12289, 16385, 24577];
  const DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13];
  const CLORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15];

  function huffman(lengths) {  // canonical code: counts per length + symbols in code order
    const count = new Uint16Array(16), symbol = new Uint16Array(lengths.length), offs = new Uint16Array(16);
    for (const l of lengths) count[l]++;
    count[0] = 0;
    for (let i = 1; i < 16; i++) offs[i] = offs[i - 1] + count[i - 1];
    for (let s = 0; s < lengths.length; s++) if (lengths[s]) symbol[offs[lengths[s]]++] = s;
    return { count, symbol };
  }
  const FIXED_L = huffman(Array.from({ length: 288 }, (_, i) => (i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8)));
  const FIXED_D = huffman(new Array(30).fill(5));

  class Inflater {
    constructor() { this.hist = new Uint8Array(0); this.header = false; }

    push(data) {
      let pos = 0, bitbuf = 0, bitcnt = 0;
      const need = (n) => {
        while (bitcnt < n) {
          if (pos >= data.length) throw new Error("inflate: truncated input");
          bitbuf |= data[pos++] << bitcnt; bitcnt += 8;
        }
      };
      const bits = (n) => { need(n); const v = bitbuf & ((1 << n) - 1); bitbuf >>>= n; bitcnt -= n; return v; };
      const decode = (h) => {
        let code = 0, first = 0, index = 0;
        for (let len = 1; len < 16; len++) {
          code |= bits(1);
          const cnt = h.count[len];
          if (code - cnt < first) return h.symbol[index + (code - first)];
          index += cnt; first += cnt; first <<= 1; code <<= 1;
        }
        throw new Error("inflate: bad code");
      };
      if (!this.header) {
        const cmf = data[0], flg = data[1];
        if ((cmf & 15) !== 8 || ((cmf << 8) | flg) % 31 !== 0 || (flg & 32)) throw new Error("inflate: bad zlib header");
        pos = 2; this.header = true;
      }
      const base = this.hist.length;
      let out = new Uint8Array(Math.max(base + data.length * 4, 65536));
      out.set(this.hist);
      let n = base;
      const grow = (k) => { if (n + k > out.length) { const o = new Uint8Array(Math.max(out.length * 2, n + k)); o.set(out.subarray(0, n)); out = o; } };
      while (pos < data.length || bitcnt >= 3) {
        if (pos >= data.length && bitcnt < 8 && (bitbuf & ((1 << bitcnt) - 1)) === 0) break;  // flush padding
        const final = bits(1), type = bits(2);
        if (type === 0) {
          bitbuf = 0; bitcnt = 0;
          const len = data[pos] | (data[pos + 1] << 8);
          pos += 4;
          grow(len); out.set(data.subarray(pos, pos + len), n); n += len; pos += len;
        } else {
          let lt = FIXED_L, dt = FIXED_D;
          if (type === 2) {
            const hlit = bits(5) + 257, hdist = bits(5) + 1, hclen = bits(4) + 4;
            const cl = new Array(19).fill(0);
            for (let i = 0; i < hclen; i++) cl[CLORDER[i]] = bits(3);
            const ct = huffman(cl);
            const lens = [];
            while (lens.length < hlit + hdist) {
              const sym = decode(ct);
              if (sym < 16) lens.push(sym);
              else if (sym === 16) { const p = lens[lens.length - 1]; for (let r = 3 + bits(2); r > 0; r--) lens.push(p); }
              else if (sym === 17) { for (let r = 3 + bits(3); r > 0; r--) lens.push(0); }
              else { for (let r = 11 + bits(7); r > 0; r--) lens.push(0); }
            }
            lt = huffman(lens.slice(0, hlit)); dt = huffman(lens.slice(hlit));
          } else if (type !== 1) throw new Error("inflate: bad block type");
          for (;;) {
            const sym = decode(lt);
            if (sym < 256) { grow(1); out[n++] = sym; continue; }
            if (sym === 256) break;
            const len = LBASE[sym - 257] + bits(LEXT[sym - 257]);
            const ds = decode(dt);
            const dist = DBASE[ds] + bits(DEXT[ds]);
            if (dist > n) throw new Error("inflate: distance too far");
            grow(len);
            for (let i = 0; i < len; i++, n++) out[n] = out[n - dist];
          }
        }
        if (final) break;
      }
      const result = out.slice(base, n);
      this.hist = out.slice(Math.max(0, n - 32768), n);
      return result;
    }
  }

  // ------------------------------------------------------------------ RFB client core
  class ByteQueue {
    constructor() { this.chunks = []; this.len = 0; this.waiter = null; this.closed = false; }
    push(u8) { this.chunks.push(u8); this.len += u8.length; this._wake(); }
    close() { this.closed = true; this._wake(); }
    _wake() { if (this.waiter) { const w = this.waiter; this.waiter = null; w(); } }
    async read(n) {
      while (this.len < n) {
        if (this.closed) throw new Error("connection closed");
        await new Promise((r) => { this.waiter = r; });
      }
      const out = new Uint8Array(n);
      let k = 0;
      while (k < n) {
        const c = this.chunks[0], take = Math.min(c.length, n - k);
        out.set(c.subarray(0, take), k); k += take;
        if (take === c.length) this.chunks.shift(); else this.chunks[0] = c.subarray(take);
      }
      this.len -= n;
      return out;
    }
  }

  const u16 = (b, o) => (b[o] << 8) | b[o + 1];
  const u32 = (b, o) => ((b[o] << 24) >>> 0) + (b[o + 1] << 16) + (b[o + 2] << 8) + b[o + 3];

  class RfbClient {
    // send(Uint8Array); opts: password, onResize(w, h), onUpdate(), onBell(), onCutText(text)
    constructor(send, opts = {}) {
      this.send = send; this.opts = opts; this.q = new ByteQueue(); this.inflater = new Inflater();
      this.width = 0; this.height = 0; this.fb = null; this.name = ""; this.updates = 0;
    }
    feed(u8) { this.q.push(u8); }
    close() { this.q.close(); }

    async run() {
      const q = this.q;
      const ver = new TextDecoder().decode(await q.read(12));
      if (!ver.startsWith("RFB 003.")) throw new Error("not an RFB server");
      this.send(new TextEncoder().encode("RFB 003.008\n"));
      const nTypes = (await q.read(1))[0];
      if (nTypes === 0) { const l = u32(await q.read(4), 0); throw new Error(new TextDecoder().decode(await q.read(l))); }
      const types = await q.read(nTypes);
      const sec = types.includes(2) ? 2 : types.includes(1) ? 1 : -1;
      if (sec < 0) throw new Error("no supported security type");
      this.send(Uint8Array.of(sec));
      if (sec === 2) this.send(vncResponse(this.opts.password || "", await q.read(16)));
      const res = u32(await q.read(4), 0);
      if (res !== 0) { const l = u32(await q.read(4), 0); throw new Error("auth: " + new TextDecoder().decode(await q.read(l))); }
      this.send(Uint8Array.of(1));  // shared
      const si = await q.read(24);
      this._resize(u16(si, 0), u16(si, 2));
      this.name = new TextDecoder().decode(await q.read(u32(si, 20)));
      // 32 bpp, depth 24, little endian, true colour, R@0 G@8 B@16: RGBX bytes = canvas RGBA order
      this.send(Uint8Array.of(0, 0, 0, 0, 32, 24, 0, 1, 0, 255, 0, 255, 0, 255, 0, 8, 16, 0, 0, 0));
      const encs = [16, 0, -223];
      const se = new DataView(new ArrayBuffer(4 + 4 * encs.length));
      se.setUint8(0, 2); se.setUint16(2, encs.length);
      encs.forEach((e, i) => se.setInt32(4 + 4 * i, e));
      this.send(new Uint8Array(se.buffer));
      this.requestUpdate(false);
      for (;;) {
        const t = (await q.read(1))[0];
        if (t === 0) await this._update();
        else if (t === 1) { const h = await q.read(5); await q.read(6 * u16(h, 3)); }
        else if (t === 2) { if (this.opts.onBell) this.opts.onBell(); }
        else if (t === 3) {
          const h = await q.read(7);
          const raw = await q.read(u32(h, 3));
          let text = ""; for (let i = 0; i < raw.length; i++) text += String.fromCharCode(raw[i]);
          if (this.opts.onCutText) this.opts.onCutText(text);
        } else throw new Error("unknown server message " + t);
      }
    }

    _resize(w, h) {
      this.width = w; this.height = h;
      this.fb = new Uint8Array(w * h * 4);
      for (let i = 3; i < this.fb.length; i += 4) this.fb[i] = 255;
      if (this.opts.onResize) this.opts.onResize(w, h);
    }

    requestUpdate(incremental = true) {
      const b = new DataView(new ArrayBuffer(10));
      b.setUint8(0, 3); b.setUint8(1, incremental ? 1 : 0); b.setUint16(6, this.width); b.setUint16(8, this.height);
      this.send(new Uint8Array(b.buffer));
    }

    pointer(x, y, mask) {
      this.send(Uint8Array.of(5, mask & 255, (x >> 8) & 255, x & 255, (y >> 8) & 255, y & 255));
    }

    key(keysym, down) {
      this.send(Uint8Array.of(4, down ? 1 : 0, 0, 0, (keysym >>> 24) & 255, (keysym >> 16) & 255, (keysym >> 8) & 255, keysym & 255));
    }

    cutText(text) {
      const t = Uint8Array.from(text, (c) => c.charCodeAt(0) & 255);
      const m = new Uint8Array(8 + t.length);
      m[0] = 6; m[4] = (t.length >>> 24) & 255; m[5] = (t.length >> 16) & 255; m[6] = (t.length >> 8) & 255; m[7] = t.length & 255;
      m.set(t, 8);
      this.send(m);
    }

    async _update() {
      const q = this.q;
      const n = u16(await q.read(3), 1);
      for (let r = 0; r < n; r++) {
        const h = await q.read(12);
        const x = u16(h, 0), y = u16(h, 2), w = u16(h, 4), hh = u16(h, 6);
        const enc = (h[8] << 24) | (h[9] << 16) | (h[10] << 8) | h[11];
        if (enc === 0) this._blitRaw(x, y, w, hh, await q.read(w * hh * 4));
        else if (enc === 16) this._zrle(x, y, w, hh, this.inflater.push(await q.read(u32(await q.read(4), 0))));
        else if (enc === -223) this._resize(w, hh);
        else throw new Error("unsupported encoding " + enc);
      }
      this.updates++;
      if (this.opts.onUpdate) this.opts.onUpdate();
      this.requestUpdate(true);
    }

    _blitRaw(x, y, w, h, px) {
      const fb = this.fb, W = this.width;
      for (let j = 0; j < h; j++) {
        const d = ((y + j) * W + x) * 4, s = j * w * 4;
        for (let i = 0; i < w; i++) {
          fb[d + 4 * i] = px[s + 4 * i]; fb[d + 4 * i + 1] = px[s + 4 * i + 1]; fb[d + 4 * i + 2] = px[s + 4 * i + 2];
        }
      }
    }

    _zrle(rx, ry, rw, rh, data) {
      const fb = this.fb, W = this.width;
      let p = 0;
      const cpix = () => { const v = (data[p] << 16) | (data[p + 1] << 8) | data[p + 2]; p += 3; return v; };  // R G B
      const put = (x, y, v) => { const o = (y * W + x) * 4; fb[o] = v >> 16; fb[o + 1] = (v >> 8) & 255; fb[o + 2] = v & 255; };
      for (let ty = ry; ty < ry + rh; ty += 64) {
        for (let tx = rx; tx < rx + rw; tx += 64) {
          const tw = Math.min(64, rx + rw - tx), th = Math.min(64, ry + rh - ty);
          const sub = data[p++];
          if (sub === 0) {
            for (let j = 0; j < th; j++) for (let i = 0; i < tw; i++) put(tx + i, ty + j, cpix());
          } else if (sub === 1) {
            const v = cpix();
            for (let j = 0; j < th; j++) for (let i = 0; i < tw; i++) put(tx + i, ty + j, v);
          } else if (sub <= 16) {
            const pal = []; for (let k = 0; k < sub; k++) pal.push(cpix());
            const bpp = sub <= 2 ? 1 : sub <= 4 ? 2 : 4, mask = (1 << bpp) - 1;
            for (let j = 0; j < th; j++) {
              let byte = 0, left = 0;
              for (let i = 0; i < tw; i++) {
                if (left === 0) { byte = data[p++]; left = 8; }
                left -= bpp;
                put(tx + i, ty + j, pal[(byte >> left) & mask]);
              }
            }
          } else if (sub === 128 || sub >= 130) {
            const pal = []; if (sub >= 130) for (let k = 0; k < sub - 128; k++) pal.push(cpix());
            let i = 0;
            const total = tw * th;
            while (i < total) {
              let v, run = 1;
              if (sub === 128) { v = cpix(); run = 0; } else {
                const idx = data[p++];
                v = pal[idx & 127];
                if (idx & 128) run = 0;
              }
              if (run === 0) { let b; run = 1; do { b = data[p++]; run += b; } while (b === 255); }
              for (let k = 0; k < run && i < total; k++, i++) put(tx + (i % tw), ty + ((i / tw) | 0), v);
            }
          } else throw new Error("bad ZRLE subencoding " + sub);
        }
      }
      if (p !== data.length) throw new Error(`ZRLE: ${data.length - p} trailing bytes`);
    }
  }

  const api = { RfbClient, Inflater, vncResponse, desBlock };
  if (typeof module !== "undefined" && module.exports) module.exports = api;
  else root.mxvnc = api;
})(typeof window !== "undefined" ? window : this);
