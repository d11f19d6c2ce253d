"""Pure-Python VP8 decoder (RFC 6386) for the subset mxdesk's VP8 encoder emits: the oracle for
its inter frames (no libvpx / ffmpeg in this image; key frames are also checked against libwebp
through Pillow, tests/test_vp8.py).

Written from the decoding side of the RFC: boolean decoder (7), frame header (9, 19.2), token
probability and motion-vector probability updates (13.4, 17.2), key-frame and inter-frame mode
parsing (11, 16) with the near-vector search (16.3), token decoding with contexts (13),
dequantisation (14.1) with per-segment quantisers (9.3), inverse WHT / DCT (14.3, 14.4), 16x16 and
chroma intra prediction with the 127 / 129 frame edges (12), and six-tap inter prediction (18).

Supported: key and inter frames, 16x16 intra modes, key-frame B_PRED macroblocks (the ten 4x4
sub-block modes of 12.3 under the contextual key-frame probabilities, no Y2 block, the Y2 entropy
context carried past them), 16x16 inter macroblocks (ZERO / NEAREST / NEAR / NEW vectors, last-frame
reference), segmentation (segment map, absolute / delta segment quantisers and loop-filter levels),
the normal loop filter (15), token partitions, probability updates, skip flags.  Raises
``NotImplementedError`` for B_PRED in inter frames, SPLITMV, the simple filter, filter sharpness,
mode / reference filter deltas and golden / altref references.  Slow; for test pictures.
"""
from __future__ import annotations

import numpy as np

from .vp8_tables import AC_Q, COEF_PROBS0, COEF_UPDATE_PROBS, DC_Q, KF_BMODE_PROB

ZIGZAG = [0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15]
BANDS = [0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0]
PCAT = [[159], [165, 145], [173, 148, 140], [176, 155, 140, 135], [180, 157, 141, 134, 130],
        [254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129]]
CAT_BASE = [5, 7, 11, 19, 35, 67]
KF_YMODE_PROB = [145, 156, 163, 128]
KF_UVMODE_PROB = [142, 114, 183]
YMODE_PROB = [112, 86, 140, 37]
UVMODE_PROB = [162, 101, 204]
MV_DEFAULT = [[162, 128, 225, 146, 172, 147, 214, 39, 156, 128, 129, 132, 75, 145, 178, 206, 239, 254, 254],
              [164, 128, 204, 170, 119, 235, 140, 230, 228, 128, 130, 130, 74, 148, 180, 203, 236, 254, 254]]
MV_UPDATE = [[237, 246, 253, 253, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 250, 250, 252, 254, 254],
             [231, 243, 245, 253, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 251, 251, 254, 254, 254]]
MODE_CONTEXTS = [[7, 1, 1, 143], [14, 18, 14, 107], [135, 64, 57, 68], [60, 56, 128, 65], [159, 134, 128, 34],
                 [234, 188, 128, 28]]
SUBPEL = [[0, 0, 128, 0, 0, 0], [0, -6, 123, 12, -1, 0], [2, -11, 108, 36, -8, 1], [0, -9, 93, 50, -6, 0],
          [3, -16, 77, 77, -16, 3], [0, -6, 50, 93, -9, 0], [1, -8, 36, 108, -11, 2], [0, -1, 12, 123, -6, 0]]
DC_PRED, V_PRED, H_PRED, TM_PRED, B_PRED = 0, 1, 2, 3, 4
# sub-block modes, in the bmode tree's leaf order (the index order of KF_BMODE_PROB [above][left][9])
B_DC, B_TM, B_VE, B_HE, B_RD, B_VR, B_LD, B_VL, B_HD, B_HU = range(10)
IMPLIED_BMODE = {DC_PRED: B_DC, V_PRED: B_VE, H_PRED: B_HE, TM_PRED: B_TM}


class Vp8Error(Exception):
    pass


class BoolDecoder:
    """RFC 6386 section 7.3."""

    def __init__(self, data: bytes, start: int = 0, end: int | None = None):
        self.d = data
        self.pos = start
        self.end = len(data) if end is None else end
        self.value = (self._byte() << 8) | self._byte()
        self.range = 255
        self.bit_count = 0

    def _byte(self) -> int:
        if self.pos < self.end:
            b = self.d[self.pos]
            self.pos += 1
            return b
        self.pos += 1
        return 0

    def bool(self, prob: int) -> int:
        split = 1 + (((self.range - 1) * prob) >> 8)
        big = split << 8
        if self.value >= big:
            ret = 1
            self.range -= split
            self.value -= big
        else:
            ret = 0
            self.range = split
        while self.range < 128:
            self.value <<= 1
            self.range <<= 1
            self.bit_count += 1
            if self.bit_count == 8:
                self.bit_count = 0
                self.value |= self._byte()
        return ret

    def lit(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bool(128)
        return v

    def signed(self, n: int) -> int:
        v = self.lit(n)
        return -v if self.bool(128) else v


def _iwht(c):
    t = [0] * 16
    for i in range(4):
        a1, b1 = c[i] + c[12 + i], c[4 + i] + c[8 + i]
        c1, d1 = c[4 + i] - c[8 + i], c[i] - c[12 + i]
        t[i], t[4 + i], t[8 + i], t[12 + i] = a1 + b1, c1 + d1, a1 - b1, d1 - c1
    out = [0] * 16
    for i in range(4):
        a1, b1 = t[4 * i] + t[4 * i + 3], t[4 * i + 1] + t[4 * i + 2]
        c1, d1 = t[4 * i + 1] - t[4 * i + 2], t[4 * i] - t[4 * i + 3]
        out[4 * i:4 * i + 4] = [(a1 + b1 + 3) >> 3, (c1 + d1 + 3) >> 3, (a1 - b1 + 3) >> 3, (d1 - c1 + 3) >> 3]
    return out


def _idct(c):
    C8, S8 = 20091, 35468
    if not any(c[1:]):
        return [(c[0] + 4) >> 3] * 16
    t = [0] * 16
    for i in range(4):
        i0, i4, i8, i12 = c[i], c[4 + i], c[8 + i], c[12 + i]
        a1, b1 = i0 + i8, i0 - i8
        c1 = ((i4 * S8) >> 16) - (i12 + ((i12 * C8) >> 16))
        d1 = (i4 + ((i4 * C8) >> 16)) + ((i12 * S8) >> 16)
        t[i], t[12 + i], t[4 + i], t[8 + i] = a1 + d1, a1 - d1, b1 + c1, b1 - c1
    out = [0] * 16
    for i in range(4):
        r = t[4 * i:4 * i + 4]
        a1, b1 = r[0] + r[2], r[0] - r[2]
        c1 = ((r[1] * S8) >> 16) - (r[3] + ((r[3] * C8) >> 16))
        d1 = (r[1] + ((r[1] * C8) >> 16)) + ((r[3] * S8) >> 16)
        out[4 * i:4 * i + 4] = [(a1 + d1 + 4) >> 3, (b1 + c1 + 4) >> 3, (b1 - c1 + 4) >> 3, (a1 - d1 + 4) >> 3]
    return out


class Decoder:
    """``decode(frames)`` -> list of (Y, U, V) uint8 planes (display size); ``frames_coded`` keeps
    the macroblock-aligned planes; ``modes`` the last frame's per-MB (ymode, mv) records."""

    def __init__(self):
        self.frames = []
        self.frames_coded = []
        self.last = None
        self.w = self.h = 0
        self.stats = {"key": 0, "inter": 0, "skip": 0, "zero": 0, "nearest": 0, "near": 0, "new": 0}

    # ------------------------------------------------------------------ frame
    def decode(self, frames: list[bytes]):
        for f in frames:
            self.decode_frame(f)
        return self.frames

    def decode_frame(self, buf: bytes):
        if len(buf) < 3:
            raise Vp8Error("truncated frame tag")
        tag = buf[0] | (buf[1] << 8) | (buf[2] << 16)
        key = not (tag & 1)
        version = (tag >> 1) & 7
        first_size = tag >> 5
        if version != 0:
            raise NotImplementedError(f"version {version} (bilinear / full-pixel filters)")
        pos = 3
        if key:
            if buf[3:6] != b"\x9d\x01\x2a":
                raise Vp8Error("bad key-frame start code")
            self.w = (buf[6] | (buf[7] << 8)) & 0x3FFF
            self.h = (buf[8] | (buf[9] << 8)) & 0x3FFF
            pos = 10
            self.coef = list(COEF_PROBS0)
            self.mvp = [list(MV_DEFAULT[0]), list(MV_DEFAULT[1])]
            self.ymode_prob, self.uvmode_prob = list(YMODE_PROB), list(UVMODE_PROB)
        elif self.last is None:
            raise Vp8Error("inter frame without a key frame")
        mw, mh = (self.w + 15) // 16, (self.h + 15) // 16
        self.mw, self.mh = mw, mh
        bd = BoolDecoder(buf, pos, pos + first_size)
        if key:
            bd.lit(1)  # color space
            self.clamping = bd.lit(1)
        seg_on = bd.lit(1)
        update_map = 0
        if key:
            self.seg_abs, self.seg_q, self.seg_lf = 0, [0, 0, 0, 0], [0, 0, 0, 0]
            self.seg_probs = [255, 255, 255]
            self.lf_deltas = [0] * 8
        if seg_on:  # 9.3: segment quantisers and loop-filter levels (absolute or delta), map probabilities
            update_map = bd.lit(1)
            if bd.lit(1):  # update_segment_feature_data
                self.seg_abs = bd.lit(1)
                self.seg_q = [(bd.signed(7) if bd.lit(1) else 0) for _ in range(4)]
                self.seg_lf = [(bd.signed(6) if bd.lit(1) else 0) for _ in range(4)]
            if update_map:
                self.seg_probs = [bd.lit(8) if bd.lit(1) else 255 for _ in range(3)]
        simple = bd.lit(1)  # filter type
        level = bd.lit(6)
        sharpness = bd.lit(3)
        if bd.lit(1):  # loop_filter_adj_enable: reference / mode level deltas (persist between frames)
            if bd.lit(1):
                for k in range(8):
                    if bd.lit(1):
                        self.lf_deltas[k] = bd.signed(6)
            if any(self.lf_deltas):
                raise NotImplementedError("loop-filter mode / reference deltas")
        if level and (simple or sharpness):
            raise NotImplementedError("simple loop filter / sharpness")
        # 15.1: per-segment filter levels (absolute or added to the frame level), 0..63
        lf_seg = [min(63, max(0, (self.seg_lf[k] if self.seg_abs else level + self.seg_lf[k]) if seg_on else level))
                  for k in range(4)]
        nparts = 1 << bd.lit(2)
        qi = bd.lit(7)
        deltas = [bd.signed(4) if bd.lit(1) else 0 for _ in range(5)]  # y_dc, y2_dc, y2_ac, uv_dc, uv_ac
        q = lambda base, d: min(127, max(0, base + d))  # noqa: E731

        def quant(qb):
            return {
                "y1dc": DC_Q[q(qb, deltas[0])], "y1ac": AC_Q[q(qb, 0)],
                "y2dc": 2 * DC_Q[q(qb, deltas[1])], "y2ac": max(8, AC_Q[q(qb, deltas[2])] * 155 // 100),
                "uvdc": min(132, DC_Q[q(qb, deltas[3])]), "uvac": AC_Q[q(qb, deltas[4])],
            }
        self.q = quant(qi)
        # per-segment quantisers (segment_feature_mode 1: absolute indices, 0: deltas on y_ac_qi)
        self.seg_quant = [quant(self.seg_q[k] if self.seg_abs else q(qi, self.seg_q[k])) for k in range(4)] \
            if seg_on else [self.q] * 4
        saved = None
        if key:
            refresh_probs = bd.lit(1)
        else:
            if bd.lit(1) or bd.lit(1):
                raise NotImplementedError("golden / altref refresh")
            bd.lit(2)
            bd.lit(2)  # copy_buffer_to_golden / altref (ignored: never referenced)
            bd.lit(1)
            bd.lit(1)  # sign bias
            refresh_probs = bd.lit(1)
            bd.lit(1)  # refresh_last
        if not refresh_probs:
            saved = (list(self.coef), [list(p) for p in self.mvp], list(self.ymode_prob), list(self.uvmode_prob))
        for i in range(1056):
            if bd.bool(COEF_UPDATE_PROBS[i]):
                self.coef[i] = bd.lit(8)
        skip_on = bd.lit(1)
        prob_skip = bd.lit(8) if skip_on else 0
        if not key:
            prob_intra, prob_last = bd.lit(8), bd.lit(8)
            bd.lit(8)  # prob_gf
            if bd.lit(1):
                self.ymode_prob = [bd.lit(8) for _ in range(4)]
            if bd.lit(1):
                self.uvmode_prob = [bd.lit(8) for _ in range(3)]
            for c in range(2):
                for k in range(19):
                    if bd.bool(MV_UPDATE[c][k]):
                        x = bd.lit(7)
                        self.mvp[c][k] = (x << 1) if x else 1
        # ---- per-MB modes
        mbs = []
        if not hasattr(self, "seg_map") or len(self.seg_map) != mw * mh or key:
            self.seg_map = [0] * (mw * mh)
        for my in range(mh):
            for mx in range(mw):
                if update_map:  # segment_id (tree {2, 4, -0, -1, -2, -3})
                    sp = self.seg_probs
                    self.seg_map[my * mw + mx] = (2 + bd.bool(sp[2])) if bd.bool(sp[0]) else bd.bool(sp[1])
                    k = "seg%d" % self.seg_map[my * mw + mx]
                    self.stats[k] = self.stats.get(k, 0) + 1
                skip = bd.bool(prob_skip) if skip_on else 0
                if key:
                    ym = self._tree_kf_ymode(bd)
                    if ym == B_PRED:  # 16 sub-block modes, each under its above / left sub-block's mode
                        bm = [0] * 16
                        for b in range(16):
                            bx, by = b & 3, b >> 2
                            a = bm[b - 4] if by else (mbs[(my - 1) * mw + mx]["b"][12 + bx] if my else B_DC)
                            lm = bm[b - 1] if bx else (mbs[my * mw + mx - 1]["b"][4 * by + 3] if mx else B_DC)
                            bm[b] = self._tree_bmode(bd, KF_BMODE_PROB[(a * 10 + lm) * 9:(a * 10 + lm) * 9 + 9])
                        self.stats["bpred"] = self.stats.get("bpred", 0) + 1
                    else:
                        bm = [IMPLIED_BMODE[ym]] * 16
                    uvm = self._tree_uv(bd, KF_UVMODE_PROB)
                    mbs.append({"inter": False, "y": ym, "uv": uvm, "skip": skip, "mv": (0, 0), "b": bm})
                    continue
                if not bd.bool(prob_intra):
                    ym = self._tree_ymode(bd)
                    uvm = self._tree_uv(bd, self.uvmode_prob)
                    self.stats["intra_p"] = self.stats.get("intra_p", 0) + 1
                    mbs.append({"inter": False, "y": ym, "uv": uvm, "skip": skip, "mv": (0, 0)})
                    continue
                if bd.bool(prob_last):
                    raise NotImplementedError("golden / altref reference")
                near, cnt = self._near_mvs(mbs, mx, my)
                p = [MODE_CONTEXTS[cnt[i]][i] for i in range(4)]
                if not bd.bool(p[0]):
                    mv, kind = (0, 0), "zero"
                elif not bd.bool(p[1]):
                    mv, kind = near[1], "nearest"
                elif not bd.bool(p[2]):
                    mv, kind = near[2], "near"
                elif not bd.bool(p[3]):
                    dy = self._mv_component(bd, self.mvp[0]) * 2
                    dx = self._mv_component(bd, self.mvp[1]) * 2
                    mv, kind = (near[0][0] + dx, near[0][1] + dy), "new"
                    lo_x, hi_x, lo_y, hi_y = self._mv_limits(mx, my)
                    if not (lo_x <= mv[0] <= hi_x and lo_y <= mv[1] <= hi_y):
                        raise NotImplementedError("vector outside the clamping range")
                else:
                    raise NotImplementedError("SPLITMV")
                self.stats[kind] += 1
                mbs.append({"inter": True, "y": None, "uv": None, "skip": skip, "mv": mv})
        self.modes = mbs
        # ---- token partitions
        p0 = pos + first_size
        sizes_at = p0
        data_at = p0 + 3 * (nparts - 1)
        parts = []
        for k in range(nparts):
            if k < nparts - 1:
                n = buf[sizes_at + 3 * k] | (buf[sizes_at + 3 * k + 1] << 8) | (buf[sizes_at + 3 * k + 2] << 16)
            else:
                n = len(buf) - data_at
            parts.append(BoolDecoder(buf, data_at, data_at + n))
            data_at += n
        # ---- reconstruction
        Y = np.zeros((mh * 16, mw * 16), np.int32)
        U = np.zeros((mh * 8, mw * 8), np.int32)
        V = np.zeros((mh * 8, mw * 8), np.int32)
        above = [[0] * 9 for _ in range(mw)]
        for my in range(mh):
            bd = parts[my % nparts]
            left = [0] * 9
            for mx in range(mw):
                m = mbs[my * mw + mx]
                has_y2 = m["y"] != B_PRED
                if m["skip"]:
                    self.stats["skip"] += 1
                    coefs = [[0] * 16 for _ in range(25)]
                    for k in range(9 if has_y2 else 8):  # contexts reset (Y2's only with a Y2 block)
                        above[mx][k] = left[k] = 0
                else:
                    coefs = self._tokens(bd, above[mx], left, has_y2)
                # inner edges are filtered where a coefficient is coded, and always in B_PRED
                m["coded"] = any(any(c) for c in coefs) or not has_y2
                self._recon(Y, U, V, mx, my, m, coefs, key)
        if level:  # section 15: after the whole frame is reconstructed (intra prediction saw it unfiltered)
            self._loop_filter(Y, U, V, mbs, [lf_seg[self.seg_map[i]] if seg_on else level for i in range(mw * mh)], key)
            self.stats["filtered"] = self.stats.get("filtered", 0) + 1
        if saved is not None:
            self.coef, self.mvp, self.ymode_prob, self.uvmode_prob = saved
        self.stats["key" if key else "inter"] += 1
        self.last = (Y, U, V)
        y8, u8, v8 = (p.astype(np.uint8) for p in (Y, U, V))
        self.frames_coded.append((y8, u8, v8))
        self.frames.append((y8[:self.h, :self.w], u8[:(self.h + 1) // 2, :(self.w + 1) // 2],
                            v8[:(self.h + 1) // 2, :(self.w + 1) // 2]))

    # ------------------------------------------------------------------ modes
    @staticmethod
    def _tree_kf_ymode(bd):
        p = KF_YMODE_PROB
        if not bd.bool(p[0]):
            return B_PRED
        if not bd.bool(p[1]):
            return V_PRED if bd.bool(p[2]) else DC_PRED
        return TM_PRED if bd.bool(p[3]) else H_PRED

    def _tree_ymode(self, bd):
        p = self.ymode_prob  # DC "0", V "100", H "101", TM "110", B_PRED "111"
        if not bd.bool(p[0]):
            return DC_PRED
        if not bd.bool(p[1]):
            return H_PRED if bd.bool(p[2]) else V_PRED
        if bd.bool(p[3]):
            raise NotImplementedError("B_PRED")
        return TM_PRED

    @staticmethod
    def _tree_bmode(bd, p):  # 11.2 bmode_tree
        if not bd.bool(p[0]):
            return B_DC
        if not bd.bool(p[1]):
            return B_TM
        if not bd.bool(p[2]):
            return B_VE
        if not bd.bool(p[3]):
            if not bd.bool(p[4]):
                return B_HE
            return B_VR if bd.bool(p[5]) else B_RD
        if not bd.bool(p[6]):
            return B_LD
        if not bd.bool(p[7]):
            return B_VL
        return B_HU if bd.bool(p[8]) else B_HD

    @staticmethod
    def _tree_uv(bd, p):
        if not bd.bool(p[0]):
            return DC_PRED
        if not bd.bool(p[1]):
            return V_PRED
        return TM_PRED if bd.bool(p[2]) else H_PRED

    def _mv_limits(self, mx, my):
        return (-((mx * 16) << 3) - 128, (((self.mw - 1 - mx) * 16) << 3) + 128,
                -((my * 16) << 3) - 128, (((self.mh - 1 - my) * 16) << 3) + 128)

    def _near_mvs(self, mbs, mx, my):
        mv = [(0, 0)] * 4
        cnt = [0, 0, 0, 0]
        idx = 0
        for nx, ny, w in ((mx, my - 1, 2), (mx - 1, my, 2), (mx - 1, my - 1, 1)):
            if nx < 0 or ny < 0:
                continue
            n = mbs[ny * self.mw + nx]
            if not n["inter"]:
                continue
            if n["mv"] != (0, 0):
                if idx == 0 or n["mv"] != mv[idx]:
                    idx += 1
                    mv[idx] = n["mv"]
                cnt[idx] += w
            else:
                cnt[0] += w
        if cnt[3] and mv[idx] == mv[1]:
            cnt[1] += 1
        cnt[3] = 0  # SPLITMV neighbours (none decoded)
        if cnt[2] > cnt[1]:
            cnt[1], cnt[2] = cnt[2], cnt[1]
            mv[1], mv[2] = mv[2], mv[1]
        if cnt[1] >= cnt[0]:
            mv[0] = mv[1]
        lo_x, hi_x, lo_y, hi_y = self._mv_limits(mx, my)
        near = [(min(max(v[0], lo_x), hi_x), min(max(v[1], lo_y), hi_y)) for v in mv[:3]]
        return near, cnt

    @staticmethod
    def _mv_component(bd, p):
        if bd.bool(p[0]):
            x = 0
            for i in range(3):
                x += bd.bool(p[9 + i]) << i
            for i in range(9, 3, -1):
                x += bd.bool(p[9 + i]) << i
            if not (x & 0xFFF0) or bd.bool(p[9 + 3]):
                x += 8
        else:
            if not bd.bool(p[2]):
                x = (2 + bd.bool(p[5])) if bd.bool(p[3]) else bd.bool(p[4])
            else:
                x = (6 + bd.bool(p[8])) if bd.bool(p[6]) else (4 + bd.bool(p[7]))
        if x and bd.bool(p[1]):
            x = -x
        return x

    # ------------------------------------------------------------------ tokens
    def _block(self, bd, typ, first, ctx):
        out = [0] * 16
        i = first
        prev_zero = False
        while i < 16:
            b0 = ((typ * 8 + BANDS[i]) * 3 + ctx) * 11
            p = self.coef[b0:b0 + 11]
            if not prev_zero and not bd.bool(p[0]):
                break  # EOB
            if not bd.bool(p[1]):
                ctx, prev_zero = 0, True
                i += 1
                continue
            if not bd.bool(p[2]):
                v = 1
            elif not bd.bool(p[3]):
                if not bd.bool(p[4]):
                    v = 2
                else:
                    v = 4 if bd.bool(p[5]) else 3
            elif not bd.bool(p[6]):
                cat = 1 if bd.bool(p[7]) else 0
                v = CAT_BASE[cat] + self._extra(bd, PCAT[cat])
            elif not bd.bool(p[8]):
                cat = 3 if bd.bool(p[9]) else 2
                v = CAT_BASE[cat] + self._extra(bd, PCAT[cat])
            else:
                cat = 5 if bd.bool(p[10]) else 4
                v = CAT_BASE[cat] + self._extra(bd, PCAT[cat])
            ctx = 1 if v == 1 else 2
            if bd.bool(128):
                v = -v
            out[i] = v
            prev_zero = False
            i += 1
        return out

    @staticmethod
    def _extra(bd, probs):
        v = 0
        for p in probs:
            v = (v << 1) | bd.bool(p)
        return v

    def _tokens(self, bd, above, left, has_y2=True):
        coefs = [None] * 25
        nz = lambda c, first: int(any(c[first:]))  # noqa: E731
        if has_y2:
            c = self._block(bd, 1, 0, above[8] + left[8])
            coefs[24] = c
            above[8] = left[8] = nz(c, 0)
        else:
            coefs[24] = [0] * 16
        typ, first = (0, 1) if has_y2 else (3, 0)
        for b in range(16):
            bx, by = b & 3, b >> 2
            c = self._block(bd, typ, first, above[bx] + left[by])
            coefs[b] = c
            above[bx] = left[by] = nz(c, first)
        for comp in range(2):
            for b in range(4):
                bx, by = b & 1, b >> 1
                k = 4 + 2 * comp
                c = self._block(bd, 2, 0, above[k + bx] + left[k + by])
                coefs[16 + 4 * comp + b] = c
                above[k + bx] = left[k + by] = nz(c, 0)
        return coefs

    # ------------------------------------------------------------------ reconstruction
    def _recon(self, Y, U, V, mx, my, m, coefs, key):
        q = self.seg_quant[self.seg_map[my * self.mw + mx]]
        x0, y0 = mx * 16, my * 16
        if m["inter"]:
            pred = self._inter_pred(self.last[0], x0, y0, 16, m["mv"][0], m["mv"][1])
            # chroma vector: the luma vector halved, rounded away from zero (18.4)
            half = lambda v: (v + 1) // 2 if v >= 0 else -((1 - v) // 2)  # noqa: E731
            cvx, cvy = half(m["mv"][0]), half(m["mv"][1])
            cpred = [self._inter_pred(P, x0 // 2, y0 // 2, 8, cvx, cvy) for P in self.last[1:]]
        elif m["y"] == B_PRED:
            cpred = [self._intra_pred(P, x0 // 2, y0 // 2, 8, m["uv"]) for P in (U, V)]
            for b in range(16):  # raster order, each sub-block predicted from the ones before it
                bx, by = b & 3, b >> 2
                c = [0] * 16
                for k in range(16):
                    c[ZIGZAG[k]] = coefs[b][k] * (q["y1dc"] if k == 0 else q["y1ac"])
                pr = self._bpred(Y, mx, my, bx, by, m["b"][b])
                xs, ys = x0 + 4 * bx, y0 + 4 * by
                Y[ys:ys + 4, xs:xs + 4] = np.clip(pr + np.array(_idct(c)).reshape(4, 4), 0, 255)
            pred = None
        else:
            pred = self._intra_pred(Y, x0, y0, 16, m["y"])
            cpred = [self._intra_pred(P, x0 // 2, y0 // 2, 8, m["uv"]) for P in (U, V)]
        if pred is None:
            self._recon_chroma(U, V, x0, y0, coefs, cpred, q)
            return
        # luma with Y2
        y2 = [0] * 16
        for k, v in enumerate(coefs[24]):
            y2[ZIGZAG[k]] = v * (q["y2dc"] if k == 0 else q["y2ac"])
        dcs = _iwht(y2)
        res = np.zeros((16, 16), np.int64)
        for b in range(16):
            c = [0] * 16
            for k in range(1, 16):
                c[ZIGZAG[k]] = coefs[b][k] * q["y1ac"]
            c[0] = dcs[b]
            r = _idct(c)
            bx, by = b & 3, b >> 2
            res[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4] = np.array(r).reshape(4, 4)
        Y[y0:y0 + 16, x0:x0 + 16] = np.clip(pred + res, 0, 255)
        self._recon_chroma(U, V, x0, y0, coefs, cpred, q)

    @staticmethod
    def _recon_chroma(U, V, x0, y0, coefs, cpred, q):
        for comp, P in enumerate((U, V)):
            cres = np.zeros((8, 8), np.int64)
            for b in range(4):
                c = [0] * 16
                for k, v in enumerate(coefs[16 + 4 * comp + b]):
                    c[ZIGZAG[k]] = v * (q["uvdc"] if k == 0 else q["uvac"])
                bx, by = b & 1, b >> 1
                cres[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4] = np.array(_idct(c)).reshape(4, 4)
            P[y0 // 2:y0 // 2 + 8, x0 // 2:x0 // 2 + 8] = np.clip(cpred[comp] + cres, 0, 255)

    def _bpred(self, Y, mx, my, bx, by, mode):
        """12.3: sub-block (bx, by) of macroblock (mx, my) in `mode` from the reconstruction Y.
        Above-right: inside the macroblock from the sub-block row above; otherwise (the top row, the
        right column) from the row above the macroblock -- the above-right macroblock's bottom row,
        at the right frame edge the above macroblock's last sample repeated, 127 above the frame."""
        x, y = mx * 16 + 4 * bx, my * 16 + 4 * by
        A = [int(v) for v in Y[y - 1, x:x + 4]] if y > 0 else [127] * 4
        if by > 0 and bx < 3:
            A += [int(v) for v in Y[y - 1, x + 4:x + 8]]
        elif my == 0:
            A += [127] * 4
        elif bx < 3:
            A += [int(v) for v in Y[my * 16 - 1, x + 4:x + 8]]
        elif mx + 1 < self.mw:
            A += [int(v) for v in Y[my * 16 - 1, mx * 16 + 16:mx * 16 + 20]]
        else:
            A += [int(Y[my * 16 - 1, mx * 16 + 15])] * 4
        L = [int(v) for v in Y[y:y + 4, x - 1]] if x > 0 else [129] * 4
        P = 127 if y == 0 else (129 if x == 0 else int(Y[y - 1, x - 1]))
        E = [L[3], L[2], L[1], L[0], P] + A  # the edge from the bottom-left around to the top-right
        a3 = lambda a, b, c: (a + 2 * b + c + 2) >> 2  # noqa: E731
        a2 = lambda a, b: (a + b + 1) >> 1  # noqa: E731
        B = np.zeros((4, 4), np.int64)
        for r in range(4):
            for c in range(4):
                if mode == B_DC:
                    v = (sum(A[:4]) + sum(L) + 4) >> 3
                elif mode == B_TM:
                    v = min(255, max(0, L[r] + A[c] - P))
                elif mode == B_VE:
                    v = a3(E[4 + c], E[5 + c], E[6 + c])
                elif mode == B_HE:
                    v = a3(E[4 - r], E[3 - r], E[2 - r]) if r < 3 else a3(L[2], L[3], L[3])
                elif mode == B_LD:
                    v = a3(A[r + c], A[r + c + 1], A[min(r + c + 2, 7)])
                elif mode == B_RD:
                    v = a3(E[3 - r + c], E[4 - r + c], E[5 - r + c])
                elif mode == B_VR:
                    z = 2 * c - r
                    if z < 0:  # down the left edge
                        v = a3(E[4 + z], E[5 + z], E[6 + z])
                    elif z & 1:
                        v = a3(E[3 + (z + 1) // 2], E[4 + (z + 1) // 2], E[5 + (z + 1) // 2])
                    else:
                        v = a2(E[4 + z // 2], E[5 + z // 2])
                elif mode == B_VL:
                    if (r, c) == (2, 3):
                        v = a3(A[4], A[5], A[6])
                    elif (r, c) == (3, 3):
                        v = a3(A[5], A[6], A[7])
                    elif r & 1:
                        v = a3(A[c + r // 2], A[c + r // 2 + 1], A[c + r // 2 + 2])
                    else:
                        v = a2(A[c + r // 2], A[c + r // 2 + 1])
                elif mode == B_HD:
                    z = 2 * r - c
                    if z < 0:  # along the top edge
                        v = a3(E[2 - z], E[3 - z], E[4 - z])
                    elif z & 1:
                        v = a3(E[3 - (z + 1) // 2], E[4 - (z + 1) // 2], E[5 - (z + 1) // 2])
                    else:
                        v = a2(E[3 - z // 2], E[4 - z // 2])
                else:  # B_HU
                    k = c + 2 * r
                    Lx = L + [L[3], L[3]]
                    v = L[3] if k > 5 else (a3(Lx[k // 2], Lx[k // 2 + 1], Lx[k // 2 + 2]) if k & 1 else a2(Lx[k // 2], Lx[k // 2 + 1]))
                B[r, c] = v
        return B

    @staticmethod
    def _intra_pred(P, x0, y0, n, mode):
        above = P[y0 - 1, x0:x0 + n].astype(np.int64) if y0 > 0 else np.full(n, 127, np.int64)
        left = P[y0:y0 + n, x0 - 1].astype(np.int64) if x0 > 0 else np.full(n, 129, np.int64)
        corner = 127 if y0 == 0 else (129 if x0 == 0 else int(P[y0 - 1, x0 - 1]))
        if mode == DC_PRED:
            s, cnt = 0, 0
            if y0 > 0:
                s += int(above.sum())
                cnt += 1
            if x0 > 0:
                s += int(left.sum())
                cnt += 1
            if cnt == 0:
                return np.full((n, n), 128, np.int64)
            shift = (3 if n == 16 else 2) + cnt
            return np.full((n, n), (s + (1 << (shift - 1))) >> shift, np.int64)
        if mode == V_PRED:
            return np.tile(above, (n, 1))
        if mode == H_PRED:
            return np.tile(left[:, None], (1, n))
        return np.clip(left[:, None] + above[None, :] - corner, 0, 255)

    # ------------------------------------------------------------------ loop filter (15)
    @staticmethod
    def _lf_edge(P, mb, level, key):
        """Filter the sample lines across one edge: P (8, n) = p3 p2 p1 p0 q0 q1 q2 q3 (int64),
        in place -- the normal filter of 15.3 (libvpx's arithmetic)."""
        lim = max(level, 1)
        elim = (level + 2) * 2 + lim if mb else level * 2 + lim
        t = ((2 if level >= 40 else 1 if level >= 15 else 0) if key else
             (3 if level >= 40 else 2 if level >= 20 else 1 if level >= 15 else 0))
        p3, p2, p1, p0, q0, q1, q2, q3 = P
        mask = ((np.abs(p0 - q0) * 2 + (np.abs(p1 - q1) >> 1) <= elim) & (np.abs(p3 - p2) <= lim)
                & (np.abs(p2 - p1) <= lim) & (np.abs(p1 - p0) <= lim) & (np.abs(q3 - q2) <= lim)
                & (np.abs(q2 - q1) <= lim) & (np.abs(q1 - q0) <= lim))
        hev = (np.abs(p1 - p0) > t) | (np.abs(q1 - q0) > t)
        s8 = lambda v: np.clip(v, -128, 127)  # noqa: E731
        ps2, ps1, ps0, qs0, qs1, qs2 = p2 - 128, p1 - 128, p0 - 128, q0 - 128, q1 - 128, q2 - 128
        if mb:
            w = s8(s8(ps1 - qs1) + 3 * (qs0 - ps0))
            a27, a18, a9 = s8((27 * w + 63) >> 7), s8((18 * w + 63) >> 7), s8((9 * w + 63) >> 7)
            n = [np.where(hev, ps2, s8(ps2 + a9)), np.where(hev, ps1, s8(ps1 + a18)),
                 np.where(hev, s8(ps0 + (s8(w + 3) >> 3)), s8(ps0 + a27)),
                 np.where(hev, s8(qs0 - (s8(w + 4) >> 3)), s8(qs0 - a27)),
                 np.where(hev, qs1, s8(qs1 - a18)), np.where(hev, qs2, s8(qs2 - a9))]
        else:
            a = s8(np.where(hev, s8(ps1 - qs1), 0) + 3 * (qs0 - ps0))
            f1, f2 = s8(a + 4) >> 3, s8(a + 3) >> 3
            o = (f1 + 1) >> 1
            n = [ps2, np.where(hev, ps1, s8(ps1 + o)), s8(ps0 + f2), s8(qs0 - f1), np.where(hev, qs1, s8(qs1 - o)), qs2]
        for k in range(6):
            P[1 + k] = np.where(mask, n[k] + 128, P[1 + k])

    def _loop_filter(self, Y, U, V, mbs, levels, key):
        """15.1: macroblocks in raster order; per macroblock and plane the left edge, the inner
        vertical edges, the top edge, the inner horizontal edges (inner ones only where the
        macroblock has coefficients)."""
        for my in range(self.mh):
            for mx in range(self.mw):
                i = my * self.mw + mx
                level = levels[i]
                if not level:
                    continue
                inner = mbs[i]["coded"]
                for P, n in ((Y, 16), (U, 8), (V, 8)):
                    x0, y0 = mx * n, my * n
                    edges_v = ([(x0, True)] if mx else []) + ([(x0 + e, False) for e in range(4, n, 4)] if inner else [])
                    for xe, mb in edges_v:
                        T = P[y0:y0 + n, xe - 4:xe + 4].T.copy()
                        self._lf_edge(T, mb, level, key)
                        P[y0:y0 + n, xe - 4:xe + 4] = T.T
                    edges_h = ([(y0, True)] if my else []) + ([(y0 + e, False) for e in range(4, n, 4)] if inner else [])
                    for ye, mb in edges_h:
                        T = P[ye - 4:ye + 4, x0:x0 + n].copy()
                        self._lf_edge(T, mb, level, key)
                        P[ye - 4:ye + 4, x0:x0 + n] = T

    @staticmethod
    def _inter_pred(P, x0, y0, n, mvx, mvy):
        """Six-tap prediction of an n x n block (vector in 1/8 samples of this plane), edge-extended."""
        H, W = P.shape
        ix, iy, fx, fy = mvx >> 3, mvy >> 3, mvx & 7, mvy & 7
        ys = np.clip(np.arange(y0 + iy - 2, y0 + iy + n + 3), 0, H - 1)
        xs = np.clip(np.arange(x0 + ix - 2, x0 + ix + n + 3), 0, W - 1)
        R = P[np.ix_(ys, xs)].astype(np.int64)  # (n+5, n+5)
        hf, vf = SUBPEL[fx], SUBPEL[fy]
        t = sum(hf[k] * R[:, k:k + n] for k in range(6))
        t = np.clip((t + 64) >> 7, 0, 255)
        o = sum(vf[k] * t[k:k + n, :] for k in range(6))
        return np.clip((o + 64) >> 7, 0, 255)


def ivf_frames(data: bytes) -> list[bytes]:
    """Frames of an IVF file (the container libvpx tools use)."""
    if data[:4] != b"DKIF":
        raise Vp8Error("not an IVF file")
    hl = data[6] | (data[7] << 8)
    pos, out = hl, []
    while pos + 12 <= len(data):
        n = int.from_bytes(data[pos:pos + 4], "little")
        out.append(data[pos + 12:pos + 12 + n])
        pos += 12 + n
    return out


def webp_container(key_frame: bytes) -> bytes:
    """Wrap a VP8 key frame in a RIFF/WEBP container (lossy WebP *is* a VP8 key frame), for
    decoding through libwebp (Pillow)."""
    chunk = key_frame + (b"\x00" if len(key_frame) & 1 else b"")
    body = b"WEBP" + b"VP8 " + len(key_frame).to_bytes(4, "little") + chunk
    return b"RIFF" + len(body).to_bytes(4, "little") + body
