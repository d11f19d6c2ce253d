"""Minimal pure-Python H.264 decoder for the Constrained-Baseline CAVLC subset that
mxdesk emits (SURVEY.md §4.2 "encoder conformance": no ffmpeg/PyAV in this image, so this
is the oracle).  Written independently of the C++/HIP encoder: tables are transcribed as
the bit strings of the spec tables (ITU-T H.264 Tables 9-5, 9-7..9-10), decoding follows
the spec's parsing/decoding processes (7.3, 8.3, 8.4, 8.5, 9.2).

Supported: SPS/PPS (baseline subset incl. VUI skip), I and P slices, I_NxN (Intra4x4),
Intra16x16, I_PCM, P_L0_16x16 / 16x8 / 8x16, P_Skip, one reference frame, CAVLC,
frame cropping, and the in-loop deblocking filter (8.7: bS derivation 8.7.2.1, the alpha / beta /
tC0 tables 8-16 / 8-17, bS < 4 and bS == 4 luma and chroma filters, disable_deblocking_filter_idc
0 / 1 / 2 with the slice's alpha / beta offsets), applied per macroblock in raster order when a
picture is complete.

Slow (pure Python); intended for small test pictures.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# ----------------------------------------------------------------------------- tables
# coeff_token: {nC class: {bitstring: (TrailingOnes, TotalCoeff)}}
_CT_SRC = {
    # (T1, TC): [0<=nC<2, 2<=nC<4, 4<=nC<8, 8<=nC, nC==-1]
    (0, 0): ["1", "11", "1111", "000011", "01"],
    (0, 1): ["000101", "001011", "001111", "000000", "000111"],
    (1, 1): ["01", "10", "1110", "000001", "1"],
    (0, 2): ["00000111", "000111", "001011", "000100", "000100"],
    (1, 2): ["000100", "00111", "01111", "000101", "000110"],
    (2, 2): ["001", "011", "1101", "000110", "001"],
    (0, 3): ["000000111", "0000111", "001000", "001000", "000011"],
    (1, 3): ["00000110", "001010", "01100", "001001", "0000011"],
    (2, 3): ["0000101", "001001", "01110", "001010", "0000010"],
    (3, 3): ["00011", "0101", "1100", "001011", "000101"],
    (0, 4): ["0000000111", "00000111", "0001111", "001100", "000010"],
    (1, 4): ["000000110", "000110", "01010", "001101", "00000011"],
    (2, 4): ["00000101", "000101", "01011", "001110", "00000010"],
    (3, 4): ["000011", "0100", "1011", "001111", "0000000"],
    (0, 5): ["00000000111", "00000100", "0001011", "010000", None],
    (1, 5): ["0000000110", "0000110", "01000", "010001", None],
    (2, 5): ["000000101", "0000101", "01001", "010010", None],
    (3, 5): ["0000100", "00110", "1010", "010011", None],
    (0, 6): ["0000000001111", "000000111", "0001001", "010100", None],
    (1, 6): ["00000000110", "00000110", "001110", "010101", None],
    (2, 6): ["0000000101", "00000101", "001101", "010110", None],
    (3, 6): ["00000100", "001000", "1001", "010111", None],
    (0, 7): ["0000000001011", "00000001111", "0001000", "011000", None],
    (1, 7): ["0000000001110", "000000110", "001010", "011001", None],
    (2, 7): ["00000000101", "000000101", "001001", "011010", None],
    (3, 7): ["000000100", "000100", "1000", "011011", None],
    (0, 8): ["0000000001000", "00000001011", "00001111", "011100", None],
    (1, 8): ["0000000001010", "00000001110", "0001110", "011101", None],
    (2, 8): ["0000000001101", "00000001101", "0001101", "011110", None],
    (3, 8): ["0000000100", "0000100", "01101", "011111", None],
    (0, 9): ["00000000001111", "000000001111", "00001011", "100000", None],
    (1, 9): ["00000000001110", "00000001010", "00001110", "100001", None],
    (2, 9): ["0000000001001", "00000001001", "0001010", "100010", None],
    (3, 9): ["00000000100", "000000100", "001100", "100011", None],
    (0, 10): ["00000000001011", "000000001011", "000001111", "100100", None],
    (1, 10): ["00000000001010", "000000001110", "00001010", "100101", None],
    (2, 10): ["00000000001101", "000000001101", "00001101", "100110", None],
    (3, 10): ["0000000001100", "00000001100", "0001100", "100111", None],
    (0, 11): ["000000000001111", "000000001000", "000001011", "101000", None],
    (1, 11): ["000000000001110", "000000001010", "000001110", "101001", None],
    (2, 11): ["00000000001001", "000000001001", "00001001", "101010", None],
    (3, 11): ["00000000001100", "00000001000", "00001100", "101011", None],
    (0, 12): ["000000000001011", "0000000001111", "000001000", "101100", None],
    (1, 12): ["000000000001010", "0000000001110", "000001010", "101101", None],
    (2, 12): ["000000000001101", "0000000001101", "000001101", "101110", None],
    (3, 12): ["00000000001000", "000000001100", "00001000", "101111", None],
    (0, 13): ["0000000000001111", "0000000001011", "0000001101", "110000", None],
    (1, 13): ["000000000000001", "0000000001010", "000000111", "110001", None],
    (2, 13): ["000000000001001", "0000000001001", "000001001", "110010", None],
    (3, 13): ["000000000001100", "0000000001100", "000001100", "110011", None],
    (0, 14): ["0000000000001011", "0000000000111", "0000001001", "110100", None],
    (1, 14): ["0000000000001110", "00000000001011", "0000001100", "110101", None],
    (2, 14): ["0000000000001101", "0000000000110", "0000001011", "110110", None],
    (3, 14): ["000000000001000", "0000000001000", "0000001010", "110111", None],
    (0, 15): ["0000000000000111", "00000000001001", "0000000101", "111000", None],
    (1, 15): ["0000000000001010", "00000000001000", "0000001000", "111001", None],
    (2, 15): ["0000000000001001", "00000000001010", "0000000111", "111010", None],
    (3, 15): ["0000000000001100", "0000000000001", "0000000110", "111011", None],
    (0, 16): ["0000000000000100", "00000000000111", "0000000001", "111100", None],
    (1, 16): ["0000000000000110", "00000000000110", "0000000100", "111101", None],
    (2, 16): ["0000000000000101", "00000000000101", "0000000011", "111110", None],
    (3, 16): ["0000000000001000", "00000000000100", "0000000010", "111111", None],
}
COEFF_TOKEN: list[dict[str, tuple[int, int]]] = [{} for _ in range(5)]
for (_t1, _tc), _codes in _CT_SRC.items():
    for _cls, _c in enumerate(_codes):
        if _c is not None:
            COEFF_TOKEN[_cls][_c] = (_t1, _tc)

# total_zeros, 4x4 blocks: TOTAL_ZEROS[tzVlcIndex-1] = list of codes indexed by total_zeros
TOTAL_ZEROS = [
    ["1", "011", "010", "0011", "0010", "00011", "00010", "000011", "000010", "0000011", "0000010", "00000011",
     "00000010", "000000011", "000000010", "000000001"],
    ["111", "110", "101", "100", "011", "0101", "0100", "0011", "0010", "00011", "00010", "000011", "000010",
     "000001", "000000"],
    ["0101", "111", "110", "101", "0100", "0011", "100", "011", "0010", "00011", "00010", "000001", "00001",
     "000000"],
    ["00011", "111", "0101", "0100", "110", "101", "100", "0011", "011", "0010", "00010", "00001", "00000"],
    ["0101", "0100", "0011", "111", "110", "101", "100", "011", "0010", "00001", "0001", "00000"],
    ["000001", "00001", "111", "110", "101", "100", "011", "010", "0001", "001", "000000"],
    ["000001", "00001", "101", "100", "011", "11", "010", "0001", "001", "000000"],
    ["000001", "0001", "00001", "011", "11", "10", "010", "001", "000000"],
    ["000001", "000000", "0001", "11", "10", "001", "01", "00001"],
    ["00001", "00000", "001", "11", "10", "01", "0001"],
    ["0000", "0001", "001", "010", "1", "011"],
    ["0000", "0001", "01", "1", "001"],
    ["000", "001", "1", "01"],
    ["00", "01", "1"],
    ["0", "1"],
]
TOTAL_ZEROS_DC = [["1", "01", "001", "000"], ["1", "01", "00"], ["1", "0"]]
RUN_BEFORE = [
    ["1", "0"],
    ["1", "01", "00"],
    ["11", "10", "01", "00"],
    ["11", "10", "01", "001", "000"],
    ["11", "10", "011", "010", "001", "000"],
    ["11", "000", "001", "011", "010", "101", "100"],
    ["111", "110", "101", "100", "011", "010", "001", "0001", "00001", "000001", "0000001", "00000001",
     "000000001", "0000000001", "00000000001"],
]


def _inv(table: list[str]) -> dict[str, int]:
    return {c: i for i, c in enumerate(table)}


TOTAL_ZEROS_D = [_inv(t) for t in TOTAL_ZEROS]
TOTAL_ZEROS_DC_D = [_inv(t) for t in TOTAL_ZEROS_DC]
RUN_BEFORE_D = [_inv(t) for t in RUN_BEFORE]

ZIGZAG = [(0, 0), (1, 0), (0, 1), (0, 2), (1, 1), (2, 0), (3, 0), (2, 1), (1, 2), (0, 3), (1, 3), (2, 2), (3, 1),
          (3, 2), (2, 3), (3, 3)]  # (x, y) per scan index
# Table 9-4, ChromaArrayType 1/2: codeNum -> (intra cbp, inter cbp)
CBP_INTRA = [47, 31, 15, 0, 23, 27, 29, 30, 7, 11, 13, 14, 39, 43, 45, 46, 16, 3, 5, 10, 12, 19, 21, 26, 28, 35, 37,
             42, 44, 1, 2, 4, 8, 17, 18, 20, 24, 6, 9, 22, 25, 32, 33, 34, 36, 40, 38, 41]
CBP_INTER = [0, 16, 1, 2, 4, 8, 32, 3, 5, 10, 12, 15, 47, 7, 11, 13, 14, 6, 9, 31, 35, 37, 42, 44, 33, 34, 36, 40,
             39, 43, 45, 46, 17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41]
QPC = list(range(30)) + [29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39]
V_SCALE = [[10, 16, 13], [11, 18, 14], [13, 20, 16], [14, 23, 18], [16, 25, 20], [18, 29, 23]]


def _vclass(x: int, y: int) -> int:
    if x % 2 == 0 and y % 2 == 0:
        return 0
    if x % 2 == 1 and y % 2 == 1:
        return 1
    return 2


# block index -> (x, y) in 4x4-block units inside a MB (6.4.3)
BLK_XY = [((b // 4 % 2) * 2 + b % 2, (b // 8) * 2 + (b % 4) // 2) for b in range(16)]


class DecodeError(Exception):
    pass


# ----------------------------------------------------------------------------- bits
def nal_units(stream: bytes) -> list[bytes]:
    """Split an Annex-B byte stream into NAL units (emulation prevention removed)."""
    out = []
    i, n = 0, len(stream)
    starts = []
    while i + 3 <= n:
        if stream[i] == 0 and stream[i + 1] == 0 and stream[i + 2] == 1:
            starts.append(i + 3)
            i += 3
        else:
            i += 1
    for k, s in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else n
        while e > s and stream[e - 1] == 0:  # trailing zero bytes / 4-byte start code
            e -= 1
        raw = stream[s:e]
        rbsp = bytearray()
        zeros = 0
        for b in raw:
            if zeros >= 2 and b == 3:
                zeros = 0
                continue
            rbsp.append(b)
            zeros = zeros + 1 if b == 0 else 0
        out.append(bytes(rbsp))
    return out


class BitReader:
    def __init__(self, data: bytes, pos: int = 0):
        self.data = data
        self.pos = pos
        self.nbits = len(data) * 8
        # index of the rbsp_stop_one_bit
        last = len(data) - 1
        while last >= 0 and data[last] == 0:
            last -= 1
        if last < 0:
            self.stop = 0
        else:
            b = data[last]
            tz = (b & -b).bit_length() - 1
            self.stop = last * 8 + (7 - tz)

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            if self.pos >= self.nbits:
                raise DecodeError("read past end of NAL")
            v = (v << 1) | ((self.data[self.pos >> 3] >> (7 - (self.pos & 7))) & 1)
            self.pos += 1
        return v

    def bit(self) -> int:
        return self.u(1)

    def ue(self) -> int:
        z = 0
        while self.bit() == 0:
            z += 1
            if z > 31:
                raise DecodeError("bad exp-golomb")
        return (1 << z) - 1 + (self.u(z) if z else 0)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)

    def more_rbsp_data(self) -> bool:
        return self.pos < self.stop

    def byte_aligned(self) -> bool:
        return self.pos % 8 == 0

    def vlc(self, table: dict[str, object], maxlen: int = 16):
        code = ""
        while len(code) < maxlen:
            code += "1" if self.bit() else "0"
            if code in table:
                return table[code]
        raise DecodeError(f"invalid VLC code {code}")


# ----------------------------------------------------------------------------- headers
@dataclass
class SPS:
    profile_idc: int = 0
    level_idc: int = 0
    log2_max_frame_num: int = 4
    poc_type: int = 0
    log2_max_poc_lsb: int = 4
    max_num_ref_frames: int = 1
    mb_w: int = 0
    mb_h: int = 0
    frame_mbs_only: int = 1
    crop: tuple[int, int, int, int] = (0, 0, 0, 0)
    vui: dict = field(default_factory=dict)

    @property
    def width(self) -> int:
        return self.mb_w * 16 - 2 * (self.crop[0] + self.crop[1])

    @property
    def height(self) -> int:
        return self.mb_h * 16 - 2 * (self.crop[2] + self.crop[3])


@dataclass
class PPS:
    entropy_coding_mode: int = 0
    num_ref_idx_l0_default: int = 1
    pic_init_qp: int = 26
    chroma_qp_offset: int = 0
    deblocking_filter_control_present: int = 0
    constrained_intra_pred: int = 0
    redundant_pic_cnt_present: int = 0
    bottom_field_pic_order: int = 0
    weighted_pred: int = 0


def parse_sps(r: BitReader) -> SPS:
    s = SPS()
    s.profile_idc = r.u(8)
    r.u(8)
    s.level_idc = r.u(8)
    r.ue()
    if s.profile_idc in (100, 110, 122, 244, 44, 83, 86, 118, 128, 138, 139, 134, 135):
        raise DecodeError("high profiles not supported")
    s.log2_max_frame_num = r.ue() + 4
    s.poc_type = r.ue()
    if s.poc_type == 0:
        s.log2_max_poc_lsb = r.ue() + 4
    elif s.poc_type == 1:
        raise DecodeError("poc type 1 not supported")
    s.max_num_ref_frames = r.ue()
    r.bit()  # gaps
    s.mb_w = r.ue() + 1
    s.mb_h = r.ue() + 1
    s.frame_mbs_only = r.bit()
    if not s.frame_mbs_only:
        raise DecodeError("interlace not supported")
    r.bit()  # direct_8x8_inference
    if r.bit():
        s.crop = (r.ue(), r.ue(), r.ue(), r.ue())
    if r.bit():  # VUI
        v = s.vui
        if r.bit():
            idc = r.u(8)
            if idc == 255:
                r.u(16)
                r.u(16)
        if r.bit():
            r.bit()
        if r.bit():
            v["video_format"] = r.u(3)
            v["full_range"] = r.bit()
            if r.bit():
                v["colour_primaries"] = r.u(8)
                v["transfer"] = r.u(8)
                v["matrix"] = r.u(8)
        if r.bit():
            r.ue()
            r.ue()
        if r.bit():
            v["num_units_in_tick"] = r.u(32)
            v["time_scale"] = r.u(32)
            v["fixed_frame_rate"] = r.bit()
        nal_hrd = r.bit()
        vcl_hrd = r.bit()
        if nal_hrd or vcl_hrd:
            raise DecodeError("HRD parameters not supported")
        r.bit()  # pic_struct_present
        if r.bit():
            r.bit()
            r.ue()
            r.ue()
            r.ue()
            r.ue()
            v["max_num_reorder_frames"] = r.ue()
            v["max_dec_frame_buffering"] = r.ue()
    return s


def parse_pps(r: BitReader) -> PPS:
    p = PPS()
    r.ue()
    r.ue()
    p.entropy_coding_mode = r.bit()
    if p.entropy_coding_mode:
        raise DecodeError("CABAC not supported")
    p.bottom_field_pic_order = r.bit()
    if r.ue() != 0:
        raise DecodeError("slice groups not supported")
    p.num_ref_idx_l0_default = r.ue() + 1
    r.ue()
    p.weighted_pred = r.bit()
    r.u(2)
    p.pic_init_qp = 26 + r.se()
    r.se()
    p.chroma_qp_offset = r.se()
    p.deblocking_filter_control_present = r.bit()
    p.constrained_intra_pred = r.bit()
    p.redundant_pic_cnt_present = r.bit()
    return p


# ----------------------------------------------------------------------------- picture
@dataclass
class MbState:
    available: bool = False
    slice_id: int = -1
    intra: bool = False
    skip: bool = False
    pcm: bool = False
    mv: tuple[int, int] = (0, 0)  # for 16x16 (per-partition mv stored in mv4)
    ref: int = -1
    mv4: list = field(default_factory=lambda: [[(0, 0)] * 4 for _ in range(4)])  # [by][bx]
    ref4: list = field(default_factory=lambda: [[-1] * 4 for _ in range(4)])
    nz_luma: list = field(default_factory=lambda: [[0] * 4 for _ in range(4)])  # [by][bx]
    nz_cb: list = field(default_factory=lambda: [[0] * 2 for _ in range(2)])
    nz_cr: list = field(default_factory=lambda: [[0] * 2 for _ in range(2)])
    i4modes: list = field(default_factory=lambda: [[2] * 4 for _ in range(4)])
    i4: bool = False
    qp: int = 0  # QP_Y of the macroblock as decoded (skipped / residual-free MBs: the predictor)


def _clip(a):
    return np.clip(a, 0, 255)


def _tap6(a, b, c, d, e, f):
    return a - 5 * b + 20 * c + 20 * d - 5 * e + f


class Decoder:
    """Decode an Annex-B stream.  ``decode(stream)`` returns a list of (Y, U, V) frames
    (cropped, uint8).  ``frames_coded`` keeps the uncropped planes."""

    PAD = 24

    def __init__(self):
        self.sps: SPS | None = None
        self.pps: PPS | None = None
        self.ref = None  # (Y, U, V) int32 planes of the reference (coded size)
        self.frames: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []
        self.frames_coded: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []
        # tests: decode a subset of a picture's slices (the missing macroblocks stay zero)
        self.allow_partial = False
        self.cur = None
        self.mbs: list[MbState] = []
        self.slice_count = 0
        self.stats = {"skip": 0, "i16": 0, "i4": 0, "p": 0, "pcm": 0}

    # ------------------------------------------------------------------ top level
    def decode(self, stream: bytes) -> list[tuple[np.ndarray, np.ndarray, np.ndarray]]:
        for nal in nal_units(stream):
            self.decode_nal(nal)
        self.finish_picture()
        return self.frames

    def decode_nal(self, nal: bytes) -> None:
        if not nal:
            return
        hdr = nal[0]
        if hdr & 0x80:
            raise DecodeError("forbidden_zero_bit set")
        nal_ref_idc = (hdr >> 5) & 3
        t = hdr & 0x1F
        r = BitReader(nal, 8)
        if t == 7:
            self.finish_picture()
            self.sps = parse_sps(r)
        elif t == 8:
            self.pps = parse_pps(r)
        elif t in (1, 5):
            self.decode_slice(r, idr=(t == 5), nal_ref_idc=nal_ref_idc)
        elif t in (6, 9, 10, 11, 12):
            pass  # SEI, AUD, end of seq/stream, filler
        else:
            raise DecodeError(f"unsupported NAL type {t}")

    def new_picture(self) -> None:
        s = self.sps
        self.cur = (
            np.zeros((s.mb_h * 16, s.mb_w * 16), np.int32),
            np.zeros((s.mb_h * 8, s.mb_w * 8), np.int32),
            np.zeros((s.mb_h * 8, s.mb_w * 8), np.int32),
        )
        self.mbs = [MbState() for _ in range(s.mb_w * s.mb_h)]
        self.decoded_mbs = 0
        self.slice_db = {}

    def finish_picture(self) -> None:
        if self.cur is None:
            return
        s = self.sps
        if self.decoded_mbs != s.mb_w * s.mb_h and not self.allow_partial:
            raise DecodeError(f"incomplete picture: {self.decoded_mbs}/{s.mb_w * s.mb_h} MBs")
        self.deblock_picture()
        y, u, v = (p.astype(np.uint8) for p in self.cur)
        self.frames_coded.append((y, u, v))
        cl, cr, ct, cb = s.crop
        y2 = y[2 * ct: y.shape[0] - 2 * cb, 2 * cl: y.shape[1] - 2 * cr]
        u2 = u[ct: u.shape[0] - cb, cl: u.shape[1] - cr]
        v2 = v[ct: v.shape[0] - cb, cl: v.shape[1] - cr]
        self.frames.append((y2, u2, v2))
        self.ref = self.cur
        self.cur = None

    # ------------------------------------------------------------------ slices
    def decode_slice(self, r: BitReader, idr: bool, nal_ref_idc: int) -> None:
        s, p = self.sps, self.pps
        if s is None or p is None:
            raise DecodeError("slice before SPS/PPS")
        first_mb = r.ue()
        slice_type = r.ue() % 5
        if slice_type not in (0, 2):
            raise DecodeError(f"slice type {slice_type} not supported")
        r.ue()  # pps id
        frame_num = r.u(s.log2_max_frame_num)
        if first_mb == 0:
            self.finish_picture()
            self.new_picture()
        if self.cur is None:
            raise DecodeError("slice does not start a picture and none is open")
        if idr:
            r.ue()  # idr_pic_id
        if s.poc_type == 0:
            r.u(s.log2_max_poc_lsb)
            if p.bottom_field_pic_order:
                r.se()
        if p.redundant_pic_cnt_present:
            r.ue()
        num_ref = p.num_ref_idx_l0_default
        if slice_type == 0:
            if r.bit():
                num_ref = r.ue() + 1
            if r.bit():
                raise DecodeError("ref_pic_list_modification not supported")
            if p.weighted_pred:
                raise DecodeError("weighted prediction not supported")
        if nal_ref_idc:
            if idr:
                r.bit()
                r.bit()
            elif r.bit():
                raise DecodeError("adaptive ref pic marking not supported")
        qp = p.pic_init_qp + r.se()
        off_a = off_b = 0
        if p.deblocking_filter_control_present:
            idc = r.ue()
            if idc not in (0, 1, 2):
                raise DecodeError(f"disable_deblocking_filter_idc {idc}")
            if idc != 1:
                off_a = r.se() * 2
                off_b = r.se() * 2
        else:
            idc = 0
        if slice_type == 0 and self.ref is None:
            raise DecodeError("P slice without reference")
        self.slice_count += 1
        sid = self.slice_count
        self.slice_db[sid] = (idc, off_a, off_b)
        self.num_ref = num_ref
        self.qp = qp
        addr = first_mb
        nmb = s.mb_w * s.mb_h
        more = True
        while more:
            if slice_type == 0:
                run = r.ue()
                for _ in range(run):
                    if addr >= nmb:
                        raise DecodeError("skip run past end of picture")
                    self.decode_skip(addr, sid)
                    addr += 1
                if run > 0:
                    more = r.more_rbsp_data()
                    if not more:
                        break
            if addr >= nmb:
                raise DecodeError("macroblock past end of picture")
            self.decode_mb(r, addr, sid, slice_type)
            addr += 1
            more = r.more_rbsp_data()

    # ------------------------------------------------------------------ neighbours
    def _nb(self, addr: int, dx: int, dy: int, sid: int) -> MbState | None:
        s = self.sps
        x, y = addr % s.mb_w + dx, addr // s.mb_w + dy
        if x < 0 or y < 0 or x >= s.mb_w or y >= s.mb_h:
            return None
        m = self.mbs[y * s.mb_w + x]
        if not m.available or m.slice_id != sid:
            return None
        return m

    def _nc(self, addr, sid, bx, by, kind):
        """nC for a 4x4 block (kind: 'y', 'cb', 'cr'); bx,by inside the MB."""
        m = self.mbs[addr]
        lim = 4 if kind == "y" else 2
        get = {"y": lambda mm: mm.nz_luma, "cb": lambda mm: mm.nz_cb, "cr": lambda mm: mm.nz_cr}[kind]

        def count(mm, x, y):
            if mm.skip:
                return 0
            if mm.pcm:
                return 16
            return get(mm)[y][x]

        if bx > 0:
            a_av, na = True, count(m, bx - 1, by)
        else:
            ma = self._nb(addr, -1, 0, sid)
            a_av, na = ma is not None, (count(ma, lim - 1, by) if ma is not None else 0)
        if by > 0:
            b_av, nb = True, count(m, bx, by - 1)
        else:
            mb = self._nb(addr, 0, -1, sid)
            b_av, nb = mb is not None, (count(mb, bx, lim - 1) if mb is not None else 0)
        if a_av and b_av:
            return (na + nb + 1) >> 1
        if a_av:
            return na
        if b_av:
            return nb
        return 0

    # ------------------------------------------------------------------ residual
    def residual_block(self, r: BitReader, nc: int, maxnum: int) -> list[int]:
        cls = 4 if nc == -1 else (0 if nc < 2 else 1 if nc < 4 else 2 if nc < 8 else 3)
        t1, total = r.vlc(COEFF_TOKEN[cls])
        coef = [0] * maxnum
        if total == 0:
            return coef
        if total > maxnum:
            raise DecodeError("TotalCoeff > maxNumCoeff")
        levels = []
        suffix_len = 1 if (total > 10 and t1 < 3) else 0
        for i in range(total):
            if i < t1:
                levels.append(-1 if r.bit() else 1)
                continue
            prefix = 0
            while r.bit() == 0:
                prefix += 1
                if prefix > 31:
                    raise DecodeError("bad level_prefix")
            size = suffix_len
            if prefix == 14 and suffix_len == 0:
                size = 4
            if prefix >= 15:
                size = prefix - 3
            code = (min(15, prefix) << suffix_len) + (r.u(size) if size > 0 else 0)
            if prefix >= 15 and suffix_len == 0:
                code += 15
            if prefix >= 16:
                code += (1 << (prefix - 3)) - 4096
            if i == t1 and t1 < 3:
                code += 2
            lvl = (code + 2) >> 1 if code % 2 == 0 else (-code - 1) >> 1
            levels.append(lvl)
            if suffix_len == 0:
                suffix_len = 1
            if abs(lvl) > (3 << (suffix_len - 1)) and suffix_len < 6:
                suffix_len += 1
        if total < maxnum:
            tab = TOTAL_ZEROS_DC_D[total - 1] if maxnum == 4 else TOTAL_ZEROS_D[total - 1]
            total_zeros = r.vlc(tab)
        else:
            total_zeros = 0
        runs = []
        zl = total_zeros
        for i in range(total - 1):
            if zl > 0:
                rb = r.vlc(RUN_BEFORE_D[min(zl, 7) - 1])
            else:
                rb = 0
            runs.append(rb)
            zl -= rb
            if zl < 0:
                raise DecodeError("run_before exceeds zerosLeft")
        runs.append(zl)
        pos = -1
        for i in range(total - 1, -1, -1):
            pos += runs[i] + 1
            if pos >= maxnum:
                raise DecodeError("coefficient index out of range")
            coef[pos] = levels[i]
        return coef

    # ------------------------------------------------------------------ transforms
    @staticmethod
    def idct4(d: np.ndarray) -> np.ndarray:
        d = d.astype(np.int64)
        if not d.any():
            return np.zeros((4, 4), np.int64)
        if not d.ravel()[1:].any():  # DC only: every output sample is (dc + 32) >> 6
            return np.full((4, 4), (int(d[0, 0]) + 32) >> 6, np.int64)
        f = np.zeros((4, 4), np.int64)
        for i in range(4):
            e0 = d[i, 0] + d[i, 2]
            e1 = d[i, 0] - d[i, 2]
            e2 = (d[i, 1] >> 1) - d[i, 3]
            e3 = d[i, 1] + (d[i, 3] >> 1)
            f[i] = [e0 + e3, e1 + e2, e1 - e2, e0 - e3]
        h = np.zeros((4, 4), np.int64)
        for j in range(4):
            g0 = f[0, j] + f[2, j]
            g1 = f[0, j] - f[2, j]
            g2 = (f[1, j] >> 1) - f[3, j]
            g3 = f[1, j] + (f[3, j] >> 1)
            h[:, j] = [g0 + g3, g1 + g2, g1 - g2, g0 - g3]
        return (h + 32) >> 6

    @staticmethod
    def scan_to_matrix(levels: list[int], start: int) -> np.ndarray:
        c = np.zeros((4, 4), np.int64)
        for k, v in enumerate(levels):
            x, y = ZIGZAG[start + k]
            c[y, x] = v
        return c

    @staticmethod
    def dequant(c: np.ndarray, qp: int, skip_dc: bool) -> np.ndarray:
        d = np.zeros((4, 4), np.int64)
        if not c.any():
            return d
        for y in range(4):
            for x in range(4):
                if skip_dc and x == 0 and y == 0:
                    continue
                d[y, x] = (int(c[y, x]) * V_SCALE[qp % 6][_vclass(x, y)]) << (qp // 6)
        return d

    # ------------------------------------------------------------------ intra prediction
    def _luma_nb(self, addr, sid):
        s = self.sps
        Y = self.cur[0]
        x0, y0 = (addr % s.mb_w) * 16, (addr // s.mb_w) * 16
        left = self._nb(addr, -1, 0, sid) is not None
        top = self._nb(addr, 0, -1, sid) is not None
        tl = self._nb(addr, -1, -1, sid) is not None
        tr = self._nb(addr, 1, -1, sid) is not None
        return Y, x0, y0, left, top, tl, tr

    def pred16(self, addr, sid, mode) -> np.ndarray:
        Y, x0, y0, left, top, tl, _ = self._luma_nb(addr, sid)
        T = Y[y0 - 1, x0: x0 + 16] if top else None
        L = Y[y0: y0 + 16, x0 - 1] if left else None
        if mode == 0:
            if not top:
                raise DecodeError("I16 vertical without top")
            return np.tile(T, (16, 1))
        if mode == 1:
            if not left:
                raise DecodeError("I16 horizontal without left")
            return np.tile(L[:, None], (1, 16))
        if mode == 2:
            if top and left:
                dc = (int(T.sum()) + int(L.sum()) + 16) >> 5
            elif left:
                dc = (int(L.sum()) + 8) >> 4
            elif top:
                dc = (int(T.sum()) + 8) >> 4
            else:
                dc = 128
            return np.full((16, 16), dc, np.int64)
        if not (top and left and tl):
            raise DecodeError("I16 plane needs all neighbours")
        P = lambda x, y: int(Y[y0 + y, x0 + x])  # noqa: E731  (x,y may be -1)
        H = sum((xp + 1) * (P(8 + xp, -1) - P(6 - xp, -1)) for xp in range(8))
        V = sum((yp + 1) * (P(-1, 8 + yp) - P(-1, 6 - yp)) for yp in range(8))
        a = 16 * (P(-1, 15) + P(15, -1))
        b = (5 * H + 32) >> 6
        c = (5 * V + 32) >> 6
        yy, xx = np.mgrid[0:16, 0:16]
        return _clip((a + b * (xx - 7) + c * (yy - 7) + 16) >> 5)

    def pred_chroma(self, addr, sid, mode, comp) -> np.ndarray:
        s = self.sps
        C = self.cur[1 + comp]
        x0, y0 = (addr % s.mb_w) * 8, (addr // s.mb_w) * 8
        left = self._nb(addr, -1, 0, sid) is not None
        top = self._nb(addr, 0, -1, sid) is not None
        tl = self._nb(addr, -1, -1, sid) is not None
        out = np.zeros((8, 8), np.int64)
        if mode == 0:
            for by in range(2):
                for bx in range(2):
                    xo, yo = bx * 4, by * 4
                    st = int(C[y0 - 1, x0 + xo: x0 + xo + 4].sum()) if top else None
                    sl = int(C[y0 + yo: y0 + yo + 4, x0 - 1].sum()) if left else None
                    if (xo, yo) in ((0, 0), (4, 4)):
                        if st is not None and sl is not None:
                            dc = (st + sl + 4) >> 3
                        elif sl is not None:
                            dc = (sl + 2) >> 2
                        elif st is not None:
                            dc = (st + 2) >> 2
                        else:
                            dc = 128
                    elif xo > 0:
                        dc = (st + 2) >> 2 if st is not None else ((sl + 2) >> 2 if sl is not None else 128)
                    else:
                        dc = (sl + 2) >> 2 if sl is not None else ((st + 2) >> 2 if st is not None else 128)
                    out[yo: yo + 4, xo: xo + 4] = dc
            return out
        if mode == 1:
            if not left:
                raise DecodeError("chroma horizontal without left")
            return np.tile(C[y0: y0 + 8, x0 - 1][:, None], (1, 8)).astype(np.int64)
        if mode == 2:
            if not top:
                raise DecodeError("chroma vertical without top")
            return np.tile(C[y0 - 1, x0: x0 + 8], (8, 1)).astype(np.int64)
        if not (top and left and tl):
            raise DecodeError("chroma plane needs all neighbours")
        P = lambda x, y: int(C[y0 + y, x0 + x])  # noqa: E731
        H = sum((xp + 1) * (P(4 + xp, -1) - P(2 - xp, -1)) for xp in range(4))
        V = sum((yp + 1) * (P(-1, 4 + yp) - P(-1, 2 - yp)) for yp in range(4))
        a = 16 * (P(-1, 7) + P(7, -1))
        b = (34 * H + 32) >> 6
        c = (34 * V + 32) >> 6
        yy, xx = np.mgrid[0:8, 0:8]
        return _clip((a + b * (xx - 3) + c * (yy - 3) + 16) >> 5)

    def pred4x4(self, addr, sid, bx, by, mode) -> np.ndarray:
        """Intra 4x4 prediction for the block at (bx, by) of MB addr (8.3.1.2)."""
        s = self.sps
        Y = self.cur[0]
        mbx, mby = addr % s.mb_w, addr // s.mb_w
        X0, Y0 = mbx * 16 + bx * 4, mby * 16 + by * 4

        def avail(px, py):  # sample position relative to the picture
            if px < 0 or py < 0 or px >= s.mb_w * 16 or py >= s.mb_h * 16:
                return False
            nx, ny = px // 16, py // 16
            if (nx, ny) == (mbx, mby):
                # inside current MB: available if that 4x4 block is already decoded
                lbx, lby = (px % 16) // 4, (py % 16) // 4
                return self._blk_done.get((lbx, lby), False)
            m = self._nb(addr, nx - mbx, ny - mby, sid)
            return m is not None

        def p(x, y):
            return int(Y[Y0 + y, X0 + x])

        top = avail(X0, Y0 - 1)
        left = avail(X0 - 1, Y0)
        tl = avail(X0 - 1, Y0 - 1)
        tr = avail(X0 + 4, Y0 - 1)
        T = [p(x, -1) for x in range(4)] if top else None
        if top:
            TR = [p(x, -1) for x in range(4, 8)] if tr else [p(3, -1)] * 4
            T8 = T + TR
        L = [p(-1, y) for y in range(4)] if left else None
        Q = p(-1, -1) if tl else None
        o = np.zeros((4, 4), np.int64)
        if mode == 0:
            if not top:
                raise DecodeError("I4 vertical without top")
            o[:] = T
        elif mode == 1:
            if not left:
                raise DecodeError("I4 horizontal without left")
            o[:] = np.array(L)[:, None]
        elif mode == 2:
            if top and left:
                dc = (sum(T) + sum(L) + 4) >> 3
            elif left:
                dc = (sum(L) + 2) >> 2
            elif top:
                dc = (sum(T) + 2) >> 2
            else:
                dc = 128
            o[:] = dc
        elif mode == 3:  # diagonal down left
            if not top:
                raise DecodeError("I4 DDL without top")
            for y in range(4):
                for x in range(4):
                    if x == 3 and y == 3:
                        o[y, x] = (T8[6] + 3 * T8[7] + 2) >> 2
                    else:
                        o[y, x] = (T8[x + y] + 2 * T8[x + y + 1] + T8[x + y + 2] + 2) >> 2
        elif mode in (4, 5, 6):
            if not (top and left and tl):
                raise DecodeError(f"I4 mode {mode} needs top/left/top-left")

            def P(x, y):
                if y == -1:
                    return Q if x == -1 else T8[x]
                return L[y]

            for y in range(4):
                for x in range(4):
                    if mode == 4:  # diagonal down right
                        if x > y:
                            v = (P(x - y - 2, -1) + 2 * P(x - y - 1, -1) + P(x - y, -1) + 2) >> 2
                        elif x < y:
                            v = (P(-1, y - x - 2) + 2 * P(-1, y - x - 1) + P(-1, y - x) + 2) >> 2
                        else:
                            v = (P(0, -1) + 2 * P(-1, -1) + P(-1, 0) + 2) >> 2
                    elif mode == 5:  # vertical right
                        z = 2 * x - y
                        if z >= 0 and z % 2 == 0:
                            v = (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1
                        elif z >= 0:
                            v = (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2
                        elif z == -1:
                            v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                        else:
                            v = (P(-1, y - 1) + 2 * P(-1, y - 2) + P(-1, y - 3) + 2) >> 2
                    elif mode == 6:  # horizontal down
                        z = 2 * y - x
                        if z >= 0 and z % 2 == 0:
                            v = (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1
                        elif z >= 0:
                            v = (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2
                        elif z == -1:
                            v = (P(-1, 0) + 2 * P(-1, -1) + P(0, -1) + 2) >> 2
                        else:
                            v = (P(x - 1, -1) + 2 * P(x - 2, -1) + P(x - 3, -1) + 2) >> 2
                    o[y, x] = v
            return o
        elif mode == 7:  # vertical left
            if not top:
                raise DecodeError("I4 VL without top")
            for y in range(4):
                for x in range(4):
                    i = x + (y >> 1)
                    if y % 2 == 0:
                        o[y, x] = (T8[i] + T8[i + 1] + 1) >> 1
                    else:
                        o[y, x] = (T8[i] + 2 * T8[i + 1] + T8[i + 2] + 2) >> 2
        elif mode == 8:  # horizontal up
            if not left:
                raise DecodeError("I4 HU without left")
            for y in range(4):
                for x in range(4):
                    z = x + 2 * y
                    if z > 5:
                        o[y, x] = L[3]
                    elif z == 5:
                        o[y, x] = (L[2] + 3 * L[3] + 2) >> 2
                    elif z % 2 == 0:
                        o[y, x] = (L[y + (x >> 1)] + L[y + (x >> 1) + 1] + 1) >> 1
                    else:
                        o[y, x] = (L[y + (x >> 1)] + 2 * L[y + (x >> 1) + 1] + L[y + (x >> 1) + 2] + 2) >> 2
        return o

    # ------------------------------------------------------------------ inter prediction
    def _ref_padded(self):
        # keyed by the reference object itself (held, so its id cannot be reused by a new picture)
        if getattr(self, "_ref_key", None) is not self.ref:
            P = self.PAD
            self._refp = [np.pad(pl.astype(np.int64), P, mode="edge") for pl in self.ref]
            self._ref_key = self.ref
        return self._refp

    def pred_luma_inter(self, x0, y0, w, h, mvx, mvy) -> np.ndarray:
        P = self.PAD
        R = self._ref_padded()[0]
        xi, yi = x0 + (mvx >> 2) + P, y0 + (mvy >> 2) + P
        xf, yf = mvx & 3, mvy & 3

        def G(dx, dy, ww=w, hh=h):
            return R[yi + dy: yi + dy + hh, xi + dx: xi + dx + ww]

        def b1_at(dy):  # horizontal half intermediate at rows yi+dy.., cols xi..
            return _tap6(G(-2, dy), G(-1, dy), G(0, dy), G(1, dy), G(2, dy), G(3, dy))

        def h1_at(dx):
            return _tap6(G(dx, -2), G(dx, -1), G(dx, 0), G(dx, 1), G(dx, 2), G(dx, 3))

        def half(v1):
            return _clip((v1 + 16) >> 5)

        if xf == 0 and yf == 0:
            return G(0, 0).copy()
        b = half(b1_at(0))
        hh = half(h1_at(0))
        if yf == 0:
            if xf == 2:
                return b
            return (G(0, 0) + b + 1) >> 1 if xf == 1 else (G(1, 0) + b + 1) >> 1
        if xf == 0:
            if yf == 2:
                return hh
            return (G(0, 0) + hh + 1) >> 1 if yf == 1 else (G(0, 1) + hh + 1) >> 1
        j1 = _tap6(b1_at(-2), b1_at(-1), b1_at(0), b1_at(1), b1_at(2), b1_at(3))
        j = _clip((j1 + 512) >> 10)
        s = half(b1_at(1))
        m = half(h1_at(1))
        table = {
            (2, 2): j,
            (2, 1): (b + j + 1) >> 1,
            (2, 3): (j + s + 1) >> 1,
            (1, 2): (hh + j + 1) >> 1,
            (3, 2): (j + m + 1) >> 1,
            (1, 1): (b + hh + 1) >> 1,
            (3, 1): (b + m + 1) >> 1,
            (1, 3): (hh + s + 1) >> 1,
            (3, 3): (m + s + 1) >> 1,
        }
        return table[(xf, yf)]

    def pred_chroma_inter(self, comp, xc0, yc0, w, h, mvx, mvy) -> np.ndarray:
        P = self.PAD
        R = self._ref_padded()[1 + comp]
        xi, yi = xc0 + (mvx >> 3) + P, yc0 + (mvy >> 3) + P
        xf, yf = mvx & 7, mvy & 7
        A = R[yi: yi + h, xi: xi + w]
        B = R[yi: yi + h, xi + 1: xi + 1 + w]
        C = R[yi + 1: yi + 1 + h, xi: xi + w]
        D = R[yi + 1: yi + 1 + h, xi + 1: xi + 1 + w]
        return ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * C + xf * yf * D + 32) >> 6

    # ------------------------------------------------------------------ motion vectors
    def _mv_at(self, addr, sid, px, py, cur_parts):
        """(available, ref, mv) of the 4x4 block covering luma position (px,py) relative to
        the current MB's top-left; cur_parts = dict (bx,by)->(ref,mv) already decoded in this MB."""
        if 0 <= px < 16 and 0 <= py < 16:
            k = (px // 4, py // 4)
            if k in cur_parts:
                return True, cur_parts[k][0], cur_parts[k][1]
            return False, -1, (0, 0)
        dx = -1 if px < 0 else (1 if px >= 16 else 0)
        dy = -1 if py < 0 else 0
        m = self._nb(addr, dx, dy, sid)
        if m is None:
            return False, -1, (0, 0)
        if m.intra:
            return True, -1, (0, 0)
        bx, by = (px % 16) // 4, (py % 16) // 4
        return True, m.ref4[by][bx], m.mv4[by][bx]

    def _mvp(self, addr, sid, x, y, w, h, cur_parts, shape=None):
        A = self._mv_at(addr, sid, x - 1, y, cur_parts)
        B = self._mv_at(addr, sid, x, y - 1, cur_parts)
        C = self._mv_at(addr, sid, x + w, y - 1, cur_parts)
        if not C[0]:
            C = self._mv_at(addr, sid, x - 1, y - 1, cur_parts)
        if shape == "16x8_top" and B[1] == 0:
            return B[2]
        if shape == "16x8_bot" and A[1] == 0:
            return A[2]
        if shape == "8x16_left" and A[1] == 0:
            return A[2]
        if shape == "8x16_right" and C[1] == 0:
            return C[2]
        if not B[0] and not C[0] and A[0]:
            B = A
            C = A
        refs = [A[1], B[1], C[1]]
        if refs.count(0) == 1:
            return [A, B, C][refs.index(0)][2]
        mvs = [A[2], B[2], C[2]]
        return (sorted(v[0] for v in mvs)[1], sorted(v[1] for v in mvs)[1])

    def _skip_mv(self, addr, sid):
        A = self._mv_at(addr, sid, -1, 0, {})
        B = self._mv_at(addr, sid, 0, -1, {})
        if not A[0] or not B[0]:
            return (0, 0)
        if A[1] == 0 and A[2] == (0, 0):
            return (0, 0)
        if B[1] == 0 and B[2] == (0, 0):
            return (0, 0)
        return self._mvp(addr, sid, 0, 0, 16, 16, {})

    # ------------------------------------------------------------------ macroblocks
    def _store_inter(self, addr, sid, parts, skip=False):
        m = self.mbs[addr]
        m.available = True
        m.slice_id = sid
        m.intra = False
        m.skip = skip
        for (bx, by), (ref, mv) in parts.items():
            m.ref4[by][bx] = ref
            m.mv4[by][bx] = mv

    def decode_skip(self, addr, sid):
        s = self.sps
        mv = self._skip_mv(addr, sid)
        parts = {(bx, by): (0, mv) for by in range(4) for bx in range(4)}
        self._store_inter(addr, sid, parts, skip=True)
        self.mbs[addr].qp = self.qp
        self.mbs[addr].nz_luma = [[0] * 4 for _ in range(4)]
        x0, y0 = (addr % s.mb_w) * 16, (addr // s.mb_w) * 16
        self.cur[0][y0: y0 + 16, x0: x0 + 16] = self.pred_luma_inter(x0, y0, 16, 16, mv[0], mv[1])
        for c in range(2):
            self.cur[1 + c][y0 // 2: y0 // 2 + 8, x0 // 2: x0 // 2 + 8] = self.pred_chroma_inter(
                c, x0 // 2, y0 // 2, 8, 8, mv[0], mv[1])
        self.decoded_mbs += 1
        self.stats["skip"] += 1

    def decode_mb(self, r: BitReader, addr: int, sid: int, slice_type: int) -> None:
        s = self.sps
        mb_type = r.ue()
        m = self.mbs[addr]
        x0, y0 = (addr % s.mb_w) * 16, (addr // s.mb_w) * 16
        if slice_type == 0:
            if mb_type < 5:
                return self.decode_inter_mb(r, addr, sid, mb_type, x0, y0)
            mb_type -= 5
        # ---- intra
        m.available = True
        m.slice_id = sid
        m.intra = True
        m.ref = -1
        if mb_type == 25:  # I_PCM
            while not r.byte_aligned():
                r.bit()
            for y in range(16):
                for x in range(16):
                    self.cur[0][y0 + y, x0 + x] = r.u(8)
            for c in range(2):
                for y in range(8):
                    for x in range(8):
                        self.cur[1 + c][y0 // 2 + y, x0 // 2 + x] = r.u(8)
            m.pcm = True
            m.qp = 0  # qPp of an I_PCM macroblock (8.7.2.2)
            m.nz_luma = [[16] * 4 for _ in range(4)]
            self.decoded_mbs += 1
            self.stats["pcm"] += 1
            return
        i16 = mb_type > 0
        if i16:
            t = mb_type - 1
            pred_mode = t % 4
            cbp_c = (t // 4) % 3
            cbp_l = 15 if t >= 12 else 0
            cmode = r.ue()
            self.stats["i16"] += 1
        else:
            modes = []
            for _ in range(16):
                if r.bit():
                    modes.append(-1)
                else:
                    modes.append(r.u(3))
            cmode = r.ue()
            cbp = CBP_INTRA[r.ue()]
            cbp_l, cbp_c = cbp & 15, cbp >> 4
            self.stats["i4"] += 1
        if i16 or cbp_l or cbp_c:
            self.qp = (self.qp + r.se() + 52) % 52
        qp = self.qp
        m.qp = qp
        if i16:
            nc = self._nc(addr, sid, 0, 0, "y")
            dcl = self.residual_block(r, nc, 16)
        ac = {}
        for b in range(16):
            bx, by = BLK_XY[b]
            if cbp_l & (1 << (b // 4)):
                nc = self._nc(addr, sid, bx, by, "y")
                lv = self.residual_block(r, nc, 15 if i16 else 16)
                m.nz_luma[by][bx] = sum(1 for v in lv if v)
                ac[b] = lv
            else:
                m.nz_luma[by][bx] = 0
        chroma = self._parse_chroma(r, addr, sid, cbp_c)
        # ---- reconstruction
        if i16:
            pred = self.pred16(addr, sid, pred_mode)
            c = self.scan_to_matrix(dcl, 0)
            f = self._hadamard(c)
            ls = 16 * V_SCALE[qp % 6][0]
            if qp >= 36:
                dcy = (f * ls) << (qp // 6 - 6)
            else:
                dcy = (f * ls + (1 << (5 - qp // 6))) >> (6 - qp // 6)
            res = np.zeros((16, 16), np.int64)
            for b in range(16):
                bx, by = BLK_XY[b]
                cm = self.scan_to_matrix(ac[b], 1) if b in ac else np.zeros((4, 4), np.int64)
                d = self.dequant(cm, qp, skip_dc=True)
                d[0, 0] = dcy[by, bx]
                res[by * 4: by * 4 + 4, bx * 4: bx * 4 + 4] = self.idct4(d)
            self.cur[0][y0: y0 + 16, x0: x0 + 16] = _clip(pred + res)
        else:
            self._blk_done = {}
            for b in range(16):
                bx, by = BLK_XY[b]
                mode = self._i4_mode(addr, sid, bx, by, modes[b])
                m.i4modes[by][bx] = mode
                pred = self.pred4x4(addr, sid, bx, by, mode)
                cm = self.scan_to_matrix(ac[b], 0) if b in ac else np.zeros((4, 4), np.int64)
                d = self.dequant(cm, qp, skip_dc=False)
                self.cur[0][y0 + by * 4: y0 + by * 4 + 4, x0 + bx * 4: x0 + bx * 4 + 4] = _clip(pred + self.idct4(d))
                self._blk_done[(bx, by)] = True
            m.i4 = True
        for comp in range(2):
            pred = self.pred_chroma(addr, sid, cmode, comp)
            self._recon_chroma(comp, addr, pred, chroma, qp)
        self.decoded_mbs += 1

    def _i4_mode(self, addr, sid, bx, by, coded):
        def nb_mode(dx, dy):
            lx, ly = bx + dx, by + dy
            if 0 <= lx < 4 and 0 <= ly < 4:
                return self.mbs[addr].i4modes[ly][lx], True
            m = self._nb(addr, -1 if lx < 0 else 0, -1 if ly < 0 else 0, sid)
            if m is None:
                return None, False
            if not m.intra or not m.i4:
                return 2, True
            return m.i4modes[ly % 4][lx % 4], True

        a, aa = nb_mode(-1, 0)
        b, ba = nb_mode(0, -1)
        if not aa or not ba:
            pred = 2
        else:
            pred = min(a, b)
        if coded == -1:
            return pred
        return coded if coded < pred else coded + 1

    @staticmethod
    def _hadamard(c):
        H = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]], np.int64)
        return H @ c @ H

    def _parse_chroma(self, r, addr, sid, cbp_c):
        out = {"dc": [[0] * 4, [0] * 4], "ac": [[None] * 4, [None] * 4]}
        m = self.mbs[addr]
        if cbp_c & 3:
            for comp in range(2):
                out["dc"][comp] = self.residual_block(r, -1, 4)
        for comp in range(2):
            for b in range(4):
                bx, by = b % 2, b // 2
                tgt = m.nz_cb if comp == 0 else m.nz_cr
                if cbp_c & 2:
                    nc = self._nc(addr, sid, bx, by, "cb" if comp == 0 else "cr")
                    lv = self.residual_block(r, nc, 15)
                    out["ac"][comp][b] = lv
                    tgt[by][bx] = sum(1 for v in lv if v)
                else:
                    tgt[by][bx] = 0
        return out

    def _recon_chroma(self, comp, addr, pred, chroma, qp):
        s = self.sps
        qpc = QPC[max(0, min(51, qp + self.pps.chroma_qp_offset))]
        c = np.array(chroma["dc"][comp], np.int64).reshape(2, 2)
        f = np.array([[1, 1], [1, -1]], np.int64) @ c @ np.array([[1, 1], [1, -1]], np.int64)
        dcc = ((f * (16 * V_SCALE[qpc % 6][0])) << (qpc // 6)) >> 5
        res = np.zeros((8, 8), np.int64)
        for b in range(4):
            bx, by = b % 2, b // 2
            lv = chroma["ac"][comp][b]
            cm = self.scan_to_matrix(lv, 1) if lv is not None else np.zeros((4, 4), np.int64)
            d = self.dequant(cm, qpc, skip_dc=True)
            d[0, 0] = dcc[by, bx]
            res[by * 4: by * 4 + 4, bx * 4: bx * 4 + 4] = self.idct4(d)
        x0, y0 = (addr % s.mb_w) * 8, (addr // s.mb_w) * 8
        self.cur[1 + comp][y0: y0 + 8, x0: x0 + 8] = _clip(pred + res)

    # ------------------------------------------------------------------ deblocking (8.7)
    def deblock_picture(self) -> None:
        """8.7 over the whole picture.  The process is defined macroblock by macroblock in raster
        order; macroblocks on one anti-diagonal x + 2y = t never touch each other's samples (a
        macroblock depends on its left, upper and upper-right neighbours only), so each diagonal
        is filtered as one vectorised step -- the same result as the raster order, in
        mb_w + 2 mb_h steps instead of mb_w * mb_h."""
        s = self.sps
        mw, mh = s.mb_w, s.mb_h
        n = mw * mh
        off_c = self.pps.chroma_qp_offset
        # per-MB records
        idc = np.ones(n, int)
        offa = np.zeros(n, int)
        offb = np.zeros(n, int)
        qp = np.zeros(n, int)
        for i, m in enumerate(self.mbs):
            if m.available:
                idc[i], offa[i], offb[i] = self.slice_db.get(m.slice_id, (1, 0, 0))
                qp[i] = m.qp
        if (idc == 1).all():
            return
        bsv = np.zeros((n, 4, 4), int)  # [mb, edge, segment]
        bsh = np.zeros((n, 4, 4), int)
        for i, m in enumerate(self.mbs):
            if idc[i] == 1 or not m.available:
                continue
            mx, my = i % mw, i // mw
            left = self.mbs[i - 1] if mx > 0 else None
            top = self.mbs[i - mw] if my > 0 else None
            if left is not None and (not left.available or (idc[i] == 2 and left.slice_id != m.slice_id)):
                left = None
            if top is not None and (not top.available or (idc[i] == 2 and top.slice_id != m.slice_id)):
                top = None
            for sg in range(4):
                bsv[i, 0, sg] = _bs(left, 3, sg, m, 0, sg, True) if left is not None else 0
                bsh[i, 0, sg] = _bs(top, sg, 3, m, sg, 0, True) if top is not None else 0
                for e in range(1, 4):
                    bsv[i, e, sg] = _bs(m, e - 1, sg, m, e, sg, False)
                    bsh[i, e, sg] = _bs(m, sg, e - 1, m, sg, e, False)
        qpc = np.array(QPC)[np.clip(qp + off_c, 0, 51)]
        Yp = np.pad(self.cur[0], ((4, 0), (4, 0)))
        Cp = [np.pad(c, ((2, 0), (2, 0))) for c in self.cur[1:]]
        for t in range(mw + 2 * (mh - 1) + 1):
            ys = np.arange(max(0, (t - mw + 2) // 2), min(mh - 1, t // 2) + 1)
            xs = t - 2 * ys
            ok = (xs >= 0) & (xs < mw)
            ys, xs = ys[ok], xs[ok]
            if len(ys) == 0:
                continue
            ids = ys * mw + xs
            keep = idc[ids] != 1
            ys, xs, ids = ys[keep], xs[keep], ids[keep]
            if len(ids) == 0:
                continue
            qn = qp[ids]
            ql = qp[np.maximum(ids - 1, 0)]
            qt = qp[np.maximum(ids - mw, 0)]
            # luma: region rows 16y-4 .. 16y+15, cols 16x-4 .. 16x+15 (padded coordinates + 4)
            rr = (ys[:, None] * 16 + np.arange(20))[:, :, None]
            cc = (xs[:, None] * 16 + np.arange(20))[:, None, :]
            R = Yp[rr, cc].astype(np.int64)
            for vert, bsx in ((True, bsv), (False, bsh)):
                for e in range(4):
                    b = np.repeat(bsx[ids, e], 4, axis=1)  # (k, 16 lines)
                    if not b.any():
                        continue
                    qa = (((ql if vert else qt) if e == 0 else qn) + qn + 1) >> 1
                    k = 4 + 4 * e
                    if vert:
                        pl = R[:, 4:20, k - 4:k][:, :, ::-1]
                        qd = R[:, 4:20, k:k + 4]
                    else:
                        pl = R[:, k - 4:k, 4:20][:, ::-1, :].transpose(0, 2, 1)
                        qd = R[:, k:k + 4, 4:20].transpose(0, 2, 1)
                    P2, Q2 = pl.reshape(-1, 4).copy(), qd.reshape(-1, 4).copy()
                    _filter_lines(P2, Q2, b.reshape(-1), np.repeat(qa, 16), np.repeat(offa[ids], 16),
                                  np.repeat(offb[ids], 16), False)
                    if vert:
                        R[:, 4:20, k - 4:k] = P2.reshape(-1, 16, 4)[:, :, ::-1]
                        R[:, 4:20, k:k + 4] = Q2.reshape(-1, 16, 4)
                    else:
                        R[:, k - 4:k, 4:20] = P2.reshape(-1, 16, 4).transpose(0, 2, 1)[:, ::-1, :]
                        R[:, k:k + 4, 4:20] = Q2.reshape(-1, 16, 4).transpose(0, 2, 1)
            Yp[rr, cc] = R
            # chroma: region rows 8y-2 .. 8y+7, cols 8x-2 .. 8x+7; edges 0 / 4 take luma edges 0 / 8
            rr = (ys[:, None] * 8 + np.arange(10))[:, :, None]
            cc = (xs[:, None] * 8 + np.arange(10))[:, None, :]
            qcn, qcl, qct = qpc[ids], qpc[np.maximum(ids - 1, 0)], qpc[np.maximum(ids - mw, 0)]
            for Pc in Cp:
                R = Pc[rr, cc].astype(np.int64)
                for vert, bsx in ((True, bsv), (False, bsh)):
                    for ce in range(2):
                        b = np.repeat(bsx[ids, 2 * ce], 2, axis=1)  # (k, 8 lines)
                        if not b.any():
                            continue
                        qa = (((qcl if vert else qct) if ce == 0 else qcn) + qcn + 1) >> 1
                        k = 2 + 4 * ce
                        z = np.zeros((len(ids), 8, 2), np.int64)
                        if vert:
                            pl = np.concatenate([R[:, 2:10, k - 2:k][:, :, ::-1], z], axis=2)
                            qd = np.concatenate([R[:, 2:10, k:k + 2], z], axis=2)
                        else:
                            pl = np.concatenate([R[:, k - 2:k, 2:10][:, ::-1, :].transpose(0, 2, 1), z], axis=2)
                            qd = np.concatenate([R[:, k:k + 2, 2:10].transpose(0, 2, 1), z], axis=2)
                        P2, Q2 = pl.reshape(-1, 4).copy(), qd.reshape(-1, 4).copy()
                        _filter_lines(P2, Q2, b.reshape(-1), np.repeat(qa, 8), np.repeat(offa[ids], 8),
                                      np.repeat(offb[ids], 8), True)
                        if vert:
                            R[:, 2:10, k - 2:k] = P2.reshape(-1, 8, 4)[:, :, 1::-1]
                            R[:, 2:10, k:k + 2] = Q2.reshape(-1, 8, 4)[:, :, :2]
                        else:
                            R[:, k - 2:k, 2:10] = P2.reshape(-1, 8, 4)[:, :, 1::-1].transpose(0, 2, 1)
                            R[:, k:k + 2, 2:10] = Q2.reshape(-1, 8, 4)[:, :, :2].transpose(0, 2, 1)
                Pc[rr, cc] = R
        self.cur = (Yp[4:, 4:], Cp[0][2:, 2:], Cp[1][2:, 2:])

    def decode_inter_mb(self, r, addr, sid, mb_type, x0, y0):
        if mb_type >= 3:
            raise DecodeError("P_8x8 not supported")
        nparts = 1 if mb_type == 0 else 2
        refs = []
        for _ in range(nparts):
            if self.num_ref > 1:
                refs.append(r.ue() if self.num_ref > 2 else 1 - r.bit())
            else:
                refs.append(0)
        if any(x != 0 for x in refs):
            raise DecodeError("only reference index 0 supported")
        if mb_type == 0:
            geo = [(0, 0, 16, 16, None)]
        elif mb_type == 1:
            geo = [(0, 0, 16, 8, "16x8_top"), (0, 8, 16, 8, "16x8_bot")]
        else:
            geo = [(0, 0, 8, 16, "8x16_left"), (8, 0, 8, 16, "8x16_right")]
        cur_parts: dict = {}
        mvs = []
        for (px, py, w, h, shape) in geo:
            mvdx, mvdy = r.se(), r.se()
            mvp = self._mvp(addr, sid, px, py, w, h, cur_parts, shape)
            mv = (mvp[0] + mvdx, mvp[1] + mvdy)
            mvs.append((px, py, w, h, mv))
            for by in range(py // 4, (py + h) // 4):
                for bx in range(px // 4, (px + w) // 4):
                    cur_parts[(bx, by)] = (0, mv)
        self._store_inter(addr, sid, cur_parts)
        m = self.mbs[addr]
        cbp = CBP_INTER[r.ue()]
        cbp_l, cbp_c = cbp & 15, cbp >> 4
        if cbp:
            self.qp = (self.qp + r.se() + 52) % 52
        qp = self.qp
        m.qp = qp
        ac = {}
        for b in range(16):
            bx, by = BLK_XY[b]
            if cbp_l & (1 << (b // 4)):
                nc = self._nc(addr, sid, bx, by, "y")
                lv = self.residual_block(r, nc, 16)
                m.nz_luma[by][bx] = sum(1 for v in lv if v)
                ac[b] = lv
            else:
                m.nz_luma[by][bx] = 0
        chroma = self._parse_chroma(r, addr, sid, cbp_c)
        pred = np.zeros((16, 16), np.int64)
        cpred = [np.zeros((8, 8), np.int64), np.zeros((8, 8), np.int64)]
        for (px, py, w, h, mv) in mvs:
            pred[py: py + h, px: px + w] = self.pred_luma_inter(x0 + px, y0 + py, w, h, mv[0], mv[1])
            for c in range(2):
                cpred[c][py // 2: (py + h) // 2, px // 2: (px + w) // 2] = self.pred_chroma_inter(
                    c, (x0 + px) // 2, (y0 + py) // 2, w // 2, h // 2, mv[0], mv[1])
        res = np.zeros((16, 16), np.int64)
        for b in range(16):
            bx, by = BLK_XY[b]
            if b in ac:
                d = self.dequant(self.scan_to_matrix(ac[b], 0), qp, skip_dc=False)
                res[by * 4: by * 4 + 4, bx * 4: bx * 4 + 4] = self.idct4(d)
        self.cur[0][y0: y0 + 16, x0: x0 + 16] = _clip(pred + res)
        for comp in range(2):
            self._recon_chroma(comp, addr, cpred[comp], chroma, qp)
        self.decoded_mbs += 1
        self.stats["p"] += 1


# ----------------------------------------------------------------------------- deblocking (8.7)
# Table 8-16 (alpha', beta' by indexA / indexB) and Table 8-17 (tC0' by indexA and bS = 1, 2, 3),
# 8-bit video; typed in from the tables, independently of the encoder's copy.
_DB_ALPHA = [0] * 16 + [4, 4, 5, 6, 7, 8, 9, 10, 12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71,
                        80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255]
_DB_BETA = [0] * 16 + [2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12,
                       13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18]
_DB_TC0 = [(0, 0, 0)] * 17 + [
    (0, 0, 1), (0, 0, 1), (0, 0, 1), (0, 0, 1), (0, 1, 1), (0, 1, 1), (1, 1, 1), (1, 1, 1), (1, 1, 1),
    (1, 1, 1), (1, 1, 2), (1, 1, 2), (1, 1, 2), (1, 1, 2), (1, 2, 3), (1, 2, 3), (2, 2, 3), (2, 2, 4),
    (2, 3, 4), (2, 3, 4), (3, 3, 5), (3, 4, 6), (3, 4, 6), (4, 5, 7), (4, 5, 8), (4, 6, 9), (5, 7, 10),
    (6, 8, 11), (6, 8, 13), (7, 10, 14), (8, 11, 16), (9, 12, 18), (10, 13, 20), (11, 15, 23), (13, 17, 25)]
assert len(_DB_ALPHA) == len(_DB_BETA) == len(_DB_TC0) == 52


_A_T = np.array(_DB_ALPHA)
_B_T = np.array(_DB_BETA)
_TC_T = np.array(_DB_TC0)


def _filter_lines(pl, qd, bs, qpav, off_a, off_b, chroma):
    """Vectorised 8.7.2.3 / 8.7.2.4 over lines with per-line bS, qPav and slice offsets;
    ``pl`` / ``qd``: (lines, 4) p0..p3 / q0..q3 (index 0 nearest the edge).  In place."""
    ia = np.clip(qpav + off_a, 0, 51)
    ib = np.clip(qpav + off_b, 0, 51)
    alpha, beta = _A_T[ia], _B_T[ib]
    p0, p1, p2, p3 = (pl[:, i].copy() for i in range(4))
    q0, q1, q2, q3 = (qd[:, i].copy() for i in range(4))
    f = (bs > 0) & (np.abs(p0 - q0) < alpha) & (np.abs(p1 - p0) < beta) & (np.abs(q1 - q0) < beta)
    if not f.any():
        return
    ap, aq = np.abs(p2 - p0) < beta, np.abs(q2 - q0) < beta
    weak = f & (bs < 4)
    strong = f & (bs == 4)
    if weak.any():
        tc0 = np.where(bs > 0, _TC_T[ia, np.clip(bs - 1, 0, 2)], 0)
        tc = tc0 + 1 if chroma else tc0 + ap + aq
        d = np.clip((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc)
        pl[weak, 0] = np.clip(p0 + d, 0, 255)[weak]
        qd[weak, 0] = np.clip(q0 - d, 0, 255)[weak]
        if not chroma:
            mp = weak & ap
            pl[mp, 1] = (p1 + np.clip((p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1, -tc0, tc0))[mp]
            mq = weak & aq
            qd[mq, 1] = (q1 + np.clip((q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1, -tc0, tc0))[mq]
    if strong.any():
        if chroma:
            pl[strong, 0] = ((2 * p1 + p0 + q1 + 2) >> 2)[strong]
            qd[strong, 0] = ((2 * q1 + q0 + p1 + 2) >> 2)[strong]
            return
        small = np.abs(p0 - q0) < ((alpha >> 2) + 2)
        sp, wp = strong & ap & small, strong & ~(ap & small)
        pl[sp, 0] = ((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3)[sp]
        pl[sp, 1] = ((p2 + p1 + p0 + q0 + 2) >> 2)[sp]
        pl[sp, 2] = ((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3)[sp]
        pl[wp, 0] = ((2 * p1 + p0 + q1 + 2) >> 2)[wp]
        sq, wq = strong & aq & small, strong & ~(aq & small)
        qd[sq, 0] = ((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3)[sq]
        qd[sq, 1] = ((p0 + q0 + q1 + q2 + 2) >> 2)[sq]
        qd[sq, 2] = ((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3)[sq]
        qd[wq, 0] = ((2 * q1 + q0 + p1 + 2) >> 2)[wq]


def _bs(mp: MbState, bxp, byp, mq: MbState, bxq, byq, mb_edge: bool) -> int:
    """Boundary strength (8.7.2.1, frame macroblocks, one reference list)."""
    if mp.intra or mq.intra:
        return 4 if mb_edge else 3
    if mp.nz_luma[byp][bxp] or mq.nz_luma[byq][bxq]:
        return 2
    if mp.ref4[byp][bxp] != mq.ref4[byq][bxq]:
        return 1
    a, b = mp.mv4[byp][bxp], mq.mv4[byq][bxq]
    return 1 if (abs(a[0] - b[0]) >= 4 or abs(a[1] - b[1]) >= 4) else 0


def decode_annexb(stream: bytes) -> list[tuple[np.ndarray, np.ndarray, np.ndarray]]:
    return Decoder().decode(stream)


def psnr(a: np.ndarray, b: np.ndarray) -> float:
    mse = float(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2))
    return 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)
