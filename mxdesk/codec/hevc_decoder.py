"""Pure-Python HEVC (H.265 Main profile subset) decoder: the oracle for mxdesk's HIP and
CPU HEVC encoders (there is no ffmpeg/libde265 in this image).

Written from the decoding side of ITU-T H.265: NAL/RBSP parsing (7.3), CABAC parsing with
context selection per 9.3.4.2, and the decoding processes for intra prediction (8.4.4.2,
all 35 modes with reference substitution and filtering), inter prediction with merge and
AMVP spatial candidates (8.5.3.2) and 8-tap / 4-tap interpolation (8.5.3.3.3), scaling
and the inverse core transform (8.6).  The encoder side (csrc/codec/hevc_core.h) shares
no code with this file.

Supported: VPS/SPS/PPS (incl. VUI), I and P slices (one reference picture, short-term RPS
from the SPS), coding quadtrees with split_cu_flag, PartMode 2Nx2N (intra and inter),
transform trees with split_transform_flag, residual coding for 4x4..32x32 TUs (scanIdx
0/1/2, no sign hiding, no transform skip), cu_qp_delta, conformance window cropping.
Both in-loop filters are implemented: deblocking (8.7.2) and sample adaptive offset (8.7.3,
band and edge offsets with CTB merge-left/up, 7.3.8.3).  TMVP must be off (mxdesk's encoder
guarantees it); anything else raises ``NotImplementedError``.  Slow; meant for small test pictures.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# ----------------------------------------------------------------------------- CABAC tables
_RANGE_LPS = [
    (128, 176, 208, 240), (128, 167, 197, 227), (128, 158, 187, 216), (123, 150, 178, 205),
    (116, 142, 169, 195), (111, 135, 160, 185), (105, 128, 152, 175), (100, 122, 144, 166),
    (95, 116, 137, 158), (90, 110, 130, 150), (85, 104, 123, 142), (81, 99, 117, 135),
    (77, 94, 111, 128), (73, 89, 105, 122), (69, 85, 100, 116), (66, 80, 95, 110),
    (62, 76, 90, 104), (59, 72, 86, 99), (56, 69, 81, 94), (53, 65, 77, 89),
    (51, 62, 73, 85), (48, 59, 69, 80), (46, 56, 66, 76), (43, 53, 63, 72),
    (41, 50, 59, 69), (39, 48, 56, 65), (37, 45, 54, 62), (35, 43, 51, 59),
    (33, 41, 48, 56), (32, 39, 46, 53), (30, 37, 43, 50), (29, 35, 41, 48),
    (27, 33, 39, 45), (26, 31, 37, 43), (24, 30, 35, 41), (23, 28, 33, 39),
    (22, 27, 32, 37), (21, 26, 30, 35), (20, 24, 29, 33), (19, 23, 27, 31),
    (18, 22, 26, 30), (17, 21, 25, 28), (16, 20, 23, 27), (15, 19, 22, 25),
    (14, 18, 21, 24), (14, 17, 20, 23), (13, 16, 19, 22), (12, 15, 18, 21),
    (12, 14, 17, 20), (11, 14, 16, 19), (11, 13, 15, 18), (10, 12, 15, 17),
    (10, 12, 14, 16), (9, 11, 13, 15), (9, 11, 12, 14), (8, 10, 12, 14),
    (8, 9, 11, 13), (7, 9, 11, 12), (7, 9, 10, 12), (7, 8, 10, 11),
    (6, 8, 9, 11), (6, 7, 9, 10), (6, 7, 8, 9), (2, 2, 2, 2),
]
_TRANS_LPS = [0, 0, 1, 2, 2, 4, 4, 5, 6, 7, 8, 9, 9, 11, 11, 12, 13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21,
              21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33, 33, 33,
              34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63]

# initValue per syntax element: (initType 0 values, initType 1 values, initType 2 values)
_INIT = {
    "split_cu_flag": ([139, 141, 157], [107, 139, 126], [107, 139, 126]),
    "cu_skip_flag": ([154, 154, 154], [197, 185, 201], [197, 185, 201]),
    "merge_flag": ([154], [110], [154]),
    "merge_idx": ([154], [122], [137]),
    "pred_mode_flag": ([154], [149], [134]),
    "part_mode": ([184, 154, 154, 154], [154, 139, 154, 154], [154, 139, 154, 154]),
    "prev_intra_luma_pred_flag": ([184], [154], [183]),
    "intra_chroma_pred_mode": ([63], [152], [152]),
    "rqt_root_cbf": ([154], [79], [79]),
    "mvp_flag": ([154], [168], [168]),
    "ref_idx": ([154, 154], [153, 153], [153, 153]),
    "abs_mvd_greater0_flag": ([154], [140], [169]),
    "abs_mvd_greater1_flag": ([154], [198], [198]),
    "split_transform_flag": ([153, 138, 138], [124, 138, 94], [224, 167, 122]),
    "cbf_luma": ([111, 141], [153, 111], [153, 111]),
    "cbf_chroma": ([94, 138, 182, 154], [149, 107, 167, 154], [149, 92, 167, 154]),
    "cu_qp_delta_abs": ([154, 154], [154, 154], [154, 154]),
    "last_sig_coeff_x_prefix": (
        [110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63],
        [125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108],
        [125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93]),
    "coded_sub_block_flag": ([91, 171, 134, 141], [121, 140, 61, 154], [121, 140, 61, 154]),
    "sig_coeff_flag": (
        [111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153,
         125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139, 111, 136,
         139, 111],
        [155, 154, 139, 153, 139, 123, 123, 63, 153, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153,
         154, 166, 183, 140, 136, 153, 154, 170, 153, 123, 123, 107, 121, 107, 121, 167, 151, 183, 140, 151,
         183, 140],
        [170, 154, 139, 153, 139, 123, 123, 63, 124, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153,
         154, 166, 183, 140, 136, 153, 154, 170, 153, 138, 138, 122, 121, 122, 121, 167, 151, 183, 140, 151,
         183, 140]),
    "coeff_abs_level_greater1_flag": (
        [140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166, 182, 140,
         227, 122, 197],
        [154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137, 169, 194, 166, 167,
         154, 167, 137, 182],
        [154, 196, 167, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 122, 169, 208, 166, 167,
         154, 152, 167, 182]),
    "coeff_abs_level_greater2_flag": ([138, 153, 136, 167, 152, 152], [107, 167, 91, 122, 107, 167],
                                      [107, 167, 91, 107, 107, 167]),
    "sao_merge_flag": ([153], [153], [153]),       # sao_merge_left_flag and sao_merge_up_flag share it
    "sao_type_idx": ([200], [185], [160]),          # first bin of sao_type_idx_luma / _chroma
}
_INIT["last_sig_coeff_y_prefix"] = _INIT["last_sig_coeff_x_prefix"]

_INTRA_ANGLE = [0, 0, 32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26, -32, -26, -21, -17, -13,
                -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32]
_INV_ANGLE = {-2: -4096, -5: -1638, -9: -910, -13: -630, -17: -482, -21: -390, -26: -315, -32: -256}
_LUMA_FILTER = [[0, 0, 0, 64, 0, 0, 0, 0], [-1, 4, -10, 58, 17, -5, 1, 0], [-1, 4, -11, 40, 40, -11, 4, -1],
                [0, 1, -5, 17, 58, -10, 4, -1]]
_CHROMA_FILTER = [[0, 64, 0, 0], [-2, 58, 10, -2], [-4, 54, 16, -2], [-6, 46, 28, -4], [-4, 36, 36, -4],
                  [-4, 28, 46, -6], [-2, 16, 54, -4], [-2, 10, 58, -2]]
_LEVEL_SCALE = [40, 45, 51, 57, 64, 72]
# deblocking beta' (Table 8-12, Q = 0..51) and tC' (Q = 0..53)
_DB_BETA = [0] * 16 + [6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18] + list(range(20, 66, 2))
_DB_TC = [0] * 18 + [1] * 9 + [2] * 4 + [3] * 4 + [4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24]
# SAO edge classes (Table 8-13 hPos/vPos): neighbours a, b of each sample
_SAO_EO_NB = [((-1, 0), (1, 0)), ((0, -1), (0, 1)), ((-1, -1), (1, 1)), ((1, -1), (-1, 1))]
_SAO_EDGE_CAT = np.array([1, 2, 0, 3, 4])  # edgeIdx 2 + sign + sign -> offset category (8.7.3.2)
_QPC_TABLE = {30: 29, 31: 30, 32: 31, 33: 32, 34: 33, 35: 33, 36: 34, 37: 34, 38: 35, 39: 35, 40: 36, 41: 36,
              42: 37, 43: 37}

# 32x32 core transform matrix (8.6.4.2, eq. 8-315 ff.): 31 distinct magnitudes
_T32_ODD_ROW1 = [90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4]


def _transform_matrix() -> np.ndarray:
    # magnitudes c[m] = |entry| of angle index m (cos(pi*m/64)) from the rows 1, 2, 4, 8, 16
    c = {0: 64}
    for i, v in enumerate(_T32_ODD_ROW1):
        c[2 * i + 1] = v
    for i, v in enumerate([90, 87, 80, 70, 57, 43, 25, 9]):
        c[4 * i + 2] = v
    for i, v in enumerate([89, 75, 50, 18]):
        c[8 * i + 4] = v
    for i, v in enumerate([83, 36]):
        c[16 * i + 8] = v
    c[16] = 64
    c[32] = 0
    m = np.zeros((32, 32), dtype=np.int64)
    for k in range(32):
        for n in range(32):
            if k == 0:
                m[k, n] = 64
                continue
            a = (k * (2 * n + 1)) % 128
            s = 1
            if a > 64:
                a = 128 - a
            if a > 32:
                a = 64 - a
                s = -1
            m[k, n] = s * c[a]
    return m


_T32 = _transform_matrix()


# 4x4 DST-VII (8.6.4.2, trType 1: intra 4x4 luma), rows = basis functions
_DST4 = np.array([[29, 55, 74, 84], [74, 74, 0, -74], [84, -29, -74, 55], [55, -84, 74, -29]], np.int64)


def _tmat(n: int) -> np.ndarray:
    return _T32[:: 32 // n, :n]


# ----------------------------------------------------------------------------- bitstream
def split_nal_units(stream: bytes) -> list[bytes]:
    """Annex-B byte stream -> NAL unit payloads (start codes removed, EPB kept)."""
    out = []
    i, n = 0, len(stream)
    starts = []
    while i + 2 < n:
        if stream[i] == 0 and stream[i + 1] == 0 and stream[i + 2] == 1:
            starts.append(i + 3)
            i += 3
        else:
            i += 1
    for k, s in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else n
        nal = stream[s:e]
        while nal and nal[-1] == 0:  # trailing zero_byte of the next 4-byte start code
            nal = nal[:-1]
        out.append(bytes(nal))
    return out


def escape(rbsp: bytes) -> bytes:
    """Emulation prevention (7.4.2): 0x03 after two zero bytes before a byte <= 3."""
    out = bytearray()
    zeros = 0
    for b in rbsp:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


def unescape(nal: bytes) -> bytes:
    out = bytearray()
    zeros = 0
    for b in nal:
        if zeros >= 2 and b == 3:
            zeros = 0
            continue
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


class BitReader:
    def __init__(self, data: bytes, pos: int = 0):
        self.data = data
        self.pos = pos  # bit position

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            byte = self.data[self.pos >> 3] if (self.pos >> 3) < len(self.data) else 0
            v = (v << 1) | ((byte >> (7 - (self.pos & 7))) & 1)
            self.pos += 1
        return v

    def ue(self) -> int:
        lz = 0
        while self.u(1) == 0:
            lz += 1
            if lz > 32:
                raise ValueError("bad Exp-Golomb code")
        return (1 << lz) - 1 + self.u(lz)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)

    def byte_alignment(self) -> None:
        if self.u(1) != 1:
            raise ValueError("alignment_bit_equal_to_one missing")
        while self.pos & 7:
            if self.u(1) != 0:
                raise ValueError("nonzero alignment bit")


# ----------------------------------------------------------------------------- parameter sets
@dataclass
class SPS:
    width: int = 0
    height: int = 0
    conf: tuple = (0, 0, 0, 0)
    chroma_format_idc: int = 1
    log2_max_poc_lsb: int = 8
    log2_min_cb: int = 3
    log2_ctb: int = 4
    log2_min_tb: int = 2
    log2_max_tb: int = 5
    max_th_depth_inter: int = 0
    max_th_depth_intra: int = 0
    amp: int = 0
    sao: int = 0
    pcm: int = 0
    st_rps: list = field(default_factory=list)  # list of list of (delta_poc, used)
    long_term: int = 0
    tmvp: int = 0
    strong_intra_smoothing: int = 0


@dataclass
class PPS:
    dependent_slices: int = 0
    output_flag_present: int = 0
    num_extra_slice_header_bits: int = 0
    sign_data_hiding: int = 0
    cabac_init_present: int = 0
    num_ref_idx_l0_default: int = 1
    init_qp: int = 26
    constrained_intra_pred: int = 0
    transform_skip: int = 0
    cu_qp_delta_enabled: int = 0
    diff_cu_qp_delta_depth: int = 0
    cb_qp_offset: int = 0
    cr_qp_offset: int = 0
    slice_chroma_qp_offsets_present: int = 0
    weighted_pred: int = 0
    transquant_bypass: int = 0
    tiles: int = 0
    entropy_sync: int = 0
    loop_filter_across_slices: int = 0
    deblocking_override_enabled: int = 0
    deblocking_disabled: int = 0
    beta_offset_div2: int = 0
    tc_offset_div2: int = 0
    lists_modification_present: int = 0
    log2_parallel_merge_level: int = 2


def _profile_tier_level(r: BitReader, max_sub_layers_minus1: int) -> None:
    r.u(2 + 1 + 5 + 32 + 4 + 43 + 1)
    r.u(8)  # general_level_idc
    if max_sub_layers_minus1:
        raise NotImplementedError("sub-layers")


def _parse_vui(r: BitReader) -> None:
    if r.u(1):  # aspect_ratio_info_present_flag
        if r.u(8) == 255:
            r.u(32)
    if r.u(1):  # overscan_info_present_flag
        r.u(1)
    if r.u(1):  # video_signal_type_present_flag
        r.u(3 + 1)
        if r.u(1):
            r.u(24)
    if r.u(1):  # chroma_loc_info_present_flag
        r.ue()
        r.ue()
    r.u(3)  # neutral_chroma_indication, field_seq, frame_field_info_present
    if r.u(1):  # default_display_window_flag
        for _ in range(4):
            r.ue()
    if r.u(1):  # vui_timing_info_present_flag
        r.u(32)
        r.u(32)
        if r.u(1):
            r.ue()
        if r.u(1):
            raise NotImplementedError("HRD parameters")
    if r.u(1):  # bitstream_restriction_flag
        r.u(3)
        for _ in range(5):
            r.ue()


def _st_ref_pic_set(r: BitReader, idx: int, sets: list) -> list:
    if idx != 0 and r.u(1):
        raise NotImplementedError("inter RPS prediction")
    nneg, npos = r.ue(), r.ue()
    out, poc = [], 0
    for _ in range(nneg):
        poc -= r.ue() + 1
        out.append((poc, r.u(1)))
    poc = 0
    for _ in range(npos):
        poc += r.ue() + 1
        out.append((poc, r.u(1)))
    return out


def parse_sps(rbsp: bytes) -> SPS:
    r = BitReader(rbsp, 16)
    s = SPS()
    r.u(4)
    msl = r.u(3)
    r.u(1)
    _profile_tier_level(r, msl)
    r.ue()
    s.chroma_format_idc = r.ue()
    if s.chroma_format_idc != 1:
        raise NotImplementedError("only 4:2:0")
    s.width, s.height = r.ue(), r.ue()
    if r.u(1):
        s.conf = (r.ue(), r.ue(), r.ue(), r.ue())
    if r.ue() or r.ue():
        raise NotImplementedError("only 8-bit")
    s.log2_max_poc_lsb = r.ue() + 4
    sub = r.u(1)
    for _ in range(0 if sub else msl, msl + 1):
        r.ue()
        r.ue()
        r.ue()
    s.log2_min_cb = r.ue() + 3
    s.log2_ctb = s.log2_min_cb + r.ue()
    s.log2_min_tb = r.ue() + 2
    s.log2_max_tb = s.log2_min_tb + r.ue()
    s.max_th_depth_inter = r.ue()
    s.max_th_depth_intra = r.ue()
    if r.u(1):
        raise NotImplementedError("scaling lists")
    s.amp = r.u(1)
    s.sao = r.u(1)
    s.pcm = r.u(1)
    if s.pcm:
        raise NotImplementedError("PCM")
    n = r.ue()
    for i in range(n):
        s.st_rps.append(_st_ref_pic_set(r, i, s.st_rps))
    s.long_term = r.u(1)
    if s.long_term:
        raise NotImplementedError("long-term references")
    s.tmvp = r.u(1)
    s.strong_intra_smoothing = r.u(1)
    if r.u(1):
        _parse_vui(r)
    return s


def parse_pps(rbsp: bytes) -> PPS:
    r = BitReader(rbsp, 16)
    p = PPS()
    r.ue()
    r.ue()
    p.dependent_slices = r.u(1)
    p.output_flag_present = r.u(1)
    p.num_extra_slice_header_bits = r.u(3)
    p.sign_data_hiding = r.u(1)
    p.cabac_init_present = r.u(1)
    p.num_ref_idx_l0_default = r.ue() + 1
    r.ue()
    p.init_qp = 26 + r.se()
    p.constrained_intra_pred = r.u(1)
    p.transform_skip = r.u(1)
    p.cu_qp_delta_enabled = r.u(1)
    if p.cu_qp_delta_enabled:
        p.diff_cu_qp_delta_depth = r.ue()
    p.cb_qp_offset = r.se()
    p.cr_qp_offset = r.se()
    p.slice_chroma_qp_offsets_present = r.u(1)
    p.weighted_pred = r.u(1)
    r.u(1)
    p.transquant_bypass = r.u(1)
    p.tiles = r.u(1)
    p.entropy_sync = r.u(1)
    if p.tiles:
        raise NotImplementedError("tiles")
    p.loop_filter_across_slices = r.u(1)
    if r.u(1):  # deblocking_filter_control_present_flag
        p.deblocking_override_enabled = r.u(1)
        p.deblocking_disabled = r.u(1)
        if not p.deblocking_disabled:
            p.beta_offset_div2 = r.se()
            p.tc_offset_div2 = r.se()
    if r.u(1):
        raise NotImplementedError("PPS scaling lists")
    p.lists_modification_present = r.u(1)
    p.log2_parallel_merge_level = r.ue() + 2
    return p


# ----------------------------------------------------------------------------- CABAC engine
class Cabac:
    def __init__(self, data: bytes, byte_pos: int, slice_type: int, qp: int, cabac_init_flag: int = 0):
        self.data = data
        self.init_contexts(slice_type, qp, cabac_init_flag)
        self.init_engine(byte_pos)

    def init_engine(self, byte_pos: int) -> None:
        """Arithmetic decoding engine initialisation (9.3.2.5) at a byte position."""
        self.pos = byte_pos * 8
        self.range = 510
        self.offset = self.bits(9)

    def init_contexts(self, slice_type: int, qp: int, cabac_init_flag: int = 0) -> None:
        init_type = 0 if slice_type == 2 else (2 if cabac_init_flag else 1) if slice_type == 1 else (
            1 if cabac_init_flag else 2)
        self.ctx: dict[str, list[list[int]]] = {}
        qpc = min(max(qp, 0), 51)
        for name, vals in _INIT.items():
            states = []
            for iv in vals[init_type]:
                m = (iv >> 4) * 5 - 45
                n = ((iv & 15) << 3) - 16
                pre = min(max(((m * qpc) >> 4) + n, 1), 126)
                states.append([pre - 64, 1] if pre > 63 else [63 - pre, 0])
            self.ctx[name] = states

    def save_contexts(self) -> dict:
        return {k: [list(s) for s in v] for k, v in self.ctx.items()}

    def restore_contexts(self, saved: dict) -> None:
        self.ctx = {k: [list(s) for s in v] for k, v in saved.items()}

    def end_substream(self) -> int:
        """After end_of_subset_one_bit == 1: the last bit read is alignment_bit_equal_to_one, zero
        bits follow up to the byte boundary; returns the byte position of the next substream."""
        last = self.pos - 1
        if (self.data[last >> 3] >> (7 - (last & 7))) & 1 != 1:
            raise ValueError("substream does not end with alignment_bit_equal_to_one")
        while self.pos & 7:
            if self.bit():
                raise ValueError("nonzero alignment bit after a substream")
        return self.pos >> 3

    def bit(self) -> int:
        i = self.pos >> 3
        b = (self.data[i] >> (7 - (self.pos & 7))) & 1 if i < len(self.data) else 0
        self.pos += 1
        return b

    def bits(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bit()
        return v

    def decision(self, name: str, inc: int = 0) -> int:
        st = self.ctx[name][inc]
        s, mps = st
        lps = _RANGE_LPS[s][(self.range >> 6) & 3]
        self.range -= lps
        if self.offset >= self.range:
            b = 1 - mps
            self.offset -= self.range
            self.range = lps
            if s == 0:
                st[1] = 1 - mps
            st[0] = _TRANS_LPS[s]
        else:
            b = mps
            st[0] = min(s + 1, 62)
        while self.range < 256:
            self.range <<= 1
            self.offset = (self.offset << 1) | self.bit()
        return b

    def bypass(self) -> int:
        self.offset = (self.offset << 1) | self.bit()
        if self.offset >= self.range:
            self.offset -= self.range
            return 1
        return 0

    def bypass_bits(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bypass()
        return v

    def terminate(self) -> int:
        self.range -= 2
        if self.offset >= self.range:
            return 1
        while self.range < 256:
            self.range <<= 1
            self.offset = (self.offset << 1) | self.bit()
        return 0

    def check_slice_end(self) -> None:
        """After end_of_slice_segment_flag == 1 (9.3.4.3.5): the last bit read into ivlOffset
        is the rbsp_stop_one_bit; only zero alignment bits may follow, then the NAL ends."""
        last = self.pos - 1
        if (self.data[last >> 3] >> (7 - (last & 7))) & 1 != 1:
            raise ValueError("the last bit of the slice data is not rbsp_stop_one_bit")
        while self.pos & 7:
            if self.bit():
                raise ValueError("nonzero alignment bit after the slice data")
        if (self.pos >> 3) != len(self.data):
            raise ValueError(f"{len(self.data) - (self.pos >> 3)} trailing bytes after the slice data")

    def egk(self, k: int) -> int:
        v = 0
        while self.bypass():
            v += 1 << k
            k += 1
        return v + self.bypass_bits(k)


# ----------------------------------------------------------------------------- picture state
@dataclass
class Picture:
    y: np.ndarray
    u: np.ndarray
    v: np.ndarray
    poc: int


def _scan_diag(blk: int) -> list[tuple[int, int]]:
    out = []
    x = y = 0
    while len(out) < blk * blk:
        while y >= 0:
            if x < blk and y < blk:
                out.append((x, y))
            y -= 1
            x += 1
        y, x = x, 0
    return out


_SCANS = {}
for _b in (1, 2, 4, 8):
    _SCANS[(_b, 0)] = _scan_diag(_b)
    _SCANS[(_b, 1)] = [(x, y) for y in range(_b) for x in range(_b)]  # horizontal
    _SCANS[(_b, 2)] = [(x, y) for x in range(_b) for y in range(_b)]  # vertical
_CTX_IDX_MAP_4X4 = [0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8]


class Decoder:
    """Decode an Annex-B HEVC stream; ``frames`` holds cropped (Y, U, V) uint8 planes in
    output order, ``frames_coded`` the uncropped reconstructions."""

    def __init__(self):
        self.sps: SPS | None = None
        self.pps: PPS | None = None
        self.frames: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []
        self.frames_coded: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []
        self.ref: Picture | None = None
        self.cur: Picture | None = None
        self.prev_poc_tid0 = 0
        self.stats = {"skip": 0, "merge": 0, "amvp": 0, "intra": 0, "slices": 0}

    # ---------------------------------------------------------------- top level
    def decode(self, stream: bytes) -> list[tuple[np.ndarray, np.ndarray, np.ndarray]]:
        start = len(self.frames)
        for nal in split_nal_units(stream):
            self._nal(nal)
        self._finish_picture()
        return self.frames[start:]

    def _nal(self, nal: bytes) -> None:
        if len(nal) < 2:
            return
        if nal[0] & 0x80:
            raise ValueError("forbidden_zero_bit set")
        typ = (nal[0] >> 1) & 63
        rbsp = unescape(nal)
        if typ == 32:
            return  # VPS: nothing needed for decoding
        if typ == 33:
            self.sps = parse_sps(rbsp)
        elif typ == 34:
            self.pps = parse_pps(rbsp)
        elif typ in (0, 1, 19, 20):
            self._slice(typ, rbsp)
        elif typ in (35, 39, 40):
            pass  # AUD / SEI
        else:
            raise NotImplementedError(f"NAL unit type {typ}")

    def _finish_picture(self) -> None:
        if self.cur is None:
            return
        s = self.sps
        p = self.cur
        if any(not sp["db_disabled"] for sp in self.slice_params.values()):
            self._deblock()
        if self.sao_params:
            self._sao()
        self.frames_coded.append((p.y.copy(), p.u.copy(), p.v.copy()))
        l, r, t, b = s.conf
        h, w = p.y.shape
        self.frames.append((p.y[2 * t:h - 2 * b, 2 * l:w - 2 * r].copy(),
                            p.u[t:h // 2 - b, l:w // 2 - r].copy(), p.v[t:h // 2 - b, l:w // 2 - r].copy()))
        self.ref = p
        self.cur = None

    # ---------------------------------------------------------------- SAO (8.7.3)
    def _sao(self) -> None:
        """Sample adaptive offset over the deblocked picture: every CTB reads the deblocked
        samples (never an already offset neighbour) and writes the output picture."""
        s = self.sps
        ctbs_w = (s.width + (1 << s.log2_ctb) - 1) >> s.log2_ctb
        planes = (self.cur.y, self.cur.u, self.cur.v)
        src = [pl.copy() for pl in planes]
        for ctb, params in self.sao_params.items():
            cx, cy = ctb % ctbs_w, ctb // ctbs_w
            x_l, y_l = cx << s.log2_ctb, cy << s.log2_ctb
            prm = self.slice_params[int(self.slice_map[y_l >> 2, x_l >> 2])]
            for c in range(3):
                if not (prm["sao_luma"] if c == 0 else prm["sao_chroma"]):
                    continue
                typ, off, band, eo = params[c]
                if typ == 0:
                    continue
                sh = 0 if c == 0 else 1
                pic = src[c]
                H, W = pic.shape
                sz = 1 << (s.log2_ctb - sh)
                x0, y0 = cx * sz, cy * sz
                x1, y1 = min(x0 + sz, W), min(y0 + sz, H)
                blk = pic[y0:y1, x0:x1]
                if typ == 1:  # band offset: four consecutive bands of width 8 from sao_band_position
                    table = np.zeros(32, np.int32)
                    for k in range(4):
                        table[(k + band) & 31] = off[k]
                    delta = table[blk >> 3]
                else:  # edge offset along class eo
                    ys, xs = np.mgrid[y0:y1, x0:x1]
                    cur_sid = self.slice_map[(ys << sh) >> 2, (xs << sh) >> 2]
                    valid = np.ones(blk.shape, bool)
                    signs = 2
                    for dx, dy in _SAO_EO_NB[eo]:
                        ny, nx = ys + dy, xs + dx
                        inside = (ny >= 0) & (ny < H) & (nx >= 0) & (nx < W)
                        nyc, nxc = np.clip(ny, 0, H - 1), np.clip(nx, 0, W - 1)
                        nb_sid = self.slice_map[(nyc << sh) >> 2, (nxc << sh) >> 2]
                        # across a slice border the later slice's slice_loop_filter_across_slices_enabled_flag rules
                        later = np.maximum(cur_sid, nb_sid)
                        across = np.vectorize(lambda a: self.slice_params[int(a)]["lf_across"])(later) if (
                            (nb_sid != cur_sid).any()) else np.ones(blk.shape, np.int32)
                        valid &= inside & ((nb_sid == cur_sid) | (across != 0))
                        signs = signs + np.sign(blk - pic[nyc, nxc])
                    offv = np.array([0, off[0], off[1], off[2], off[3]], np.int32)
                    delta = np.where(valid, offv[_SAO_EDGE_CAT[signs]], 0)
                planes[c][y0:y1, x0:x1] = np.clip(blk + delta, 0, 255)

    def _sao_syntax(self, cab: Cabac, ctb: int, ctbs_w: int, slice_addr: int, luma: int, chroma: int) -> None:
        """sao(rx, ry) (7.3.8.3): merge left / up, else per component type, offsets, band
        position or edge class.  Stored as (SaoTypeIdx, SaoOffsetVal[1..4], band, eo_class)."""
        rx, ry = ctb % ctbs_w, ctb // ctbs_w
        if rx > 0 and ctb - 1 >= slice_addr and cab.decision("sao_merge_flag"):
            self.sao_params[ctb] = self.sao_params[ctb - 1]
            self.stats["sao_merge"] = self.stats.get("sao_merge", 0) + 1
            return
        if ry > 0 and ctb - ctbs_w >= slice_addr and cab.decision("sao_merge_flag"):
            self.sao_params[ctb] = self.sao_params[ctb - ctbs_w]
            self.stats["sao_merge"] = self.stats.get("sao_merge", 0) + 1
            return
        out = []
        for c in range(3):
            if not (luma if c == 0 else chroma):
                out.append((0, (0, 0, 0, 0), 0, 0))
                continue
            if c == 2:
                typ, eo = out[1][0], out[1][3]
            else:
                typ = 0 if not cab.decision("sao_type_idx") else (1 if not cab.bypass() else 2)
                eo = 0
            if typ == 0:
                out.append((0, (0, 0, 0, 0), 0, 0))
                continue
            absv = []
            for _ in range(4):  # TR, cMax = (1 << (min(bitDepth, 10) - 5)) - 1 = 7, bypass
                v = 0
                while v < 7 and cab.bypass():
                    v += 1
                absv.append(v)
            band = 0
            if typ == 1:
                offs = tuple(-a if a and cab.bypass() else a for a in absv)
                band = cab.bypass_bits(5)
            else:
                offs = (absv[0], absv[1], -absv[2], -absv[3])
                if c < 2:
                    eo = cab.bypass_bits(2)
            out.append((typ, offs, band, eo))
            key = "sao_band" if typ == 1 else "sao_edge"
            self.stats[key] = self.stats.get(key, 0) + 1
        self.sao_params[ctb] = tuple(out)

    # ---------------------------------------------------------------- deblocking (8.7.2)
    def _deblock(self) -> None:
        for vertical in (True, False):  # all vertical edges of the picture first, then horizontal
            self._deblock_dir(vertical)

    def _deblock_dir(self, vertical: bool) -> None:
        y, u, v = self.cur.y, self.cur.u, self.cur.v
        H, W = y.shape
        emap = self.edge_v if vertical else self.edge_h
        for e in range(8, W if vertical else H, 8):  # 8x8 luma grid, picture borders excluded
            for t in range(0, H if vertical else W, 4):  # 4-sample segments along the edge
                xq, yq = (e, t) if vertical else (t, e)
                xp, yp = (e - 1, t) if vertical else (t, e - 1)
                if not emap[yq >> 2, xq >> 2]:
                    continue
                sq, sp_ = self.slice_map[yq >> 2, xq >> 2], self.slice_map[yp >> 2, xp >> 2]
                prm = self.slice_params[int(sq)]
                if prm["db_disabled"] or (sq != sp_ and not prm["lf_across"]):
                    continue
                bq, bp = (yq >> 2, xq >> 2), (yp >> 2, xp >> 2)
                if self.pred_intra[bq] or self.pred_intra[bp]:
                    bs = 2
                elif self.cbf_map[bq] or self.cbf_map[bp]:
                    bs = 1
                else:
                    mq, mp = self.mv_map[bq], self.mv_map[bp]
                    bs = 1 if abs(int(mq[0]) - int(mp[0])) >= 4 or abs(int(mq[1]) - int(mp[1])) >= 4 else 0
                if bs == 0:
                    continue
                qpl = (int(self.qp_map[bq]) + int(self.qp_map[bp]) + 1) >> 1
                self._db_luma(y, vertical, e, t, bs, qpl, prm)
                if bs == 2 and e % 16 == 0:  # chroma: 8-sample chroma grid, intra edges only
                    for plane, off in ((u, self.pps.cb_qp_offset), (v, self.pps.cr_qp_offset)):
                        qpi = qpl + off
                        qpc = qpi if qpi < 30 else (qpi - 6 if qpi > 43 else _QPC_TABLE[qpi])
                        tc = _DB_TC[min(max(qpc + 2 + prm["tc_offset"], 0), 53)]
                        for k in range(2):
                            if vertical:
                                row, c = plane[t // 2 + k], e // 2
                                p0, p1, q0, q1 = int(row[c - 1]), int(row[c - 2]), int(row[c]), int(row[c + 1])
                            else:
                                col, c = plane[:, t // 2 + k], e // 2
                                p0, p1, q0, q1 = int(col[c - 1]), int(col[c - 2]), int(col[c]), int(col[c + 1])
                            d = min(max((((q0 - p0) * 4) + p1 - q1 + 4) >> 3, -tc), tc)
                            (row if vertical else col)[c - 1] = min(max(p0 + d, 0), 255)
                            (row if vertical else col)[c] = min(max(q0 - d, 0), 255)

    @staticmethod
    def _db_luma(y, vertical: bool, e: int, t: int, bs: int, qpl: int, prm: dict) -> None:
        beta = _DB_BETA[min(max(qpl + prm["beta_offset"], 0), 51)]
        tc = _DB_TC[min(max(qpl + 2 * (bs - 1) + prm["tc_offset"], 0), 53)]
        lines = [y[t + k, e - 4: e + 4] if vertical else y[e - 4: e + 4, t + k] for k in range(4)]
        vals = [[int(x) for x in ln] for ln in lines]  # p3 p2 p1 p0 q0 q1 q2 q3
        def dp(k):
            return abs(vals[k][1] - 2 * vals[k][2] + vals[k][3])
        def dq(k):
            return abs(vals[k][6] - 2 * vals[k][5] + vals[k][4])
        dpq0, dpq3 = dp(0) + dq(0), dp(3) + dq(3)
        if dpq0 + dpq3 >= beta:
            return
        def strong(k, dpq):
            a = vals[k]
            return (2 * dpq < (beta >> 2) and abs(a[0] - a[3]) + abs(a[4] - a[7]) < (beta >> 3)
                    and abs(a[3] - a[4]) < ((5 * tc + 1) >> 1))
        de2 = strong(0, dpq0) and strong(3, dpq3)
        dep = dp(0) + dp(3) < ((beta + (beta >> 1)) >> 3)
        deq = dq(0) + dq(3) < ((beta + (beta >> 1)) >> 3)
        def c3(lo, hi, x):
            return min(max(x, lo), hi)
        for k in range(4):
            p3, p2, p1, p0, q0, q1, q2, q3 = vals[k]
            out = lines[k]
            if de2:
                out[3] = c3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3)
                out[2] = c3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2)
                out[1] = c3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3)
                out[4] = c3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3)
                out[5] = c3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2)
                out[6] = c3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3)
            else:
                d = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4
                if abs(d) >= tc * 10:
                    continue
                d = c3(-tc, tc, d)
                out[3] = c3(0, 255, p0 + d)
                out[4] = c3(0, 255, q0 - d)
                if dep:
                    out[2] = c3(0, 255, p1 + c3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + d) >> 1))
                if deq:
                    out[5] = c3(0, 255, q1 + c3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - d) >> 1))

    # ---------------------------------------------------------------- slice
    def _slice(self, typ: int, rbsp: bytes) -> None:
        s, p = self.sps, self.pps
        r = BitReader(rbsp, 16)
        first = r.u(1)
        if 16 <= typ <= 23:
            r.u(1)
        r.ue()
        ctbs_w = (s.width + (1 << s.log2_ctb) - 1) >> s.log2_ctb
        ctbs_h = (s.height + (1 << s.log2_ctb) - 1) >> s.log2_ctb
        addr = 0
        if not first:
            if p.dependent_slices and r.u(1):
                raise NotImplementedError("dependent slice segments")
            nb = (ctbs_w * ctbs_h - 1).bit_length()
            addr = r.u(nb)
        r.u(p.num_extra_slice_header_bits)
        slice_type = r.ue()
        if p.output_flag_present:
            r.u(1)
        idr = typ in (19, 20)
        if idr:
            poc = 0
        else:
            lsb = r.u(s.log2_max_poc_lsb)
            max_lsb = 1 << s.log2_max_poc_lsb
            prev_lsb, prev_msb = self.prev_poc_tid0 % max_lsb, self.prev_poc_tid0 - self.prev_poc_tid0 % max_lsb
            if lsb < prev_lsb and prev_lsb - lsb >= max_lsb // 2:
                msb = prev_msb + max_lsb
            elif lsb > prev_lsb and lsb - prev_lsb > max_lsb // 2:
                msb = prev_msb - max_lsb
            else:
                msb = prev_msb
            poc = msb + lsb
            if r.u(1):  # short_term_ref_pic_set_sps_flag
                rps = s.st_rps[r.u((len(s.st_rps) - 1).bit_length()) if len(s.st_rps) > 1 else 0]
            else:
                rps = _st_ref_pic_set(r, len(s.st_rps), s.st_rps)
            if s.tmvp and r.u(1):
                raise NotImplementedError("TMVP")
        if first:
            self._finish_picture()
            h = ctbs_h << s.log2_ctb
            w = ctbs_w << s.log2_ctb
            if s.width % (1 << s.log2_min_cb) or s.height % (1 << s.log2_min_cb):
                raise ValueError("picture size not a multiple of MinCbSizeY")
            self.cur = Picture(np.zeros((s.height, s.width), np.int32), np.zeros((s.height // 2, s.width // 2), np.int32),
                               np.zeros((s.height // 2, s.width // 2), np.int32), poc)
            n4 = (h // 4, w // 4)
            self.slice_map = np.full(n4, -1, np.int32)   # slice address per 4x4 block (-1 = not decoded)
            self.pred_intra = np.zeros(n4, bool)
            self.skip_map = np.zeros(n4, bool)
            self.depth_map = np.zeros(n4, np.int32)
            self.mv_map = np.zeros(n4 + (2,), np.int32)
            self.intra_mode_map = np.full(n4, 1, np.int32)
            self.qp_map = np.zeros(n4, np.int32)
            self.cbf_map = np.zeros(n4, bool)    # luma TU with nonzero levels covering the 4x4 block
            self.edge_v = np.zeros(n4, bool)     # transform/prediction edge on the left of the 4x4 block
            self.edge_h = np.zeros(n4, bool)     # ... on the top
            self.slice_params = {}
            self.sao_params = {}
            self.prev_poc_tid0 = poc
        elif self.cur is None:
            raise ValueError("slice of a picture whose first slice is missing")
        sao_luma = sao_chroma = 0
        if s.sao:
            sao_luma, sao_chroma = r.u(1), r.u(1)
        max_merge = 5
        if slice_type != 2:
            if slice_type != 1:
                raise NotImplementedError("B slices")
            num_ref = p.num_ref_idx_l0_default
            if r.u(1):
                num_ref = r.ue() + 1
            if num_ref != 1:
                raise NotImplementedError("more than one reference index")
            if p.cabac_init_present and r.u(1):
                raise NotImplementedError("cabac_init_flag")
            if p.weighted_pred:
                raise NotImplementedError("weighted prediction")
            max_merge = 5 - r.ue()
            if self.ref is None:
                raise ValueError("P slice without a reference picture")
            if not any(used for _, used in rps):
                raise ValueError("P slice with an empty RPS")
            if rps[0][0] + poc != self.ref.poc:
                raise NotImplementedError("reference is not the previous picture")
        slice_qp = p.init_qp + r.se()
        if p.slice_chroma_qp_offsets_present:
            r.se()
            r.se()
        db_disabled = p.deblocking_disabled
        beta_div2, tc_div2 = p.beta_offset_div2, p.tc_offset_div2
        if p.deblocking_override_enabled and r.u(1):  # deblocking_filter_override_flag
            db_disabled = r.u(1)  # slice_deblocking_filter_disabled_flag
            if not db_disabled:
                beta_div2, tc_div2 = r.se(), r.se()
        lf_across = p.loop_filter_across_slices
        if p.loop_filter_across_slices and (sao_luma or sao_chroma or not db_disabled):
            lf_across = r.u(1)
        entry = []
        if p.entropy_sync:
            n_entry = r.ue()
            if n_entry:
                olen = r.ue() + 1
                entry = [r.u(olen) + 1 for _ in range(n_entry)]
        self.slice_params[addr] = {"db_disabled": db_disabled, "lf_across": lf_across,
                                   "sao_luma": sao_luma, "sao_chroma": sao_chroma,
                                   "beta_offset": 2 * beta_div2, "tc_offset": 2 * tc_div2}
        r.byte_alignment()
        self.stats["slices"] += 1
        self.slice_type = slice_type
        self.slice_addr = addr
        self.max_merge = max_merge
        self.qp_y = slice_qp
        self.qp_prev = slice_qp
        cab = Cabac(rbsp, r.pos >> 3, slice_type, slice_qp)
        ctb = addr
        sub_starts = [r.pos >> 3]  # rbsp byte position of every substream (WPP)
        wpp_saved = None
        while True:
            cx, cy = ctb % ctbs_w, ctb // ctbs_w
            if p.entropy_sync and cx == 0 and ctb != addr:
                # 9.3.1: the contexts of a CTU row's first CTB come from the row above after its
                # second CTB when the top-right CTB is available (same slice), else fresh
                tr_ok = ctbs_w >= 2 and (ctb - ctbs_w + 1) >= addr
                if tr_ok and wpp_saved is not None:
                    cab.restore_contexts(wpp_saved)
                else:
                    cab.init_contexts(slice_type, slice_qp)
                wpp_saved = None
                self.qp_prev = slice_qp  # 8.6.1: first QG of a CTB row with WPP
            if sao_luma or sao_chroma:
                self._sao_syntax(cab, ctb, ctbs_w, addr, sao_luma, sao_chroma)
            self._coding_quadtree(cab, cx << s.log2_ctb, cy << s.log2_ctb, s.log2_ctb, 0)
            if p.entropy_sync and cx == 1:
                wpp_saved = cab.save_contexts()  # storage after the row's second CTB (9.3.2.2)
            if cab.terminate():
                cab.check_slice_end()
                break
            ctb += 1
            if ctb >= ctbs_w * ctbs_h:
                raise ValueError("slice runs past the last CTB")
            if p.entropy_sync and ctb % ctbs_w == 0:
                if not cab.terminate():
                    raise ValueError("end_of_subset_one_bit is not 1")
                nxt = cab.end_substream()
                sub_starts.append(nxt)
                cab.init_engine(nxt)
        if p.entropy_sync:
            # entry points = substream sizes after emulation prevention (7.4.7.1)
            if len(entry) != len(sub_starts) - 1:
                raise ValueError(f"{len(entry)} entry points for {len(sub_starts)} substreams")
            for k, e in enumerate(entry):
                got = len(escape(rbsp[sub_starts[k]:sub_starts[k + 1]]))
                if got != e:
                    raise ValueError(f"entry point {k}: {e} bytes signalled, substream is {got}")
            self.stats["substreams"] = self.stats.get("substreams", 0) + len(sub_starts)

    # ---------------------------------------------------------------- availability (6.4.1)
    def _avail(self, xc: int, yc: int, xn: int, yn: int) -> bool:
        s = self.sps
        if xn < 0 or yn < 0 or xn >= s.width or yn >= s.height:
            return False
        sid = self.slice_map[yn >> 2, xn >> 2]
        return sid == self.slice_addr

    # ---------------------------------------------------------------- coding tree
    def _coding_quadtree(self, cab: Cabac, x0: int, y0: int, log2: int, depth: int) -> None:
        s, p = self.sps, self.pps
        size = 1 << log2
        if x0 + size <= s.width and y0 + size <= s.height and log2 > s.log2_min_cb:
            inc = 0
            if self._avail(x0, y0, x0 - 1, y0) and self.depth_map[y0 >> 2, (x0 - 1) >> 2] > depth:
                inc += 1
            if self._avail(x0, y0, x0, y0 - 1) and self.depth_map[(y0 - 1) >> 2, x0 >> 2] > depth:
                inc += 1
            split = cab.decision("split_cu_flag", inc)
        else:
            split = 1 if log2 > s.log2_min_cb else 0
        if p.cu_qp_delta_enabled and log2 >= s.log2_ctb - p.diff_cu_qp_delta_depth:
            self.qg_coded = False
            self.cu_qp_delta = 0
            self._qg_start(x0, y0)
        if split:
            h = size >> 1
            for dx, dy in ((0, 0), (h, 0), (0, h), (h, h)):
                if x0 + dx < s.width and y0 + dy < s.height:
                    self._coding_quadtree(cab, x0 + dx, y0 + dy, log2 - 1, depth + 1)
        else:
            self._coding_unit(cab, x0, y0, log2, depth)

    def _qg_start(self, x0: int, y0: int) -> None:
        # qPY_PRED (8.6.1): previous QG's QpY unless first QG of the slice; left/above if in the same CTB
        s = self.sps
        prev = self.qp_prev
        ctb_mask = ~((1 << s.log2_ctb) - 1)
        def nb(xn, yn):
            if self._avail(x0, y0, xn, yn) and (xn & ctb_mask) == (x0 & ctb_mask) and (yn & ctb_mask) == (y0 & ctb_mask):
                return int(self.qp_map[yn >> 2, xn >> 2])
            return prev
        self.qp_pred = (nb(x0 - 1, y0) + nb(x0, y0 - 1) + 1) >> 1
        self.qp_y = self.qp_pred

    def _coding_unit(self, cab: Cabac, x0: int, y0: int, log2: int, depth: int) -> None:
        s, p = self.sps, self.pps
        size = 1 << log2
        if p.transquant_bypass:
            raise NotImplementedError("transquant bypass")
        skip = 0
        if self.slice_type != 2:
            inc = 0
            if self._avail(x0, y0, x0 - 1, y0) and self.skip_map[y0 >> 2, (x0 - 1) >> 2]:
                inc += 1
            if self._avail(x0, y0, x0, y0 - 1) and self.skip_map[(y0 - 1) >> 2, x0 >> 2]:
                inc += 1
            skip = cab.decision("cu_skip_flag", inc)
        b4 = (slice(y0 >> 2, (y0 + size) >> 2), slice(x0 >> 2, (x0 + size) >> 2))
        self.edge_v[b4[0], x0 >> 2] = True  # prediction-unit (= CU) edges
        self.edge_h[y0 >> 2, b4[1]] = True
        self.cbf_map[b4] = False
        if skip:
            self.stats["skip"] += 1
            mv = self._prediction_unit(cab, x0, y0, size, size, merge_flag=1)
            self._inter_predict(x0, y0, size, mv)
            self.qp_map[b4] = self.qp_y
            self._mark(b4, intra=False, skip=True, depth=depth, mv=mv)
            self.qp_prev = self.qp_y
            return
        intra = 1 if self.slice_type == 2 else cab.decision("pred_mode_flag")
        if not intra or log2 == s.log2_min_cb:
            if intra:
                pm = 0 if cab.decision("part_mode", 0) else 1
            else:
                if not cab.decision("part_mode", 0):
                    raise NotImplementedError("inter PartMode other than 2Nx2N")
                pm = 0
            if pm != 0:
                raise NotImplementedError("intra NxN")
        if intra:
            self.stats["intra"] += 1
            prev_flag = cab.decision("prev_intra_luma_pred_flag")
            if prev_flag:
                mpm_idx = 0
                while mpm_idx < 2 and cab.bypass():
                    mpm_idx += 1
            else:
                rem = cab.bypass_bits(5)
            cand = self._mpm(x0, y0)
            if prev_flag:
                mode = cand[mpm_idx]
            else:
                mode = rem
                for c in sorted(cand):
                    if mode >= c:
                        mode += 1
            if cab.decision("intra_chroma_pred_mode"):
                cm = cab.bypass_bits(2)
                mode_c = [0, 26, 10, 1][cm]
                if mode_c == mode:
                    mode_c = 34
            else:
                mode_c = mode
            self.intra_mode_map[b4] = mode
            self._mark(b4, intra=True, skip=False, depth=depth, mv=(0, 0), decoded=False)
            root = 1
            merge = 0
            mv = (0, 0)
        else:
            merge = cab.decision("merge_flag")
            mv = self._prediction_unit(cab, x0, y0, size, size, merge_flag=merge)
            self.stats["merge" if merge else "amvp"] += 1
            self._inter_predict(x0, y0, size, mv)
            self._mark(b4, intra=False, skip=False, depth=depth, mv=mv, decoded=False)
            root = 1 if merge else cab.decision("rqt_root_cbf")
            mode = mode_c = None
        self.cu_intra_modes = (mode, mode_c)
        if root:
            max_depth = s.max_th_depth_intra if intra else s.max_th_depth_inter
            self._transform_tree(cab, x0, y0, x0, y0, log2, 0, 0, max_depth, intra, (1, 1), x0, y0, log2)
        elif intra:
            raise AssertionError
        self.qp_map[b4] = self.qp_y
        self.qp_prev = self.qp_y
        self.slice_map[b4] = self.slice_addr

    def _mark(self, b4, intra: bool, skip: bool, depth: int, mv, decoded: bool = True) -> None:
        self.pred_intra[b4] = intra
        self.skip_map[b4] = skip
        self.depth_map[b4] = depth
        self.mv_map[b4] = mv
        if decoded:
            self.slice_map[b4] = self.slice_addr

    def _mpm(self, x0: int, y0: int) -> list[int]:
        s = self.sps
        def cand(xn, yn, above):
            if not self._avail(x0, y0, xn, yn) or not self.pred_intra[yn >> 2, xn >> 2]:
                return 1
            if above and yn < ((y0 >> s.log2_ctb) << s.log2_ctb):
                return 1
            return int(self.intra_mode_map[yn >> 2, xn >> 2])
        a, b = cand(x0 - 1, y0, False), cand(x0, y0 - 1, True)
        if a == b:
            if a < 2:
                return [0, 1, 26]
            return [a, 2 + ((a + 29) % 32), 2 + ((a - 2 + 1) % 32)]
        third = 0 if (a != 0 and b != 0) else (1 if (a != 1 and b != 1) else 26)
        return [a, b, third]

    # ---------------------------------------------------------------- prediction units (inter)
    def _nb_motion(self, xp: int, yp: int, xn: int, yn: int):
        if not self._avail(xp, yp, xn, yn) or self.pred_intra[yn >> 2, xn >> 2]:
            return None
        return tuple(int(v) for v in self.mv_map[yn >> 2, xn >> 2])

    def _prediction_unit(self, cab: Cabac, x: int, y: int, w: int, h: int, merge_flag: int):
        pml = self.pps.log2_parallel_merge_level
        def par(xn, yn):  # same merge estimation region -> unavailable
            return (x >> pml) == (xn >> pml) and (y >> pml) == (yn >> pml)
        if merge_flag:
            idx = 0  # merge_idx: truncated rice, cMax MaxNumMergeCand - 1, first bin context coded
            if self.max_merge > 1 and cab.decision("merge_idx"):
                idx = 1
                while idx < self.max_merge - 1 and cab.bypass():
                    idx += 1
            a1 = None if par(x - 1, y + h - 1) else self._nb_motion(x, y, x - 1, y + h - 1)
            b1 = None if par(x + w - 1, y - 1) else self._nb_motion(x, y, x + w - 1, y - 1)
            b0 = None if par(x + w, y - 1) else self._nb_motion(x, y, x + w, y - 1)
            a0 = None if par(x - 1, y + h) else self._nb_motion(x, y, x - 1, y + h)
            b2 = None if par(x - 1, y - 1) else self._nb_motion(x, y, x - 1, y - 1)
            cands = []
            if a1 is not None:
                cands.append(a1)
            if b1 is not None and b1 != a1:
                cands.append(b1)
            if b0 is not None and b0 != b1:
                cands.append(b0)
            if a0 is not None and a0 != a1:
                cands.append(a0)
            if b2 is not None and len(cands) < 4 and b2 != a1 and b2 != b1:
                cands.append(b2)
            while len(cands) < self.max_merge:
                cands.append((0, 0))
            return cands[idx]
        # AMVP (one reference picture -> no scaling)
        mvd = self._mvd_coding(cab)
        mvp_flag = cab.decision("mvp_flag")
        a0 = self._nb_motion(x, y, x - 1, y + h)
        a1 = self._nb_motion(x, y, x - 1, y + h - 1)
        mva = a0 if a0 is not None else a1
        scaled_flag = a0 is not None or a1 is not None
        mvb = None
        for xn, yn in ((x + w, y - 1), (x + w - 1, y - 1), (x - 1, y - 1)):
            m = self._nb_motion(x, y, xn, yn)
            if m is not None:
                mvb = m
                break
        if not scaled_flag and mvb is not None:
            mva = mvb
        if not scaled_flag:
            mvb = None
            for xn, yn in ((x + w, y - 1), (x + w - 1, y - 1), (x - 1, y - 1)):
                m = self._nb_motion(x, y, xn, yn)
                if m is not None:
                    mvb = m
                    break
        lst = []
        if mva is not None:
            lst.append(mva)
        if mvb is not None and not (mva is not None and mva == mvb):
            lst.append(mvb)
        while len(lst) < 2:
            lst.append((0, 0))
        mvp = lst[mvp_flag]
        return (((mvp[0] + mvd[0] + 32768) & 0xffff) - 32768, ((mvp[1] + mvd[1] + 32768) & 0xffff) - 32768)

    def _mvd_coding(self, cab: Cabac):
        g0 = [cab.decision("abs_mvd_greater0_flag"), cab.decision("abs_mvd_greater0_flag")]
        g1 = [cab.decision("abs_mvd_greater1_flag") if g0[0] else 0,
              cab.decision("abs_mvd_greater1_flag") if g0[1] else 0]
        out = []
        for c in range(2):
            v = 0
            if g0[c]:
                v = 1
                if g1[c]:
                    v = 2 + cab.egk(1)
                if cab.bypass():
                    v = -v
            out.append(v)
        return out

    def _inter_predict(self, x0: int, y0: int, size: int, mv) -> None:
        ref = self.ref
        mvx, mvy = mv
        H, W = ref.y.shape
        yi = np.clip(np.arange(y0 + (mvy >> 2) - 3, y0 + (mvy >> 2) + size + 5), 0, H - 1)
        xi = np.clip(np.arange(x0 + (mvx >> 2) - 3, x0 + (mvx >> 2) + size + 5), 0, W - 1)
        blk = ref.y[np.ix_(yi, xi)].astype(np.int64)
        fx, fy = mvx & 3, mvy & 3
        fh, fv = _LUMA_FILTER[fx], _LUMA_FILTER[fy]
        if fx == 0 and fy == 0:
            pred = blk[3:3 + size, 3:3 + size] << 6
        elif fy == 0:
            pred = sum(fh[i] * blk[3:3 + size, i:i + size] for i in range(8))
        elif fx == 0:
            pred = sum(fv[i] * blk[i:i + size, 3:3 + size] for i in range(8))
        else:
            tmp = sum(fh[i] * blk[:, i:i + size] for i in range(8))
            pred = sum(fv[i] * tmp[i:i + size, :] for i in range(8)) >> 6
        self.cur.y[y0:y0 + size, x0:x0 + size] = np.clip((pred + 32) >> 6, 0, 255)
        cs = size // 2
        xc, yc = x0 // 2, y0 // 2
        for plane_ref, plane in ((ref.u, self.cur.u), (ref.v, self.cur.v)):
            Hc, Wc = plane_ref.shape
            yi = np.clip(np.arange(yc + (mvy >> 3) - 1, yc + (mvy >> 3) + cs + 3), 0, Hc - 1)
            xi = np.clip(np.arange(xc + (mvx >> 3) - 1, xc + (mvx >> 3) + cs + 3), 0, Wc - 1)
            blk = plane_ref[np.ix_(yi, xi)].astype(np.int64)
            fx, fy = mvx & 7, mvy & 7
            fh, fv = _CHROMA_FILTER[fx], _CHROMA_FILTER[fy]
            if fx == 0 and fy == 0:
                pred = blk[1:1 + cs, 1:1 + cs] << 6
            elif fy == 0:
                pred = sum(fh[i] * blk[1:1 + cs, i:i + cs] for i in range(4))
            elif fx == 0:
                pred = sum(fv[i] * blk[i:i + cs, 1:1 + cs] for i in range(4))
            else:
                tmp = sum(fh[i] * blk[:, i:i + cs] for i in range(4))
                pred = sum(fv[i] * tmp[i:i + cs, :] for i in range(4)) >> 6
            plane[yc:yc + cs, xc:xc + cs] = np.clip((pred + 32) >> 6, 0, 255)

    # ---------------------------------------------------------------- transform tree
    def _transform_tree(self, cab, x0, y0, xb, yb, log2, depth, blk, max_depth, intra, parent_cbf, xcu, ycu,
                        log2cu):
        s = self.sps
        if log2 <= s.log2_max_tb and log2 > s.log2_min_tb and depth < max_depth:
            split = cab.decision("split_transform_flag", 5 - log2)
        else:
            split = 1 if log2 > s.log2_max_tb else 0
        cbf_cb = cbf_cr = 0
        if log2 > 2:
            if depth == 0 or parent_cbf[0]:
                cbf_cb = cab.decision("cbf_chroma", depth)
            if depth == 0 or parent_cbf[1]:
                cbf_cr = cab.decision("cbf_chroma", depth)
        else:
            cbf_cb, cbf_cr = parent_cbf
        if split:
            self.stats["tu_split"] = self.stats.get("tu_split", 0) + 1
            h = 1 << (log2 - 1)
            for k, (dx, dy) in enumerate(((0, 0), (h, 0), (0, h), (h, h))):
                self._transform_tree(cab, x0 + dx, y0 + dy, x0, y0, log2 - 1, depth + 1, k, max_depth, intra,
                                     (cbf_cb, cbf_cr), xcu, ycu, log2cu)
            return
        cbf_luma = 1
        if intra or depth != 0 or cbf_cb or cbf_cr:
            cbf_luma = cab.decision("cbf_luma", 1 if depth == 0 else 0)
        self._transform_unit(cab, x0, y0, xb, yb, log2, depth, blk, intra, cbf_luma, cbf_cb, cbf_cr)

    def _transform_unit(self, cab, x0, y0, xb, yb, log2, depth, blk, intra, cbf_luma, cbf_cb, cbf_cr):
        p = self.pps
        if (cbf_luma or cbf_cb or cbf_cr) and p.cu_qp_delta_enabled and not self.qg_coded:
            a = 0
            while a < 5 and cab.decision("cu_qp_delta_abs", 1 if a else 0):
                a += 1
            if a == 5:
                a += cab.egk(0)
            if a and cab.bypass():
                a = -a
            self.qg_coded = True
            self.qp_y = ((self.qp_pred + a + 52) % 52)
        mode, mode_c = self.cu_intra_modes
        n = 1 << log2
        # luma
        res = self._residual(cab, log2, 0, mode if intra else None) if cbf_luma else None
        tb4 = (slice(y0 >> 2, (y0 + n) >> 2), slice(x0 >> 2, (x0 + n) >> 2))
        self.cbf_map[tb4] = bool(cbf_luma)
        self.edge_v[tb4[0], x0 >> 2] = True
        self.edge_h[y0 >> 2, tb4[1]] = True
        if intra:
            self._intra_predict(x0, y0, log2, 0, mode)
        self._add_residual(self.cur.y, x0, y0, n, res, self.qp_y, log2, dst=intra and log2 == 2)
        b4 = (slice(y0 >> 2, (y0 + n) >> 2), slice(x0 >> 2, (x0 + n) >> 2))
        self.slice_map[b4] = self.slice_addr
        # chroma (4:2:0)
        if log2 > 2:
            xc, yc, lc = x0 // 2, y0 // 2, log2 - 1
        elif blk == 3:
            xc, yc, lc = xb // 2, yb // 2, 2
        else:
            return
        for comp, cbf in ((1, cbf_cb), (2, cbf_cr)):
            r = self._residual(cab, lc, comp, mode_c if intra else None) if cbf else None
            plane = self.cur.u if comp == 1 else self.cur.v
            if intra:
                self._intra_predict(xc, yc, lc, comp, mode_c)
            off = p.cb_qp_offset if comp == 1 else p.cr_qp_offset
            qpi = min(max(self.qp_y + off, 0), 57)
            qpc = qpi if qpi < 30 else (qpi - 6 if qpi > 43 else _QPC_TABLE[qpi])
            self._add_residual(plane, xc, yc, 1 << lc, r, qpc, lc)

    def _add_residual(self, plane, x0, y0, n, levels, qp, log2, dst=False):
        """Scaling (8.6.2/8.6.3) and the inverse transform (8.6.4.2): the DCT-like core transform,
        or for a 4x4 intra luma TU the DST-VII matrix (8.6.4.2 trType 1)."""
        if levels is None:
            return
        d = (levels.astype(np.int64) * 16 * _LEVEL_SCALE[qp % 6]) << (qp // 6)
        bd = 8 + log2 - 5
        d = np.clip((d + (1 << (bd - 1))) >> bd, -32768, 32767)
        t = _DST4 if dst else _tmat(n)
        # d is indexed [y][x] (row = vertical frequency); columns first, then rows
        e = t.T @ d
        g = np.clip((e + 64) >> 7, -32768, 32767)
        r = (g @ t + 2048) >> 12
        plane[y0:y0 + n, x0:x0 + n] = np.clip(plane[y0:y0 + n, x0:x0 + n] + r, 0, 255)

    # ---------------------------------------------------------------- residual_coding (7.3.8.11)
    def _residual(self, cab: Cabac, log2: int, cidx: int, intra_mode):
        n = 1 << log2
        scan_idx = 0
        if intra_mode is not None and (log2 == 2 or (log2 == 3 and cidx == 0)):
            if 6 <= intra_mode <= 14:
                scan_idx = 2
            elif 22 <= intra_mode <= 30:
                scan_idx = 1
        # last significant position
        def prefix(name):
            off = 3 * (log2 - 2) + ((log2 - 1) >> 2) if cidx == 0 else 15
            shift = (log2 + 1) >> 2 if cidx == 0 else log2 - 2
            v = 0
            while v < (log2 << 1) - 1 and cab.decision(name, off + (v >> shift)):
                v += 1
            return v
        px, py = prefix("last_sig_coeff_x_prefix"), prefix("last_sig_coeff_y_prefix")
        def full(pre):
            if pre <= 3:
                return pre
            nb = (pre >> 1) - 1
            return (1 << nb) * (2 + (pre & 1)) + cab.bypass_bits(nb)
        lx = full(px)
        ly = full(py)
        if scan_idx == 2:
            lx, ly = ly, lx
        coef = np.zeros((n, n), np.int64)
        nsb = 1 << (log2 - 2)
        sb_scan = _SCANS[(nsb, scan_idx)]
        pos_scan = _SCANS[(4, scan_idx)]
        # locate the last sub-block / position
        last_sb = nsb * nsb - 1
        last_pos = 16
        while True:
            if last_pos == 0:
                last_pos = 16
                last_sb -= 1
            last_pos -= 1
            xs, ys = sb_scan[last_sb]
            xp, yp = pos_scan[last_pos]
            if (xs << 2) + xp == lx and (ys << 2) + yp == ly:
                break
        csbf = np.zeros((nsb, nsb), np.int32)
        greater1_ctx_prev = None
        for i in range(last_sb, -1, -1):
            xs, ys = sb_scan[i]
            infer_dc = False
            right = csbf[ys, xs + 1] if xs + 1 < nsb else 0
            below = csbf[ys + 1, xs] if ys + 1 < nsb else 0
            if 0 < i < last_sb:
                csbf[ys, xs] = cab.decision("coded_sub_block_flag", min(right + below, 1) + (2 if cidx else 0))
                infer_dc = True
            else:
                csbf[ys, xs] = 1
            sig = [0] * 16
            if i == last_sb:
                sig[last_pos] = 1
            start = last_pos - 1 if i == last_sb else 15
            for nn in range(start, -1, -1):
                xp, yp = pos_scan[nn]
                xc, yc = (xs << 2) + xp, (ys << 2) + yp
                if csbf[ys, xs] and (nn > 0 or not infer_dc):
                    if log2 == 2:
                        sc = _CTX_IDX_MAP_4X4[(yc << 2) + xc]
                    elif xc + yc == 0:
                        sc = 0
                    else:
                        prev = right + 2 * below
                        if prev == 0:
                            sc = 2 if xp + yp == 0 else (1 if xp + yp < 3 else 0)
                        elif prev == 1:
                            sc = 2 if yp == 0 else (1 if yp == 1 else 0)
                        elif prev == 2:
                            sc = 2 if xp == 0 else (1 if xp == 1 else 0)
                        else:
                            sc = 2
                        if cidx == 0:
                            if xs > 0 or ys > 0:
                                sc += 3
                            sc += (9 if scan_idx == 0 else 15) if log2 == 3 else 21
                        else:
                            sc += 9 if log2 == 3 else 12
                    sig[nn] = cab.decision("sig_coeff_flag", sc if cidx == 0 else 27 + sc)
                    if sig[nn]:
                        infer_dc = False
                elif nn == 0 and infer_dc and csbf[ys, xs]:
                    sig[0] = 1
            sig_pos = [nn for nn in range(15, -1, -1) if sig[nn]]
            if not sig_pos:
                continue
            # greater1 / greater2 (9.3.4.2.6 / 9.3.4.2.7)
            ctx_set = 0 if (i == 0 or cidx > 0) else 2
            if greater1_ctx_prev is not None and greater1_ctx_prev == 0:
                ctx_set += 1
            greater1_ctx = 1
            g1 = {}
            first_g1 = None
            for k, nn in enumerate(sig_pos[:8]):
                inc = ctx_set * 4 + min(3, greater1_ctx) + (16 if cidx else 0)
                f = cab.decision("coeff_abs_level_greater1_flag", inc)
                g1[nn] = f
                if f:
                    greater1_ctx = 0
                    if first_g1 is None:
                        first_g1 = nn
                elif greater1_ctx > 0:
                    greater1_ctx += 1
            greater1_ctx_prev = greater1_ctx
            g2 = {}
            if first_g1 is not None:
                g2[first_g1] = cab.decision("coeff_abs_level_greater2_flag", ctx_set + (4 if cidx else 0))
            signs = {nn: cab.bypass() for nn in sig_pos}
            num_sig = 0
            rice = 0
            for nn in sig_pos:
                base = 1 + g1.get(nn, 0) + g2.get(nn, 0)
                thr = (3 if nn == first_g1 else 2) if num_sig < 8 else 1
                level = base
                if base == thr:
                    # coeff_abs_level_remaining (9.3.3.11)
                    pre = 0
                    while pre < 4 and cab.bypass():
                        pre += 1
                    if pre < 4:
                        rem = (pre << rice) + cab.bypass_bits(rice)
                    else:
                        rem = (4 << rice) + cab.egk(rice + 1)
                    level = base + rem
                    if level > 3 * (1 << rice):
                        rice = min(rice + 1, 4)
                xp, yp = pos_scan[nn]
                coef[(ys << 2) + yp, (xs << 2) + xp] = -level if signs[nn] else level
                num_sig += 1
        return coef

    # ---------------------------------------------------------------- intra prediction (8.4.4.2)
    def _intra_predict(self, x0: int, y0: int, log2: int, cidx: int, mode: int) -> None:
        s = self.sps
        n = 1 << log2
        plane = self.cur.y if cidx == 0 else (self.cur.u if cidx == 1 else self.cur.v)
        sub = 0 if cidx == 0 else 1
        xl, yl = x0 << sub, y0 << sub  # luma location of the block
        # reference samples p[x][y] for x = -1, y = -1..2n-1 and y = -1, x = 0..2n-1
        coords = [(-1, y) for y in range(2 * n - 1, -2, -1)] + [(x, -1) for x in range(0, 2 * n)]
        vals, avail = [], []
        for (x, y) in coords:
            xn, yn = x0 + x, y0 + y
            ok = self._avail(xl, yl, xn << sub, yn << sub)
            if ok and self.pps.constrained_intra_pred and not self.pred_intra[(yn << sub) >> 2, (xn << sub) >> 2]:
                ok = False
            avail.append(ok)
            vals.append(int(plane[yn, xn]) if ok else 0)
        if not any(avail):
            vals = [128] * len(vals)
        else:
            if not avail[0]:
                for k in range(1, len(vals)):
                    if avail[k]:
                        vals[0] = vals[k]
                        break
            for k in range(1, len(vals)):
                if not avail[k]:
                    vals[k] = vals[k - 1]
        pl = {}  # (x, y) -> value
        for (x, y), v in zip(coords, vals):
            pl[(x, y)] = v
        # filtering (8.4.4.2.3)
        if cidx == 0 and mode != 1 and n != 4:
            min_dist = min(abs(mode - 26), abs(mode - 10))
            thres = {8: 7, 16: 1, 32: 0}[n]
            if min_dist > thres:
                if s.strong_intra_smoothing and n == 32:
                    raise NotImplementedError("strong intra smoothing")
                f = dict(pl)
                f[(-1, -1)] = (pl[(-1, 0)] + 2 * pl[(-1, -1)] + pl[(0, -1)] + 2) >> 2
                for y in range(0, 2 * n - 1):
                    f[(-1, y)] = (pl[(-1, y + 1)] + 2 * pl[(-1, y)] + pl[(-1, y - 1)] + 2) >> 2
                for x in range(0, 2 * n - 1):
                    f[(x, -1)] = (pl[(x - 1, -1)] + 2 * pl[(x, -1)] + pl[(x + 1, -1)] + 2) >> 2
                pl = f
        pred = np.zeros((n, n), np.int64)
        if mode == 0:
            for y in range(n):
                for x in range(n):
                    pred[y, x] = ((n - 1 - x) * pl[(-1, y)] + (x + 1) * pl[(n, -1)] + (n - 1 - y) * pl[(x, -1)]
                                  + (y + 1) * pl[(-1, n)] + n) >> (log2 + 1)
        elif mode == 1:
            dc = (sum(pl[(x, -1)] for x in range(n)) + sum(pl[(-1, y)] for y in range(n)) + n) >> (log2 + 1)
            pred[:, :] = dc
            if cidx == 0 and n < 32:
                pred[0, 0] = (pl[(-1, 0)] + 2 * dc + pl[(0, -1)] + 2) >> 2
                for x in range(1, n):
                    pred[0, x] = (pl[(x, -1)] + 3 * dc + 2) >> 2
                for y in range(1, n):
                    pred[y, 0] = (pl[(-1, y)] + 3 * dc + 2) >> 2
        else:
            ang = _INTRA_ANGLE[mode]
            ref = {}
            if mode >= 18:
                for x in range(0, n + 1):
                    ref[x] = pl[(-1 + x, -1)]
                if ang < 0:
                    if (n * ang) >> 5 < -1:
                        inv = _INV_ANGLE[ang]
                        for x in range((n * ang) >> 5, 0):
                            ref[x] = pl[(-1, -1 + ((x * inv + 128) >> 8))]
                else:
                    for x in range(n + 1, 2 * n + 1):
                        ref[x] = pl[(-1 + x, -1)]
                for y in range(n):
                    idx, fact = ((y + 1) * ang) >> 5, ((y + 1) * ang) & 31
                    for x in range(n):
                        if fact:
                            pred[y, x] = ((32 - fact) * ref[x + idx + 1] + fact * ref[x + idx + 2] + 16) >> 5
                        else:
                            pred[y, x] = ref[x + idx + 1]
                if mode == 26 and cidx == 0 and n < 32:
                    for y in range(n):
                        pred[y, 0] = min(max(pl[(0, -1)] + ((pl[(-1, y)] - pl[(-1, -1)]) >> 1), 0), 255)
            else:
                for x in range(0, n + 1):
                    ref[x] = pl[(-1, -1 + x)]
                if ang < 0:
                    if (n * ang) >> 5 < -1:
                        inv = _INV_ANGLE[ang]
                        for x in range((n * ang) >> 5, 0):
                            ref[x] = pl[(-1 + ((x * inv + 128) >> 8), -1)]
                else:
                    for x in range(n + 1, 2 * n + 1):
                        ref[x] = pl[(-1, -1 + x)]
                for x in range(n):
                    idx, fact = ((x + 1) * ang) >> 5, ((x + 1) * ang) & 31
                    for y in range(n):
                        if fact:
                            pred[y, x] = ((32 - fact) * ref[y + idx + 1] + fact * ref[y + idx + 2] + 16) >> 5
                        else:
                            pred[y, x] = ref[y + idx + 1]
                if mode == 10 and cidx == 0 and n < 32:
                    for x in range(n):
                        pred[0, x] = min(max(pl[(-1, 0)] + ((pl[(x, -1)] - pl[(-1, -1)]) >> 1), 0), 255)
        plane[y0:y0 + n, x0:x0 + n] = pred


def psnr(a: np.ndarray, b: np.ndarray) -> float:
    d = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if d == 0 else float(10 * np.log10(255.0 ** 2 / d))
