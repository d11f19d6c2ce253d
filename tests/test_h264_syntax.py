"""Bit-level H.264 syntax: exp-Golomb, CAVLC residual blocks and transforms, checked
against the independent pure-Python decoder (mxdesk.codec.h264_decoder)."""
import re
from pathlib import Path

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from mxdesk.codec import h264_decoder as D

ROOT = Path(__file__).resolve().parent.parent


def _reader(data: bytes, nbits: int) -> D.BitReader:
    r = D.BitReader(data + b"\x80")  # append a stop bit so more_rbsp_data works
    return r


@pytest.mark.parametrize("k", [0, 1, 2, 3, 6, 7, 254, 255, 65535, 1 << 20])
def test_ue_roundtrip(native, k):
    data, n = native.h264.ue(k)
    r = _reader(data, n)
    assert r.ue() == k
    assert r.pos == n


@pytest.mark.parametrize("v", [0, 1, -1, 2, -2, 100, -100, 4095, -4096])
def test_se_roundtrip(native, v):
    data, n = native.h264.se(v)
    r = _reader(data, n)
    assert r.se() == v
    assert r.pos == n


def _blocks(maxnum):
    level = st.one_of(st.integers(-3, 3), st.integers(-2047, 2047), st.just(0), st.just(0), st.just(0))
    return st.lists(level, min_size=maxnum, max_size=maxnum)


@pytest.mark.parametrize("maxnum,nc", [(16, 0), (16, 1), (16, 2), (16, 3), (16, 5), (16, 9), (15, 0), (15, 4),
                                       (15, 8), (4, -1)])
@settings(max_examples=60, deadline=None)
@given(data=st.data())
def test_cavlc_block_roundtrip(native, maxnum, nc, data):
    coef = data.draw(_blocks(maxnum))
    raw, n = native.h264.cavlc_block(coef, nc)
    r = _reader(raw, n)
    dec = D.Decoder().residual_block(r, nc, maxnum)
    assert dec == coef
    assert r.pos == n


def test_cavlc_dense_large_levels(native):
    rng = np.random.default_rng(7)
    for _ in range(200):
        coef = [int(x) for x in rng.integers(-2047, 2048, 16)]
        raw, n = native.h264.cavlc_block(coef, 0)
        assert D.Decoder().residual_block(_reader(raw, n), 0, 16) == coef


def test_transform_pair(native):
    rng = np.random.default_rng(3)
    for _ in range(50):
        x = rng.integers(-255, 256, 16).astype(np.int32)
        y = native.h264.fdct4x4(x)
        cf = np.array([[1, 1, 1, 1], [2, 1, -1, -2], [1, -1, -1, 1], [1, -2, 2, -1]])
        assert np.array_equal(y.reshape(4, 4), cf @ x.reshape(4, 4) @ cf.T)
        d = rng.integers(-2000, 2000, 16).astype(np.int32)
        assert np.array_equal(native.h264.idct4x4(d).reshape(4, 4), D.Decoder.idct4(d.reshape(4, 4)))


def _parse_cpp_vlcs(text):
    return [(int(c, 16) if c.startswith("0x") else 0, int(n)) for c, n in re.findall(r"\{(0x[0-9a-f]+|0), (\d+)\}", text)]


def test_tables_match_spec_strings():
    """The encoder's (code,len) tables and the decoder's spec bit strings agree and the
    decoder tables are prefix-free codes."""
    src = (ROOT / "csrc/codec/h264_tables.h").read_text()
    body = src[src.index("constexpr Vlc kCoeffToken[5][16][4]"): src.index("// total_zeros for 4x4")]
    ents = _parse_cpp_vlcs(body)
    assert len(ents) == 5 * 16 * 4
    for cls in range(5):
        for tc in range(1, 17):
            for t1 in range(4):
                code, ln = ents[(cls * 16 + tc - 1) * 4 + t1]
                py = D._CT_SRC.get((t1, tc), [None] * 5)[cls]
                if ln == 0:
                    assert py is None
                else:
                    assert format(code, f"0{ln}b") == py, (cls, t1, tc)
    for tab in D.COEFF_TOKEN + [dict.fromkeys(t) for t in D.TOTAL_ZEROS + D.TOTAL_ZEROS_DC + D.RUN_BEFORE]:
        codes = list(tab)
        assert not any(a != b and b.startswith(a) for a in codes for b in codes)
        assert sum(2.0 ** -len(c) for c in codes) <= 1.0
    assert sorted(D.CBP_INTER) == list(range(48)) and sorted(D.CBP_INTRA) == list(range(48))


def test_luma_qpel_matches_decoder(native):
    rng = np.random.default_rng(5)
    plane = rng.integers(0, 256, (24, 24)).astype(np.uint8)
    dec = D.Decoder()
    dec.ref = (plane.astype(np.int32), np.zeros((12, 12), np.int32), np.zeros((12, 12), np.int32))
    for mvx in range(-9, 10):
        for mvy in (-7, -2, 0, 1, 3, 6):
            blk = dec.pred_luma_inter(4, 4, 4, 4, mvx, mvy)
            for y in range(4):
                for x in range(4):
                    assert blk[y, x] == native.h264.luma_qpel(plane, (4 + x) * 4 + mvx, (4 + y) * 4 + mvy)
