"""VP8 boolean encoder (csrc/codec/vp8_encoder.h BoolEncoder: mask-selected update, whole-shift
normalisation into a 64-bit low end, deferred byte emission) against the one-bit-at-a-time
encoder of RFC 6386 section 7.3, written out here in Python, over random, skewed and
carry-heavy streams."""
import numpy as np
import pytest


def rfc_bool_encode(probs, bits) -> bytes:
    out = bytearray()
    rng, bottom, bit_count = 255, 0, 24

    def add_one():
        i = len(out) - 1
        while i >= 0 and out[i] == 255:
            out[i] = 0
            i -= 1
        out[i] += 1

    def put(prob, bit):
        nonlocal rng, bottom, bit_count
        split = 1 + (((rng - 1) * prob) >> 8)
        if bit:
            bottom += split
            rng -= split
        else:
            rng = split
        while rng < 128:
            rng <<= 1
            if bottom & (1 << 31):
                add_one()
            bottom = (bottom << 1) & 0xFFFFFFFF
            bit_count -= 1
            if bit_count == 0:
                out.append((bottom >> 24) & 0xFF)
                bottom &= (1 << 24) - 1
                bit_count = 8

    for p, b in zip(probs, bits):
        put(int(p), int(b))
    for _ in range(32):  # flush
        put(128, 0)
    return bytes(out)


@pytest.mark.parametrize("mode", ["random", "skewed", "ones", "follow"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bool_encoder_matches_rfc(native, mode, seed):
    rs = np.random.default_rng(seed)
    n = int(rs.integers(1, 4000))
    if mode == "random":
        probs = rs.integers(1, 256, n)
        bits = rs.integers(0, 2, n)
    elif mode == "skewed":  # extreme probabilities, both outcomes
        probs = np.where(rs.integers(0, 2, n) == 1, 1, 255)
        bits = rs.integers(0, 2, n)
    elif mode == "ones":  # long runs of the likely-one branch: carries through 0xff bytes
        probs = rs.integers(1, 8, n)
        bits = np.ones(n, np.int64)
    else:  # bits drawn from the stated probability (the coder's real regime)
        probs = rs.integers(1, 256, n)
        bits = (rs.integers(0, 256, n) >= probs).astype(np.int64)
    got = native.vp8_bool_encode(probs.astype(np.int32), bits.astype(np.int32))
    assert got == rfc_bool_encode(probs, bits)
