"""CPU check of the matcher's fp4 packed-key arithmetic (mageslam_amd/csrc/match.hip,
tile_mfma_fp4 / Keys16): the MX MFMA adds 256 products of +-2^-21 (fp4 +-1 elements, E8M0 scales
2^-11 and 2^-10) to the inline constant 1/(2 pi).  Restated here in float32 with numpy, in every
order the hardware could use (ascending, descending, blockwise by K = 64 instruction), for every
Hamming distance 0..256: each partial sum must be exact and the result's low 16 bits, read as
i16, must be (128 - d - 26) << 6 | 3 -- the key layout Keys16 relies on."""
import numpy as np

C0 = np.float32(0.15915494309189535)  # the 1/(2 pi) inline constant, f32 0x3E22F983
UNIT = np.float32(2.0 ** -21)
FP4_K0 = 26


def accumulate(terms, start):
    acc = np.float32(start)
    for t in terms:
        nxt = np.float32(acc + t)
        # exact: the f32 sum equals the real sum (both operands are multiples of 2^-26 here)
        assert float(nxt) == float(acc) + float(t)
        acc = nxt
    return acc


def low16_i16(x):
    u = int(np.float32(x).view(np.uint32)) & 0xFFFF
    return u - 0x10000 if u >= 0x8000 else u


def test_inline_constant_bits():
    assert int(C0.view(np.uint32)) == 0x3E22F983


def test_fp4_accumulator_keys_exact_for_every_distance():
    rng = np.random.default_rng(7)
    keys = []
    for d in range(257):
        signs = np.ones(256, np.float32)
        signs[rng.permutation(256)[:d]] = -1.0  # d differing bits contribute -1
        terms = signs * UNIT
        results = set()
        # ascending, descending, and four K = 64 blocks each summed first, then chained through C
        results.add(float(accumulate(terms, C0)))
        results.add(float(accumulate(terms[::-1], C0)))
        acc = C0
        for blk in range(4):
            part = accumulate(terms[64 * blk:64 * (blk + 1)], 0.0)
            acc = accumulate([part], acc)
        results.add(float(acc))
        assert len(results) == 1, d
        k = low16_i16(acc)
        assert k == ((128 - d - FP4_K0) << 6) | 3, (d, k)
        # the flush / export decode: (k >> 6) + FP4_K0 = 128 - d
        assert (k >> 6) + FP4_K0 == 128 - d
        keys.append(k)
    # strictly decreasing in d: a larger key is a smaller distance; every key is above NONE
    assert all(a > b for a, b in zip(keys, keys[1:]))
    assert min(keys) > -32768


def test_index_xor_replaces_low_bits():
    # the row / column index (0..63, stored as 63 - index) replaces the constant 3 by one XOR
    for d in (0, 30, 127, 128, 256):
        base = ((128 - d - FP4_K0) << 6) | 3
        for idx in range(64):
            key = base ^ ((63 - idx) ^ 3)
            assert key >> 6 == base >> 6 and key & 63 == 63 - idx
