"""The hit mask's bit stream (wcsph_tiled.hip), restated in Python with the kernels' integer arithmetic:
pass 1's writer (a 64-bit shift register of two u32 advanced by v_alignbit, newest bit at bit 0; a word
leaves once 32 are pending, bit-reversed so the oldest candidate lands at bit 0; the last, partial word has
zeros above its bits) and pass 2's reader (64-bit buffer refilled from a queue of words; takes of 0..32 bits; pieces of 16
for the hit loop). Random candidate streams cut into random windows, in the scan's groups of 4 plus a scalar
tail, must come back bit for bit, and a reader skipping planes must stay aligned."""
import numpy as np
import pytest

HM_WORDS = 8
M64 = (1 << 64) - 1


def alignbit(a, b, c):
    """v_alignbit_b32: ({a, b} >> (c & 31))[31:0]"""
    return (((a << 32) | b) >> (c & 31)) & 0xFFFFFFFF


def bitrev32(x):
    return int(f"{x:032b}"[::-1], 2)


def write_mask(windows):
    """The kernel's writer. windows: list of bool arrays (one per window, visit order); the sign bit of
    r² − 4h² is the hit. Returns the HM_WORDS words."""
    mh, ml, mn, mw = 0, 0, 0, 0
    words = [0] * HM_WORDS

    def bit(h):
        nonlocal ml
        d = 0x80000000 if h else 0x3F800000          # r² − 4h² < 0 (sign set) or > 0
        ml = alignbit(ml, d, 31)

    def emit():
        nonlocal mn, mw
        if mn >= 32:
            mn -= 32
            if mw < HM_WORDS:
                words[mw] = bitrev32(alignbit(mh, ml, mn))
            mw += 1

    for w in windows:
        t, ln = 0, len(w)
        while t + 4 <= ln:                      # the 4-wide group
            mh = alignbit(mh, ml, 28)
            for k in range(4):
                bit(w[t + k])
            mn += 4
            emit()
            t += 4
        while t < ln:                           # the scalar tail
            mh = alignbit(mh, ml, 31)
            bit(w[t])
            mn += 1
            emit()
            t += 1
    if mn > 0 and mw < HM_WORDS:
        words[mw] = bitrev32((ml << (32 - mn)) & 0xFFFFFFFF)
    return words


def write_mask_uniform(windows):
    """The kernel's writer since round 3: a window's 4-wide groups store a word after every eighth group
    (the test is wave-uniform: all lanes still scanning are at the same group) with the mn bits pending
    before the scan above it, the bits since the last such store are settled once after the groups, and
    the 0-3 remaining candidates enter as one group (k bits in one 64-bit shift)."""
    mh, ml, mn, mw = 0, 0, 0, 0
    words = [0] * HM_WORDS

    def store(sh):
        nonlocal mw
        if mw < HM_WORDS:
            words[mw] = bitrev32(alignbit(mh, ml, sh))
        mw += 1

    def sign(h):
        return 1 if h else 0

    for w in windows:
        ln = len(w)
        n4 = ln // 4
        for it in range(n4):
            mh = alignbit(mh, ml, 28)
            for k in range(4):
                ml = alignbit(ml, 0x80000000 if w[4 * it + k] else 0x3F800000, 31)
            if it % 8 == 7:
                store(mn)
        pend = mn + 4 * (n4 % 8)
        if pend >= 32:
            store(pend - 32)
        mn = pend & 31
        k = ln % 4
        if k:
            t = 4 * n4
            bits = [sign(w[t + j]) if j < k else 0 for j in range(3)]
            f = (bits[0] << 2 | bits[1] << 1 | bits[2]) >> (3 - k)
            m = (((mh << 32) | ml) << k | f) & M64
            mh, ml = m >> 32, m & 0xFFFFFFFF
            mn += k
            if mn >= 32:
                mn -= 32
                store(mn)
    if mn > 0 and mw < HM_WORDS:
        words[mw] = bitrev32((ml << (32 - mn)) & 0xFFFFFFFF)
    return words


def write_mask_plain(windows):
    """The stream's definition (oldest bit first, 32 to a word, zeros past the end) with a 64-bit
    register that takes the newest bit at bit 63 (the round-2 writer before v_alignbit)."""
    mb, mn, mw = 0, 0, 0
    words = [0] * HM_WORDS

    def bit(h):
        nonlocal mb
        mb = ((mb >> 1) | ((1 << 63) if h else 0)) & M64

    def emit():
        nonlocal mb, mn, mw
        if mn >= 32:
            if mw < HM_WORDS:
                words[mw] = (mb >> (64 - mn)) & 0xFFFFFFFF
            mw += 1
            mn -= 32

    for w in windows:
        t, ln = 0, len(w)
        while t + 4 <= ln:                      # the 4-wide group
            for k in range(4):
                bit(w[t + k])
            mn += 4
            emit()
            t += 4
        while t < ln:                           # the scalar tail
            bit(w[t])
            mn += 1
            emit()
            t += 1
    if mn > 0 and mw < HM_WORDS:
        words[mw] = (mb >> (64 - mn)) & ((1 << mn) - 1)
    return words


class Reader:
    def __init__(self, words):
        self.q = list(words)
        self.rb = self.q[0] | (self.q[1] << 32)
        self.rn = 64

    def take(self, ln):
        assert 0 <= ln <= 32
        v = self.rb & (0xFFFFFFFF if ln >= 32 else (1 << ln) - 1)
        self.rb >>= ln
        self.rn -= ln
        if self.rn <= 32:
            self.rb |= self.q[2] << self.rn
            self.rn += 32
            self.q[2:] = self.q[3:] + [0]
        return v

    def hits(self, ln):                          # 16 candidates at a time, as the hit loop
        out = []
        off = 0
        while off < ln:
            m = self.take(min(16, ln - off))
            while m:
                t = (m & -m).bit_length() - 1
                out.append(off + t)
                m &= m - 1
            off += 16
        return out

    def skip(self, ln):
        off = 0
        while off < ln:
            self.take(min(32, ln - off))
            off += 32


def _windows(rng, total):
    """random window lengths (0..60) summing to total, as 3 planes of 3 rows"""
    cuts = np.sort(rng.integers(0, total + 1, 8))
    lens = np.diff(np.concatenate([[0], cuts, [total]]))
    return [rng.random(int(n)) < 0.3 for n in lens]


@pytest.mark.parametrize("total", [0, 1, 5, 31, 32, 33, 180, 241, 255, 256])
def test_round_trip(total):
    rng = np.random.default_rng(total)
    for _ in range(50):
        wins = _windows(rng, total)
        words = write_mask(wins)
        r = Reader(words)
        for w in wins:
            assert r.hits(len(w)) == [int(i) for i in np.flatnonzero(w)]


def test_skip_keeps_alignment():
    """a plane scanned by distance passes over its bits; the next plane's bits are still in place"""
    rng = np.random.default_rng(7)
    for _ in range(100):
        wins = _windows(rng, 240)
        words = write_mask(wins)
        r = Reader(words)
        for p in range(3):
            plane = wins[3 * p: 3 * p + 3]
            if p == 1:
                r.skip(sum(len(w) for w in plane))
                continue
            for w in plane:
                assert r.hits(len(w)) == [int(i) for i in np.flatnonzero(w)]


@pytest.mark.parametrize("total", [0, 3, 32, 35, 100, 255, 256, 300])
def test_alignbit_writer_equals_plain_definition(total):
    rng = np.random.default_rng(100 + total)
    for _ in range(50):
        wins = _windows(rng, total)
        assert write_mask(wins) == write_mask_plain(wins)


def test_budget_words_beyond_256_are_not_written():
    wins = [np.ones(300, bool)]
    words = write_mask(wins)
    assert words == [0xFFFFFFFF] * HM_WORDS


@pytest.mark.parametrize("total", [0, 3, 32, 35, 100, 255, 256, 300])
def test_uniform_store_writer_equals_plain_definition(total):
    """the round-3 schedule (wave-uniform stores every eighth group, grouped tail) writes the same words"""
    rng = np.random.default_rng(200 + total)
    for _ in range(50):
        wins = _windows(rng, total)
        assert write_mask_uniform(wins) == write_mask_plain(wins)
    long = [rng.random(n) < 0.3 for n in (37, 70, 5, 0, 64, 33)]   # windows of more than eight groups
    assert write_mask_uniform(long) == write_mask_plain(long)
