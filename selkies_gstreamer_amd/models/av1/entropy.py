"""AV1 symbol decoder written from the AV1 specification's decoding process
(section 8.2: init_symbol, read_symbol, read_bool / read_literal, the CDF update
rule) -- the independent oracle for the native multi-symbol encoder
(csrc/codec/av1_ec.h). It shares no code with the encoder: the spec keeps the
decoder state as a complemented window (SymbolValue) read most significant bit
first, the encoder keeps a carry-propagating low end.
"""
from __future__ import annotations

EC_PROB_SHIFT = 6
EC_MIN_PROB = 4


def floor_log2(x: int) -> int:
    return x.bit_length() - 1


def update_cdf(cdf: list, n: int, symbol: int) -> None:
    rate = 3 + (cdf[n] > 15) + (cdf[n] > 31) + min(floor_log2(n), 2)
    tmp = 0
    for i in range(n - 1):
        tmp = (1 << 15) if i == symbol else tmp
        if tmp < cdf[i]:
            cdf[i] -= (cdf[i] - tmp) >> rate
        else:
            cdf[i] += (tmp - cdf[i]) >> rate
    cdf[n] += cdf[n] < 32


class SymbolDecoder:
    def __init__(self, data: bytes):
        self.data = data
        self.bitpos = 0
        sz = len(data)
        num_bits = min(sz * 8, 15)
        buf = self._f(num_bits)
        padded = buf << (15 - num_bits)
        self.value = ((1 << 15) - 1) ^ padded
        self.range = 1 << 15
        self.max_bits = 8 * sz - 15

    def _f(self, n: int) -> int:
        v = 0
        for _ in range(n):
            byte = self.data[self.bitpos >> 3] if (self.bitpos >> 3) < len(self.data) else 0
            v = (v << 1) | ((byte >> (7 - (self.bitpos & 7))) & 1)
            self.bitpos += 1
        return v

    def read_symbol(self, cdf: list, n: int, adapt: bool = True) -> int:
        cur = self.range
        symbol = -1
        while True:
            symbol += 1
            prev = cur
            f = (1 << 15) - cdf[symbol]
            cur = ((self.range >> 8) * (f >> EC_PROB_SHIFT) >> (7 - EC_PROB_SHIFT)) + EC_MIN_PROB * (n - symbol - 1)
            if self.value >= cur:
                break
        self.range = prev - cur
        self.value -= cur
        bits = 15 - floor_log2(self.range)
        self.range <<= bits
        num_bits = min(bits, max(0, self.max_bits))
        new_data = self._f(num_bits)
        padded = new_data << (bits - num_bits)
        self.value = padded ^ (((self.value + 1) << bits) - 1)
        self.max_bits -= bits
        if adapt:
            update_cdf(cdf, n, symbol)
        return symbol

    def read_bool(self) -> int:
        return self.read_symbol([1 << 14, 1 << 15, 0], 2, adapt=False)

    def read_literal(self, n: int) -> int:
        x = 0
        for _ in range(n):
            x = 2 * x + self.read_bool()
        return x

    def exit_ok(self) -> bool:
        """Spec exit_symbol: the padding after the last symbol is consistent
        (trailing bits beyond the data are zero) -- checked loosely here as
        'the decoder never needed more than the data plus its 15-bit window'."""
        return self.max_bits >= -15
