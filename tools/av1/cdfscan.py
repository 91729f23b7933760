"""Scan helper: parse a uint16 region of a binary as libaom-style CDF groups
(inverted CDF values strictly decreasing to 0, then a 0 adaptation counter)."""
import sys
import numpy as np

LIB = '/usr/local/lib/python3.10/dist-packages/pillow.libs/libavif-a883386a.so.16.4.1'


def load():
    return open(LIB, 'rb').read()


def groups(b, off, maxbytes):
    a = np.frombuffer(b[off:off + maxbytes], dtype='<u2')
    out = []
    i = 0
    while i < len(a):
        j = i
        # values strictly decreasing, positive, until a 0
        while j < len(a) and a[j] != 0 and (j == i or a[j] < a[j - 1]) and a[j] <= 32768:
            j += 1
        if j < len(a) - 1 and a[j] == 0 and a[j + 1] == 0 and j > i:
            out.append((off + 2 * i, [32768 - int(x) for x in a[i:j]] + [32768]))
            i = j + 2
        else:
            out.append((off + 2 * i, None))
            break
    return out


if __name__ == '__main__':
    b = load()
    off = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    for o, g in groups(b, off, n):
        print(o, len(g) if g else None, g)
