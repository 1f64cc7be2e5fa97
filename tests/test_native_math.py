"""Host-side checks of the integer math the kernels rely on (no GPU).

``FastDiv`` (csrc/common.h): x / d as (mulhi(x, m) + x) >> l with a 33-bit sum, m and l precomputed on
the host.  The kernels use it for the row -> (n, h, w) decomposition of the pooling kernels; it must be
exact for every 32-bit x."""
import random


def _fastdiv(d):
    l = 0
    while (1 << l) < d:
        l += 1
    m = ((1 << 32) * ((1 << l) - d)) // d + 1
    assert m < (1 << 32) or d == 1
    return m & 0xFFFFFFFF, l


def test_fastdiv_exact():
    rng = random.Random(0)
    divisors = list(range(1, 300)) + [3136, 12544, 802816, 65535, 65536, 65537, 2 ** 31 - 1]
    for d in divisors:
        m, l = _fastdiv(d)
        xs = [0, 1, d - 1, d, d + 1, 2 ** 31 - 1, 2 ** 32 - 1] + [rng.randrange(2 ** 32) for _ in range(500)]
        for x in xs:
            assert ((((x * m) >> 32) + x) >> l) == x // d, (d, x)
