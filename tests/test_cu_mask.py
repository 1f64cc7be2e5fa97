"""The CU mask of the weight-gradient side stream (ops/_hip/streams.py IMGCLS_WGRAD_CU_FRAC): k of every 8 CUs
of each XCD, whether the driver numbers CUs XCD-major or XCD-interleaved."""
import pytest

from pytorch_imageclassification_distributed_amd.ops._hip.streams import cu_mask_words


def _on(words, i):
    return (words[i // 32] >> (i % 32)) & 1


@pytest.mark.parametrize("frac,k", [(1.0, 8), (0.875, 7), (0.75, 6), (0.5, 4), (0.1, 1)])
def test_cu_mask_words_per_xcd(frac, k):
    n = 256  # MI355X: 8 XCDs x 32 CUs
    w = cu_mask_words(n, frac)
    assert len(w) == 8 and all(0 <= x < 2 ** 32 for x in w)
    assert sum(_on(w, i) for i in range(n)) == 32 * k
    for xcd in range(8):
        assert sum(_on(w, i) for i in range(n) if i // 32 == xcd) == 4 * k  # XCD-major numbering
        assert sum(_on(w, i) for i in range(n) if i % 8 == xcd) == 4 * k  # XCD-interleaved numbering


def test_cu_mask_words_partial_word():
    w = cu_mask_words(40, 0.5)
    assert len(w) == 2 and w[1] < 2 ** 8
