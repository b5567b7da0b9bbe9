"""The dropout mask generator restated in the oracle (kernels.h mix32 / drop_site /
drop_keep): keep rate, independence across sites and known answers that pin the function
the HIP kernels implement (the GPU parity tests compare the two end to end)."""
import numpy as np

from oracle import refcpu


def test_keep_rate_and_sites():
    idx = np.arange(1 << 20, dtype=np.uint64)
    for p in (0.1, 0.2, 0.5):
        keep = refcpu.drop_keep(refcpu.drop_site(7, 2, 3, 1), idx, p)
        assert abs(keep.mean() - (1 - p)) < 3e-3
    a = refcpu.drop_keep(refcpu.drop_site(7, 2, 3, 1), idx, 0.5)
    b = refcpu.drop_keep(refcpu.drop_site(7, 2, 4, 1), idx, 0.5)   # another inner step
    c = refcpu.drop_keep(refcpu.drop_site(8, 2, 3, 1), idx, 0.5)   # another meta-step seed
    assert abs((a == b).mean() - 0.5) < 3e-3 and abs((a == c).mean() - 0.5) < 3e-3
    assert refcpu.drop_keep(refcpu.drop_site(7, 1, 0, 0), idx, 0.0).all()


def _mix(x):  # kernels.h mix32 on Python ints (an independent restatement)
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    return x ^ (x >> 16)


def test_known_answers():
    assert int(refcpu._mix32(np.uint64(0))) == 0
    assert int(refcpu._mix32(np.uint64(1))) == _mix(1) == 0x688990C0
    site = refcpu.drop_site(12345, 2, 1, 0)
    assert int(site) == _mix(12345 ^ _mix((2 << 24) ^ (1 << 8))) == 0x47ECF3F3
    keep = refcpu.drop_keep(site, np.arange(16, dtype=np.uint64), 0.2)
    assert keep.astype(int).tolist() == [1, 1, 1, 1, 1, 1, 1, 1, 0, 1, 0, 1, 1, 1, 1, 1]
    # 64-bit element indices use the high word too
    big = np.array([(1 << 40) + 5], dtype=np.uint64)
    s2 = refcpu.drop_site(3, 1, 0, 2)
    h = _mix(int(s2) ^ 5 ^ ((256 * 0x9E3779B9) & 0xFFFFFFFF))
    assert bool(refcpu.drop_keep(s2, big, 0.5)[0]) == ((h >> 8) >= (1 << 23))
