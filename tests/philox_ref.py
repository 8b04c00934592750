"""Host (numpy) reference of beekern's counter-based uniform streams
(csrc/kernels/bk_philox.hpp + random.hip): Philox4x32-10 and the numpy-style
53-bit / 24-bit uniform constructions, vectorised over counters."""

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
TAG_F64, TAG_F32 = 0x62656B65, 0x62656B66
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32 with 10 rounds (Salmon et al., SC'11; Random123 layout) on
    uint32 arrays; returns the four output words as uint32 arrays."""
    x = [np.asarray(c, dtype=np.uint64) & _MASK for c in (c0, c1, c2, c3)]
    for _ in range(10):
        p0 = M0 * x[0]
        p1 = M1 * x[2]
        x = [((p1 >> np.uint64(32)) ^ x[1] ^ np.uint64(k0)) & _MASK, p1 & _MASK,
             ((p0 >> np.uint64(32)) ^ x[3] ^ np.uint64(k1)) & _MASK, p0 & _MASK]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return [v.astype(np.uint32) for v in x]


def uniform_f64(n: int, seed: int, offset: int = 0, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    """What bk_rand_uniform(dtype=f64) writes: counter p -> elements 2p, 2p+1."""
    pairs = (n + 1) // 2
    ctr = np.arange(offset, offset + pairs, dtype=np.uint64)
    r = philox4x32_10(ctr & _MASK, ctr >> np.uint64(32), np.full(pairs, TAG_F64), np.zeros(pairs), seed & 0xFFFFFFFF,
                      (seed >> 32) & 0xFFFFFFFF)

    def u53(a, b):
        return ((a >> 5).astype(np.float64) * 67108864.0 + (b >> 6).astype(np.float64)) * (1.0 / 9007199254740992.0)

    out = np.empty(2 * pairs)
    out[0::2] = lo + (hi - lo) * u53(r[0], r[1])
    out[1::2] = lo + (hi - lo) * u53(r[2], r[3])
    return out[:n]


def uniform_f32(n: int, seed: int, offset: int = 0, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    """What bk_rand_uniform(dtype=f32) writes: counter q -> elements 4q..4q+3,
    computed in f32 like the kernel (lo + span * u24)."""
    quads = (n + 3) // 4
    ctr = np.arange(offset, offset + quads, dtype=np.uint64)
    r = philox4x32_10(ctr & _MASK, ctr >> np.uint64(32), np.full(quads, TAG_F32), np.zeros(quads), seed & 0xFFFFFFFF,
                      (seed >> 32) & 0xFFFFFFFF)
    lo32, span = np.float32(lo), np.float32(hi - lo)
    out = np.empty(4 * quads, dtype=np.float32)
    for j in range(4):
        u = (r[j] >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)
        out[j::4] = lo32 + span * u
    return out[:n]
