"""Replayable random draws for the sequence fixtures (test infrastructure).

tests/golden/gen_golden.py runs the reference's own modules with their torch.randint /
torch.randn / torch.rand calls (utils/mapper.py:244,331-338, utils/data_sampler.py:52,81,95)
answered by a ``ReplayDraws`` instead of torch's generator; the GPU tests hand the same draws, in
the same call order, to pin_slam_amd's Mapper (``Mapper._randint``) and DataSampler
(``process_frame(draws=...)``).  Nothing has to be recorded: call c of a stream is a function of
(seed, c) alone, built from PCG64 integer output and exact float32 arithmetic, so it is the same
on every machine.

  randint(high, n) -> int64 [n] in [0, high)
  rand(n)          -> float32 [n] in [0, 1), multiples of 2^-24
  randn(n)         -> float32 [n], Irwin-Hall(12) - 6 (zero mean, unit variance, |x| <= 6): the
                      twelve 24-bit uniforms are added one at a time in float32
"""
import numpy as np


class ReplayDraws:
    def __init__(self, seed: int):
        self.seed = int(seed)
        self.calls = 0

    def _gen(self):
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence([self.seed, self.calls])))
        self.calls += 1
        return g

    def randint(self, high: int, n: int) -> np.ndarray:
        return self._gen().integers(0, int(high), size=int(n), dtype=np.int64)

    @staticmethod
    def _u24(g, shape):
        bits = g.integers(0, 1 << 24, size=shape, dtype=np.int64)
        return bits.astype(np.float32) * np.float32(2.0 ** -24)

    def rand(self, n: int) -> np.ndarray:
        return self._u24(self._gen(), (int(n),))

    def randn(self, n: int) -> np.ndarray:
        u = self._u24(self._gen(), (12, int(n)))
        s = u[0].copy()
        for k in range(1, 12):
            s = s + u[k]
        return s - np.float32(6.0)


def mapping_pool(P, n, pool_seed):
    """A training-sample pool around map points P [M,3] f32 for the mapping() fixtures (float32
    arithmetic on ReplayDraws draws, so the GPU test rebuilds it bit for bit): coord = P[i] +
    0.25 randn along z, label = -offset, ts in [0, 10), weight in [0.5, 1.5)."""
    d = ReplayDraws(pool_seed)
    idx = d.randint(P.shape[0], n)
    off = d.randn(n) * np.float32(0.25)
    coord = P[idx].astype(np.float32).copy()
    coord[:, 2] = coord[:, 2] + off
    ts = d.randint(10, n)
    weight = d.rand(n) + np.float32(0.5)
    return coord, (-off).astype(np.float32), ts, weight
