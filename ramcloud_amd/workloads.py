"""Synthetic inputs for the benchmarks and parity tests (no datasets exist offline).

Shared definitions so that bench.py, the tests and the oracle agree byte for
byte:

* splitmix64 streams: word j of a stream with seed s is
  mix64(s + (j+1) * 0x9E3779B97F4A7C15), stored little-endian
  (SURVEY.md section 8(c)).
* bench segments (BASELINE configs 1/2/4): segment i is the splitmix64 stream
  with seed 0x52414D43 + i, 8 MiB each.
* mixed log entries (config 3): 1,000,000 lengths drawn i.i.d. from
  {100, 1024, 4096} with Zipf s=1 weights 6/11, 3/11, 2/11 using
  numpy.random.default_rng(20251015); entries packed back to back (unaligned
  starts, as in a log); the bytes are the splitmix64 stream with seed
  0x4C4F4745 ("LOGE").
"""
import numpy as np

GAMMA = 0x9E3779B97F4A7C15
MIX1 = 0xBF58476D1CE4E5B9
MIX2 = 0x94D049BB133111EB
SEGMENT_SEED = 0x52414D43
ENTRY_SEED = 0x4C4F4745
ENTRY_RNG_SEED = 20251015
MiB = 1 << 20


def _s64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def _srl(t, k):
    """Logical right shift of an int64 tensor."""
    return (t >> k) & ((1 << (64 - k)) - 1)


def _mix64_torch(z):
    z = (z ^ _srl(z, 30)) * _s64(MIX1)
    z = (z ^ _srl(z, 27)) * _s64(MIX2)
    return z ^ _srl(z, 31)


def splitmix_fill_segments(out_u8, seg_bytes, first_seed, slice_segments=64):
    """Fill a CUDA uint8 tensor laid out as consecutive segments of seg_bytes
    (multiple of 8): segment i gets the splitmix64 stream of seed first_seed + i."""
    import torch

    assert seg_bytes % 8 == 0
    nseg = out_u8.numel() // seg_bytes
    words = seg_bytes // 8
    view = out_u8[: nseg * seg_bytes].view(torch.int64).view(nseg, words)
    j = torch.arange(1, words + 1, dtype=torch.int64, device=out_u8.device) * _s64(GAMMA)
    for s0 in range(0, nseg, slice_segments):
        s1 = min(nseg, s0 + slice_segments)
        seeds = torch.arange(s0, s1, dtype=torch.int64, device=out_u8.device) + first_seed
        z = seeds[:, None] + j[None, :]
        view[s0:s1] = _mix64_torch(z)
    return out_u8


def splitmix_bytes_np(seed, nbytes):
    """Host reference generator (numpy, vectorised) -- same stream as above."""
    words = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(1, words + 1, dtype=np.uint64) * np.uint64(GAMMA))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(MIX1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(MIX2)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()


def entry_lengths(n=1_000_000, seed=ENTRY_RNG_SEED):
    rng = np.random.default_rng(seed)
    sizes = np.array([100, 1024, 4096], dtype=np.uint64)
    p = np.array([6.0, 3.0, 2.0]) / 11.0
    return sizes[rng.choice(3, size=n, p=p)]


def packed_offsets(lengths):
    off = np.zeros(lengths.size, dtype=np.uint64)
    if lengths.size > 1:
        np.cumsum(lengths[:-1], out=off[1:])
    return off
