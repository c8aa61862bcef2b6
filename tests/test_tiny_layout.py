"""CPU checks of the tiny phases' LDS addressing (ramcloud_amd/csrc/ramcrc_device.hip,
RAMCRC_TINY_WR and RAMCRC_TINY_LD16): the one-v_perm address of every lookup
equals the table position it must read, the 32 lanes of a half-wave read 32
distinct banks at every lookup instruction, and the fill writes every position
exactly once inside the 128 KiB table.  The formulas are restated from the
kernel source (TwRows, tiny_win_wr, tw_addr, tiny_fill_wr)."""


def perm(s0, s1, sel):
    """v_perm_b32: result byte i = byte sel_i of {s0 (bytes 4-7), s1 (bytes 0-3)};
    0x0C -> 0x00, >= 0x0D -> 0xFF (the codes these kernels use)."""
    src = [(s1 >> (8 * i)) & 0xFF for i in range(4)] + [(s0 >> (8 * i)) & 0xFF for i in range(4)]
    out = 0
    for i in range(4):
        c = (sel >> (8 * i)) & 0xFF
        b = src[c] if c < 8 else (0 if c == 0x0C else 0xFF)
        out |= b << (8 * i)
    return out


def alignbyte(hi, lo, s):
    return ((((hi << 32) | lo) >> (8 * (s & 3))) & 0xFFFFFFFF)


# --- RAMCRC_TINY_WR (the default): lane u holds dwords u, u + 8, u + 16, u + 24
def wr_addr(q, b):
    return ((q >> 6) << 16) | (b << 8) | ((q & 63) << 2)


def test_wr_addresses_and_banks():
    for j in range(4):
        for k in range(4):
            banks = {}
            for lane in range(32):
                gl, g4 = lane & 7, (lane >> 3) & 3
                lr = ((j >> 1) << 16) | (16 * gl + 4 * ((k + g4) & 3))
                for data in (0x03020100, 0xA1B2C3D4, 0xFFFFFFFF):
                    xr = alignbyte(data, data, g4)
                    a = perm(xr, lr, 0x0C020000 | ((4 + k) << 8)) + 128 * (j & 1)
                    kk = (k + g4) & 3
                    q = 32 * j + 4 * gl + kk
                    assert a == wr_addr(q, (data >> (8 * kk)) & 0xFF)
                banks.setdefault((a >> 2) & 31, []).append(lane)
            assert len(banks) == 32, (j, k, banks)


# --- RAMCRC_TINY_LD16: lane u holds window bytes 16 u .. 16 u + 15
def ld16_addr(q, b):
    return (((q & 3) >> 1) << 16) | (b << 8) | ((q & 1) << 7) | ((q >> 2) << 2)


def test_ld16_addresses_and_banks():
    for j in range(4):
        for k in range(4):
            banks = set()
            sel = 0x0C000000 | (0x00020000 if k >> 1 else 0x000C0000) | ((4 + k) << 8) | (k & 1)
            for lane in range(32):
                gl, g4 = lane & 7, (lane >> 3) & 3
                o = 16 * gl + 4 * ((j + g4) & 3)
                P = 0x00010000 | ((o | 128) << 8) | o
                for data in (0x03020100, 0xA1B2C3D4, 0xFFFFFFFF):
                    a = perm(data, P, sel)
                    assert a == ld16_addr(o + k, (data >> (8 * k)) & 0xFF)
                    assert a < 128 * 1024
                banks.add((a >> 2) & 31)
            assert len(banks) == 32, (j, k)


def test_ld16_fill_covers_table_once():
    seen = {}
    for i in range(4 * 256 * 8):
        kk, b, c = i >> 11, (i >> 3) & 255, i & 7
        base = ld16_addr(16 * c + kk, b)
        for r in range(4):   # the chunk's four words: rows 4 c + r, position 4 (4 c + r) + kk
            q = 4 * (4 * c + r) + kk
            addr = base + 4 * r
            assert addr == ld16_addr(q, b)
            assert addr not in seen
            seen[addr] = (q, b)
    assert len(seen) == 128 * 256 and max(seen) < 128 * 1024


def test_ld16_dword_rotation():
    # instruction j of group g4 takes dword (j + g4) & 3 (two cndmask levels)
    for g4 in range(4):
        w = [10, 11, 12, 13]
        b0, b1 = g4 & 1, g4 & 2
        t = [w[1], w[2], w[3], w[0]] if b0 else w
        ws = [t[2], t[3], t[0], t[1]] if b1 else t
        assert ws == [w[(j + g4) & 3] for j in range(4)]
