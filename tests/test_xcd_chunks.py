"""The XCD-interleaved chunk map of K1t and the K2b scan (csrc/spatial.hip xcd_chunk_block,
k1t_xcb / k1t_grid and the scan's device-side chunk size): restated here, it must be a bijection
from the launched blocks onto the logical blocks, so every tile (wave) is processed exactly once
whatever the grid, chunk count or XCD placement.  Host arithmetic only (no GPU)."""
import pytest


def ceil_div(a, b):
    return (a + b - 1) // b


def chunk_block(b, xcb):  # xcd_chunk_block
    if xcb <= 0:
        return b
    j, x = b >> 3, b & 7
    q, o = j // xcb, j % xcb
    return ((q << 3) + x) * xcb + o


def k1t_xcb(ntiles, m):
    return max(1, ceil_div(ceil_div(ntiles, 4), 8 * m)) if m > 0 else 0


def k1t_grid(ntiles, xcb):
    g = ceil_div(ntiles, 4)
    return ceil_div(g, 8 * xcb) * 8 * xcb if xcb > 0 else g


@pytest.mark.parametrize("ntiles", [1, 3, 4, 5, 63, 64, 65, 1000, 15625, 31251])
@pytest.mark.parametrize("m", [0, 1, 3, 8, 16])
def test_k1t_map_covers_every_tile_once(ntiles, m):
    xcb = k1t_xcb(ntiles, m)
    grid = k1t_grid(ntiles, xcb)
    seen = [chunk_block(b, xcb) for b in range(grid)]
    assert sorted(seen) == list(range(grid))  # a bijection on the launched blocks
    tiles = sorted(t for L in seen for t in range(4 * L, 4 * L + 4) if t < ntiles)
    assert tiles == list(range(ntiles))


@pytest.mark.parametrize("max_waves", [4, 100, 2048, 15625])
@pytest.mark.parametrize("nw", [0, 1, 5, 64, 257, 2048])
@pytest.mark.parametrize("xm", [0, 1, 8])
def test_scan_map_covers_every_wave_once(max_waves, nw, xm):
    if nw > max_waves:
        pytest.skip("the scan never has more waves than its worst case")
    grid = ceil_div(max_waves, 4) + 8 * xm  # the host's scan grid
    waves = []
    for blk in range(grid):
        if xm > 0:
            xcb = max(1, ceil_div(ceil_div(nw, 4), 8 * xm))
            if blk >= 8 * xm * xcb:
                continue
            blk = chunk_block(blk, xcb)
        waves += [t for t in range(4 * blk, 4 * blk + 4) if t < nw]
    assert sorted(waves) == list(range(nw))
