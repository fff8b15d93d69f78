"""Every volume gather of the march stays inside the volume allocation (CPU
check). The byte range each layout's gather reads
(csrc/kernels.hip vol_fetch: the clamped cell (cx, cy, cz) in [0, W] x [0, H]
x [0, D], 8 bytes from the cell's address; LINEAR: 8 single bytes) is
evaluated with the kernel's own address formulas — the 32-bit u24
multiply-add forms where the host selects them (make_params' vol32), the
64-bit forms otherwise — and compared with the allocation volume_begin makes,
for every cell of small ragged volumes and for the extreme cells (the last
brick / column / slab on every axis) of large ones up to the 8192 limit. The
guard build (tests/test_gpu_guard.py) checks the same on the GPU at run time.
"""
import itertools

import pytest

BRICK = 4  # kBrickCells


def u24(x):
    return x & 0xFFFFFF


def mad_u24(a, b, c):  # v_mad_u32_u24: low 24 bits of a and b, 32-bit result
    return (u24(a) * u24(b) + c) & 0xFFFFFFFF


def alloc_bytes(layout, W, H, D):
    """volume_begin_one's allocation (vptmcm.cpp): ncell 8-byte units."""
    if layout == "linear":
        return W * H * D
    if layout == "brick8":
        bw, bh, bd = (W + BRICK) // BRICK, (H + BRICK) // BRICK, (D + BRICK) // BRICK
        return bw * bh * bd * 64 * 8
    if layout == "column4":
        return ((W + 1) * (H + 1) * (D + 2) + 1) // 2 * 8
    return (W + 1) * (H + 1) * (D + 1) * 8


def vol32(layout, W, H, D):
    """make_params' choice of the 32-bit address forms (vptmcm.cpp)."""
    w1, h1, d1 = W + 1, H + 1, D + 1
    if layout == "brick8":
        bw, bh, bd = (w1 + BRICK - 1) // BRICK, (h1 + BRICK - 1) // BRICK, (d1 + BRICK - 1) // BRICK
        return bw * bh * bd * 512 < 2 ** 32 and bd * bh < 2 ** 24
    if layout == "column4":
        return w1 * h1 * (d1 + 1) * 4 < 2 ** 32 and w1 * h1 < 2 ** 24
    return w1 * h1 * d1 * 8 < 2 ** 32 and d1 * h1 < 2 ** 24 and w1 < 2 ** 24


def brick_inner(cx, cy, cz):
    return (cx & 3) | ((cy & 1) << 2) | ((cz & 1) << 3) | ((cy & 2) << 3) | ((cz & 2) << 4)


def gather_end(layout, W, H, D, cx, cy, cz, narrow):
    """One past the last byte the gather of cell (cx, cy, cz) reads."""
    if layout == "brick8":
        BW, BH = (W + 1 + BRICK - 1) // BRICK, (H + 1 + BRICK - 1) // BRICK
        if narrow:
            brick = (u24(mad_u24(cz >> 2, BH, cy >> 2)) * u24(BW) + (cx >> 2)) & 0xFFFFFFFF
            off = ((brick << 9) | (brick_inner(cx, cy, cz) << 3)) & 0xFFFFFFFF
        else:
            brick = ((cz >> 2) * BH + (cy >> 2)) * BW + (cx >> 2)
            off = (brick << 9) | (brick_inner(cx, cy, cz) << 3)
        return off + 8
    if layout == "column4":
        W1, D2 = W + 1, D + 2
        if narrow:
            off = ((u24(mad_u24(cy, W1, cx)) * u24(D2) + cz) << 2) & 0xFFFFFFFF
        else:
            off = ((cy * W1 + cx) * D2 + cz) << 2
        return off + 8
    if layout == "corner8":
        W1, H1 = W + 1, H + 1
        if narrow:
            off = ((u24(mad_u24(cz, H1, cy)) * u24(W1) + cx) << 3) & 0xFFFFFFFF
        else:
            off = ((cz * H1 + cy) * W1 + cx) * 8
        return off + 8
    # LINEAR: x0, x1 = clamp(ix, W-1), clamp(ix+1, W-1); the largest byte index read
    x1, y1, z1 = min(cx, W - 1), min(cy, H - 1), min(cz, D - 1)
    return (z1 * H + y1) * W + x1 + 1


def cells(W, H, D, small):
    if small:
        return itertools.product(range(W + 1), range(H + 1), range(D + 1))
    ax = lambda n: sorted(c for c in {0, 1, 2, 3, 4, n // 2} | set(range(max(0, n - 8), n + 1)) if c <= n)
    return itertools.product(ax(W), ax(H), ax(D))


DIMS = [(1, 1, 1), (2, 3, 5), (7, 3, 2), (37, 29, 23), (48, 48, 48), (64, 1, 64),
        (512, 512, 512), (1024, 1024, 1024), (8192, 8, 8), (8, 8192, 8), (8, 8, 8192),
        (8192, 8192, 1), (2048, 2048, 2048)]


@pytest.mark.parametrize("layout", ["column4", "corner8", "brick8", "linear"])
@pytest.mark.parametrize("dims", DIMS, ids=lambda d: "x".join(map(str, d)))
def test_every_gather_inside_the_volume_allocation(layout, dims):
    W, H, D = dims
    limit = alloc_bytes(layout, W, H, D)
    narrow = layout != "linear" and vol32(layout, W, H, D)
    small = W * H * D <= 64 ** 3
    worst = 0
    for cx, cy, cz in cells(W, H, D, small):
        end = gather_end(layout, W, H, D, cx, cy, cz, narrow)
        if narrow:  # the 32-bit form must equal the exact 64-bit address
            assert end == gather_end(layout, W, H, D, cx, cy, cz, False), (layout, dims, cx, cy, cz)
        worst = max(worst, end)
    assert worst <= limit, (layout, dims, worst, limit)
    if layout in ("corner8", "column4"):
        assert worst == limit or layout == "column4"  # corner8: the last cell ends the array
