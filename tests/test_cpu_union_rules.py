"""Host-side rules of the union-staged conv kernels (``csrc/kernels/conv3d.hip``: ``k_conv_wgrad_tri``,
``k_conv_fwd_tri``, ``k_conv_fwd_slab``): the union size of a band of output positions (which decides eligibility and the kernel's U) against
an independent Python model of the padded-input rows the three kw taps read, and the launch-choice rules measured in
``profiles/r2_ab_wgrad_tri.txt`` / ``profiles/r2_ab_fwd_tri.txt``.  Runs on the CPU (host functions of the built
extension; skipped when it is not built)."""
import pytest


def _ext():
    from neuroimagedisttraining_amd import ops
    try:
        return ops.ext()
    except Exception as e:  # noqa: BLE001 - extension not built in this environment
        pytest.skip("HIP extension not built: %s" % e)


def _union_rows(B, D, H, W, pad, P, slab=False):
    """Largest number of distinct padded-input rows {b(p) + kw} (``slab``: the whole window b(p) .. b(p) + 2 Wp + 2)
    over the bands of P consecutive output positions."""
    Dp, Hp, Wp = D + 2 * pad, H + 2 * pad, W + 2 * pad
    Do, Ho, Wo = Dp - 2, Hp - 2, Wp - 2
    S, vol = Do * Ho * Wo, Dp * Hp * Wp
    mg = B * S
    best = 0
    for m0 in range(0, mg, P):
        rows = set()
        for m in range(m0, min(m0 + P, mg)):
            n, r = divmod(m, S)
            od, r = divmod(r, Ho * Wo)
            oh, ow = divmod(r, Wo)
            base = n * vol + (od * Hp + oh) * Wp + ow
            rows.update(range(base, base + (2 * Wp + 3 if slab else 3)))
        best = max(best, len(rows))
    return best


@pytest.mark.parametrize("shape", [(16, 19, 23, 19, 0), (3, 19, 23, 19, 0), (16, 17, 21, 17, 2), (16, 5, 7, 5, 1),
                                   (2, 5, 7, 5, 2), (1, 9, 6, 11, 1)])
@pytest.mark.parametrize("P", [64, 256])
def test_union_size_matches_python_model(shape, P):
    m = _ext()
    assert m.conv3d_union_umax(*shape, P) == _union_rows(*shape, P)


def test_union_kernel_choices():
    m = _ext()
    conv2 = (16, 19, 23, 19, 64, 128, 0)        # AlexNet3D conv2 forward / wgrad geometry (B=16)
    conv2_dgrad = (16, 17, 21, 17, 128, 64, 2)  # its data gradient: a pad-2 forward
    conv4 = (16, 5, 7, 5, 192, 192, 1)
    for G in (64, 8, 1):
        assert m.conv3d_wgrad_tri_pick(G, *conv2) == 1          # unpadded wgrad: always
        assert m.conv3d_fwd_tri_ok(*conv2_dgrad) == 1           # supported ...
        assert m.conv3d_fwd_tri_pick(G, *conv2_dgrad) == 0      # ... but not chosen (no consistent gain)
    assert m.conv3d_fwd_tri_pick(64, *conv2) == 1
    # padded wgrad: only with >= 8 K output positions per launch (64 K before the overlapped stage DMA, [ADMA])
    assert m.conv3d_wgrad_tri_pick(64, *conv4) == 1
    assert m.conv3d_wgrad_tri_pick(8, *conv4) == 1              # 22 K positions
    assert m.conv3d_wgrad_tri_pick(1, *conv4) == 0              # 2.8 K positions
    assert m.conv3d_fwd_tri_pick(64, *conv4) == 0               # padded forwards stay on the per-tap kernel
    # split factors stay within the model's bounds and keep >= 8 steps per block
    for G in (64, 8, 1):
        ns = m.conv3d_wgrad_tri_nsplit(G, *conv2)
        assert 1 <= ns <= 64 and 16 * 17 * 21 * 17 // ns >= 512
    # table sizes: one entry per band, 2U + P ints with U a multiple of 8 covering the largest union
    n_bands = -(-16 * 17 * 21 * 17 // 64)
    per = m.conv3d_wgrad_tri_table_size(16, 19, 23, 19, 0) // n_bands
    assert per * n_bands == m.conv3d_wgrad_tri_table_size(16, 19, 23, 19, 0)
    assert (per - 64) % 16 == 0 and (per - 64) // 2 >= m.conv3d_union_umax(16, 19, 23, 19, 0, 64)


@pytest.mark.parametrize("shape", [(16, 19, 23, 19, 0), (16, 17, 21, 17, 2), (5, 10, 12, 11, 1), (16, 8, 14, 20, 1),
                                   (3, 19, 23, 19, 0), (16, 5, 7, 5, 1), (4, 31, 37, 31, 1), (4, 16, 19, 16, 1)])
def test_slab_union_matches_python_model(shape):
    """kd-slab unions: size vs the Python model, and the addressing invariant the kernel relies on — every tap
    (kh, kw) of a position reads union row idx(p) + kh Wp + kw (whole windows make the union contiguous there)."""
    m = _ext()
    B, D, H, W, pad = shape
    um = _union_rows(*shape, 256, slab=True)
    assert m.conv3d_slab_umax(*shape) == um
    assert m.conv3d_fwd_slab_ok(B, D, H, W, 64, 64, pad) == (1 if um <= 416 else 0)      # 64-channel blocks
    assert m.conv3d_fwd_slab_ok(B, D, H, W, 64, 128, pad) == (1 if um <= 384 else 0)     # 128-channel blocks
    Dp, Hp, Wp = D + 2 * pad, H + 2 * pad, W + 2 * pad
    Do, Ho, Wo = Dp - 2, Hp - 2, Wp - 2
    S, vol = Do * Ho * Wo, Dp * Hp * Wp
    for m0 in range(0, B * S, 256):
        bases = []
        for q in range(m0, min(m0 + 256, B * S)):
            n, r = divmod(q, S)
            od, r = divmod(r, Ho * Wo)
            oh, ow = divmod(r, Wo)
            bases.append(n * vol + (od * Hp + oh) * Wp + ow)
        union = sorted({b + e for b in bases for e in range(2 * Wp + 3)})
        pos = {r: i for i, r in enumerate(union)}
        for b in bases:
            for kh in range(3):
                for kw in range(3):
                    assert pos[b + kh * Wp + kw] == pos[b] + kh * Wp + kw


def test_slab_kernel_choice():
    m = _ext()
    conv2 = (16, 19, 23, 19, 64, 128, 0)
    conv2_dgrad = (16, 17, 21, 17, 128, 64, 2)
    for G in (64, 8):
        assert m.conv3d_fwd_slab_ok(*conv2) == 1 and m.conv3d_fwd_slab_ok(*conv2_dgrad) == 1
        assert m.conv3d_fwd_slab_pick(G, *conv2_dgrad) == 1      # padded data gradient: the slab kernel
    assert m.conv3d_fwd_slab_ok(16, 5, 7, 5, 192, 192, 1) == 0   # 5x7x5 bands: unions of ~470 rows
    n_bands = -(-16 * 19 * 23 * 19 // 256)
    assert m.conv3d_fwd_slab_table_size(16, 17, 21, 17, 2) == n_bands * (2 * 384 + 256)


def test_conv2d_slab_choice():
    """2-D 3x3 convs on the slab kernel (D = 1 volumes, pad 1): eligible when every 256-position block lies in one
    sample and the band union fits; picked for 64-channel blocks always and 128-channel blocks from 160 blocks up."""
    m = _ext()
    assert m.conv3d_slab_umax(16, 1, 32, 32, 1) == _union_rows(16, 1, 32, 32, 1, 256, slab=True) == 340
    assert m.conv3d_slab_umax(16, 1, 64, 64, 1) == 396                      # Tiny layer 1: the 416-row variant
    assert m.conv2d_fwd_slab_ok(16, 32, 32, 64, 64) == 1
    assert m.conv2d_fwd_slab_ok(16, 64, 64, 64, 64) == 1
    assert m.conv2d_fwd_slab_ok(16, 64, 64, 128, 128) == 0                  # 416-row unions only for 64-ch blocks
    assert m.conv2d_fwd_slab_ok(16, 8, 8, 256, 256) == 0                    # 64-position samples: blocks straddle
    assert m.conv2d_fwd_slab_ok(16, 16, 16, 256, 256) == 1
    assert m.conv2d_fwd_slab_pick(1, 16, 32, 32, 64, 64) == 1              # 64-channel blocks: any grid
    assert m.conv2d_fwd_slab_pick(4, 16, 16, 16, 128, 128) == 0            # 64 blocks of 128 channels
    assert m.conv2d_fwd_slab_pick(10, 16, 16, 16, 128, 128) == 1           # 160 blocks
    assert m.conv2d_fwd_slab_pick(2, 16, 16, 16, 256, 256) == 0            # 64 blocks
    assert m.conv2d_fwd_slab_pick(10, 16, 16, 16, 256, 256) == 1
    n_bands = 16 * 32 * 32 // 256
    assert m.conv3d_fwd_slab_table_size(16, 1, 32, 32, 1) == n_bands * (2 * 384 + 256)


def test_vol_kernel_rule():
    """Whole-sample union kernel (k_conv_fwd_vol): padded sample <= 448 rows and <= 256 output positions; opt-in."""
    m = _ext()
    assert m.conv3d_fwd_vol_ok(16, 5, 7, 5, 128, 192, 1) == 1      # AlexNet conv3: 7x9x7 = 441 rows, 175 positions
    assert m.conv3d_fwd_vol_ok(16, 5, 7, 5, 192, 128, 1) == 1
    assert m.conv3d_fwd_vol_ok(16, 6, 8, 7, 64, 64, 1) == 0        # 8x10x9 = 720 padded rows
    assert m.conv3d_fwd_vol_ok(16, 5, 7, 5, 96, 128, 1) == 0       # channels not a multiple of 64
    assert m.conv3d_fwd_vol_pick(64, 16, 5, 7, 5, 128, 192, 1) == 0  # off unless NIDT_FWD_VOL=1
