"""CPU tests of the mouth-region post-process restatement (oracle/post.py): hand-computed known
answers for cv2.pyrDown / cv2.pyrUp / cv2.resize(INTER_LINEAR) and the blend's algebra.

cv2 is not importable in this image, so these pin the restatement to OpenCV's documented formulas
(reflect-101 borders, [1 4 6 4 1] kernels, 11-bit resize weights); parity against cv2 itself is
unpinned."""
import numpy as np
import pytest

from oracle import post


def test_border_reflect_101():
    assert list(post.bi101(np.arange(-3, 8), 5)) == [3, 2, 1, 0, 1, 2, 3, 4, 3, 2, 1]
    assert list(post.bi101(np.array([-2, -1, 2, 3]), 2)) == [0, 1, 0, 1]
    assert list(post.bi101(np.array([-2, 5]), 1)) == [0, 0]


def test_pyr_down_known_answers():
    assert (post.pyr_down(np.full((8, 6, 3), 77, np.uint8)) == 77).all()
    x = np.zeros((9, 9), np.uint8)
    x[4, 4] = 255
    y = post.pyr_down(x)
    assert y.shape == (5, 5)
    assert y[2, 2] == (255 * 36 + 128) >> 8          # centre weight 6*6
    assert y[1, 2] == (255 * 6 + 128) >> 8           # row weight 1 (dy = 4), column weight 6
    assert y[0, 0] == 0
    # reflect-101 at the border: an impulse at (0, 0) reaches output (0, 0) with weight 6*6 only
    x0 = np.zeros((4, 4), np.uint8)
    x0[0, 0] = 200
    assert post.pyr_down(x0)[0, 0] == (200 * 36 + 128) >> 8
    # x1 at (1, 1): rows -1 -> 1 and 1 both weight 4 -> 8, same for columns -> 64
    x1 = np.zeros((4, 4), np.uint8)
    x1[1, 1] = 100
    assert post.pyr_down(x1)[0, 0] == (100 * 64 + 128) >> 8
    f = post.pyr_down(x.astype(np.float32))
    assert f.dtype == np.float32 and f[2, 2] == np.float32(255 * 36 / 256)
    assert post.pyr_down(np.zeros((1, 1), np.float32)).shape == (1, 1)
    assert post.pyr_down(np.zeros((7, 5), np.uint8)).shape == (4, 3)


def test_pyr_up_known_answers():
    c = post.pyr_up(np.full((3, 4, 3), 5.0, np.float32))
    assert c.shape == (6, 8, 3) and (c == 5.0).all()
    x = np.zeros((3, 3), np.float32)
    x[1, 1] = 64.0
    y = post.pyr_up(x)
    assert y[2, 2] == 36.0 and y[3, 3] == 16.0 and y[2, 3] == 24.0
    assert (post.pyr_up(np.full((1, 1), 3.0, np.float32)) == 3.0).all()
    # right edge (even): s[w-2] + s[w-1]*7, (odd): s[w-1]*8; bottom rows reflect
    r = post.pyr_up(np.array([[0.0, 8.0]], np.float32))
    assert list(r[0]) == [16 / 8.0, 32 / 8.0, 56 / 8.0, 64 / 8.0]


def test_resize_linear_known_answers():
    img = np.arange(16, dtype=np.uint8).reshape(4, 4) * 10
    assert (post.resize_linear(img, (4, 4)) == img).all()
    half = post.resize_linear(img, (2, 2))           # exact 2x2 box average, rounded half up
    box = (img.astype(np.int64).reshape(2, 2, 2, 2).sum((1, 3)) + 2) // 4
    assert (half == box).all()
    up = post.resize_linear(np.array([[0.0, 4.0]], np.float32), (4, 1))
    assert list(up[0]) == [0.0, 1.0, 3.0, 4.0]
    rgb = np.random.default_rng(0).integers(0, 256, (5, 7, 3), dtype=np.uint8)
    out = post.resize_linear(rgb, (11, 9))
    assert out.shape == (9, 11, 3) and out.dtype == np.uint8
    # per channel == the single-channel resize
    assert (out[..., 1] == post.resize_linear(np.ascontiguousarray(rgb[..., 1]), (11, 9))).all()


@pytest.mark.parametrize("levels", [1, 3, 6])
def test_blend_algebra(levels):
    rng = np.random.default_rng(levels)
    A = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    B = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    ones, zeros = np.ones((64, 96), np.float32), np.zeros((64, 96), np.float32)
    # pyramid values are multiples of 2^-6 well inside fp32's exact range, so the telescoping
    # Laplacian sum reconstructs the selected image exactly
    assert (post.laplacian_blend(A, B, ones, levels) == A).all()
    assert (post.laplacian_blend(A, B, zeros, levels) == B).all()
    half = post.laplacian_blend(A, B, np.full((64, 96), 0.5, np.float32), levels)
    assert np.abs(half - (A.astype(np.float64) + B) / 2).max() < 1e-3


def test_blend_needs_sizes_divisible_by_the_pyramid():
    # like the reference: cv2.pyrUp doubles, so np.subtract fails on a ragged level
    A = np.zeros((32, 24, 3), np.uint8)
    with pytest.raises(ValueError):
        post.laplacian_blend(A, A, np.zeros((32, 24), np.float32), 6)


def test_mouth_mask_paste_keeps_only_255():
    tmp = np.zeros((512, 512), np.uint8)
    tmp[200:300, 100:400] = 255
    tmp[300:310, 100:400] = 254                      # 254 / 255. stored into uint8 -> 0
    full = post.mouth_mask_full(tmp, (360, 640), (40, 296, 100, 356))
    assert full.dtype == np.float32 and set(np.unique(full)) <= {0.0, 1.0}
    assert full[:40].sum() == 0 and full[:, :100].sum() == 0 and full.sum() > 0


def test_img2tensor_and_tenor2mask():
    img = np.array([[[0, 128, 255]]], np.uint8)      # BGR
    t = post.img2tensor(img)
    assert t.shape == (1, 3, 1, 1) and t[0, 0, 0, 0] == np.float32(1.0) and t[0, 2, 0, 0] == np.float32(-1.0)
    logits = np.zeros((1, 19, 2, 2), np.float32)
    logits[0, 11, 0, 0] = 1.0
    logits[0, 3, 1, 1] = 2.0
    m = post.tenor2mask(logits, post.MOUTH_MM)[0]
    assert m.dtype == np.uint8 and m[0, 0] == 255 and m[1, 1] == 0 and m[0, 1] == 0
