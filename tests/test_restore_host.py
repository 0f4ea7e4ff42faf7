"""GFPGANer restore composition, host side (gfpgan/utils.py:97-143 and facexlib 0.2.5's
FaceRestoreHelper, which is not vendored): the host geometry of s2v_amd.restore against the CPU
restatement (oracle/restore.py) and against closed-form cases.  Parity UNPINNED: neither facexlib
nor OpenCV is importable here, so these check the restatement's own invariants."""
import numpy as np
import pytest

import s2v_import  # noqa: F401
from oracle import restore as OR


def _sim(angle, scale, tx, ty):
    c, s = np.cos(angle) * scale, np.sin(angle) * scale
    return np.array([[c, -s, tx], [s, c, ty]])


def _apply(M, p):
    return p @ M[:, :2].T + M[:, 2]


@pytest.mark.parametrize("M", [_sim(0.0, 1.0, 0, 0), _sim(0.2, 1.7, -40.5, 12.0), _sim(-0.4, 0.6, 300.0, -7.25)])
def test_lmeds_fit_recovers_an_exact_similarity(M):
    from s2v_amd import restore
    src = np.random.default_rng(1).uniform(50, 450, (5, 2)).astype(np.float32)
    dst = _apply(M, src.astype(np.float64))
    got = restore.estimate_affine_partial_2d(src, dst)
    assert np.array_equal(got, OR.estimate_affine_partial_2d(src, dst))
    np.testing.assert_allclose(got, M, rtol=0, atol=2e-4 * max(1.0, np.abs(M).max()))
    assert got[0, 0] == got[1, 1] and got[0, 1] == -got[1, 0]              # 4-DOF (rotation part antisymmetric)


def test_lmeds_fit_drops_an_outlier():
    """One landmark far off the similarity: LMeDS's median ignores it, the inlier test drops it and the
    refinement is the least-squares similarity over the other four."""
    from s2v_amd import restore
    M = _sim(0.3, 1.2, 20.0, -10.0)
    src = np.float32(OR.FFHQ_TEMPLATE_512 * 0.4 + 30.0)
    dst = _apply(M, src.astype(np.float64))
    dst = dst + np.random.default_rng(2).normal(0, 0.3, dst.shape)          # landmark noise
    bad = dst.copy()
    bad[3] += (35.0, -28.0)
    got = restore.estimate_affine_partial_2d(src, bad)
    exp4 = OR._ls_partial(src[[0, 1, 2, 4]], np.float32(bad[[0, 1, 2, 4]]))
    np.testing.assert_allclose(got, exp4, rtol=1e-12, atol=1e-9)
    assert np.array_equal(got, OR.estimate_affine_partial_2d(src, bad))
    allfit = OR._ls_partial(src, np.float32(bad))
    assert np.abs(allfit - exp4).max() > 1e-3                              # the outlier would have moved the fit


def test_lmeds_degenerate_inputs():
    from s2v_amd import restore
    assert restore.estimate_affine_partial_2d(np.zeros((1, 2)), np.zeros((1, 2))) is None
    assert restore.estimate_affine_partial_2d(np.ones((5, 2)), np.zeros((5, 2))) is None


def test_inverse_affine_matches_the_restatement():
    from s2v_amd import restore
    M = _sim(0.7, 0.9, 11.0, -3.0)
    inv = restore.invert_affine_transform(M)
    assert np.array_equal(inv, OR.invert_affine_transform(M))
    np.testing.assert_allclose(_apply(inv, _apply(M, np.array([[3.0, 4.0]]))), [[3.0, 4.0]], atol=1e-12)


def test_center_face_choice():
    from s2v_amd import restore
    dets = [np.array([0, 0, 20, 20, 0.99]), np.array([90, 40, 130, 80, 0.98]), np.array([200, 0, 260, 30, 0.99])]
    for fn in (restore.get_center_face, OR.get_center_face):
        det, idx = fn(dets, 120, 220)
        assert idx == 1 and det is dets[1]


def test_gaussian_taps_follow_opencv_sigma_zero_rules():
    from s2v_amd import restore
    for k in (3, 5, 7, 9, 21, 51):
        got = restore.gaussian_taps_auto(k, "cpu").numpy()
        exp = OR.gaussian_taps_auto(k)
        assert got.dtype == np.float32 and np.array_equal(got, exp), k
        assert abs(float(exp.astype(np.float64).sum()) - 1.0) < 1e-6
    assert np.array_equal(OR.gaussian_taps_auto(5), np.float32([0.0625, 0.25, 0.375, 0.25, 0.0625]))


@pytest.mark.parametrize("k", [0, 2, 3, 4, 9])
def test_erode_restatement_matches_a_direct_window_min(k):
    g = np.random.default_rng(k)
    x = g.random((13, 17)).astype(np.float32)
    got = OR.erode(x, k)
    kk = 3 if k == 0 else k
    a = kk // 2
    exp = np.empty_like(x)
    for y in range(13):
        for xx in range(17):
            exp[y, xx] = x[max(0, y - a): y - a + kk, max(0, xx - a): xx - a + kk].min()
    assert np.array_equal(got, exp)


def test_paste_restatement_keeps_the_frame_outside_the_face():
    """Identity-sized face pasted well inside a frame: pixels the soft mask never reaches are the input,
    the face interior is the restored face."""
    g = np.random.default_rng(3)
    img = g.integers(0, 256, (200, 220, 3), dtype=np.uint8)
    face = g.integers(0, 256, (64, 64, 3), dtype=np.uint8)
    M = _sim(0.0, 1.0, -70.0, -60.0)               # frame (70 + cx, 60 + cy) -> crop (cx, cy)
    inv = OR.invert_affine_transform(M)
    trace = []
    out = OR.paste_faces(img, [face], [inv], (64, 64), trace)
    assert trace[0]["area"] == 63 * 63 and trace[0]["w_edge"] == 3
    assert np.array_equal(out[:50], img[:50]) and np.array_equal(out[:, 145:], img[:, 145:])
    assert np.array_equal(out[80:100, 90:110], face[20:40, 20:40])


def test_largest_face_clips_boxes_to_the_image():
    """A box hanging off the frame loses the area outside it (facexlib get_largest_face)."""
    from s2v_amd import restore
    dets = [np.array([-300, -300, 60, 60, 0.99]), np.array([100, 50, 190, 150, 0.98])]
    for fn in (restore.get_largest_face, OR.get_largest_face):
        det, idx = fn(dets, 200, 220)
        assert idx == 1 and det is dets[1]


def test_edge_boundary_guard():
    """w_edge = int(sqrt(area)) // 20 flips at multiples of 20; near them the paste recomputes the area as
    numpy's pairwise fp32 sum (facexlib's np.sum) instead of trusting the device sum's last bits."""
    from s2v_amd.restore import edge_boundary
    assert edge_boundary(np.float32(3600.0)) and edge_boundary(np.float32(3600.3)) and edge_boundary(np.float32(3599.8))
    assert not edge_boundary(np.float32(3700.0)) and not edge_boundary(np.float32(63 * 63))
    assert not edge_boundary(np.float32(0.0)) and not edge_boundary(np.float32(399.0))
