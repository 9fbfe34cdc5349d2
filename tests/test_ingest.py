"""Video frame ingest (utilities.py:43-52 cv2_to_tensor; infer_video.py:80): BGR->RGB, INTER_AREA
resize, toTensor255.  cv2 is not installed here, so PARITY WITH cv2 IS UNPINNED: the oracle
restates OpenCV's area-average definition (oracle.resize_area) and the HIP kernel is held to it
exactly, except for outputs within 1e-3 of a rounding tie (cvRound's half-to-even against cv2's
vectorised fast paths is itself ambiguous there), which may differ by one level."""
import numpy as np
import pytest
import torch

from oracle import mhada_oracle as O


def _frame(seed, H, W):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, size=(H, W, 3), dtype=np.uint8)


def test_oracle_resize_area_definition():
    img = _frame(1, 12, 18)
    # integer factor: plain box mean
    got = O.resize_area(img, 6, 4)
    ref = img.astype(np.float64).reshape(4, 3, 6, 3, 3).mean(axis=(1, 3))
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)
    # same size: identity; fractional factor: weights sum to one, means stay in range
    np.testing.assert_array_equal(O.resize_area(img, 18, 12), img.astype(np.float64))
    frac = O.resize_area(img, 7, 5)
    assert frac.shape == (5, 7, 3) and frac.min() >= 0 and frac.max() <= 255
    # a constant image stays constant under any area resize
    const = np.full((13, 17, 3), 77, np.uint8)
    np.testing.assert_allclose(O.resize_area(const, 5, 4), 77.0, atol=1e-12)
    # cv2_to_tensor: BGR -> RGB, CHW, float32 values of the u8 levels
    t = O.cv2_to_tensor(img)
    assert t.shape == (3, 12, 18) and t.dtype == np.float32
    np.testing.assert_array_equal(t[0], img[..., 2].astype(np.float32))


def test_oracle_resize_area_up_definition():
    """INTER_AREA enlarging (OpenCV's area-mode 2-tap path, oracle.resize_area_up): an integer
    factor replicates pixels (area-mode weights are 0/1 there), a constant image stays constant,
    and values stay between the neighbouring source levels."""
    img = _frame(3, 5, 7)
    up = O.resize_area_up(img, 14, 10)
    np.testing.assert_array_equal(up, img.repeat(2, axis=0).repeat(2, axis=1))
    const = np.full((6, 9, 3), 200, np.uint8)
    np.testing.assert_array_equal(O.resize_area_up(const, 20, 13), 200)
    frac = O.resize_area_up(img, 11, 8).astype(int)
    assert frac.shape == (8, 11, 3) and frac.min() >= int(img.min()) and frac.max() <= int(img.max())
    mixed = O.resize_area_up(img, 3, 9)  # width shrinks, height grows: same generic path
    assert mixed.shape == (9, 3, 3)
    t = O.cv2_to_tensor(img, resize=(14, 10))
    np.testing.assert_array_equal(t[0], up[..., 2].astype(np.float32))


def _check_against_oracle(frame, resize, got):
    rgb = frame[..., ::-1]
    if resize is not None and (resize[0] > frame.shape[1] or resize[1] > frame.shape[0]):
        np.testing.assert_array_equal(got, O.cv2_to_tensor(frame, resize))  # integer path: bit-exact
        return
    if resize is None:
        ref = O.cv2_to_tensor(frame)
        np.testing.assert_array_equal(got, ref)  # exact, bit for bit (both fp32 /255 *255)
        return
    mean = O.resize_area(rgb, *resize).transpose(2, 0, 1)
    ref = np.rint(mean)
    tie = np.abs(mean - np.floor(mean) - 0.5) < 1e-3
    diff = np.abs(got.astype(np.float64) - ref)
    assert np.all(diff[~tie] == 0), float(diff[~tie].max())
    assert np.all(diff[tie] <= 1)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,resize", [(1080, 1920, None), (1080, 1920, (512, 256)), (1080, 1920, (960, 540)),
                                        (37, 53, (20, 11)), (64, 64, (64, 64)), (7, 5, (1, 1)),
                                        (240, 320, (512, 256)), (37, 53, (100, 41)), (5, 7, (14, 10)),
                                        (40, 100, (60, 90))])
def test_frame_ingest_matches_oracle(H, W, resize):
    from mhada_hip import video
    frame = _frame(H * W, H, W)
    got = video.cv2_to_tensor(frame, resize=resize).cpu().numpy()
    h, w = (H, W) if resize is None else (resize[1], resize[0])
    assert got.shape == (3, h, w) and got.dtype == np.float32
    _check_against_oracle(frame, resize, got)


@pytest.mark.gpu
def test_frame_ingest_batched_padded_rows_and_errors():
    from mhada_hip import ops
    frames = torch.from_numpy(np.stack([_frame(s, 30, 40) for s in range(3)]))
    padded = torch.zeros(3, 30, 48, 3, dtype=torch.uint8)
    padded[:, :, :40] = frames
    dev = padded.cuda()[:, :, :40]  # rows of 48*3 bytes, 40 pixels used
    out = ops.frame_ingest(dev, (15, 20), bgr=True).cpu().numpy()
    for i in range(3):
        _check_against_oracle(frames[i].numpy(), (20, 15), out[i])
    keep = ops.frame_ingest(dev, None, bgr=False).cpu().numpy()  # RGB order kept
    np.testing.assert_array_equal(keep[1, 0], frames[1, :, :, 0].numpy().astype(np.float32))
    up = ops.frame_ingest(dev, (60, 80), bgr=True).cpu().numpy()  # enlarging: area-mode 2-tap path
    for i in range(3):
        _check_against_oracle(frames[i].numpy(), (80, 60), up[i])
    with pytest.raises(ValueError):
        ops.frame_ingest(dev.float(), None)
