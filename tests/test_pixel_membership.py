"""prepare_data's loop_idx (reference analysis.py:117-125: a Python set
lookup per disp pixel): the masked form (keys over the whole union, masked
once) equals the set lookup over row[mask], col[mask]."""
import numpy as np

from hic3defdr_amd.util.clusters import pixel_membership


def test_masked_membership_equals_set_lookup():
    rng = np.random.default_rng(5)
    n_bins = 3000
    row = np.repeat(np.arange(n_bins), 7).astype(np.int32)
    col = (row + np.tile(np.arange(7), n_bins) * 3).astype(np.int32)
    mask = rng.random(len(row)) < 0.6
    clusters = [rng.integers(0, len(row), 400), rng.integers(0, len(row), 50)]
    cl = [np.stack([row[c], col[c]], 1).astype(np.int64) for c in clusters]
    cl.append(np.array([[n_bins + 5, n_bins + 9]], dtype=np.int64))  # no match
    want_set = set(map(tuple, np.concatenate(cl).tolist()))
    want = np.array([(int(r), int(c)) in want_set
                     for r, c in zip(row[mask], col[mask])])
    got = pixel_membership(row, col, cl, mask=mask)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(
        pixel_membership(row[mask], col[mask], cl), want)
    empty = np.zeros(len(row), dtype=bool)
    assert pixel_membership(row, col, cl, mask=empty).shape == (0,)
    assert pixel_membership(row, col, [], mask=mask).shape == (int(mask.sum()),)
