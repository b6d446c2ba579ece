"""libh3d's one-column text reader (h3d_read_text_column, load_bias's bias
files; reference core.py:35-60 reads them with np.loadtxt) against
np.loadtxt: the same doubles bit for bit, and None (the caller's np.loadtxt)
for anything that is not one decimal number per line. Host code only."""
import glob
import os

import numpy as np
import pytest

from hic3defdr_amd import _native

HERE = os.path.dirname(os.path.abspath(__file__))


def _same(a, b):
    a, b = np.atleast_1d(a), np.atleast_1d(b)
    return a.shape == b.shape and np.array_equal(a.view(np.int64),
                                                 b.view(np.int64))


def test_golden_bias_files_bit_for_bit():
    files = sorted(glob.glob(os.path.join(HERE, 'golden', 'data', '*', '*',
                                          '*.bias')))
    assert files
    for f in files:
        assert _same(_native.read_text_column(f), np.loadtxt(f)), f


def test_savetxt_values_and_specials(tmp_path):
    v = np.random.default_rng(1).lognormal(sigma=3, size=20000)
    v[[3, 5, 8]] = [np.nan, np.inf, -0.0]
    v[100:110] = np.random.default_rng(2).uniform(-1e-300, 1e300, 10)
    f = str(tmp_path / 'x.bias')
    for fmt in ('%.18e', '%r', '%.6g'):
        np.savetxt(f, v, fmt=fmt if fmt != '%r' else '%s')
        assert _same(_native.read_text_column(f), np.loadtxt(f)), fmt


def test_comments_blank_lines_whitespace(tmp_path):
    f = str(tmp_path / 'x.bias')
    with open(f, 'w') as fh:
        fh.write('# header\n1.5  # trailing\n\n\t 2e-3 \r\n-inf\nnan\n')
    assert _same(_native.read_text_column(f), np.loadtxt(f))


@pytest.mark.parametrize('text', ['1 2\n', '0x10\n', '1.5abc\n', 'foo\n'])
def test_other_files_left_to_loadtxt(tmp_path, text):
    f = str(tmp_path / 'x.bias')
    with open(f, 'w') as fh:
        fh.write(text)
    assert _native.read_text_column(f) is None


def test_missing_and_empty(tmp_path):
    assert _native.read_text_column(str(tmp_path / 'none.bias')) is None
    f = str(tmp_path / 'e.bias')
    open(f, 'w').close()
    assert _native.read_text_column(f).shape == (0,)
