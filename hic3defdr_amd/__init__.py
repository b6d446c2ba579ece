"""hic3defdr_amd — MI355X-native drop-in for hic3defdr's run_to_qvalues() path.

``HiC3DeFDR`` keeps the reference's class surface (constructor kwargs,
prepare_data / estimate_disp / lrt / bh / run_to_qvalues, load / load_data /
save_data / load_disp_fn) and its outdir file contract; the per-pixel
numerics run in hand-written gfx950 kernels behind the C ABI of libh3d.so
(include/h3d.h), bound with ctypes in ``hic3defdr_amd._native``.
"""
from hic3defdr_amd.analysis.constructor import HiC3DeFDR  # noqa: F401

__version__ = '0.1.0'
