"""Phase timing of the device smoother (H3D_TABLE_STAMPS) on the golden
full-size cfg2 dispersion table, and its wall time per call."""
import os
import time

import numpy as np
import torch

os.environ.setdefault('H3D_TABLE_STAMPS', '1')
from hic3defdr_amd import _native  # noqa: E402

ctx = _native.context(0)
dpd = np.load(os.path.join(os.path.dirname(__file__), '..', 'tests', 'golden',
                           'full_cfg2.npz'))['disp_per_dist']
dev = torch.device('cuda', 0)
t_in = torch.from_numpy(dpd).to(dev)
t_out = torch.empty_like(t_in)
torch.cuda.synchronize()
D, C = dpd.shape
for i in range(3):
    ctx.disp_tables_dev(t_in.data_ptr(), D, C, t_out.data_ptr())
    ctx.disp_tables_wait()
os.environ.pop('H3D_TABLE_STAMPS')
t = time.perf_counter()
for i in range(20):
    ctx.disp_tables_dev(t_in.data_ptr(), D, C, t_out.data_ptr())
    ctx.disp_tables_wait()
print('device table call: %.1f us' % ((time.perf_counter() - t) / 20 * 1e6))
t = time.perf_counter()
for i in range(20):
    _native.disp_tables(dpd)
print('host tables call: %.1f us' % ((time.perf_counter() - t) / 20 * 1e6))
