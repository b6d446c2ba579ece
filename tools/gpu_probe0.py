"""Minimal bring-up probe: prints before every step (diagnostics only)."""
import os
import sys
import time

T0 = time.time()


def log(*a):
    print('[probe0 %.1fs]' % (time.time() - T0), *a, flush=True)


log('start')
import ctypes  # noqa: E402
log('ctypes')
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(REPO, 'hic3defdr_amd', 'lib', 'libh3d.so'))
log('lib loaded')
lib.h3d_open.restype = ctypes.c_void_p
log('device count', lib.h3d_device_count())
h = lib.h3d_open(0)
log('open ->', h)
import numpy  # noqa: E402,F401
log('numpy')
import scipy.special  # noqa: E402,F401
log('scipy')
import pandas  # noqa: E402,F401
log('pandas')
