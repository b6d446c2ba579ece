"""In-tree build of the native libraries (no cmake; plain hipcc / g++).

- ``libh3d.so``          the product: C-ABI host code + gfx950 HIP kernels
                          (csrc/h3d_api.hip), loaded by hic3defdr_amd._native.
- ``libh3d_hosttest.so`` the device numerics compiled for the host, used only
                          by CPU unit tests (tests/test_special_host.py).

Both land in ``hic3defdr_amd/lib/`` so they travel to the GPU box with the
repo snapshot (they are git-ignored, not gpurun-ignored).
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, 'csrc')
LIBDIR = os.path.join(PKG, 'lib')
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')
HIPCC = os.path.join(ROCM, 'bin', 'hipcc')
ARCH = os.environ.get('H3D_OFFLOAD_ARCH', 'gfx950')

NATIVE_SRCS = ['h3d_api.hip']
HEADERS = ['h3d_special.h', 'h3d_model.h', 'h3d_kernels.h', 'h3d_host.h',
           'h3d_prepare.h', 'h3d_prepare_api.h']


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd):
    print('[h3d build]', ' '.join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)


def build_hosttest(force=False):
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, 'libh3d_hosttest.so')
    src = os.path.join(CSRC, 'h3d_hosttest.cpp')
    deps = [src] + [os.path.join(CSRC, h) for h in HEADERS]
    if force or _stale(out, deps):
        _run(['g++', '-O2', '-std=c++17', '-shared', '-fPIC',
              '-ffp-contract=off', '-o', out, src])
    return out


def build_native(force=False):
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, 'libh3d.so')
    srcs = [os.path.join(CSRC, s) for s in NATIVE_SRCS]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(os.path.dirname(PKG), 'include', 'h3d.h')]
    if force or _stale(out, deps):
        _run([HIPCC, '--offload-arch=%s' % ARCH, '-O3', '-std=c++17',
              '-shared', '-fPIC', '-munsafe-fp-atomics',
              '-I', os.path.join(os.path.dirname(PKG), 'include'),
              '-o', out] + srcs)
    return out


def build_all(force=False):
    return build_native(force), build_hosttest(force)


if __name__ == '__main__':
    build_all(force='--force' in sys.argv)
