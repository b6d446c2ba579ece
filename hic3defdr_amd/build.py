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

# (source, compiler): device TU through hipcc, host-only TUs through g++
NATIVE_SRCS = [('h3d_api.hip', 'hipcc'), ('h3d_alt.hip', 'hipcc'),
               ('h3d_calls.cpp', 'g++')]
HEADERS = ['h3d_special.h', 'h3d_model.h', 'h3d_kernels.h', 'h3d_host.h',
           'h3d_prepare.h', 'h3d_prepare_api.h', 'h3d_errors.h',
           'h3d_ctx.h']


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
    """Compiles each TU to an object (rebuilt only when it or a header is
    newer), then links libh3d.so with hipcc."""
    os.makedirs(os.path.join(LIBDIR, 'obj'), exist_ok=True)
    out = os.path.join(LIBDIR, 'libh3d.so')
    inc = os.path.join(os.path.dirname(PKG), 'include')
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(inc, 'h3d.h')]
    objs = []
    for src, cc in NATIVE_SRCS:
        s = os.path.join(CSRC, src)
        o = os.path.join(LIBDIR, 'obj', src + '.o')
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            if cc == 'hipcc':
                _run([HIPCC, '--offload-arch=%s' % ARCH, '-O3', '-std=c++17',
                      '-fPIC', '-munsafe-fp-atomics', '-I', inc, '-c', '-o', o,
                      s])
            else:
                _run(['g++', '-O2', '-std=c++17', '-fPIC', '-I', inc, '-c',
                      '-o', o, s])
    if force or _stale(out, objs):
        _run([HIPCC, '--offload-arch=%s' % ARCH, '-shared', '-fPIC', '-o', out]
             + objs)
    return out


def build_all(force=False):
    return build_native(force), build_hosttest(force)


if __name__ == '__main__':
    build_all(force='--force' in sys.argv)
