"""In-tree build of the native libraries (no cmake; plain hipcc / g++).

- ``libh3d.so``          the product: C-ABI host code + gfx950 HIP kernels
                          (csrc/h3d_api.hip, h3d_alt.hip, h3d_calls.cpp,
                          h3d_npz.cpp; links zlib), loaded
                          by hic3defdr_amd._native.
- ``libh3d_hosttest.so`` the device numerics compiled for the host, used only
                          by CPU unit tests (tests/test_special_host.py).
- ``libh3d_selftest.so`` the same numerics compiled for gfx950 behind the same
                          test ABI, used only by GPU unit tests.
- ``libh3d_peak.so``     bench.py's measured roofline denominators (an FP64
                          FMA-chain kernel and a 16 B/lane copy); measurement
                          only, never loaded by the product.

All land in ``hic3defdr_amd/lib/`` so they travel to the GPU box with the
repo snapshot (they are git-ignored, not gpurun-ignored).

Staleness is decided by CONTENT, not mtimes: every output carries a
``.stamp`` file holding the sha256 of its compile command and of every source
and header it is built from, and is rebuilt whenever that digest changes. A
binary copied from another tree (or a stale one whose sources were edited
with an older mtime) is therefore never silently reused.
"""
import concurrent.futures
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, 'csrc')
LIBDIR = os.path.join(PKG, 'lib')
INC = os.path.join(os.path.dirname(PKG), 'include')
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')
HIPCC = os.path.join(ROCM, 'bin', 'hipcc')
ARCH = os.environ.get('H3D_OFFLOAD_ARCH', 'gfx950')

# (source, compiler): device TUs through hipcc, host-only TUs through g++
NATIVE_SRCS = [('h3d_api.hip', 'hipcc'), ('h3d_lrt.hip', 'hipcc'),
               ('h3d_prepare_api.hip', 'hipcc'), ('h3d_alt.hip', 'hipcc'),
               ('h3d_bh.hip', 'hipcc'), ('h3d_table.hip', 'hipcc'),
               ('h3d_calls.cpp', 'g++'), ('h3d_npz.cpp', 'g++')]
HEADERS = ['h3d_special.h', 'h3d_model.h', 'h3d_kernels.h', 'h3d_host.h',
           'h3d_prepare.h', 'h3d_errors.h', 'h3d_ctx.h', 'h3d_lrt_group.h', 'h3d_logtab.h']
# concurrent compiles (each hipcc TU is single-threaded; the box sets
# MAX_JOBS=16, this container has 8 CPUs)
JOBS = max(1, min(int(os.environ.get('MAX_JOBS', '8')), os.cpu_count() or 1))
HIP_FLAGS = ['--offload-arch=%s' % ARCH, '-O3', '-std=c++17', '-fPIC',
             '-munsafe-fp-atomics']


def _digest(cmd, deps):
    h = hashlib.sha256(' '.join(cmd).encode())
    for d in sorted(deps):
        if os.path.exists(d):
            h.update(d.encode())
            with open(d, 'rb') as fh:
                h.update(fh.read())
    return h.hexdigest()


def _fresh(target, digest):
    try:
        with open(target + '.stamp') as fh:
            return os.path.exists(target) and fh.read().strip() == digest
    except OSError:
        return False


def _run(cmd, target, digest):
    print('[h3d build]', ' '.join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    with open(target + '.stamp', 'w') as fh:
        fh.write(digest + '\n')


def _build(target, cmd, deps, force):
    dig = _digest(cmd, deps)
    if force or not _fresh(target, dig):
        _run(cmd, target, dig)
    return target


def _headers():
    return [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(INC, 'h3d.h')]


def build_hosttest(force=False):
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, 'libh3d_hosttest.so')
    src = os.path.join(CSRC, 'h3d_hosttest.cpp')
    cmd = ['g++', '-O2', '-std=c++17', '-shared', '-fPIC',
           '-ffp-contract=off', '-o', out, src]
    return _build(out, cmd, [src] + _headers(), force)


def build_selftest(force=False):
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, 'libh3d_selftest.so')
    src = os.path.join(CSRC, 'h3d_selftest.hip')
    cmd = [HIPCC] + HIP_FLAGS + ['-shared', '-o', out, src]
    return _build(out, cmd, [src] + _headers(), force)


def build_peak(force=False):
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, 'libh3d_peak.so')
    src = os.path.join(CSRC, 'h3d_peak.hip')
    cmd = [HIPCC] + HIP_FLAGS + ['-shared', '-o', out, src]
    return _build(out, cmd, [src], force)


def _native_objects(objdir=None, extra=()):
    """(object, compile command, deps) of every TU of libh3d.so."""
    hdrs = _headers()
    objdir = objdir or os.path.join(LIBDIR, 'obj')
    jobs = []
    for src, cc in NATIVE_SRCS:
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src + '.o')
        if cc == 'hipcc':
            cmd = [HIPCC] + HIP_FLAGS + list(extra) + ['-I', INC, '-c', '-o',
                                                       o, s]
        else:
            cmd = ['g++', '-O2', '-std=c++17', '-fPIC', '-I', INC, '-c', '-o',
                   o, s]
        jobs.append((o, cmd, [s] + hdrs))
    return jobs


def _link_native(force):
    out = os.path.join(LIBDIR, 'libh3d.so')
    objs = [o for o, _, _ in _native_objects()]
    cmd = [HIPCC, '--offload-arch=%s' % ARCH, '-shared', '-fPIC', '-o', out] \
        + objs + ['-lz', '-ldl']
    return _build(out, cmd, objs, force)


def build_native(force=False):
    """Compiles each TU to an object (concurrently), then links libh3d.so
    with hipcc; each step is skipped when its content digest is unchanged."""
    os.makedirs(os.path.join(LIBDIR, 'obj'), exist_ok=True)
    with concurrent.futures.ThreadPoolExecutor(JOBS) as ex:
        for f in [ex.submit(_build, o, c, d, force)
                  for o, c, d in _native_objects()]:
            f.result()
    return _link_native(force)


def build_variant(name, extra=()):
    """A measurement variant of libh3d.so built from the current sources
    with extra hipcc flags (e.g. -DH3D_SECPROF) into
    lib/variants/libh3d_<name>.so (objects under lib/obj_<name>); selected at
    run time by H3D_LIB (tools/ab_lib.sh, tools/secprof.py)."""
    objdir = os.path.join(LIBDIR, 'obj_' + name)
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.join(LIBDIR, 'variants'), exist_ok=True)
    jobs = _native_objects(objdir, extra)
    with concurrent.futures.ThreadPoolExecutor(JOBS) as ex:
        for f in [ex.submit(_build, o, c, d, False) for o, c, d in jobs]:
            f.result()
    out = os.path.join(LIBDIR, 'variants', 'libh3d_%s.so' % name)
    objs = [o for o, _, _ in jobs]
    cmd = [HIPCC, '--offload-arch=%s' % ARCH, '-shared', '-fPIC', '-o', out] \
        + objs + ['-lz', '-ldl']
    return _build(out, cmd, objs, False)


def build_all(force=False):
    """libh3d.so, libh3d_hosttest.so and libh3d_selftest.so; every compile
    step of the three runs concurrently."""
    os.makedirs(os.path.join(LIBDIR, 'obj'), exist_ok=True)
    with concurrent.futures.ThreadPoolExecutor(JOBS) as ex:
        futs = [ex.submit(_build, o, c, d, force)
                for o, c, d in _native_objects()]
        futs += [ex.submit(build_hosttest, force),
                 ex.submit(build_selftest, force),
                 ex.submit(build_peak, force)]
        for f in futs:
            f.result()
    return (_link_native(force), os.path.join(LIBDIR, 'libh3d_hosttest.so'),
            os.path.join(LIBDIR, 'libh3d_selftest.so'))


if __name__ == '__main__':
    build_all(force='--force' in sys.argv)
