"""Host threads on the NUMA node of the process's GPU.

One process drives one GPU; its host work (the NPZ inflate, the union
staging, the device-to-host result copies into pageable memory and the
outdir writes) moves hundreds of MB per chromosome through host memory.
On a two-socket host a process left to the scheduler may run on, and
first-touch its pages on, the socket far from its GPU. ``bind(device)``
restricts every thread of the process (the existing ones and, by
inheritance, the ones created later) to the CPUs of the GPU's node, within
the affinity the process was given. Opt-in for library users
(``H3D_NUMA_BIND=1``); ``bench.py`` binds by default (cfg2 through the
class, r06x, three interleaved processes each: run_to_qvalues 0.11-0.12 s
bound against 0.15-0.16 s unbound, estimate_disp 9-25 ms against 34-37).
"""
import os


def _cpulist(text):
    cpus = set()
    for part in text.strip().split(','):
        if not part:
            continue
        if '-' in part:
            a, b = part.split('-')
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def gpu_node(device=0):
    """NUMA node of torch device ``device`` from its PCI address, or None
    (no sysfs entry, a single-node host, no device)."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device)
        bdf = '%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id,
                                    p.pci_device_id)
        with open('/sys/bus/pci/devices/%s/numa_node' % bdf) as fh:
            node = int(fh.read().strip())
    except (ImportError, RuntimeError, AttributeError, OSError, ValueError):
        return None
    return node if node >= 0 else None


def node_cpus(node):
    try:
        with open('/sys/devices/system/node/node%d/cpulist' % node) as fh:
            return _cpulist(fh.read())
    except OSError:
        return set()


def bind(device=0):
    """Binds every thread of this process to the CPUs of ``device``'s NUMA
    node (intersected with the current affinity). Returns {'node', 'cpus'}
    or None when there is nothing to bind to."""
    node = gpu_node(device)
    if node is None:
        return None
    allowed = os.sched_getaffinity(0)
    cpus = node_cpus(node) & allowed
    if not cpus or cpus == allowed:
        return None
    # sched_setaffinity(0) sets the calling thread only: every existing
    # thread of the process in turn, later threads inherit
    for tid in os.listdir('/proc/self/task'):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:
            pass
    return {'node': node, 'cpus': len(cpus)}


def maybe_bind(device=0, default=False):
    """bind(device) when H3D_NUMA_BIND=1 (unset: ``default``)."""
    env = os.environ.get('H3D_NUMA_BIND')
    if env == '1' or (env is None and default):
        return bind(device)
    return None
