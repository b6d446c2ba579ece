cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1
python3 - <<'PY'
import numpy as np, time, os
try:
    from numpy._core.multiarray import _get_madvise_hugepage
    print('numpy madvise hugepage', _get_madvise_hugepage())
except Exception as e: print(e)
for k in range(3):
    t=time.perf_counter(); a=np.empty(2**27); a.fill(1.0); t1=time.perf_counter(); b=np.count_nonzero(a); t2=time.perf_counter()
    print('1 GiB alloc+fill %.1f ms, count %.1f ms' % ((t1-t)*1e3, (t2-t1)*1e3)); del a
t=time.perf_counter(); [os.stat('/tmp') for _ in range(1000)]; print('stat us', (time.perf_counter()-t)*1e3)
print(os.cpu_count(), len(os.sched_getaffinity(0)))
PY
