ls /sys/devices/system/node/ | grep node
for n in /sys/devices/system/node/node*; do echo $n $(cat $n/cpulist); done
python3 - <<'PY'
import os, glob
print('affinity', len(os.sched_getaffinity(0)))
for d in glob.glob('/sys/class/drm/card*/device'):
    try:
        print(d, open(d+'/numa_node').read().strip(), os.path.realpath(d))
    except Exception as e: print(d, e)
PY
cat /sys/fs/cgroup/cpu.max 2>/dev/null
rocm-smi --showtoponuma 2>/dev/null | head -20
