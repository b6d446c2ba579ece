"""Idle gaps between kernels in a rocprofv3 --kernel-trace CSV, per bench
step (a step starts at the k_iota launch of estimate_disp's sort): kernel
busy time, span, and the gaps longer than a threshold with the kernels on
either side -- where the host holds the GPU up.

    python tools/trace_gaps.py <kernel_trace.csv> [min_gap_us]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    rows = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                    r['Kernel_Name'].split('(')[0].split('<')[0][-40:])
                   for r in csv.DictReader(open(path))), key=lambda t: t[0])
    steps, cur = [], []
    for r in rows:
        if r[2].endswith('k_iota') and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
    steps.append(cur)
    for k, st in enumerate(steps[-4:]):
        busy = sum(e - s for s, e, _ in st) / 1e3
        span = (st[-1][1] - st[0][0]) / 1e3
        gaps = [((b[0] - a[1]) / 1e3, a[2], b[2]) for a, b in zip(st, st[1:])
                if (b[0] - a[1]) / 1e3 > min_gap]
        tot = sum(g for g, _, _ in gaps)
        print('step %d: %d kernels, busy %.3f ms, span %.3f ms, gaps > %g us: '
              '%.3f ms' % (k, len(st), busy / 1e3, span / 1e3, min_gap,
                           tot / 1e3))
        for g, a, b in gaps:
            print('   %8.1f us  %s -> %s' % (g, a, b))


if __name__ == '__main__':
    main()
