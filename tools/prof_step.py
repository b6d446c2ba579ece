"""Per-launch summary of the last bench step from a rocprofv3 SQLite trace:
python tools/prof_step.py gpurun_out/<dir>/run_results.db"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, duration, grid_x from kernels "
                 "order by start").fetchall()
lrt = [i for i, r in enumerate(rows) if 'k_lrt' in r[0]]
step = rows[lrt[-2] + 1:lrt[-1] + 1]
span = step[-1][2] - step[0][1]
print('kernels in last step', len(step), 'span ms %.3f' % (span / 1e6),
      'busy frac %.3f' % (sum(r[3] for r in step) / span))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    n = r[0].split('(')[0][:60]
    agg[n][0] += 1
    agg[n][1] += r[3] / 1e6
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print('%-60s %4d %8.3f ms' % (k, v[0], v[1]))
for tag in ('k_disp_work<4, 4, 0>', 'k_disp_work<4, 1, 1>'):
    sel = [r for r in step if tag in r[0]]
    if sel:
        print(tag, 'grid', sel[0][4], 'us:', [round(r[3] / 1e3) for r in sel])
