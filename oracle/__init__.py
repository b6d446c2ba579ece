"""CPU oracle for the hic3defdr hot path — TEST INFRASTRUCTURE ONLY.

This package is a from-scratch numpy/scipy/pandas restatement of the
reference's ``HiC3DeFDR.run_to_qvalues()`` path (prepare_data ->
estimate_disp -> lrt -> bh). Every function cites the reference file:line it
restates (reference = thomasgilgenast/hic3defdr 0.2.1 at /root/reference).

Who may use it: ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — and only as the checker / the timed CPU
baseline, never as the product path. The product (``hic3defdr_amd``) never
imports this package and fails loudly when its HIP library is missing.

Pinning: the restatement is checked against golden vectors produced by the
reference itself in this container (``tests/golden/make_golden.py``; scipy
1.7.1 / statsmodels 0.12.2 / pandas 2.3.3 under python 3.9, with lib5c
restated by ``tests/golden/refshim``). One deliberate deviation, shared with
the goldens: ``equal_bin`` uses a stable tie order (SURVEY.md finding 4).
"""
from oracle.restatement import *  # noqa: F401,F403
