"""stderr progress messages (reference hic3defdr/util/printing.py:5-19)."""
import sys


def eprint(*args, **kwargs):
    if kwargs.pop('skip', False):
        return
    print(*args, file=sys.stderr, **kwargs)
