import os


def check_outdir(filename):
    d = os.path.dirname(filename)
    if d and not os.path.exists(d):
        os.makedirs(d)
