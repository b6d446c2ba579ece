def plotter(fn):
    return fn
