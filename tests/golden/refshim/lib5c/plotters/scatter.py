def scatter(*a, **k):
    pass
