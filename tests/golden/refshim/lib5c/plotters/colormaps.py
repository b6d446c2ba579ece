def get_colormap(*a, **k):
    pass
