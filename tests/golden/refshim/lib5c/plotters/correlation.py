def plot_correlation_matrix(*a, **k):
    pass
