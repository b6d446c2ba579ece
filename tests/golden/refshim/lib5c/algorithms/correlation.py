def make_pairwise_correlation_matrix_from_counts_matrix(*a, **k):
    pass
