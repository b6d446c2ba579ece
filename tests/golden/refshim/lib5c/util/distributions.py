def freeze_distribution(dist, mean, var):
    n = mean ** 2 / (var - mean)
    p = mean / var
    return dist(n, p)
