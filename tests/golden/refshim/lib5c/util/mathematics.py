import numpy as np


def gmean(x, pseudocount=1, axis=None):
    return np.exp(np.nanmean(np.log(x + pseudocount), axis=axis)) - pseudocount
