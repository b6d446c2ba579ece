from statsmodels.nonparametric.smoothers_lowess import lowess as _lowess


def lowess(endog, exog, **kwargs):
    return _lowess(endog, exog, **kwargs)
