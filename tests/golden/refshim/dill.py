from cloudpickle import dumps, loads, dump  # noqa: F401
from pickle import load  # noqa: F401
