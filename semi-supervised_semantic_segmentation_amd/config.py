"""config.fromfile (reference config.py:6-25): import a python config module, return its globals."""
import os
import sys
from importlib import import_module


def fromfile(filename):
    if not os.path.exists(filename):
        raise ValueError('Config path does not exist')
    if not filename.endswith('.py'):
        raise IOError('Only .py type are supported now!')
    module_name = os.path.basename(filename)[:-3]
    if '.' in module_name:
        raise ValueError('Dots are not allowed in config file path.')
    sys.path.insert(0, os.path.dirname(filename))
    try:
        mod = import_module(module_name)
    finally:
        sys.path.pop(0)
    return {k: v for k, v in mod.__dict__.items() if not k.startswith('__')}
