"""ssseg: MI355X-native kernels behind the reference's Python API (see include/ssseg.h)."""
from . import native  # noqa: F401
