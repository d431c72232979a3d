from . import dicl  # noqa: F401
