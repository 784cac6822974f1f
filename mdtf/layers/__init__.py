from . import tools  # noqa: F401
