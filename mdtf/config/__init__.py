from . import annotations, constants, flags  # noqa: F401
from .flags import FLAGS  # noqa: F401
